#!/usr/bin/env python3
"""ISA of k_scan_v4's epilogue-pad variants, side by side.

Compiles fx_scan.hip for gfx950 (device only, -O3, the product flags) with
explicit instances of one scan shape at ablation bits 0 (product: one
accumulator wait-state pad), 2048 (no pad) and 8192 (two pads), and prints per
instance: VGPR / AGPR / SGPR counts, scratch, and the instruction mix of the
whole kernel and of its tile loop (the block between the loop header and its
back edge).  The three instances differ only in the epilogue's s_nop pad, so
any other difference is the compiler's doing.
usage: tools/isa_pad_diff.py [DT METRIC KSTEPS]   (default 2 1 12: fp16 L2 d=384, config (e))
"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "rag-faiss-embedding_amd" / "csrc"
dt, metric, ks = (sys.argv[1:4] if len(sys.argv) >= 4 else ("2", "1", "12"))
ABLS = [("pad (product)", 0), ("no pad", 2048), ("two pads", 8192)]

src = f'#include "{CSRC}/fx_scan.hip"\n' + "".join(
    f"template __global__ void fx::k_scan_v4<{dt}, {metric}, {ks}, {a}, 1>(fx::ScanParams);\n" for _, a in ABLS)
tmp = Path(tempfile.mkdtemp(prefix="fx_isa_"))
(tmp / "probe.hip").write_text(src)
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DFX_SCAN_DEV", "--cuda-device-only",
       "-S", str(tmp / "probe.hip"), "-o", str(tmp / "probe.s"), "-Rpass-analysis=kernel-resource-usage"]
r = subprocess.run(cmd, capture_output=True, text=True)
if r.returncode:
    sys.exit(r.stderr)
asm = (tmp / "probe.s").read_text()

# resource remarks, in order of the functions in the remark stream
res = collections.defaultdict(dict)
cur = None
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
    for key in ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m2 = re.search(key + r": (\d+)", line)
        if m2 and cur:
            res[cur][key.split(" ")[0]] = int(m2.group(1))


def body(name):
    i = asm.index(name + ":")
    return asm[i:asm.index(".Lfunc_end", i)]


def mix(text):
    ins = [l.strip() for l in text.splitlines()]
    ins = [l for l in ins if l and not l.startswith((";", ".")) and not l.endswith(":")]
    c = collections.Counter(l.split()[0] for l in ins)
    nops = sum(int(l.split()[1]) + 1 for l in ins if l.startswith("s_nop"))
    return len(ins), c, nops


def tile_loop(text):
    """The outer tile loop: from its header label to the last branch back to it."""
    m = re.search(r"^(\.LBB\d+_\d+):[^\n]*=>This Loop Header: Depth=1", text, re.M)
    if not m:
        return ""
    lab = m.group(1)
    end = text.rfind(lab, m.end())
    return text[m.start():text.find("\n", end)]


print(f"k_scan_v4<{dt}, {metric}, {ks}, ABL, 1> on gfx950 (hipcc -O3): {' / '.join(n for n, _ in ABLS)}")
rows = []
for label, a in ABLS:
    name = f"_ZN2fx9k_scan_v4ILi{dt}ELi{metric}ELi{ks}ELi{a}ELi1EEEvNS_10ScanParamsE"
    b = body(name)
    n_all, c_all, nop_all = mix(b)
    n_loop, c_loop, nop_loop = mix(tile_loop(b))
    rows.append((label, res.get(name, {}), n_all, n_loop, c_loop, nop_loop))
keys = ["VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize", "Occupancy"]
print(f"{'':16s}" + "".join(f"{k:>12s}" for k in keys) + f"{'instr':>8s}{'loop':>8s}{'loop s_nop states':>19s}")
for label, rr, n_all, n_loop, _, nop_loop in rows:
    print(f"{label:16s}" + "".join(f"{rr.get(k, -1):12d}" for k in keys) + f"{n_all:8d}{n_loop:8d}{nop_loop:19d}")
ops = sorted(set().union(*(r[4] for r in rows)))
print("tile-loop opcodes whose counts differ between the instances:")
for op in ops:
    v = [r[4].get(op, 0) for r in rows]
    if len(set(v)) > 1:
        print(f"  {op:32s}" + "".join(f"{x:8d}" for x in v))
