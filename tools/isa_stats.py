#!/usr/bin/env python3
"""Instruction mix of the scan kernels' main loops, from gfx950 assembly.

For every kernel symbol matching a pattern, finds the outermost loop (the
block range from a ";=>This Loop Header" label to the last branch back to it)
and counts instruction classes in it: MFMA, LDS-DMA, other VMEM, LDS reads /
writes, waits, barriers, s_nop, VALU, SALU, AGPR moves.  A cheap way to see
what a source change did to the hot loop before any hardware run.

usage: tools/isa_stats.py file.s [symbol-substring]
    (file.s from: hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S x.hip -o file.s)
"""
import re
import sys
from collections import Counter

CLASSES = [
    ("mfma", re.compile(r"^v_mfma")),
    ("lds_dma", re.compile(r"^(global|buffer)_load_lds")),
    ("vmem", re.compile(r"^(global|buffer|flat)_")),
    ("ds_read", re.compile(r"^ds_read")),
    ("ds_write/atomic", re.compile(r"^ds_")),
    ("s_waitcnt", re.compile(r"^s_waitcnt")),
    ("s_barrier", re.compile(r"^s_barrier")),
    ("s_nop", re.compile(r"^s_nop")),
    ("agpr_move", re.compile(r"^v_accvgpr")),
    ("valu", re.compile(r"^v_")),
    ("salu", re.compile(r"^s_")),
]


def classify(op):
    for name, rx in CLASSES:
        if rx.match(op):
            return name
    return "other"


def functions(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur is not None:
            body.append(ln)
            if ln.strip().startswith("s_endpgm"):
                yield cur, body
                cur, body = None, []


def loop_blocks(body):
    """{root depth-1 loop header: [instruction lines]} from LLVM's block
    annotations ("in Loop: Header=BBx Depth=d", "Parent Loop BBy", "Loop Header")."""
    parent, owner, cur = {}, {}, None
    out = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):\s*;?(.*)$", ln)
        if m:
            name = m.group(1).lstrip(".").replace("; %bb.", "bb")
            note = m.group(2) + (body[i + 1] if i + 1 < len(body) else "")
            h = re.search(r"Header=(BB\w+)", note)
            if "Loop Header" in note:
                cur = name
                pm = re.search(r"Parent Loop (BB\w+)", note)
                if pm:
                    parent[name] = pm.group(1)
            elif h:
                cur = h.group(1)
            else:
                cur = None
            continue
        if cur is None:
            continue
        root = cur
        while root in parent:
            root = parent[root]
        out.setdefault(root, []).append(ln)
    return out


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_scan"
    lines = open(path).read().splitlines()
    for name, body in functions(lines):
        if pat not in name:
            continue
        best = None
        for root, lines_ in loop_blocks(body).items():
            c = Counter()
            for ln in lines_:
                t = ln.split(";")[0].strip()
                if not t or t.endswith(":") or t.startswith("."):
                    continue
                c[classify(t.split()[0])] += 1
            if best is None or c["mfma"] > best[1]["mfma"]:
                best = (root, c)
        if not best:
            continue
        root, c = best
        print(name)
        print(f"  main loop {root}: " + ", ".join(f"{k} {c[k]}" for k, _ in CLASSES + [("other", 0)] if c[k]))


if __name__ == "__main__":
    main()
