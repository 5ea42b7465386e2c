#!/usr/bin/env python3
"""Static check of the two gfx950 hazards that faulted hand-written LDS-DMA
code in this repo ("hardware facts"):

1. an SGPR written by a VALU instruction (v_readlane / v_readfirstlane /
   v_cmp / ...) and then used as the base of a VMEM instruction needs 5 wait
   states; the compiler inserts them for its own loads but not in front of
   inline asm, so a spilled-and-reloaded DMA base can reach the load early;
2. a write of M0 immediately followed by an LDS-DMA load (needs one wait
   state, the asm puts an s_nop 0 there).

Usage: check_dma_hazards.py file.s [kernel-substring]
Parses the device assembly linearly (a hazard across a branch target is
reported too, conservatively) and prints each offending DMA with the
instruction that wrote its base.  Exit status 1 if any hazard is found.
"""
import re
import sys

VMEM_RE = re.compile(r"^\s*(global_load_lds_dword\w*|global_load\w*|global_store\w*|buffer_\w+)\s+(.*)$")
SBASE_RE = re.compile(r"s\[(\d+):(\d+)\]")
VALU_SDST_RE = re.compile(r"^\s*(v_\w+)\s+(s\[(\d+):(\d+)\]|s(\d+)|vcc)\b")
NOP_RE = re.compile(r"^\s*s_nop\s+(\w+)")
M0_WRITE_RE = re.compile(r"^\s*s_\w+\s+m0\b")


def sgprs(tok_lo, tok_hi):
    return set(range(int(tok_lo), int(tok_hi) + 1))


def instructions(lines):
    for no, line in enumerate(lines, 1):
        s = line.split(";")[0].rstrip()
        if not s.strip() or s.strip().startswith(".") or s.rstrip().endswith(":"):
            if s.rstrip().endswith(":"):
                yield no, None  # label
            continue
        yield no, s


def check(path, kernel_filter=""):
    lines = open(path).read().splitlines()
    issues = []
    cur_fn = None
    window = []  # (lineno, text, wait_states_it_provides, written_sgprs, is_m0_write)
    for no, s in instructions(lines):
        if s is None:
            continue
        if re.match(r"^\s*s_endpgm", s):
            window = []
            continue
        # function boundaries: the .type/.globl lines are skipped; detect by symbol labels
        m = VMEM_RE.match(s)
        if m and (kernel_filter == "" or cur_fn is None or kernel_filter in (cur_fn or "")):
            ops = m.group(2)
            sb = SBASE_RE.search(ops)
            if sb:
                base = sgprs(sb.group(1), sb.group(2))
                ws = 0
                for (pno, ptxt, pws, pw, pm0) in reversed(window):
                    if pw & base and ws < 5:
                        issues.append((no, s.strip(), pno, ptxt.strip(), ws))
                        break
                    ws += pws
                    if ws >= 5:
                        break
            if m.group(1).startswith("global_load_lds") and window and window[-1][4]:
                issues.append((no, s.strip(), window[-1][0], window[-1][1].strip(), 0))
        nm = NOP_RE.match(s)
        wsprov = (int(nm.group(1), 0) + 1) if nm else 1
        written = set()
        vm = VALU_SDST_RE.match(s)
        if vm and not vm.group(1).startswith("v_cmpx"):
            if vm.group(3):
                written = sgprs(vm.group(3), vm.group(4))
            elif vm.group(5):
                written = {int(vm.group(5))}
        window.append((no, s, wsprov, written, bool(M0_WRITE_RE.match(s))))
        if len(window) > 16:
            window.pop(0)
    return issues


def main():
    path = sys.argv[1]
    kf = sys.argv[2] if len(sys.argv) > 2 else ""
    issues = check(path, kf)
    for no, dma, pno, prod, ws in issues:
        print(f"{path}:{no}: {dma}\n    <- line {pno}: {prod} ({ws} wait states)")
    print(f"{len(issues)} hazard(s)")
    sys.exit(1 if issues else 0)


if __name__ == "__main__":
    main()
