#!/usr/bin/env python3
"""Table of a tools/gpu_multi.sh run: per arm the scan ms (main scan kernel,
HIP events) and the whole search's ms per step of each repetition."""
import json, sys
from pathlib import Path
d = Path(sys.argv[1])
arms = [l.split(": ", 1)[1] for l in (d / "arms_1.txt").read_text().splitlines()]
for i, a in enumerate(arms):
    ms, st = [], []
    for r in (1, 2):
        f = d / f"arm{i}_{r}.json"
        lines = [l for l in f.read_text().splitlines() if l.startswith("{")] if f.exists() else []
        j = json.loads(lines[-1]) if lines else None
        ms.append(j["roofline"]["kernel_ms_avg"] if j else float("nan"))
        st.append(j["ms_per_step"] if j else float("nan"))
    print(f"{i}: scan {ms[0]:8.3f} {ms[1]:8.3f}  step {st[0]:8.3f} {st[1]:8.3f}  {a}")
