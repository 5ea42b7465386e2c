#!/usr/bin/env python3
"""Table of a tools/gpu_multi.sh run: per arm the scan ms of each repetition."""
import json, sys
from pathlib import Path
d = Path(sys.argv[1])
arms = [l.split(": ", 1)[1] for l in (d / "arms_1.txt").read_text().splitlines()]
for i, a in enumerate(arms):
    ms = []
    for r in (1, 2):
        f = d / f"arm{i}_{r}.json"
        lines = [l for l in f.read_text().splitlines() if l.startswith("{")] if f.exists() else []
        ms.append(json.loads(lines[-1])["roofline"]["kernel_ms_avg"] if lines else float("nan"))
    print(f"{i}: {ms[0]:8.2f} {ms[1]:8.2f}  {a}")
