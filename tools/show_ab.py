#!/usr/bin/env python3
"""Print value / scan ms / frac for every bench JSON of an ab_env.sh run."""
import json, sys
from pathlib import Path
d = Path(sys.argv[1])
idx = {}
if (d / "index.txt").exists():
    for l in (d / "index.txt").read_text().splitlines():
        k, _, v = l.partition(": ")
        idx[k] = v
for f in sorted(d.glob("bench*.json")):
    lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
    if not lines:
        print(f.name, "NO OUTPUT"); continue
    j = json.loads(lines[-1]); r = j.get("roofline", {})
    tag = idx.get(f.stem.rsplit("_", 1)[-1], "")
    print(f"{f.name:28s} {j['value']:>12.1f} {r.get('kernel_ms_avg', 0):>9.3f} ms frac {r.get('frac', 0):.4f}  {tag}")
