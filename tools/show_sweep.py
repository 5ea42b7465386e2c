#!/usr/bin/env python3
"""Table of a tools/sweep_nq.sh run: per config and nq the scan time, the
roofline fraction and the qps."""
import json, sys
from pathlib import Path
d = Path(sys.argv[1])
for f in sorted(d.glob("sweep_*.jsonl")):
    for l in f.read_text().splitlines():
        if not l.startswith("{"):
            continue
        j = json.loads(l)
        r = j["roofline"]
        print(f"{f.stem:18s} nq {j['config']['nq']:6d}  scan {r['kernel_ms_avg']:8.3f} ms  {r['bound']} "
              f"{r['achieved']:9.1f} {r['unit']}  frac {r['frac']:.3f}  qps {j['value']:10.1f}  "
              f"merge+refine {r['merge_refine_ms_avg']:.3f} ms  fb {j['fallback_queries_last_step']}")
