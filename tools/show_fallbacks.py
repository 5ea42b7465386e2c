#!/usr/bin/env python3
"""Fallback counts of every line of a tools/gpu_multi.sh run (a scan change
that breaks the pruning thresholds shows as uncertified queries)."""
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
for f in sorted(d.glob("arm*_*.json")):
    lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
    if lines:
        j = json.loads(lines[-1])
        print(f.name, "fallbacks", j.get("fallback_queries_last_step"), "dropped", j.get("dropped_candidate_ids_last_step"),
              "scan_ms", j["roofline"]["kernel_ms_avg"])
