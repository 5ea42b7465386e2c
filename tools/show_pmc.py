#!/usr/bin/env python3
"""Summarise a tools/ab_pmc.sh run: per variant the bench value and scan ms,
the scan kernel's L2 hit rate, HBM-side bytes (2 x FETCH_SIZE, gfx950), MFMA
busy fraction, wave-state fractions and effective clock (medians per launch)."""
import csv, json, statistics, sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
kern = sys.argv[2] if len(sys.argv) > 2 else "k_scan_"
idx = dict(l.split(": ", 1) if ": " in l else (l.rstrip(":"), "") for l in (d / "index.txt").read_text().splitlines())


def pmc(sub):
    f = d / sub / "run_counter_collection.csv"
    agg, dur = defaultdict(list), []
    if not f.exists():
        return {}
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in agg.items()}


for i in sorted(idx, key=int):
    bj = d / f"{next(iter(sorted(d.glob(f'bench_*_{i}.json'))), Path('x')).name}"
    line = [l for l in bj.read_text().splitlines() if l.startswith("{")] if bj.exists() else []
    j = json.loads(line[-1]) if line else {}
    r = j.get("roofline", {})
    c = {**pmc(f"tcc_{i}"), **pmc(f"fetch_{i}"), **pmc(f"sq_{i}")}
    out = {"env": idx[i], "value": j.get("value"), "scan_ms": r.get("kernel_ms_avg"), "frac": r.get("frac")}
    if "TCC_HIT_sum" in c:
        out["l2_hit"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
    if "FETCH_SIZE" in c:
        out["hbm_GB"] = round(2 * c["FETCH_SIZE"] * 1024 / 1e9, 1)
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        out.update(wait=round(c["SQ_WAIT_ANY"] / w, 3), stall=round(c["SQ_WAIT_INST_ANY"] / w, 3),
                   active=round(c["SQ_ACTIVE_INST_ANY"] / w, 3))
        if "GRBM_GUI_ACTIVE" in c and r.get("kernel_ms_avg"):
            per_xcd = c["GRBM_GUI_ACTIVE"] / 8
            out["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / per_xcd, 3)
    print(json.dumps(out))
