#!/usr/bin/env python3
"""Turn a tools/profile_scan.sh output directory into committed evidence:

  profiles/<round>_<tag>_kernel_stats.csv   rocprofv3 --stats summary (verbatim)
  profiles/<round>_<tag>_summary.json       per-kernel averages + PMC per launch
  profiles/pmc_scan_<tag>.json              HBM bytes per scan launch (read by
                                            bench.py for roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream, so it
is doubled; Infinity-Cache (MALL) hits are counted in it, not excluded.
usage: tools/summarize_profile.py <prof_dir> <tag> <round> <rows_per_gpu> <nq>
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SCAN = os.environ.get("FX_PROFILE_KERNEL", "k_scan_")  # k_scan_v4 / k_scan_q32
# fx_scan.hip RESCAN / SEED: the re-scan's and the threshold-seeding scan's own instances
OTHER_MARKS = (", 4096,", "Li4096E", ", 8192,", "Li8192E")


def is_scan(name):
    """The main scan's launches, not the re-scan of uncertified queries or the
    threshold-seeding scan."""
    return SCAN in name and not any(m in name for m in OTHER_MARKS)


def counters(path, grid=None):
    """Per kernel name, per counter: the values of every dispatch (only the
    dispatches of grid size `grid` when given)."""
    agg = defaultdict(lambda: defaultdict(list))
    if not path.exists():
        return agg
    with open(path) as f:
        for r in csv.DictReader(f):
            if grid is not None and "Grid_Size" in r and int(float(r["Grid_Size"])) != grid:
                continue
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main_grid(trace, scan_name):
    """The scan's grid size that holds the most kernel time (the bench's own
    launches, not its side legs' one-query searches), and those dispatches'
    mean duration in ms."""
    by = defaultdict(list)
    with open(trace) as f:
        for r in csv.DictReader(f):
            if r["Kernel_Name"] != scan_name:
                continue
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            by[g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    g = max(by, key=lambda k: sum(by[k]))
    return g, statistics.mean(by[g]), len(by[g])


def main():
    prof, tag, rnd, rows, nq = Path(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    out = ROOT / "profiles"
    out.mkdir(exist_ok=True)
    stats = prof / "trace" / "run_kernel_stats.csv"
    shutil.copy(stats, out / f"{rnd}_{tag}_kernel_stats.csv")
    kern = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            kern[r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                               "pct": float(r["Percentage"])}
    scan_name = next(n for n in kern if is_scan(n))
    grid, avg_ms, n = main_grid(prof / "trace" / "run_kernel_trace.csv", scan_name)
    kern[scan_name]["avg_ms_all_launches"] = kern[scan_name]["avg_ms"]
    kern[scan_name]["avg_ms"] = avg_ms
    kern[scan_name]["bench_launches"] = n
    kern[scan_name]["bench_grid_threads"] = grid
    pmc = {}
    for sub in ("fetch", "write", "tcc", "sq", "lds", "ta"):
        for name, cs in counters(prof / sub / "run_counter_collection.csv", grid).items():
            if name == scan_name:
                for c, vals in cs.items():
                    pmc[c] = statistics.median(vals)
    res = {"kernels": kern, "scan_kernel": scan_name, "scan_pmc_median_per_launch": pmc,
           "rows_per_gpu": rows, "nq": nq}
    # provenance: the profiled tree's source digest (profile_scan.sh, on the box)
    # and the commit the summary was made at (here; the digest is the binding key)
    prov = prof / "provenance.json"
    if prov.exists():
        res.update(json.loads(prov.read_text()))
    try:
        import subprocess
        res["git_head_at_summary"] = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short=12", "HEAD"],
                                                    capture_output=True, text=True, check=True).stdout.strip()
    except Exception:  # noqa: BLE001
        pass
    if "FETCH_SIZE" in pmc:
        fetch = pmc["FETCH_SIZE"] * 1024 * 2          # gfx950: FETCH_SIZE = 1/2 of streamed bytes
        write = pmc.get("WRITE_SIZE", 0.0) * 1024
        res["hbm_bytes_per_launch"] = fetch + write
        res["hbm_note"] = ("(2*FETCH_SIZE + WRITE_SIZE) KiB -> bytes; includes Infinity-Cache hits "
                           "(MI355X_MICROARCH.md HBM section)")
    if "TCC_HIT_sum" in pmc:
        res["l2_hit_rate"] = pmc["TCC_HIT_sum"] / (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"])
    if "SQ_VALU_MFMA_BUSY_CYCLES" in pmc and "GRBM_GUI_ACTIVE" in pmc:
        # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy cycles sum the 1024 SIMDs
        per_xcd = pmc["GRBM_GUI_ACTIVE"] / 8
        res["mfma_busy_frac"] = pmc["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / per_xcd
        res["effective_clock_ghz"] = per_xcd / (kern[scan_name]["avg_ms"] * 1e6)
    if "SQ_WAIT_ANY" in pmc:
        res["wave_wait_frac"] = pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
        res["wave_issue_stall_frac"] = pmc["SQ_WAIT_INST_ANY"] / pmc["SQ_WAVE_CYCLES"]
        res["wave_active_frac"] = pmc["SQ_ACTIVE_INST_ANY"] / pmc["SQ_WAVE_CYCLES"]
    if "SQ_LDS_BANK_CONFLICT" in pmc and pmc.get("SQ_LDS_IDX_ACTIVE"):
        res["lds_bank_conflict_frac"] = pmc["SQ_LDS_BANK_CONFLICT"] / pmc["SQ_LDS_IDX_ACTIVE"]
    (out / f"{rnd}_{tag}_summary.json").write_text(json.dumps(res, indent=1))
    if "hbm_bytes_per_launch" in res:
        (out / f"pmc_scan_{tag}.json").write_text(json.dumps(
            {"rows_per_gpu": rows, "nq": nq, "hbm_bytes_per_launch": res["hbm_bytes_per_launch"],
             "source": f"profiles/{rnd}_{tag}_summary.json", "csrc_digest": res.get("csrc_digest"),
             "lib_digest": res.get("lib_digest"), "git_head_at_summary": res.get("git_head_at_summary")},
            indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
