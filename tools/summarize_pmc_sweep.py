#!/usr/bin/env python3
"""Small-batch (HBM-bound) points with counter evidence: for every
tools/pmc_sweep.sh output directory gpurun_out/prof_<cfg>_nq<N>, run
tools/summarize_profile.py (-> profiles/<round>_<cfg>_nq<N>_{kernel_stats.csv,
summary.json}, profiles/pmc_scan_<cfg>_nq<N>.json, read by bench.py as
roofline.traffic) and print, per point, the scan's rocprof average, the HBM
bytes per launch from the PMC passes (2*FETCH_SIZE + WRITE_SIZE, gfx950
correction of MI355X_MICROARCH.md) against the algorithmic bytes (the corpus
rows once: N*d*s), and both as GB/s.

usage: tools/summarize_pmc_sweep.py <round> [gpurun_out]
"""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CFG = {"d": (10_000_000, 768, 2), "e": (100_000_000, 384, 2), "b": (1_000_000, 384, 4)}


def main():
    rnd = sys.argv[1]
    base = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out"
    rows = []
    for cfg in ("d", "e", "b"):
        n, d, s = CFG[cfg]
        for nq in (1, 16, 64, 256, 1024):
            prof = base / f"prof_{cfg}_nq{nq}"
            if not (prof / "trace" / "run_kernel_stats.csv").exists():
                continue
            out = subprocess.run([sys.executable, str(ROOT / "tools" / "summarize_profile.py"), str(prof),
                                  f"{cfg}_nq{nq}", rnd, str(n), str(nq)], capture_output=True, text=True)
            if out.returncode != 0:
                print(f"{cfg} nq={nq}: summarize failed: {out.stderr.strip()[-200:]}")
                continue
            res = json.loads(out.stdout)
            ms = res["kernels"][res["scan_kernel"]]["avg_ms"]
            alg = n * d * s + nq * d * s + nq * 10 * 12
            hbm = res.get("hbm_bytes_per_launch")
            rows.append((cfg, nq, ms, alg, hbm))
    print(f"{'cfg':>3} {'nq':>5} {'scan ms':>9} {'alg GB':>8} {'PMC GB':>8} {'PMC/alg':>8} "
          f"{'alg GB/s':>9} {'PMC GB/s':>9} {'frac(alg)':>9}")
    for cfg, nq, ms, alg, hbm in rows:
        hb = f"{hbm / 1e9:8.2f}" if hbm else "     n/a"
        ratio = f"{hbm / alg:8.3f}" if hbm else "     n/a"
        pg = f"{hbm / ms / 1e6:9.0f}" if hbm else "      n/a"
        print(f"{cfg:>3} {nq:>5} {ms:9.3f} {alg / 1e9:8.2f} {hb} {ratio} {alg / ms / 1e6:9.0f} {pg} "
              f"{alg / ms / 1e6 / 8000:9.3f}")


if __name__ == "__main__":
    main()
