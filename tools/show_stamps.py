#!/usr/bin/env python3
"""Summarise an FX_SCAN_STAMPS dump of a -DFX_ABLATION build run with
FX_SCAN_DBG & 64: per-wave s_memtime cycle sums of k_scan_v4's phases
[stage wait + barrier, half 0, mid-stage LDS wait, half 1, epilogue, stages,
slow-path tiles, slow-path cycles, compaction calls, compaction cycles,
group pushes] (argv[2]: stages per tile, default 12).
Prints the mean cycles per stage of each phase over all waves that ran
(half 0 / half 1 each hold 16 MFMAs = 256 cycles at the MFMA issue rate)."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16).astype(np.float64)
a = a[(a[:, 5] > 0) | (a[:, 14] > 0)]
st = np.maximum(a[:, 5], 1)
names = ["wait+barrier", "half0", "mid lgkm wait", "half1", "epilogue"]
tot = a[:, :5].sum(1)
print(f"waves {len(a)}, stages/wave {st.mean():.0f}, cycles/stage total {np.mean(tot / st):.1f}")
for i, n in enumerate(names):
    per = a[:, i] / st
    print(f"  {n:14s} {per.mean():8.1f} cyc/stage  (p10 {np.percentile(per, 10):7.1f}  p90 {np.percentile(per, 90):7.1f})  "
          f"{100 * a[:, i].sum() / tot.sum():5.1f} %")
tiles = st / 12 if len(sys.argv) < 3 else st / int(sys.argv[2])
print(f"  slow-path tiles {np.mean(a[:, 6] / tiles):.3f} of tiles, {np.mean(a[:, 7] / np.maximum(a[:, 6], 1)):.0f} cyc each, "
      f"{100 * a[:, 7].sum() / tot.sum():.1f} % of wave time")
print(f"  compactions {np.mean(a[:, 8] / tiles):.4f} per tile, {np.mean(a[:, 9] / np.maximum(a[:, 8], 1)):.0f} cyc each, "
      f"{100 * a[:, 9].sum() / tot.sum():.1f} % of wave time; group pushes {np.mean(a[:, 10] / np.maximum(a[:, 6], 1)):.2f} per slow tile")
print(f"  slow path before any compaction: {np.mean(a[:, 11] / np.maximum(a[:, 6], 1)):.0f} cyc per slow tile")
print(f"  fast epilogue (tile end -> ballot decided): {np.mean(a[:, 12] / tiles):.0f} cyc per tile")
if a.shape[1] > 14 and a[:, 13].sum() > 0:  # ABL & 1024: slow-path-only stamps + whole-wave cycles
    tot = a[:, 13]
    print(f"[slow-path stamps] wave cycles {tot.mean():.0f}, tiles/wave {a[:, 14].mean():.0f}, "
          f"cycles/tile {np.mean(tot / np.maximum(a[:, 14], 1)):.0f}")
    print(f"  slow tiles {a[:, 6].sum() / a[:, 14].sum():.4f} of wave-tiles; slow-path cycles = "
          f"{100 * a[:, 7].sum() / tot.sum():.2f} % of wave cycles ({a[:, 7].sum() / max(a[:, 6].sum(), 1):.0f} per slow tile; "
          f"before compaction {a[:, 11].sum() / max(a[:, 6].sum(), 1):.0f})")
    print(f"  compactions {a[:, 8].sum() / a[:, 14].sum():.5f} per wave-tile, {a[:, 9].sum() / max(a[:, 8].sum(), 1):.0f} cyc each")
    if a[:, 12].sum() > 0:  # s_memrealtime ticks (100 MHz) of each wave's life
        clk = a[:, 13] / np.maximum(a[:, 12], 1) * 0.1
        print(f"  in-kernel clock {np.median(clk):.3f} GHz median over waves (p10 {np.percentile(clk, 10):.3f}, "
              f"p90 {np.percentile(clk, 90):.3f}; s_memtime / s_memrealtime x 100 MHz)")
