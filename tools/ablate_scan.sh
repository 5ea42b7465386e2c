#!/bin/bash
# Scan ablations on a -DFX_ABLATION build (timing only, results invalid):
# FX_SCAN_DBG = 1 L2-resident corpus, 2 no corpus DMA, 4 no MFMA, 8 no
# epilogue, 10 = 2+8, 14 = 2+4+8 (ring/barrier skeleton).
# usage: tools/ablate_scan.sh <tag> <ablation .so>
set -euo pipefail
o=gpurun_out/${1:-abl}; mkdir -p $o
for d in ${DBGS:-0 1 2 4 8 10 14}; do
  FX_INDEX_LIB=$2 FX_SCAN_DBG=$d timeout -k 10 120 python -u bench.py --no-cpu --steps 3 --warmup 1 > $o/dbg$d.json 2>$o/dbg$d.err
done
echo ok
