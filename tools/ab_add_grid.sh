#!/bin/bash
# Same-box A/B of the add() conversion grid cap (FX_CONVERT_GRID) and the
# 8-chunk variant (FX_CONVERT_WIDE), then the GPU parity suite at a small cap.
# usage: tools/ab_add_grid.sh <tag>
set -euo pipefail
o=gpurun_out/$1
mkdir -p $o
for rep in 1 2; do
  for g in 65536 4096 1024; do
    for w in 0 $([ $g = 1024 ] && echo 1); do
      for shape in "--dim 768" "--dim 384" "--dtype float32 --dim 384"; do
        FX_CONVERT_GRID=$g FX_CONVERT_WIDE=$w timeout -k 10 120 python -u tools/add_probe.py --reps 6 $shape \
          | sed "s/^/grid=$g wide=$w /" >> $o/add_grid.txt
      done
    done
  done
done
FX_CONVERT_GRID=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_f32_split.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $o/pytest_grid.log 2>&1
echo ab_add_grid done
