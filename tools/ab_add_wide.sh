#!/bin/bash
# Same-box A/B of the add() conversion kernel: 4 vs 8 chunks in flight per
# lane (FX_CONVERT_WIDE), then the GPU parity suite with the wide variant.
# usage: tools/ab_add_wide.sh <tag>
set -euo pipefail
o=gpurun_out/$1
mkdir -p $o
for rep in 1 2; do
  for w in 0 1; do
    FX_CONVERT_WIDE=$w timeout -k 10 120 python -u tools/add_probe.py | sed "s/^/wide=$w /" >> $o/add_wide.txt
    FX_CONVERT_WIDE=$w timeout -k 10 120 python -u tools/add_probe.py --dim 384 | sed "s/^/wide=$w /" >> $o/add_wide.txt
    FX_CONVERT_WIDE=$w timeout -k 10 120 python -u tools/add_probe.py --dtype float32 --dim 384 | sed "s/^/wide=$w /" >> $o/add_wide.txt
  done
done
FX_CONVERT_WIDE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_f32_split.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $o/pytest_wide.log 2>&1
echo ab_add_wide done
