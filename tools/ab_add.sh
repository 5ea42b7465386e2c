#!/bin/bash
# Same-box A/B of the add() conversion kernel: cached vs nontemporal loads /
# stores (FX_CONVERT_NT), wall-clock probe and rocprofv3 kernel stats of each,
# then the GPU parity suite with the nontemporal variant.
# usage: tools/ab_add.sh <tag>
set -euo pipefail
o=gpurun_out/$1
mkdir -p $o
export TMPDIR=/tmp
for rep in 1 2; do
  for nt in 0 1; do
    FX_CONVERT_NT=$nt timeout -k 10 120 python -u tools/add_probe.py >> $o/add_probe.jsonl 2>> $o/add_probe.err
    FX_CONVERT_NT=$nt timeout -k 10 120 python -u tools/add_probe.py --dtype float32 --dim 384 >> $o/add_probe.jsonl 2>> $o/add_probe.err
  done
done
for nt in 0 1; do
  FX_CONVERT_NT=$nt timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $o/prof_nt$nt -o run -- \
    python -u tools/add_probe.py > $o/prof_nt$nt.log 2>&1
done
FX_CONVERT_NT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $o/pytest_nt1.log 2>&1
echo ab_add done
