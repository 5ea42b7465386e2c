#!/bin/bash
# Round 3: the k > FX_MAX_K sort path on the GPU (test_big_k.py) and the
# rocprofv3 evidence of the small-batch (HBM-bound) points (tools/pmc_sweep.sh).
# usage: tools/r3_hugek.sh <tag> [nosweep]
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_big_k.py -x -v -s --timeout 200 --timeout-method thread > $o/bigk.log 2>&1 \
    || { tail -40 $o/bigk.log; exit 1; }
grep -E "passed|failed" $o/bigk.log | tail -3
if [ "${2:-}" != nosweep ]; then
  timeout -k 10 900 tools/pmc_sweep.sh
fi
echo hugek done
