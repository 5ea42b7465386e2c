#!/bin/bash
# Round-3 check on the GPU box: the parity subset that covers the scan, the
# refine, the re-scan and the exact fallback, then same-box A/B bench arms.
# usage: tools/r3_check.sh <tag> [arm ...]   (arms as tools/gpu_multi.sh)
set -euo pipefail
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests/test_lane_swap.py tests/test_rescan.py tests/test_big_k.py \
    tests/test_search_graph.py tests/test_gpu_parity.py tests/test_cert_stress.py -q -x -s --timeout 280 \
    --timeout-method thread -rf > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
grep -E "rescan|cert-stress|passed" $o/tests.log | tail -16
if [ $# -gt 0 ]; then
  timeout -k 10 400 tools/gpu_multi.sh $tag/ab d "$@"
  python3 tools/show_multi.py $o/ab
fi
