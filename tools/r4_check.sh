#!/bin/bash
# Round-4 GPU check: the scan-epilogue ablation (tools/r4_ablate.sh), then the
# whole -m gpu suite on the current build.  Stops at the first failure.
# usage: tools/r4_check.sh <tag>
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
tools/r4_ablate.sh ${t}abl
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -3 $o/pytest.log
echo check done
