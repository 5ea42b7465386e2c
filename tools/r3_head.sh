#!/bin/bash
# Round-3 HEAD evidence on the GPU box: the whole -m gpu suite, then the full
# rocprofv3 evidence (trace + FETCH/WRITE/TCC/SQ passes) of the default bench.
# usage: tools/r3_head.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 500 tools/profile_scan.sh ${tag}_d --steps 5 --warmup 2
echo head done
