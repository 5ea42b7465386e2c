#!/bin/bash
# Round 3: default prune rank max(6k/5, 12) -- whole -m gpu suite (certification
# stress asserted), clustered (d) line (fallbacks), default (d) line.
# usage: tools/r3_rank3.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
grep -E "cert-stress" $o/pytest.log | tail -10
timeout -k 10 300 python -u bench.py --data clustered --no-cpu > $o/bench_d_clustered.json 2> $o/bench_d_clustered.err
grep -o '"fallback_queries_last_step": [0-9]*' $o/bench_d_clustered.json
timeout -k 10 300 python -u bench.py --no-cpu > $o/bench_d.json 2> $o/bench_d.err
tail -c 300 $o/bench_d.json
echo rank3 done
