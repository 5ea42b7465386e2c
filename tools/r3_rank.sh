#!/bin/bash
# Round 3: prune rank max(3k/2, 16) as the default -- the whole -m gpu suite
# (certification stress asserts <= 1 % fallbacks), the clustered (d) line
# (fallbacks), and same-box (d) / (b) against FX_PRUNE_RANK=20 (the old default).
# usage: tools/r3_rank.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
grep -E "cert-stress|rescan" $o/pytest.log | tail -14
timeout -k 10 300 python -u bench.py --data clustered --no-cpu > $o/bench_d_clustered.json 2> $o/bench_d_clustered.err
grep -o '"fallback_queries_last_step": [0-9]*' $o/bench_d_clustered.json
L=rag-faiss-embedding_amd/libfx_index.so
timeout -k 10 400 tools/gpu_multi.sh $tag/d d "$L|-" "$L|FX_PRUNE_RANK=20"
python3 tools/show_multi.py $o/d
BENCH_ARGS="--nq 1000" timeout -k 10 300 tools/gpu_multi.sh $tag/b b "$L|-" "$L|FX_PRUNE_RANK=20"
python3 tools/show_multi.py $o/b
echo rank done
