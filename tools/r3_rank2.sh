#!/bin/bash
# Round 3: lower prune ranks (12, 14) at k = 10 -- certification stress under
# each (fallbacks asserted <= 1 %), then same-box (d) / (b) against the default 16.
# usage: tools/r3_rank2.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
for r in 12 14; do
  FX_PRUNE_RANK=$r timeout -k 10 400 python -u -m pytest tests/test_cert_stress.py -x -q -s --timeout 200 \
      --timeout-method thread > $o/cert_$r.log 2>&1 || { tail -30 $o/cert_$r.log; exit 1; }
  echo "rank $r:"; grep "cert-stress" $o/cert_$r.log
done
L=rag-faiss-embedding_amd/libfx_index.so
timeout -k 10 500 tools/gpu_multi.sh $tag/d d "$L|-" "$L|FX_PRUNE_RANK=14" "$L|FX_PRUNE_RANK=12"
python3 tools/show_multi.py $o/d
BENCH_ARGS="--nq 1000" timeout -k 10 300 tools/gpu_multi.sh $tag/b b "$L|-" "$L|FX_PRUNE_RANK=14" "$L|FX_PRUNE_RANK=12"
python3 tools/show_multi.py $o/b
grep -h -o '"fallback_queries_last_step": [0-9]*' $o/d/*.json $o/b/*.json | sort | uniq -c
echo rank2 done
