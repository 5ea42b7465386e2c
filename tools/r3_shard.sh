#!/bin/bash
# Round 3: list / placement knobs on the N = 8 per-rank shard (1.25M x 768
# bf16, nq 10k), same box.
# usage: tools/r3_shard.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
BENCH_ARGS="--rows 1250000" timeout -k 10 600 tools/gpu_multi.sh $tag/d8 d "$L|-" "$L|FX_COMPACT_AT=48" \
    "$L|FX_UNION_W=64" "$L|FX_SCAN_SX=4" "$L|FX_SCAN_SX=1"
python3 tools/show_multi.py $o/d8
grep -h -o '"fallback_queries_last_step": [0-9]*' $o/d8/*.json | sort | uniq -c
echo shard done
