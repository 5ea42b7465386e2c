#!/bin/bash
# Round 3: config (b) list knobs (prune rank, compaction trigger) same-box.
# usage: tools/r3_knobs2.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
BENCH_ARGS="--nq 1000" timeout -k 10 400 tools/gpu_multi.sh $tag/b b "$L|-" "$L|FX_PRUNE_RANK=16" "$L|FX_COMPACT_AT=48" "$L|FX_PRUNE_RANK=16 FX_COMPACT_AT=48"
python3 tools/show_multi.py $o/b
grep -h -o '"fallback_queries_last_step": [0-9]*' $o/b/*.json | sort | uniq -c
echo knobs2 done
