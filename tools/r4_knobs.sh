#!/bin/bash
# Same-box sweep of the list-maintenance knobs under the deferred union bound
# (prune rank 10 / 11 against the default 12, compaction trigger, union window) on the N = 8 shard and (d);
# fallback counts of every line.
# usage: tools/r4_knobs.sh <tag>
set -euo pipefail
t=$1
L=rag-faiss-embedding_amd/libfx_index.so
A=("$L|-" "$L|FX_PRUNE_RANK=10" "$L|FX_PRUNE_RANK=11" "$L|FX_COMPACT_AT=48" "$L|FX_UNION_W=32")
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}_shard
tools/gpu_multi.sh ${t}_d d "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}_d
echo knobs done
