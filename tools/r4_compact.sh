#!/bin/bash
# Same-box sweep of the compaction trigger under the deferred union bound
# (a compaction no longer waits for its union reads, so compacting earlier
# may pay): compact_at 64 (default) / 56 / 48 / 40 on (d), the N = 8 shard and
# (b); fallback counts of every line.
# usage: tools/r4_compact.sh <tag>
set -euo pipefail
t=$1
L=rag-faiss-embedding_amd/libfx_index.so
A=("$L|-" "$L|FX_COMPACT_AT=56" "$L|FX_COMPACT_AT=48" "$L|FX_COMPACT_AT=40")
tools/gpu_multi.sh ${t}_d d "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}_d
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}_shard
tools/gpu_multi.sh ${t}_b b "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}_b
L3=rag-faiss-embedding_amd/libfx_index_r3.so
tools/gpu_multi.sh ${t}_e e "$L3|-" "$L|FX_UNION_DEFER=0" "$L|-"
python tools/show_fallbacks.py gpurun_out/${t}_e
echo compact done
