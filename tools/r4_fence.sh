#!/bin/bash
# Same-box A/B of the scan epilogue's accumulator wait-state pad
# (acc_fence_v before the group minima; libfx_index_bf.so = HEAD built with
# -DFX_BISECT_FENCE) against HEAD without it, on (d), the N = 8 shard, (b)
# and (e), with fallback counts.
# usage: tools/r4_fence.sh <tag>
set -euo pipefail
t=$1
L=rag-faiss-embedding_amd
A=("$L/libfx_index.so|-" "$L/libfx_index_bf.so|-")
tools/gpu_multi.sh ${t}_d d "${A[@]}"
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "${A[@]}"
tools/gpu_multi.sh ${t}_b b "${A[@]}"
tools/gpu_multi.sh ${t}_e e "${A[@]}"
for c in d shard b e; do echo "## $c"; python tools/show_multi.py gpurun_out/${t}_$c; python tools/show_fallbacks.py gpurun_out/${t}_$c; done
echo fence done
