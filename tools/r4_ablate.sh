#!/bin/bash
# Same-box ceilings of the scan's parts: the product scan against the
# ablation build (timing only, results invalid): FX_SCAN_DBG=8 no epilogue
# (keys computed, nothing selected), 256 fast path only (slow tiles counted,
# no pushes), 2 no corpus DMA, 10 neither DMA nor epilogue -- on config (d)
# and on its N = 8 per-rank shard (1.25M rows).
# usage: tools/r4_ablate.sh <tag>
set -euo pipefail
t=$1
P=rag-faiss-embedding_amd/libfx_index.so
A=rag-faiss-embedding_amd/libfx_index_abl.so
tools/gpu_multi.sh ${t}_d d "$P|-" "$A|FX_SCAN_DBG=8" "$A|FX_SCAN_DBG=256" "$A|FX_SCAN_DBG=2"
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "$P|-" "$A|FX_SCAN_DBG=8" "$A|FX_SCAN_DBG=256"
echo ablate done
