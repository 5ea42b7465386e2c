#!/bin/bash
# Same-box ceiling of the scan's epilogue: the product scan against the
# ablation build with no epilogue (FX_SCAN_DBG=8: keys computed, nothing
# selected; results invalid) and with the fast path only (256: slow tiles
# counted, no pushes; results invalid), on config (d) and on its N = 8
# per-rank shard (1.25M rows).
# usage: tools/r4_ablate.sh <tag>
set -euo pipefail
t=$1
P=rag-faiss-embedding_amd/libfx_index.so
A=rag-faiss-embedding_amd/libfx_index_abl.so
tools/gpu_multi.sh ${t}_d d "$P|-" "$A|FX_SCAN_DBG=8" "$A|FX_SCAN_DBG=256"
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "$P|-" "$A|FX_SCAN_DBG=8" "$A|FX_SCAN_DBG=256"
echo ablate done
