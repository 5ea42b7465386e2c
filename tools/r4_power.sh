#!/bin/bash
# Same-box power/clock A/B of the epilogue pad on (e) and (d) through the
# ablation build (results valid for every arm): the product's single pad
# (dbg 0), no pad (2048) and the pad twice (8192).
# usage: tools/r4_power.sh <tag>
set -euo pipefail
t=$1
A=rag-faiss-embedding_amd/libfx_index_abl.so
tools/gpu_multi.sh ${t}_e e "$A|-" "$A|FX_SCAN_DBG=2048" "$A|FX_SCAN_DBG=8192"
tools/gpu_multi.sh ${t}_d d "$A|-" "$A|FX_SCAN_DBG=2048" "$A|FX_SCAN_DBG=8192"
for c in e d; do echo "## $c"; python tools/show_multi.py gpurun_out/${t}_$c; done
echo power done
