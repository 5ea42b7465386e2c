#!/bin/bash
# Round-4 GPU check: A/B of the round-3 product (libfx_index_r3.so) against
# the current build with and without the deferred union bound, the whole
# -m gpu suite on the current build, then the scan-epilogue ablation
# (tools/r4_ablate.sh).  Stops at the first failure.
# usage: tools/r4_check.sh <tag>
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
L=rag-faiss-embedding_amd
tools/r4_ab.sh ${t}ab "$L/libfx_index_r3.so|-" "$L/libfx_index.so|FX_UNION_DEFER=0" "$L/libfx_index.so|-"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -3 $o/pytest.log
tools/r4_ablate.sh ${t}abl
echo check done
