#!/bin/bash
# Round-4 GPU check: same-box A/B of the round-3 product (libfx_index_r3.so),
# the round-4 push + deferred union bound (libfx_index_r4b.so, with and
# without the deferral) and the current build (corpus pieces fused into MFMA
# pairs), then the whole -m gpu suite on the current build.  Stops at the
# first failure.
# usage: tools/r4_check.sh <tag>
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
L=rag-faiss-embedding_amd
tools/r4_ab.sh ${t}ab "$L/libfx_index_r3.so|-" "$L/libfx_index_r4b.so|-" "$L/libfx_index_r4f.so|-" "$L/libfx_index.so|-"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -3 $o/pytest.log
echo check done
