#!/bin/bash
# Round-4 GPU check: same-box A/B on (d), the N = 8 per-rank shard and (b) of
# the round-3 product against the current build with the union bound waited
# for in place (default) and deferred (union_defer = 1); the fallback counts
# of every line; then the -m gpu suite on the current build.
# usage: tools/r4_check.sh <tag>
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
L=rag-faiss-embedding_amd
A=("$L/libfx_index_r3.so|-" "$L/libfx_index.so|-" "$L/libfx_index.so|FX_UNION_DEFER=1")
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}ab_shard d "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}ab_shard
# the deferred arm only where the shard certified every query (a broken bound
# sends every query to the exact scan: minutes on (d))
if grep -q "arm2_1.json fallbacks 0 " <(python tools/show_fallbacks.py gpurun_out/${t}ab_shard); then :; else A=("${A[@]:0:2}"); fi
tools/gpu_multi.sh ${t}ab_d d "${A[@]}"
python tools/show_fallbacks.py gpurun_out/${t}ab_d
tools/gpu_multi.sh ${t}ab_b b "${A[@]}"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -3 $o/pytest.log
echo check done
