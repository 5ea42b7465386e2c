#!/bin/bash
# Round 3: the whole -m gpu suite at this build (6-slot DMA ring with 56-entry
# lists where a tile has >= 5 stages), then same-box A/B against the previous
# build (libfx_index_ns5.so: 5 slots, 64-entry lists) on config (d) (also with
# forced threshold seeding), (b), the (d) N=8 shard and (d) at nq = 256, then
# the rocprofv3 small-batch sweep.
# usage: tools/r3_ns6.sh <tag> [nosweep]
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
L=rag-faiss-embedding_amd/libfx_index.so
P=rag-faiss-embedding_amd/libfx_index_ns5.so
timeout -k 10 500 tools/gpu_multi.sh $tag/d d "$P|-" "$L|-" "$L|FX_SEED_TILES=256"
python3 tools/show_multi.py $o/d
BENCH_ARGS="--nq 1000" timeout -k 10 300 tools/gpu_multi.sh $tag/b b "$P|-" "$L|-" "$L|FX_SEED_TILES=-1"
python3 tools/show_multi.py $o/b
BENCH_ARGS="--rows 1250000" timeout -k 10 300 tools/gpu_multi.sh $tag/d8 d "$P|-" "$L|-" "$L|FX_SEED_TILES=-1"
python3 tools/show_multi.py $o/d8
BENCH_ARGS="--nq 256" timeout -k 10 300 tools/gpu_multi.sh $tag/d256 d "$P|-" "$L|-" "$L|FX_SEED_TILES=-1"
python3 tools/show_multi.py $o/d256
if [ "${2:-}" != nosweep ]; then
  timeout -k 10 600 tools/pmc_sweep.sh
fi
echo ns6 done
