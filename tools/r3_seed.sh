#!/bin/bash
# Round 3: the whole -m gpu suite at this build (k > FX_MAX_K sort path,
# threshold-seeding scan on by default), then same-box A/B of the seeding scan
# (FX_SEED_TILES=-1: off) on config (b), the config (d) N=8 shard (1.25M rows)
# and config (d) at nq = 256.
# usage: tools/r3_seed.sh <tag> [full|sweep]   (full: also config (d) at nq 10k with forced seeding;
#        sweep: that and the rocprofv3 small-batch sweep, tools/pmc_sweep.sh)
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
L=rag-faiss-embedding_amd/libfx_index.so
BENCH_ARGS="--nq 1000" timeout -k 10 300 tools/gpu_multi.sh $tag/b b "$L|-" "$L|FX_SEED_TILES=-1"
python3 tools/show_multi.py $o/b
BENCH_ARGS="--rows 1250000" timeout -k 10 300 tools/gpu_multi.sh $tag/d8 d "$L|-" "$L|FX_SEED_TILES=-1"
python3 tools/show_multi.py $o/d8
BENCH_ARGS="--nq 256" timeout -k 10 300 tools/gpu_multi.sh $tag/d256 d "$L|-" "$L|FX_SEED_TILES=-1"
python3 tools/show_multi.py $o/d256
if [ "${2:-}" = full ] || [ "${2:-}" = sweep ]; then
  timeout -k 10 500 tools/gpu_multi.sh $tag/d d "$L|-" "$L|FX_SEED_TILES=256" "$L|FX_SEED_TILES=1024"
  python3 tools/show_multi.py $o/d
fi
if [ "${2:-}" = sweep ]; then
  timeout -k 10 600 tools/pmc_sweep.sh
fi
echo seed done
