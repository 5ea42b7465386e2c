#!/bin/bash
# Round 3: pacing of a split's query-tile blocks (FX_PACE_W, 2-4 query tiles):
# parity under pacing (GPU parity subset + a bench line with oracle recall at
# nq = 256), then same-box A/B of the pacing window on (d), (e), (b) at nq = 256,
# then the instruction-cache counters of the default (d) scan (tools/icache_pass.sh).
# usage: tools/r3_pace.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
FX_PACE_W=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -x -q --timeout 200 \
    --timeout-method thread > $o/pytest_pace.log 2>&1 || { tail -40 $o/pytest_pace.log; exit 1; }
tail -1 $o/pytest_pace.log
FX_PACE_W=4 timeout -k 10 300 python -u bench.py --nq 256 --recall-queries 64 --cpu-seconds 3 > $o/bench_d256_pace.json 2> $o/bench_d256_pace.err
tail -c 400 $o/bench_d256_pace.json
L=rag-faiss-embedding_amd/libfx_index.so
BENCH_ARGS="--nq 256" timeout -k 10 400 tools/gpu_multi.sh $tag/d256 d "$L|-" "$L|FX_PACE_W=2" "$L|FX_PACE_W=4" "$L|FX_PACE_W=8"
python3 tools/show_multi.py $o/d256
BENCH_ARGS="--nq 256" timeout -k 10 400 tools/gpu_multi.sh $tag/e256 e "$L|-" "$L|FX_PACE_W=4"
python3 tools/show_multi.py $o/e256
BENCH_ARGS="--nq 256" timeout -k 10 300 tools/gpu_multi.sh $tag/b256 b "$L|-" "$L|FX_PACE_W=4"
python3 tools/show_multi.py $o/b256
timeout -k 10 300 tools/icache_pass.sh ${tag}_icache --steps 3 --warmup 1
echo pace done
