#!/bin/bash
# Round 3: same-box A/B of existing placement / list knobs at the mid-batch
# point (nq = 256: splits per XCD) and at the headline (compaction trigger).
# usage: tools/r3_knobs.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
BENCH_ARGS="--nq 256" timeout -k 10 400 tools/gpu_multi.sh $tag/d256 d "$L|-" "$L|FX_SCAN_SX=16" "$L|FX_SCAN_SX=32"
python3 tools/show_multi.py $o/d256
BENCH_ARGS="--nq 256" timeout -k 10 400 tools/gpu_multi.sh $tag/e256 e "$L|-" "$L|FX_SCAN_SX=16"
python3 tools/show_multi.py $o/e256
timeout -k 10 400 tools/gpu_multi.sh $tag/d d "$L|-" "$L|FX_COMPACT_AT=48"
python3 tools/show_multi.py $o/d
echo knobs done
