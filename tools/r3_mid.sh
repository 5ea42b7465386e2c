#!/bin/bash
# Mid-batch A/B (round 3): config (b) and config (d) at nq = 256, arms as
# "lib|env", then slow-path stamps of the ablation build on (d).
# usage: tools/r3_mid.sh <tag> <arm>...
set -euo pipefail
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_multi.sh $tag/b b "$@"
BENCH_ARGS="--nq 256" tools/gpu_multi.sh $tag/d256 d "$@"
FX_INDEX_LIB=rag-faiss-embedding_amd/libfx_index_abl.so FX_SCAN_DBG=1024 FX_SCAN_STAMPS=$o/st.bin timeout -k 10 200 \
    python -u bench.py --no-cpu --steps 1 --warmup 1 > $o/st.json 2> $o/st.err
echo mid done
