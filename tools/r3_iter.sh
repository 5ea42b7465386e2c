#!/bin/bash
# One round-3 scan iteration on the GPU box (repo root): same-box A/B of the
# previous and current library (and option arms) on config (d), slow-path
# stamps of the ablation build, and one FETCH_SIZE pass of the current library.
# usage: tools/r3_iter.sh <tag> [extra arms "lib|env"...]
set -euo pipefail
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=rag-faiss-embedding_amd
tools/gpu_multi.sh $tag/ab d "$L/libfx_index_prev.so|-" "$L/libfx_index.so|-" "$@"
FX_INDEX_LIB=$L/libfx_index_abl.so FX_SCAN_DBG=1024 FX_SCAN_STAMPS=$o/st.bin timeout -k 10 200 \
    python -u bench.py --no-cpu --steps 1 --warmup 1 > $o/st.json 2> $o/st.err
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- \
    python3 bench.py --no-cpu --steps 3 --warmup 1 > $o/fetch.log 2>&1
echo iter done
