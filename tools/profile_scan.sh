#!/bin/bash
# Collect the rocprofv3 evidence for the bench's dominant kernel (run on the
# GPU box from the repo root).  Kernel trace + stats in one pass; HBM traffic
# counters in their own passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC
# pass on gfx950); no --pmc together with any trace domain.
# usage: tools/profile_scan.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --no-cpu "$@" > "$out/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --no-cpu "$@" > "$out/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 bench.py --no-cpu "$@" > "$out/write.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc" -o run -- \
    python3 bench.py --no-cpu "$@" > "$out/tcc.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$out/sq" -o run -- python3 bench.py --no-cpu "$@" > "$out/sq.log" 2>&1
echo "profile $tag done"
