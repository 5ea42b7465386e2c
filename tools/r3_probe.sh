#!/bin/bash
# Round-3 scan probe (run on the GPU box from the repo root): per-wave phase
# stamps of k_scan_v4 (-DFX_ABLATION build) on synthetic and clustered config
# (d), and rocprofv3 FETCH_SIZE / SQ passes of the default kernel with and
# without the published-list union threshold (FX_SCAN_PUB=0).
# usage: tools/r3_probe.sh <tag>
set -euo pipefail
o=gpurun_out/$1; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ABL=rag-faiss-embedding_amd/libfx_index_abl.so
FX_INDEX_LIB=$ABL FX_SCAN_DBG=64 FX_SCAN_STAMPS=$o/stamps_syn.bin timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 1 > $o/st_syn.json 2> $o/st_syn.err
FX_INDEX_LIB=$ABL FX_SCAN_DBG=64 FX_SCAN_STAMPS=$o/stamps_clu.bin timeout -k 10 200 python -u bench.py --no-cpu --data clustered --steps 1 --warmup 1 > $o/st_clu.json 2> $o/st_clu.err
pmc() {  # <subdir> <env> <bench args> -- <counters...>
    local sub=$1 envs=$2 args=$3; shift 3
    env $envs timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$o/$sub" -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 $args > "$o/$sub.log" 2>&1
}
pmc fetch_def "FX_X=0" "" FETCH_SIZE
pmc fetch_nopub "FX_SCAN_PUB=0" "" FETCH_SIZE
pmc fetch_clu "FX_X=0" "--data clustered" FETCH_SIZE
pmc tcc_def "FX_X=0" "" TCC_HIT_sum TCC_MISS_sum
pmc sq_def "FX_X=0" "" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc sq_clu "FX_X=0" "--data clustered" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
echo probe done
