#!/bin/bash
# Collect the rocprofv3 evidence for the bench's dominant kernel (run on the
# GPU box from the repo root).  Kernel trace + stats in one pass; every PMC
# group in a pass of its own (FETCH_SIZE and WRITE_SIZE do not fit one TCC
# pass on gfx950; no --pmc together with any trace domain), each under a hard
# time limit (a pass over the per-block counter capacity hangs).
# Scan variants are chosen by the caller's environment (FX_* options).
# usage: tools/profile_scan.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --no-cpu --latency-calls 0 $*"
# which sources / library these counters belong to (read by summarize_profile.py)
python3 -c "import json, amd_fx; from rag_faiss_embedding_amd import _provenance as P; \
print(json.dumps({'csrc_digest': P.source_digest(), 'lib_digest': P.file_digest('rag-faiss-embedding_amd/libfx_index.so')}))" \
    > "$out/provenance.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    $B > "$out/trace.log" 2>&1
pmc() {  # <subdir> <counters...>
    local sub=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/$sub" -o run -- $B > "$out/$sub.log" 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
if [ "${FX_PROFILE_MIN:-0}" = 1 ]; then echo "profile $tag done (trace + fetch + write)"; exit 0; fi
pmc tcc TCC_HIT_sum TCC_MISS_sum
pmc sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
if [ "${FX_PROFILE_EXTRA:-0}" = 1 ]; then
  pmc lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA
  pmc ta TA_BUSY_avr TA_BUSY_max
fi
echo "profile $tag done"
