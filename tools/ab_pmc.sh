#!/bin/bash
# A/B of scan variants (environment assignments) on one bench config: a timed
# bench line, then two rocprofv3 PMC passes of a short run (L2 hits/misses,
# HBM-side fetch; SQ wave states + MFMA busy + GRBM clock), each pass its own
# process under a hard limit.  Stops at the first failure.
# usage: tools/ab_pmc.sh <tag> <config> "<envs A>" "<envs B>" ...   ("-" = none)
set -euo pipefail
out=gpurun_out/$1; cfg=$2; shift 2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for envs in "$@"; do
  [ "$envs" = "-" ] && envs=""
  echo "$i: $envs" >> "$out/index.txt"
  env $envs timeout -k 10 300 python -u bench.py --config $cfg --no-cpu > "$out/bench_${cfg}_$i.json" 2> "$out/bench_${cfg}_$i.err"
  B="python3 bench.py --config $cfg --no-cpu --steps 3 --warmup 1"
  env $envs timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc_$i" -o run -- $B > "$out/tcc_$i.log" 2>&1
  env $envs timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch_$i" -o run -- $B > "$out/fetch_$i.log" 2>&1
  env $envs timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$out/sq_$i" -o run -- $B > "$out/sq_$i.log" 2>&1
  i=$((i+1))
done
echo "ab_pmc done"
