#!/bin/bash
# One GPU call of a kernel change: the -m gpu suite on the product tree, then
# same-box A/Bs of (library, env) arms on bench workloads, each arm twice in
# alternation (tools/gpu_multi.sh).  Stops at the first failure.
# usage: tools/ab_step.sh <tag> "<workload>[:bench args]"... -- <arm>...
#   workload: d | b | e | shard (config d at 1.25M rows, the N=8 per-rank share)
#   arm: "<lib>|<env assignments or ->"; SUITE=0 skips the suite
set -euo pipefail
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o
wl=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do wl+=("$1"); shift; done
shift
if [ "${SUITE:-1}" = 1 ]; then
  if ! timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
       --durations 15 > $o/pytest.log 2>&1; then
    tail -40 $o/pytest.log; exit 1
  fi
  tail -3 $o/pytest.log
fi
for w in "${wl[@]}"; do
  name=${w%%:*}; extra=""; [ "$w" != "$name" ] && extra=${w#*:}
  cfg=$name; [ $name = shard ] && { cfg=d; extra="--rows 1250000 $extra"; }
  BENCH_ARGS="$extra" tools/gpu_multi.sh $tag/$name $cfg "$@"
  python tools/show_multi.py $o/$name | tee $o/$name/summary.txt
done
echo ab_step done
