#!/bin/bash
# Same-box comparison of several (library, environment) arms on one bench
# config, each arm run twice in alternation (box-to-box spread ~5 %).
# Arms: "<lib>|<env assignments or ->" ...  Stops at the first failure.
# usage: tools/gpu_multi.sh <tag> <config> <arm>...
set -euo pipefail
o=gpurun_out/$1; cfg=$2; shift 2
mkdir -p $o
for r in 1 2; do
  i=0
  for arm in "$@"; do
    lib=${arm%%|*}; envs=${arm#*|}; [ "$envs" = "-" ] && envs=""
    env FX_INDEX_LIB=$lib $envs timeout -k 10 150 python -u bench.py --config $cfg ${BENCH_ARGS:-} --no-cpu --latency-calls 0 --steps 6 --warmup 1 > $o/arm${i}_$r.json 2> $o/arm${i}_$r.err
    echo "$i: $arm" >> $o/arms_$r.txt
    i=$((i+1))
  done
done
echo multi done
