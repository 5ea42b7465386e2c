#!/bin/bash
# Bench config lines under several environment settings, one JSON per run.
# usage: tools/ab_env.sh <tag> <config> "<envs A>" "<envs B>" ...   ("-" = none)
set -euo pipefail
out=gpurun_out/$1; cfg=$2; shift 2
mkdir -p "$out"
i=0
for envs in "$@"; do
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python -u bench.py --config $cfg --no-cpu > "$out/bench_${cfg}_$i.json" 2> "$out/bench_${cfg}_$i.err"
  echo "$i: $envs" >> "$out/index.txt"
  i=$((i+1))
done
echo "ab_env done"
