#!/bin/bash
# A/B of a scan variant selected by an environment assignment (e.g.
# FX_SCAN_LINE=1): key-matrix + parity tests under the variant first, then
# config (d) bench lines with and without it.  Stops at the first failure.
# usage: tools/ab_scan.sh <tag> "<VAR=value ...>" [bench configs, default "d"]
set -euo pipefail
out=gpurun_out/$1
envs=$2
cfgs=${3:-d}
mkdir -p "$out"
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
env $envs timeout -k 10 300 $PYT tests/test_scan_keys.py tests/test_gpu_parity.py > "$out/tests.log" 2>&1
for c in $cfgs; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu > "$out/bench_${c}_base.json" 2> "$out/bench_${c}_base.err"
  env $envs timeout -k 10 300 python -u bench.py --config $c --no-cpu > "$out/bench_${c}_var.json" 2> "$out/bench_${c}_var.err"
done
echo "ab done"
