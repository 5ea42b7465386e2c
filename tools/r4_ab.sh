#!/bin/bash
# Same-box A/B of library builds on the (d) bench, its N = 8 per-rank shard
# (1.25M rows) and config (b); each arm twice, alternating (tools/gpu_multi.sh).
# usage: tools/r4_ab.sh <tag> <lib>...
set -euo pipefail
t=$1; shift
arms=(); for l in "$@"; do arms+=("$l|-"); done
tools/gpu_multi.sh ${t}_d d "${arms[@]}"
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "${arms[@]}"
tools/gpu_multi.sh ${t}_b b "${arms[@]}"
echo ab done
