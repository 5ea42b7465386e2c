#!/bin/bash
# Same-box A/B of library builds / options on the (d) bench, its N = 8
# per-rank shard (1.25M rows) and config (b); each arm twice, alternating
# (tools/gpu_multi.sh).  Arms: "<lib>|<env assignments or ->".
# usage: tools/r4_ab.sh <tag> <arm>...
set -euo pipefail
t=$1; shift
tools/gpu_multi.sh ${t}_d d "$@"
BENCH_ARGS="--rows 1250000" tools/gpu_multi.sh ${t}_shard d "$@"
tools/gpu_multi.sh ${t}_b b "$@"
echo ab done
