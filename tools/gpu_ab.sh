#!/bin/bash
# Same-box A/B of two builds of the library on config (d) (box-to-box spread
# is ~5 %, so only same-call comparisons count): bench lines alternating A, B,
# A, B, then an instruction-cache PMC pass of each.  Stops at the first failure.
# usage: tools/gpu_ab.sh <tag> <lib A> <lib B> [bench args...]
set -euo pipefail
o=gpurun_out/$1; A=$2; B=$3; shift 3
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    FX_INDEX_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu "$@" > $o/bench_${v}$r.json 2> $o/bench_${v}$r.err
  done
done
for v in A B; do
  L=$A; [ $v = B ] && L=$B
  FX_INDEX_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $o/ic_$v -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 "$@" > $o/ic_$v.log 2>&1
done
echo ab done
