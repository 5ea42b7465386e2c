#!/bin/bash
# Instruction-cache counters of the bench's scan (the slow path's code lies
# ~11 KB past the main loop): lists the box's counters first, then one PMC
# pass with the SQC instruction-cache counters the list offers.
# usage: tools/icache_pass.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
want=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do
  if grep -q "\b$c\b" "$out/counters.txt"; then want="$want $c"; fi
done
echo "icache counters:$want"
[ -n "$want" ] || exit 0
timeout -s KILL 240 rocprofv3 --pmc $want --output-format csv -d "$out/icache" -o run -- \
    python3 bench.py --no-cpu "$@" > "$out/icache.log" 2>&1
echo "icache pass $tag done"
