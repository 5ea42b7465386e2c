#!/bin/bash
# Single-query latency in the reference's call form (tools/latency_probe.py)
# on the shapes VERDICT r5 item 2 names, plus one rocprofv3 kernel trace of
# 200 calls on the 100k x 384 fp32 index (kernels per search).
# usage: tools/lat_trace.sh <tag>
set -euo pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 -u tools/latency_probe.py --k 10 --reps 200"
timeout -k 10 180 $P --rows 100000 --dim 384 --dtype float32 >> "$out/latency.jsonl" 2>> "$out/latency.err"
timeout -k 10 180 $P --rows 1000000 --dim 384 --dtype float32 >> "$out/latency.jsonl" 2>> "$out/latency.err"
timeout -k 10 240 $P --rows 10000000 --dim 768 --dtype bfloat16 >> "$out/latency.jsonl" 2>> "$out/latency.err"
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$out/trace" -o run -- \
    $P --rows 100000 --dim 384 --dtype float32 > "$out/trace.log" 2>&1
echo "lat $tag done"
