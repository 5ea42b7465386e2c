#!/bin/bash
# One GPU-box check of the tree: the whole -m gpu suite, then the default
# bench lines of configs (d) and (b).  Stops at the first failure.
# usage: tools/gpu_check.sh <tag>
set -euo pipefail
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d.json" 2> "$out/bench_d.err"
timeout -k 10 300 python -u bench.py --config b --no-cpu > "$out/bench_b.json" 2> "$out/bench_b.err"
echo "check done"
