#!/bin/bash
# Round-4 evidence at HEAD on one box: the -m gpu suite with the deferred
# union bound forced on (FX_UNION_DEFER=1; the default is off until this is
# green), the default bench line of (d) (CPU baseline, oracle recall,
# latency_nq1), the rocprofv3 trace + PMC passes of the (d) bench
# (tools/profile_scan.sh), and the scan's epilogue ablation
# (tools/r4_ablate.sh).  Stops at the first failure.
# usage: tools/r4_final.sh <tag>
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
FX_UNION_DEFER=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest_defer1.log 2>&1
tail -2 $o/pytest_defer1.log
timeout -k 10 400 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
tail -c 300 $o/bench_d.json
timeout -k 10 600 tools/profile_scan.sh ${t}_d --steps 5 --warmup 2
tools/r4_ablate.sh ${t}abl
echo final done
