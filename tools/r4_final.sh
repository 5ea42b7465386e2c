#!/bin/bash
# Round-4 evidence at HEAD on one box: the scan's epilogue ablation
# (tools/r4_ablate.sh: FX_SCAN_DBG 8 / 256 / 2 / 10 on (d), 8 / 256 on the
# shard), the rocprofv3 trace + PMC passes of the (d) bench
# (tools/profile_scan.sh), and the default bench line (CPU baseline, oracle
# recall, latency_nq1).
# usage: tools/r4_final.sh <tag>
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
tools/r4_ablate.sh ${t}abl
timeout -k 10 600 tools/profile_scan.sh ${t}_d --steps 5 --warmup 2
timeout -k 10 400 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
tail -c 400 $o/bench_d.json
echo final done
