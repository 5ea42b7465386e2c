#!/bin/bash
# Round-3 closing evidence at HEAD (prune rank max(6k/5, 12)): rocprofv3 trace +
# PMC passes of the default bench, the default bench line (CPU baseline +
# oracle recall), and the config (b) line.
# usage: tools/r3_final2.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 500 tools/profile_scan.sh ${tag}_d --steps 5 --warmup 2
timeout -k 10 400 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
tail -c 300 $o/bench_d.json
timeout -k 10 300 python -u bench.py --config b > $o/bench_b.json 2> $o/bench_b.err
echo final2 done
