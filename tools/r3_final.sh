#!/bin/bash
# Round-3 final evidence at HEAD on the GPU box: the whole -m gpu suite, the
# rocprofv3 trace + PMC passes of the default bench (config (d)), the default
# bench line (CPU baseline + oracle recall), and config (b) / (e) lines.
# usage: tools/r3_final.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 500 tools/profile_scan.sh ${tag}_d --steps 5 --warmup 2
timeout -k 10 400 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
tail -c 600 $o/bench_d.json
timeout -k 10 300 python -u bench.py --config b > $o/bench_b.json 2> $o/bench_b.err
timeout -k 10 300 python -u bench.py --config e --no-cpu --steps 5 > $o/bench_e.json 2> $o/bench_e.err
echo final done
