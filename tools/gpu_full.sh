#!/bin/bash
# Full GPU check of the tree: the -m gpu suite, the config (d) rocprofv3
# evidence (kernel trace + PMC passes, tools/profile_scan.sh), and the bench
# lines of configs (d), (b), (e).  Stops at the first failure.
# usage: tools/gpu_full.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
bash tools/profile_scan.sh $tag
timeout -k 10 300 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
timeout -k 10 300 python -u bench.py --config b > $o/bench_b.json 2> $o/bench_b.err
timeout -k 10 500 python -u bench.py --config e --steps 5 --warmup 1 > $o/bench_e.json 2> $o/bench_e.err
echo full done
