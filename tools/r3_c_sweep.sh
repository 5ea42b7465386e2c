#!/bin/bash
# Round 3 closing: config (c) end to end (encode 100k chunks -> add -> 1k
# queries) and the nq sweep of (d), (b), (e) at HEAD.
set -euo pipefail
o=gpurun_out/r3cs; mkdir -p $o
timeout -k 10 400 python -u tools/bench_e2e.py > $o/bench_c.json 2> $o/bench_c.err
tail -c 400 $o/bench_c.json
timeout -k 10 900 tools/sweep_nq.sh r3cs/sweep
python3 tools/show_sweep.py $o/sweep 2>/dev/null | tail -20 || true
echo c_sweep done
