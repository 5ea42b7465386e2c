#!/bin/bash
# Round-4 scan probe: the N = 8 shard bench (1.25M rows) with the deferred
# union bound off and on, then config (d); each step under its own time limit,
# chained (a timeout ends the call).  Prints each line's scan ms and fallbacks.
# usage: tools/r4_probe.sh <tag>
set -euo pipefail
o=gpurun_out/$1; mkdir -p $o
show() { python -c "import json,sys; j=json.load(open('$1')); print('$1', j['roofline']['kernel_ms_avg'], 'ms scan;', j['fallback_queries_last_step'], 'fallbacks')"; }
for d in 0 1; do
  FX_UNION_DEFER=$d timeout -k 10 100 python -u bench.py --rows 1250000 --no-cpu --steps 3 --warmup 1 --latency-calls 5 > $o/shard_defer$d.json 2> $o/shard_defer$d.err
  show $o/shard_defer$d.json
done
timeout -k 10 150 python -u bench.py --no-cpu --steps 5 --warmup 1 --latency-calls 20 > $o/d.json 2> $o/d.err
show $o/d.json
timeout -k 10 150 python -u bench.py --config b --no-cpu --steps 10 --warmup 2 --latency-calls 20 > $o/b.json 2> $o/b.err
show $o/b.json
