#!/bin/bash
# Round-4 closing evidence at HEAD on one box: the -m gpu suite, smoke(), the
# default bench line of (d), the (b) and (e) lines, the N = 8 per-rank shard of
# (d) (1.25M rows), the small-batch sweep of (d) (nq 1/16/64/256), and the
# rocprofv3 trace + PMC passes of the (d) bench.  Stops at the first failure.
# usage: PART=1|2 tools/r4_head.sh <tag>  (1: suite, smoke, bench lines; 2: nq sweep, profile)
set -euo pipefail
t=$1; o=gpurun_out/$t; mkdir -p $o
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -2 $o/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
tail -c 300 $o/bench_d.json
timeout -k 10 300 python -u bench.py --config b > $o/bench_b.json 2> $o/bench_b.err
timeout -k 10 300 python -u bench.py --config e --no-cpu > $o/bench_e.json 2> $o/bench_e.err
timeout -k 10 200 python -u bench.py --rows 1250000 --no-cpu --latency-calls 0 > $o/bench_shard.json 2> $o/bench_shard.err
echo part 1 done
exit 0
fi
for nq in 1 16 64 256; do
  timeout -k 10 200 python -u bench.py --nq $nq --steps 50 --warmup 5 --no-cpu --latency-calls 0 > $o/bench_d_nq$nq.json 2> $o/bench_d_nq$nq.err
done
timeout -k 10 600 tools/profile_scan.sh ${t}_d --steps 5 --warmup 2
FX_PROFILE_MIN=1 timeout -k 10 600 tools/profile_scan.sh ${t}_e --config e --steps 3 --warmup 1
echo head done
