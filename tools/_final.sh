# Final evidence of the round (tools/_final.sh <tag> <part>), two gpurun calls:
# part 1: the GPU suite, smoke, rocprofv3 trace + PMC passes of (d), the bench
#         line of (d) (driver default: CPU leg, 1,000-query recall), one-query
#         latencies;
# part 2: a second box's trace + FETCH/WRITE passes of (d), trace + PMC passes
#         of (e) and (b), their bench lines, the block-skew trace of (d).
# Stops at the first failure.
set -euo pipefail
tag=$1; part=${2:-1}
o=gpurun_out/$tag; mkdir -p $o
if [ "$part" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
  bash tools/profile_scan.sh ${tag}_d
  timeout -k 10 600 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
  P="python3 -u tools/latency_probe.py --k 10 --reps 300"
  timeout -k 10 120 $P --rows 100000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
  timeout -k 10 120 $P --rows 1000000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
  timeout -k 10 180 $P --rows 10000000 --dim 768 --dtype bfloat16 >> $o/latency.jsonl 2>> $o/latency.err
else
  FX_PROFILE_MIN=1 bash tools/profile_scan.sh ${tag}_d2
  bash tools/profile_scan.sh ${tag}_e --config e --steps 3 --warmup 1
  bash tools/profile_scan.sh ${tag}_b --config b
  timeout -k 10 600 python -u bench.py --config e --steps 5 --warmup 1 > $o/bench_e.json 2> $o/bench_e.err
  timeout -k 10 300 python -u bench.py --config b > $o/bench_b.json 2> $o/bench_b.err
  timeout -k 10 300 python -u tools/block_skew.py --config d > $o/skew_d.json 2> $o/skew_d.err
fi
echo "final $tag part $part done"
