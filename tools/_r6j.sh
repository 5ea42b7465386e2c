set -euo pipefail
o=gpurun_out/r6j; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
P="python3 -u tools/latency_probe.py --k 10 --reps 300"
for env in "FX_SMALL_SCAN=1" "FX_SMALL_SCAN=0" "FX_REFINE_WAVES=8" "FX_REFINE_WAVES=4" "FX_SMALL_SCAN=1" "FX_SMALL_SCAN=0"; do
  env $env timeout -k 10 120 $P --rows 100000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
done
for env in "FX_SMALL_SCAN=1" "FX_SMALL_SCAN=0"; do
  env $env timeout -k 10 120 $P --rows 1000000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
done
bash tools/lat_trace.sh r6j
B="python -u bench.py --no-cpu --latency-calls 0 --steps 20 --warmup 3"
for cfg in d e b; do
  for nq in 1 16; do
    for v in 1 0; do
      FX_SMALL_SCAN=$v timeout -k 10 240 $B --config $cfg --nq $nq >> $o/small_${cfg}.jsonl 2>> $o/sweep.err
    done
  done
done
echo r6j done
