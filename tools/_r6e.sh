set -euo pipefail
o=gpurun_out/r6e; mkdir -p $o
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_scan_options.py -m gpu > $o/pytest_first.log 2>&1
timeout -k 10 900 $T tests -m gpu > $o/pytest.log 2>&1
B="python -u bench.py --no-cpu --latency-calls 0"
for v in 1 0 1 0; do
  FX_SCAN_V5=$v timeout -k 10 300 $B --steps 10 --warmup 2 >> $o/bench_d.jsonl 2>> $o/bench.err
  FX_SCAN_V5=$v timeout -k 10 200 $B --rows 1250000 --steps 20 --warmup 3 >> $o/bench_shard.jsonl 2>> $o/bench.err
  FX_SCAN_V5=$v timeout -k 10 200 $B --nq 256 --steps 20 --warmup 3 >> $o/bench_d256.jsonl 2>> $o/bench.err
done
bash tools/lat_trace.sh r6e
echo r6e done
