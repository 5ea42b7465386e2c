set -euo pipefail
o=gpurun_out/r6f; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
P="python3 -u tools/latency_probe.py --k 10 --reps 300"
for env in "FX_SEARCH_GRAPH=1" "FX_SEARCH_GRAPH=0" "FX_SEARCH_GRAPH=1" "FX_SEARCH_GRAPH=0"; do
  env $env timeout -k 10 120 $P --rows 100000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
done
for env in "FX_SEARCH_GRAPH=1" "FX_SEARCH_GRAPH=0"; do
  env $env timeout -k 10 120 $P --rows 1000000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
done
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $o/trace -o run -- \
    $P --rows 100000 --dim 384 --dtype float32 > $o/trace.log 2>&1
B="python -u bench.py --no-cpu --latency-calls 0 --steps 20 --warmup 3"
for cfg in d e; do
  for nq in 1 16 64 256 1024; do
    for v in 1 0; do
      FX_SCAN_V5=$v timeout -k 10 240 $B --config $cfg --nq $nq >> $o/sweep_${cfg}.jsonl 2>> $o/sweep.err
    done
  done
done
echo r6f done
