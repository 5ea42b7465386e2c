set -euo pipefail
o=gpurun_out/r6c; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 -u tools/latency_probe.py --k 10 --reps 300"
for env in "FX_HOST_SPIN=0" "FX_HOST_SPIN=1" "FX_REDUCE_CAND=0" "FX_REDUCE_CAND=2" "FX_SEARCH_GRAPH=0" \
           "FX_COLD_BOUND=0" "FX_COLD_BOUND=1 FX_PRUNE_RANK=10" "FX_SCAN_PUB=0" "FX_UNION_DEFER=0" "FX_COMPACT_AT=64"; do
  env $env timeout -k 10 120 $P --rows 100000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
done
for env in "FX_REDUCE_CAND=1" "FX_REDUCE_CAND=0" "FX_REDUCE_CAND=2"; do
  env $env timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$env -o run -- \
    $P --rows 100000 --dim 384 --dtype float32 > $o/trace_$env.log 2>&1
done
timeout -k 10 120 $P --rows 1000000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
echo r6c done
