#!/bin/bash
# Measurement pass on one GPU box: config (e) bench
# line with its CPU leg, config (c) end to end, the small-batch (HBM-bound)
# sweep, and single-query latency in the reference's call form.  Every GPU step
# has its own time limit; the steps stop at the first failure.
# usage: tools/gpu_measure.sh <tag> [e|c|sweep|lat ...]   (default: all four)
set -euo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
parts=${*:-e c sweep lat}
for p in $parts; do
  case $p in
    e)
      timeout -k 10 420 python -u bench.py --config e --steps 5 --warmup 1 > "$out/bench_e.json" 2> "$out/bench_e.err" ;;
    c)
      timeout -k 10 420 python -u tools/bench_e2e.py > "$out/bench_c.json" 2> "$out/bench_c.err" ;;
    sweep)
      for cfg in d e b; do
        for nq in 1 16 64 256; do
          timeout -k 10 240 python -u bench.py --config $cfg --nq $nq --no-cpu --steps 20 --warmup 3 \
            >> "$out/sweep_$cfg.jsonl" 2>> "$out/sweep.err"
          if [ $nq -le 32 ]; then
            FX_SCAN_Q32=1 timeout -k 10 240 python -u bench.py --config $cfg --nq $nq --no-cpu --steps 20 --warmup 3 \
              >> "$out/sweep_${cfg}_q32.jsonl" 2>> "$out/sweep.err"
          fi
        done
      done ;;
    lat)
      for env in "" "FX_SEARCH_GRAPH=1" "FX_SCAN_Q32=1 FX_SEARCH_GRAPH=1"; do
        env $env timeout -k 10 180 python -u tools/latency_probe.py --rows 1000000 --dim 384 --dtype float32 \
          >> "$out/latency.jsonl" 2>> "$out/latency.err"
        env $env timeout -k 10 180 python -u tools/latency_probe.py --rows 10000000 --dim 768 --dtype bfloat16 \
          >> "$out/latency.jsonl" 2>> "$out/latency.err"
      done ;;
  esac
  echo "part $p done"
done
echo "measure done"
