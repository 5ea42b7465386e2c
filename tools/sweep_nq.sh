#!/bin/bash
# Small-batch (HBM-bound) regime, SURVEY.md 8(d): config (d) and (b) at
# nq in {1, 16, 64, 256, 1024}; one JSON line per run.
set -euo pipefail
out=gpurun_out/${1:-sweep}
mkdir -p "$out"
for cfg in d b; do
  for nq in 1 16 64 256 1024; do
    timeout -k 10 240 python -u bench.py --config $cfg --nq $nq --no-cpu --steps 20 --warmup 3 \
      >> "$out/sweep_$cfg.jsonl" 2>> "$out/sweep.err"
  done
done
echo done
