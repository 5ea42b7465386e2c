#!/bin/bash
# Small-batch (HBM-bound) regime, SURVEY.md 8(d): configs (d), (b), (e) at
# nq in {1, 16, 64, 256, 1024}; (d) and (b) also with the previous
# placement (FX_SCAN_PLACE=0) for a same-box comparison.  One JSON line per run.
set -euo pipefail
out=gpurun_out/${1:-sweep}
mkdir -p "$out"
for cfg in d b e; do
  for nq in 1 16 64 256 1024; do
    timeout -k 10 240 python -u bench.py --config $cfg --nq $nq --no-cpu --steps 20 --warmup 3 \
      >> "$out/sweep_$cfg.jsonl" 2>> "$out/sweep.err"
    if [ "$cfg" != e ] && [ $nq -ge 256 ]; then
      FX_SCAN_PLACE=0 timeout -k 10 240 python -u bench.py --config $cfg --nq $nq --no-cpu --steps 20 --warmup 3 \
        >> "$out/sweep_${cfg}_place0.jsonl" 2>> "$out/sweep.err"
    fi
  done
done
echo done
