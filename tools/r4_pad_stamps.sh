#!/bin/bash
# Slow-path stamps of the scan with and without the accumulator pad
# (ablation build: FX_SCAN_DBG 1024 = pad, 3072 = no pad) on (e) (fp16,
# 6 stages per tile) and (d) (bf16, 12): record tiles per tile and their
# cycles, to test whether the unpadded epilogue takes more record tiles.
# usage: tools/r4_pad_stamps.sh <tag>
set -euo pipefail
o=gpurun_out/$1; mkdir -p $o
A=rag-faiss-embedding_amd/libfx_index_abl.so
for cfg in e d; do
  spt=6; [ $cfg = d ] && spt=12
  for dbg in 1024 3072; do
    FX_INDEX_LIB=$A FX_SCAN_DBG=$dbg FX_SCAN_STAMPS=$o/${cfg}_$dbg.bin timeout -k 10 200 \
      python -u bench.py --config $cfg --no-cpu --latency-calls 0 --steps 2 --warmup 1 > $o/${cfg}_$dbg.json 2> $o/${cfg}_$dbg.err
    echo "## $cfg FX_SCAN_DBG=$dbg"; python tools/show_stamps.py $o/${cfg}_$dbg.bin $spt
  done
done
echo stamps done
