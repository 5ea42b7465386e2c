#!/bin/bash
# In-kernel stamps of the ablation build (libfx_index_abl.so) on one bench
# workload: per FX_SCAN_DBG value, the scan's slow-path share, compactions and
# (1024-modes) the in-kernel clock, summarised by tools/show_stamps.py.
# Stamps distort timing; their results are valid (1024 / 3072 / 9216).
# usage: tools/stamps.sh <tag> <d|e|b|shard> <dbg>...
set -euo pipefail
o=gpurun_out/$1; w=$2; shift 2; mkdir -p $o
cfg=$w; extra=""; [ $w = shard ] && { cfg=d; extra="--rows 1250000"; }
spt=12; [ $cfg = e ] && spt=6
for dbg in "$@"; do
  FX_INDEX_LIB=rag-faiss-embedding_amd/libfx_index_abl.so FX_SCAN_DBG=$dbg FX_SCAN_STAMPS=$o/${w}_$dbg.bin \
    timeout -k 10 300 python -u bench.py --config $cfg $extra --no-cpu --latency-calls 0 --steps 2 --warmup 1 \
    > $o/${w}_$dbg.json 2> $o/${w}_$dbg.err
  echo "## $w FX_SCAN_DBG=$dbg kernel_ms $(python -c "import json,sys;print(json.loads(open('$o/${w}_$dbg.json').read().splitlines()[-1])['roofline']['kernel_ms_avg'])")"
  python tools/show_stamps.py $o/${w}_$dbg.bin $spt
done
echo stamps done
