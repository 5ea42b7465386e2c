#!/bin/bash
# Same-box A/B of the corpus-partitioned placement's splits per XCD
# (FX_SCAN_SX) on configs (b) and (d); bench lines without the CPU leg.
# usage: tools/ab_sx.sh <tag>
set -euo pipefail
o=gpurun_out/$1
mkdir -p $o
for rep in 1 2; do
  for sx in "" 4 8 16 32; do
    FX_SCAN_SX=$sx timeout -k 10 120 python -u bench.py --config b --no-cpu --steps 30 --warmup 3 \
      | sed "s/^/b sx=${sx:-auto} rep=$rep /" >> $o/ab_sx.txt 2>> $o/ab_sx.err
  done
  for sx in "" 1 4; do
    FX_SCAN_SX=$sx timeout -k 10 180 python -u bench.py --config d --no-cpu --steps 5 --warmup 1 \
      | sed "s/^/d sx=${sx:-auto} rep=$rep /" >> $o/ab_sx.txt 2>> $o/ab_sx.err
  done
done
echo ab done
