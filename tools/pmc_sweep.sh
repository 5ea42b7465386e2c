#!/bin/bash
# rocprofv3 evidence for the small-batch (HBM-bound) points: kernel trace +
# FETCH_SIZE + WRITE_SIZE passes of the bench at nq in {1, 16, 256} on (d)
# and (e).  Summaries: tools/summarize_profile.py <dir> <cfg>_nq<N> r3 <rows> <nq>
set -euo pipefail
for cfg in d e; do
  for nq in 1 16 256; do
    FX_PROFILE_MIN=1 timeout -k 10 500 tools/profile_scan.sh ${cfg}_nq$nq --config $cfg --nq $nq --steps 5 --warmup 2
  done
done
echo pmc sweep done
