#!/usr/bin/env python3
"""Summarise a scan trace written with FX_SCAN_TRACE=<file> (diagnostics).

Per block: {xcc | hw_id << 8 | qtile << 32, split, t_start, t_end} in the
100 MHz wall clock.  Reports whether block b runs on XCD (b % 8)'s group,
how far apart blocks of one (XCD, split) cohort start and end (corpus
re-reads only hit that XCD's L2 while the cohort stays together), and
the per-round spread.
usage: tools/analyze_trace.py <file>
"""
import sys
from collections import defaultdict

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
live = a[:, 2] != 0
idx = np.nonzero(live)[0]
xcc = (a[:, 0] & 0xF).astype(np.int64)
hw = ((a[:, 0] >> 8) & 0xFFFFFF).astype(np.int64)
qt = (a[:, 0] >> 32).astype(np.int64)
sp = a[:, 1].astype(np.int64)
t0 = a[:, 2].astype(np.int64)
t1 = a[:, 3].astype(np.int64)
base = t0[live].min()
ts, te = (t0 - base) / 100.0, (t1 - base) / 100.0  # microseconds
print(f"blocks {len(a)}, live {live.sum()}, kernel span {te[live].max():.0f} us")
m = {}
for b in idx:
    m.setdefault(b % 8, set()).add(int(xcc[b]))
print("b%8 -> XCC ids:", {k: sorted(v) for k, v in sorted(m.items())})
dur = te[live] - ts[live]
print(f"block duration us: min {dur.min():.0f} median {np.median(dur):.0f} max {dur.max():.0f}")
coh = defaultdict(list)
for b in idx:
    coh[(int(xcc[b]), int(sp[b]))].append(b)
ss, es = [], []
for k, bs in coh.items():
    if len(bs) > 1:
        ss.append(ts[bs].max() - ts[bs].min())
        es.append(te[bs].max() - te[bs].min())
ss, es = np.array(ss), np.array(es)
print(f"cohorts (xcc, split) {len(coh)}, size median {np.median([len(v) for v in coh.values()])}")
print(f"cohort start spread us: median {np.median(ss):.1f} p90 {np.percentile(ss, 90):.1f} max {ss.max():.1f}")
print(f"cohort end spread us:   median {np.median(es):.1f} p90 {np.percentile(es, 90):.1f} max {es.max():.1f}")
# distinct CUs per XCC
cus = defaultdict(set)
for b in idx:
    cus[int(xcc[b])].add(int(hw[b]) & 0xFFFF)
print("distinct hw ids per XCC:", {k: len(v) for k, v in sorted(cus.items())})
# concurrency: at the median time, how many blocks per xcc are running with which splits
tm = np.median(ts[live]) + 1.0
run = [b for b in idx if ts[b] <= tm < te[b]]
per = defaultdict(lambda: defaultdict(int))
for b in run:
    per[int(xcc[b])][int(sp[b])] += 1
print(f"at t={tm:.0f} us: running {len(run)}")
for x in sorted(per):
    print(f"  xcc {x}: split->blocks {dict(sorted(per[x].items()))}")
