#!/usr/bin/env python3
"""Block-skew trace of the main scan: does the drift of
the workgroups that stream one corpus split explain the traffic past L2?

Runs one search of a synthetic BASELINE-config workload on the diagnostic
library with FX_SCAN_TRACE (per block: XCD, CU, query tile, split, start and
end in s_memrealtime ticks, 100 MHz), then models the fetches past L2:

  * a block's position at time t is (t - start) / its own tile time;
  * a block streams from L2 at t when another block of the SAME split, on the
    same XCD, is ahead of it by less than the L2 residency R (the time since
    that block passed the same tile: gap in tiles x its tile time); otherwise
    it fetches the tile past L2 (HBM or Infinity Cache: what FETCH_SIZE
    counts);
  * summed over samples: the modelled bytes past L2 per launch, for a few R
    (R ~ 4 MiB / the XCD's fetch rate: tens of microseconds).

Also prints the start / end spread of the blocks per dispatch round, which is
where the drift comes from (a block of round r+1 starts when one of round r
ends).  Prints one JSON line; --dump keeps the raw trace.

    python tools/block_skew.py --config d
"""
import argparse
import json
import os
import sys
import tempfile
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

CONFIGS = {"d": (10_000_000, 768, "bfloat16", 10_000), "e": (100_000_000, 384, "float16", 10_000),
           "b": (1_000_000, 384, "float32", 1_000), "shard": (1_250_000, 768, "bfloat16", 10_000)}
TICK = 1e-8  # s_memrealtime: 100 MHz


def run_trace(cfg, nq_override, path):
    os.environ["FX_SCAN_TRACE"] = str(path)  # read at index creation (diag build only)
    import torch
    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd import diag, faiss as fx
    rows, d, dtype, nq = CONFIGS[cfg]
    nq = nq_override or nq
    tdt = getattr(torch, dtype)
    ix = diag.IndexFlatL2(d, dtype=dtype)
    ix.reserve(rows)
    buf = torch.empty((min(1 << 20, rows), d), dtype=tdt, device="cuda")
    for r0 in range(0, rows, buf.shape[0]):
        part = buf[:min(buf.shape[0], rows - r0)]
        fx.synth_fill(part, r0, 1234)
        ix.add(part)
    del buf
    xq = torch.empty((nq, d), dtype=tdt, device="cuda")
    fx.synth_fill(xq, 0, 4321)
    for _ in range(3):  # warm-up (and the same clock regime as the bench's timed steps)
        ix.search(xq, 10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ix.search(xq, 10)  # the dump of this search stays in `path`
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    row_bytes = ((d * (4 if dtype == "float32" else 2) + 127) // 128) * 128
    return rows, d, dtype, nq, row_bytes, wall


def model(tr, rows, row_bytes, R_list, dt_tiles=2.0, tile_rows=128):
    xcc = (tr[:, 0] & 0xF).astype(np.int64)
    cu = ((tr[:, 0] >> 8) >> 8 & 0xFF).astype(np.int64) + 256 * xcc
    split = tr[:, 1].astype(np.int64)
    t0 = tr[:, 2].astype(np.float64) * TICK
    t1 = tr[:, 3].astype(np.float64) * TICK
    ok = (tr[:, 2] > 0) & (tr[:, 3] > tr[:, 2])
    xcc, cu, split, t0, t1 = xcc[ok], cu[ok], split[ok], t0[ok], t1[ok]
    nsplit = int(split.max()) + 1
    n_ct = (rows + tile_rows - 1) // tile_rows
    ntiles = np.array([(s + 1) * n_ct // nsplit - s * n_ct // nsplit for s in range(nsplit)])[split]
    tile_t = (t1 - t0) / np.maximum(ntiles, 1)
    T0, T1 = t0.min(), t1.max()
    dt = float(np.median(tile_t)) * dt_tiles
    tile_bytes = tile_rows * (row_bytes + 4)  # rows + their norms
    fetched = {R: 0.0 for R in R_list}
    by_split = defaultdict(list)
    for b in range(len(split)):
        by_split[split[b]].append(b)
    groups = [np.array(v) for v in by_split.values()]
    for t in np.arange(T0, T1, dt):
        for g in groups:
            act = g[(t0[g] <= t) & (t < t1[g])]
            if act.size == 0:
                continue
            pos = (t - t0[act]) / tile_t[act]
            order = np.argsort(pos)
            pos, act = pos[order], act[order]
            # time since the nearest block ahead passed this block's position
            gap = np.full(act.size, np.inf)
            gap[:-1] = (pos[1:] - pos[:-1]) * tile_t[act[1:]]
            for R in R_list:
                miss = gap > R
                fetched[R] += float(np.sum(dt / tile_t[act[miss]])) * tile_bytes
    # dispatch rounds: the blocks on each CU in start order
    rounds = defaultdict(list)
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        for r, b in enumerate(idx[np.argsort(t0[idx])]):
            rounds[r].append(b)
    spread = []
    for r in sorted(rounds):
        bs = np.array(rounds[r])
        if bs.size < 16:
            continue
        spread.append({"round": r, "blocks": int(bs.size), "start_spread_us": round(float(np.ptp(t0[bs])) * 1e6, 1),
                       "end_spread_us": round(float(np.ptp(t1[bs])) * 1e6, 1),
                       "median_block_ms": round(float(np.median(t1[bs] - t0[bs])) * 1e3, 3)})
    # nearest same-split block ahead at each block's start, in tiles
    lag = []
    for g in groups:
        for b in g:
            o = g[(t0[g] < t0[b]) & (t1[g] > t0[b])]
            if o.size:
                p = (t0[b] - t0[o]) / tile_t[o]
                lag.append(float(p.min()))
    lag = np.array(lag) if lag else np.zeros(1)
    hist = {k: int(np.sum(m)) for k, m in (("<2", lag < 2), ("2-10", (lag >= 2) & (lag < 10)),
                                             ("10-100", (lag >= 10) & (lag < 100)),
                                             ("100-1000", (lag >= 100) & (lag < 1000)), (">=1000", lag >= 1000))}
    return {"blocks": int(len(split)), "splits": nsplit, "kernel_ms_trace": round((T1 - T0) * 1e3, 3),
            "median_tile_us": round(float(np.median(tile_t)) * 1e6, 3),
            "modelled_past_l2_bytes": {f"R={R * 1e6:.0f}us": fetched[R] for R in R_list},
            "nearest_ahead_lag_tiles_at_start": hist, "rounds": spread}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d", choices=sorted(CONFIGS))
    ap.add_argument("--nq", type=int, default=0)
    ap.add_argument("--dump", default="")
    ap.add_argument("--tile-rows", type=int, default=0,
                    help="rows per scan tile (0: 64 where k_scan_v5 runs -- 16-bit rows at nq > 128 -- else 128)")
    args = ap.parse_args()
    path = Path(args.dump) if args.dump else Path(tempfile.mkdtemp()) / "scan_trace.bin"
    rows, d, dtype, nq, row_bytes, wall = run_trace(args.config, args.nq, path)
    tr = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
    v5 = os.environ.get("FX_SCAN_V5", "1") != "0" and dtype != "float32" and row_bytes in (512, 768, 1536) and nq > 128
    tile_rows = args.tile_rows or (64 if v5 else 128)
    res = model(tr, rows, row_bytes, [20e-6, 40e-6, 80e-6], tile_rows=tile_rows)
    res["tile_rows"] = tile_rows
    alg = rows * row_bytes
    res["modelled_x_algorithmic"] = {k: round(v / alg, 2) for k, v in res["modelled_past_l2_bytes"].items()}
    res.update({"config": args.config, "rows": rows, "dim": d, "dtype": dtype, "nq": nq,
                "search_wall_ms": round(wall * 1e3, 3), "algorithmic_corpus_bytes": alg})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
