#!/usr/bin/env python3
"""Single-query latency in the reference's call form: numpy float32 query in,
numpy D / I out (faiss_store.py:57-77 searches one query per call).

Times `reps` back-to-back IndexFlat.search(x[1, d], k) calls on a synthetic
index and prints one JSON line with the median / p90 latency.  The scan
variants are selected by the usual environment variables (FX_SCAN_Q32,
FX_SEARCH_GRAPH, FX_F32_SPLIT, ...), which the line records.

    python tools/latency_probe.py --rows 1000000 --dim 384 --dtype float32
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()

    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd import faiss as fx
    tdt = getattr(torch, args.dtype)
    ix = fx.IndexFlatL2(args.dim, dtype=args.dtype)
    ix.reserve(args.rows)
    buf = torch.empty((min(1 << 20, args.rows), args.dim), dtype=tdt, device="cuda")
    for r0 in range(0, args.rows, buf.shape[0]):
        part = buf[:min(buf.shape[0], args.rows - r0)]
        fx.synth_fill(part, r0, 1234)
        ix.add(part)
    torch.cuda.synchronize()
    xq = torch.empty((args.reps, args.dim), dtype=tdt, device="cuda")
    fx.synth_fill(xq, 0, 4321)
    xq = xq.float().cpu().numpy()
    for i in range(5):
        ix.search(xq[i:i + 1], args.k)
    lat = []
    for i in range(args.reps):
        t0 = time.perf_counter()
        ix.search(xq[i:i + 1], args.k)
        lat.append(time.perf_counter() - t0)
    lat = np.array(lat) * 1e3
    env = {k: v for k, v in os.environ.items() if k.startswith("FX_")}
    print(json.dumps({"metric": "single-query search latency (host in / host out)", "rows": args.rows,
                      "dim": args.dim, "dtype": args.dtype, "k": args.k, "reps": args.reps,
                      "median_ms": round(float(np.median(lat)), 4), "p90_ms": round(float(np.percentile(lat, 90)), 4),
                      "min_ms": round(float(lat.min()), 4), "env": env}), flush=True)


if __name__ == "__main__":
    main()
