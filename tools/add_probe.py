#!/usr/bin/env python3
"""Time IndexFlatL2.add of device-resident rows (the k_convert_rows_t launch
plus its stream-ordered bookkeeping) and print one JSON line: ms per add and
the effective HBM rate (input bytes read + code bytes written + norms).

usage: python tools/add_probe.py [--rows 1000000] [--dim 768] [--dtype bfloat16] [--reps 10]
(the FX_CONVERT_* environment selects the conversion kernel variant)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import amd_fx  # noqa: E402,F401
from rag_faiss_embedding_amd import faiss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    tdt = getattr(torch, a.dtype)
    x = torch.randn(a.rows, a.dim, device="cuda:0").to(tdt)
    idx = faiss.IndexFlatL2(a.dim, dtype=a.dtype, device=0)
    idx.reserve(a.rows)
    idx.add(x)  # warm-up (allocation, module load)
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        idx.reset()
        idx.reserve(a.rows)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx.add(x)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    # ceiling reference: a plain device-to-device copy of the same input bytes
    y = torch.empty_like(x)
    y.copy_(x)
    torch.cuda.synchronize()
    cms = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        y.copy_(x)
        torch.cuda.synchronize()
        cms.append((time.perf_counter() - t0) * 1e3)
    es = x.element_size()
    cbytes = a.rows * a.dim * es * 2
    nbytes = a.rows * a.dim * es * 2 + a.rows * 4
    best = min(ms)
    med = sorted(ms)[len(ms) // 2]
    print(json.dumps({"probe": "add", "rows": a.rows, "dim": a.dim, "dtype": a.dtype,
                      "nt": os.environ.get("FX_CONVERT_NT", "1"), "ms_best": round(best, 4),
                      "ms_median": round(med, 4), "tb_s_best": round(nbytes / best / 1e9, 3),
                      "tb_s_median": round(nbytes / med / 1e9, 3),
                      "copy_ms_best": round(min(cms), 4), "copy_tb_s_best": round(cbytes / min(cms) / 1e9, 3)}),
          flush=True)


if __name__ == "__main__":
    main()
