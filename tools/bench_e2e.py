#!/usr/bin/env python3
"""BASELINE config (c): encode 100k chunks with the all-MiniLM-L6-v2
architecture on PyTorch-ROCm, hand the embeddings to the HIP index on the
device, then search top-10 -- end to end on one MI355X.

Reference flow: initialize_rag.py:35-61 (generate_embeddings -> .cpu().numpy()
per batch -> FAISSVectorStore.add_vectors) and query.py:21-55 (encode one
query -> search).  Here: ragged synthetic token ids (the checkpoint and vocab
are not available offline), length-bucketed bf16 batches,
embeddings stay in HBM, one fx_index_add, one batched search.

Prints ONE JSON line: build rate (chunks/s, encode + add), query rate
(queries/s, encode + search), recall@10 / ids bit-exact against the exact CPU
oracle on the same fp32 embeddings, encoder drift of bf16 vs the same seeded
model in fp32 on the CPU, and the CPU encoder rate of that fp32 model.

    python tools/bench_e2e.py [--chunks 100000 --nq 1000 --k 10]
"""
from __future__ import annotations

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


def make_tokens(n: int, min_len: int, max_len: int, seed: int):
    """[n, max_len] int64 ids ([CLS] w... [SEP], zero padding) and lengths,
    from a seeded generator (host tensors)."""
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(min_len, max_len + 1, (n,), generator=g)
    ids = torch.randint(1000, 30522, (n, max_len), generator=g)
    pos = torch.arange(max_len)[None, :]
    ids = torch.where(pos < lens[:, None], ids, torch.zeros_like(ids))
    ids[:, 0] = 101
    ids[torch.arange(n), lens - 1] = 102
    return ids, lens


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=100_000)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--min-len", type=int, default=32)
    ap.add_argument("--max-len", type=int, default=256)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp32"])
    ap.add_argument("--check", type=int, default=64, help="queries / chunks in the parity samples")
    ap.add_argument("--cpu-chunks", type=int, default=256, help="CPU fp32 encoder sample")
    args = ap.parse_args()

    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd import faiss as fx
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    from oracle import cpu as C

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pipe = VectorizationPipeline(device="cuda", precision=args.precision, seed=0, allow_random_init=True)
    ids, lens = make_tokens(args.chunks, args.min_len, args.max_len, seed=11)
    qids, qlens = make_tokens(args.nq, 8, 64, seed=12)       # queries are short, as query.py's are
    ids_d, qids_d = ids.to(dev), qids.to(dev)

    # warm-up: kernels, autotuning, index workspace
    w = pipe.encode_lengths(ids_d[:args.batch], lens[:args.batch], args.batch)
    wi = fx.IndexFlatL2(384, device=0)
    wi.add(w)
    wi.search(w[:16], args.k)
    del wi
    torch.cuda.synchronize()

    # ---- build: encode all chunks + add (device hand-off) ---------------------
    t0 = time.perf_counter()
    emb = pipe.encode_lengths(ids_d, lens, args.batch)
    index = fx.IndexFlatL2(384, device=0)
    index.reserve(args.chunks)
    index.add(emb)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    # ---- query: encode queries + search ----------------------------------------
    t0 = time.perf_counter()
    qemb = pipe.encode_lengths(qids_d, qlens, args.batch)
    D, I = index.search(qemb, args.k)
    torch.cuda.synchronize()
    t_query = time.perf_counter() - t0
    log(f"build {t_build:.2f}s, query {t_query:.3f}s")

    # ---- parity of the search on the same fp32 embeddings ----------------------
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    xb = emb.cpu().numpy()
    sel = np.linspace(0, args.nq - 1, min(args.check, args.nq)).astype(np.int64)
    xq = qemb.cpu().numpy()[sel]
    Dr, Ir = C.knn_exact(xq, xb, args.k, nthreads)
    Ig, Dg = I.cpu().numpy()[sel], D.cpu().numpy()[sel]
    hits = sum(len(set(Ig[i].tolist()) & set(Ir[i].tolist())) for i in range(len(sel)))

    # ---- encoder drift (bf16 on GPU vs the same model in fp32 on CPU) + CPU rate
    cpu_pipe = VectorizationPipeline(device="cpu", precision="fp32", seed=0, allow_random_init=True)
    nc = min(args.cpu_chunks, args.chunks)
    t0 = time.perf_counter()
    ref = cpu_pipe.encode_lengths(ids[:nc], lens[:nc], 32).numpy()
    t_cpu = time.perf_counter() - t0
    got = emb[:nc].cpu().numpy()
    cos = np.sum(ref * got, 1) / (np.linalg.norm(ref, axis=1) * np.linalg.norm(got, axis=1))

    out = {
        "metric": "config (c): encode + add chunks/s and encode + search queries/s, 1 MI355X",
        "build_chunks_per_s": round(args.chunks / t_build, 1),
        "query_per_s": round(args.nq / t_query, 1),
        "build_s": round(t_build, 3), "query_s": round(t_query, 4),
        "unit": "chunks/s | queries/s", "n_gpus": 1, "dtype": args.precision,
        "data": "synthetic ragged token ids (seeded); MiniLM-L6 architecture with seeded weights (checkpoint offline)",
        "config": {"workload": f"{args.chunks} chunks x {args.min_len}-{args.max_len} tokens "
                               f"(mean {float(lens.float().mean()):.0f}), {args.nq} queries, top-{args.k}",
                   "batch": args.batch, "index": "IndexFlatL2 fp32 (reference storage)"},
        "recall_at_10": hits / float(len(sel) * args.k),
        "ids_bit_exact": bool((Ig == Ir).all()),
        "max_rel_dist_err": float(np.max(np.abs(Dg.astype(np.float64) - Dr) / np.maximum(1.0, np.abs(Dr)))),
        "encoder_cos_min_vs_cpu_fp32": float(cos.min()),
        "cpu_baseline": {"value": round(nc / t_cpu, 1), "unit": "chunks/s (encode only)", "cores": torch.get_num_threads(),
                         "kind": "port", "sample": f"{nc} chunks, same seeded model in fp32 on the host CPU"},
        "fallback_queries": index.last_fallbacks(),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
