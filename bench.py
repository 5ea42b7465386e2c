#!/usr/bin/env python3
"""Headline benchmark: queries/sec + recall@10 of exact flat-L2 search.

BASELINE.json metric: "queries/sec + recall@10 vs CPU FAISS, 10M x 768 flat
index, 1/2/4/8 MI355X".  Default workload = BASELINE config (d): a 10M x 768
bf16 corpus row-sharded over the N GPUs of one node (one process per GPU),
10,000-query batches, k = 10; each rank scans its shard (fused MFMA GEMM +
top-k kernel), the per-shard top-k lists are exchanged with one RCCL
all_gather over xGMI and merged on device.  The total corpus is fixed, so
scaling is "strong".

One step = one search of one 10k-query batch (queries already resident in
HBM; results left in HBM).  Corpus and queries are synthetic (counter-hash
generator shared with oracle/flat_l2.c, exact in bf16), generated on the GPU.

Launch: python bench.py [--gpus N --steps 10 --warmup 2]
          N > 1 without WORLD_SIZE: this process starts N ranks itself
          (torch.distributed.run, 127.0.0.1) before touching the GPU and
          passes rank 0's line through;
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
          (WORLD_SIZE must equal --gpus).
--data clustered: a clustered corpus (unit-norm rows around one common
direction, the shape of sentence embeddings) with fp32 queries that are NOT
exact in the storage dtype -- the certification's hard case.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# torch, torch.distributed and the HIP library are imported in main(), after
# the launcher decision: a process that starts the ranks never touches the GPU
torch = dist = fx = None

METRIC = "queries/sec + recall@10 vs CPU FAISS, 10M×768 flat index, 1/2/4/8 MI355X"
CORPUS_SEED, QUERY_SEED = 1234, 4321

# BASELINE.json configs usable as bench workloads (name -> rows, dim, dtype, nq, k)
CONFIGS = {
    "d": (10_000_000, 768, "bfloat16", 10_000, 10),   # the headline (metric's config)
    "b": (1_000_000, 384, "float32", 1_000, 10),
    "e": (100_000_000, 384, "float16", 10_000, 10),
}
# exact-oracle recall sample per config (>= 1000 queries where the
# oracle allows; the full-corpus streaming oracle costs ~0.25 s per query on (d)
# and ~1.3 s on (e) with 16 host cores: the (e) leg takes ~5 min)
RECALL_QUERIES = {"d": 1000, "b": 1000, "e": 256}
SHORT_DT = {"float32": "f32", "bfloat16": "bf16", "float16": "f16"}
# MI355X_MICROARCH.md: dense MFMA peaks (TFLOP/s) and HBM3E peak (GB/s)
MFMA_PEAK = {"float32": 157.3, "bfloat16": 2500.0, "float16": 2500.0}
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def launch_plan(gpus: int, env) -> str:
    """How to run `bench.py --gpus N`: "inproc" (N = 1, or already one rank of
    a launched world of N), "spawn" (N > 1 and no WORLD_SIZE: start the ranks
    here), or an error message (WORLD_SIZE set and != N)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "inproc"
    if int(ws) != gpus:
        return f"error: WORLD_SIZE={ws} but --gpus {gpus}"
    return "inproc"


def rank_command(gpus: int, argv, port: int):
    """The torch.distributed.run command that starts one bench rank per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + list(argv)


def spawn_ranks(gpus: int, argv) -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[bench] starting {gpus} ranks (torch.distributed.run, port {port})")
    return subprocess.call(rank_command(gpus, argv, port), env=env)


def torch_dt(dtype):
    return {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}[dtype]


CLUSTER_SEED, CLUSTER_SPREAD, CLUSTER_CHUNK = 7, 0.1, 1 << 20


def clustered_rows(chunk_id: int, nrows: int, d: int, device, base):
    """Rows of corpus chunk `chunk_id` (CLUSTER_CHUNK rows each) of the
    clustered corpus: unit-norm base + spread * N(0, I/d), fp32, generated on
    the GPU from a per-chunk seed (every rank regenerates the same rows)."""
    g = torch.Generator(device=device).manual_seed(CLUSTER_SEED * 1_000_003 + 1 + chunk_id)
    x = base[None, :] + CLUSTER_SPREAD * torch.randn((nrows, d), device=device, generator=g) / d ** 0.5
    return x / x.norm(dim=1, keepdim=True)


def clustered_base(d, device):
    g = torch.Generator(device=device).manual_seed(CLUSTER_SEED)
    b = torch.randn(d, device=device, generator=g)
    return b / b.norm()


def build_shard(ix, rank, world, n_total, d, dtype, device, data):
    lo, hi = shard_bounds(n_total, world, rank)
    ix.reserve(hi - lo)
    chunk = 1 << 20
    if data == "clustered":
        base = clustered_base(d, device)
        for c0 in range(lo // CLUSTER_CHUNK * CLUSTER_CHUNK, hi, CLUSTER_CHUNK):
            rows = clustered_rows(c0 // CLUSTER_CHUNK, min(CLUSTER_CHUNK, n_total - c0), d, device, base)
            a, b = max(lo, c0), min(hi, c0 + rows.shape[0])
            ix.add(rows[a - c0:b - c0])
            del rows
    else:
        buf = torch.empty((min(chunk, hi - lo), d), dtype=torch_dt(dtype), device=device)
        for r0 in range(lo, hi, chunk):
            nr = min(chunk, hi - r0)
            part = buf[:nr]
            fx.synth_fill(part, r0, CORPUS_SEED)
            ix.add(part)
    ix.set_id_offset(lo)
    torch.cuda.synchronize()
    return lo, hi


def make_queries(nq, d, dtype, device, data):
    if data == "clustered":  # fp32 queries of the same distribution (not exact in 16 bits)
        g = torch.Generator(device=device).manual_seed(CLUSTER_SEED * 1_000_003)
        x = clustered_base(d, device)[None, :] + CLUSTER_SPREAD * torch.randn((nq, d), device=device,
                                                                             generator=g) / d ** 0.5
        return (x / x.norm(dim=1, keepdim=True)).contiguous()
    xq = torch.empty((nq, d), dtype=torch_dt(dtype), device=device)
    fx.synth_fill(xq, 0, QUERY_SEED)
    return xq


def shard_bounds(n_total, world, rank):  # == rag_faiss_embedding_amd.sharded.shard_bounds
    return n_total * rank // world, n_total * (rank + 1) // world


def ShardedIndexFlatL2(*a, **kw):
    from rag_faiss_embedding_amd.sharded import ShardedIndexFlatL2 as S
    return S(*a, **kw)


def one_step(six, xq, k):
    # ShardedIndexFlatL2.search: local fused scan -> RCCL all_gather of the
    # (nq x k) lists -> on-device merge (world 1: local scan only)
    return six.search(xq, k)


def oracle_lib_native():
    """Compile oracle/flat_l2.c for THIS host (-march=native) into a temp dir;
    fall back to the prebuilt x86-64-v3 library."""
    from oracle import cpu as C
    try:
        out = Path(tempfile.mkdtemp(prefix="fx_oracle_"))
        p = C.build(arch="-march=native", out_dir=out)
        return C, C.load(p), "-march=native"
    except Exception as e:  # noqa: BLE001
        log("native oracle build failed, using prebuilt:", e)
        return C, C.load(), "-march=x86-64-v3"


def oracle_corpus_chunks(args, n_total, d, dtype, device, rows=None):
    """(row0, fp32 rows as stored) chunks of the clustered corpus for the CPU
    oracle, regenerated on this GPU and rounded to the storage dtype."""
    base = clustered_base(d, device)
    end = n_total if rows is None else min(rows, n_total)
    for c0 in range(0, end, CLUSTER_CHUNK):
        x = clustered_rows(c0 // CLUSTER_CHUNK, min(CLUSTER_CHUNK, n_total - c0), d, device, base)
        x = x[:end - c0].to(torch_dt(dtype)).float().cpu().numpy()
        yield c0, x


class Heartbeat:
    """A stderr line every `period` s while a long silent leg runs (the
    full-corpus recall oracle takes minutes): the GPU box's runner takes a
    process that writes nothing for 3 minutes to be hung.  The oracle's C
    calls release the GIL, so the thread gets to run."""

    def __init__(self, what, period=30.0):
        import threading
        self.what, self.period, self.t0 = what, period, time.time()
        self.stop = threading.Event()
        self.th = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self.stop.wait(self.period):
            log(f"[bench] {self.what}: {time.time() - self.t0:.0f}s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()


def cpu_baseline_and_recall(args, n_total, d, dtype, k, D, I, xq_dev, nthreads, device):
    """cpu_baseline leg (rank 0): the repo's C/OpenMP restatement of FAISS's
    IndexFlatL2 BLAS path timed on a bounded sample of the same workload, and
    recall@10 of the GPU result against the exact CPU oracle on a query
    sample over the FULL corpus."""
    import numpy as np
    from oracle import flat_l2 as F
    C, lib, march = oracle_lib_native()
    res = {}
    # recall: exact oracle over the full corpus (rows regenerated on the fly) vs GPU ids
    nr = min(args.recall_queries, D.shape[0])
    qsel = np.linspace(0, D.shape[0] - 1, nr).astype(np.int64)
    t0 = time.time()
    if args.data == "clustered":
        xq = xq_dev[torch.from_numpy(qsel).to(xq_dev.device)].float().cpu().numpy()
        Ds, Is = [], []
        for c0, xb in oracle_corpus_chunks(args, n_total, d, dtype, device):
            Dc, Ic = C.knn_exact(xq, xb, k, nthreads)
            Ds.append(Dc)
            Is.append(np.where(Ic >= 0, Ic + c0, -1))
        Dr, Ir = F.merge_topk(Ds, Is, k)
    else:
        xq = np.concatenate([F.synth(QUERY_SEED, int(q), 1, d) for q in qsel])
        Dr, Ir = C.knn_exact_synth(CORPUS_SEED, n_total, d, xq, k, nthreads)
    t_rec = time.time() - t0
    Ig = I[qsel].cpu().numpy()
    Dgpu = D[qsel].cpu().numpy()
    hits = sum(len(set(Ig[i].tolist()) & set(Ir[i].tolist())) for i in range(nr))
    res["recall_at_10"] = hits / float(nr * k)
    res["ids_bit_exact"] = bool((Ig == Ir).all())
    res["max_rel_dist_err"] = float(np.max(np.abs(Dgpu.astype(np.float64) - Dr) / np.maximum(1.0, np.abs(Dr))))
    res["recall_sample"] = f"{nr} queries x full {n_total}-row corpus, exact CPU oracle ({t_rec:.1f}s)"
    # timed baseline: BLAS-path port on a corpus slice, extrapolated to n_total
    rows = min(n_total, args.cpu_rows)
    if args.data == "clustered":
        xb = np.concatenate([x for _, x in oracle_corpus_chunks(args, n_total, d, dtype, device, rows)])
        xall = xq_dev.float().cpu().numpy()
        xcal, xpool = xall[:128], xall
    else:
        xb = C.synth(CORPUS_SEED, 0, rows, d, nthreads)
        xcal, xpool = C.synth(QUERY_SEED, 0, 128, d, nthreads), None
    # size the timed sample to ~args.cpu_seconds of CPU work (calibrated)
    t0 = time.time()
    C.knn_blas(xcal, xb, k, nthreads, lib=lib)
    tcal = max(time.time() - t0, 1e-3)
    nq_s = int(min(50_000, max(128, 128 * args.cpu_seconds / tcal)))
    if args.cpu_queries:
        nq_s = args.cpu_queries
    if xpool is not None:
        nq_s = min(nq_s, xpool.shape[0])
        xqs = np.ascontiguousarray(xpool[:nq_s])
    else:
        xqs = C.synth(QUERY_SEED, 0, nq_s, d, nthreads)
    t0 = time.time()
    C.knn_blas(xqs, xb, k, nthreads, lib=lib)
    t = time.time() - t0
    qps = nq_s / (t * (n_total / rows))
    # the reference pins OMP/BLAS to one thread: same port at 1 thread
    nq_1 = max(16, min(nq_s, int(nq_s * 0.5 / max(nthreads, 1))))
    t0 = time.time()
    C.knn_blas(xqs[:nq_1], xb, k, 1, lib=lib)
    t1 = time.time() - t0
    res["cpu_baseline"] = {
        "value": qps, "unit": "queries/s", "cores": nthreads, "kind": "port",
        "sample": (f"{nq_s} queries x first {rows} rows (fp32) of the same corpus in {t:.2f}s, "
                   f"extrapolated linearly to {n_total} rows; C/OpenMP restatement of faiss "
                   f"IndexFlatL2 BLAS path (oracle/flat_l2.c, {march}); faiss-cpu is not installed"),
        "value_1thread": nq_1 / (t1 * (n_total / rows)),
        "sample_1thread": f"{nq_1} queries, same slice, 1 thread, {t1:.2f}s",
    }
    return res


def latency_nq1(ix, xq, I_dev, k, calls):
    """The reference's own call shape (faiss_store.py:61-64,
    rag_datastore_manager.py:215-218): ONE numpy float32 query in, host D / I
    out, one search per call, on the same index -- per-call wall latency
    (H2D, query prep, scan, refine + certification, D2H).  Queries cycle
    through the bench batch; every call's ids are checked against the
    device-resident batch result of the same query."""
    import numpy as np
    xq_h = xq.float().cpu().numpy()
    I_ref = I_dev.cpu().numpy()
    nq = xq_h.shape[0]
    for q in range(3):  # workspace sizing for nq = 1
        ix.search(xq_h[q:q + 1], k)
    ts, same = [], 0
    for c in range(calls):
        q = (c * 7919) % nq
        t0 = time.perf_counter()
        _, Ih = ix.search(xq_h[q:q + 1], k)
        ts.append(time.perf_counter() - t0)
        same += int((Ih[0] == I_ref[q]).all())
    ts = np.sort(np.asarray(ts)) * 1e3
    return {"median_ms": round(float(np.median(ts)), 4), "p10_ms": round(float(ts[len(ts) // 10]), 4),
            "p99_ms": round(float(ts[min(len(ts) - 1, (len(ts) * 99) // 100)]), 4), "calls": calls,
            "qps_serial": round(1e3 / float(np.median(ts)), 1),
            "form": "numpy float32 (1, d) query -> host D/I per call (H2D + search + D2H), serial calls",
            "ids_match_device_path": same == calls}


def latency_nq1_f32(calls, device, n=100_000, d=384, k=10, nq=1000):
    """latency_nq1 on the reference's own storage dtype and call shape: an fp32
    IndexFlatL2(384) (faiss_store.py:29, rag_datastore_manager.py:138) of
    config-(c) size, one numpy float32 query per call (faiss_store.py:61-64,
    rag_datastore_manager.py:215-218), host D / I out; every call's ids
    checked against the device-resident batch search of the same queries."""
    ix = fx.IndexFlatL2(d, device=device.index)
    buf = torch.empty((n, d), dtype=torch.float32, device=device)
    fx.synth_fill(buf, 0, CORPUS_SEED)
    ix.add(buf)
    del buf
    xq = torch.empty((nq, d), dtype=torch.float32, device=device)
    fx.synth_fill(xq, 0, QUERY_SEED)
    _, I = ix.search(xq, k)
    r = latency_nq1(ix, xq, I, k, calls)
    r["index"] = f"{n} x {d} fp32 IndexFlatL2 (the reference's storage dtype), synthetic rows"
    del ix
    return r


def _lib_digest():
    from rag_faiss_embedding_amd._provenance import file_digest
    return file_digest(_lib_path())


def _lib_path():
    from rag_faiss_embedding_amd import _lib
    return Path(_lib.LIB_PATH)


def source_digest():
    from rag_faiss_embedding_amd._provenance import source_digest as sd
    return sd()


def read_pmc_traffic(cfg_name, n_local, nq, data="synthetic"):
    """HBM bytes per scan launch from a committed rocprofv3 --pmc summary of
    this same workload (profiles/pmc_scan_<cfg>[_clustered].json), and where
    that figure comes from: (bytes, source) or (None, None).  The figure is a
    lookup of an earlier profiled run, not a counter of this one; `source`
    names its file, the scan's rocprof mean duration and the effective clock
    of that profiled run (GRBM_GUI_ACTIVE / 8 / wall)."""
    base = f"pmc_scan_{cfg_name}{'' if data == 'synthetic' else '_' + data}"
    p = ROOT / "profiles" / f"{base}_nq{nq}.json"  # a small-batch sweep point
    if not p.exists():
        p = ROOT / "profiles" / f"{base}.json"
    if not p.exists():
        return None, None
    try:
        j = json.loads(p.read_text())
        if j.get("rows_per_gpu") != n_local or j.get("nq") != nq:
            return None, None
        src = {"file": str(p.relative_to(ROOT)), "summary": j.get("source"),
               "note": "committed rocprofv3 --pmc pass of the same workload (not this run)",
               "csrc_digest": j.get("csrc_digest"), "git_head_at_summary": j.get("git_head_at_summary")}
        here = source_digest()
        if j.get("csrc_digest") != here:
            # counters of other kernels than the ones this run executes: no figure
            src["reason"] = (f"profiled sources {j.get('csrc_digest')} != this build's {here}: "
                             "traffic not quoted")
            return None, src
        summ = ROOT / j["source"] if j.get("source") else None
        if summ is not None and summ.exists():
            sj = json.loads(summ.read_text())
            scan = sj.get("kernels", {}).get(sj.get("scan_kernel"), {})
            src["kernel_ms"] = round(scan["avg_ms"], 3) if "avg_ms" in scan else None
            clk = sj.get("effective_clock_ghz")
            src["clock_ghz"] = round(clk, 3) if clk else None
            src["l2_hit_rate"] = round(sj["l2_hit_rate"], 3) if sj.get("l2_hit_rate") else None
        return j.get("hbm_bytes_per_launch"), src
    except Exception:  # noqa: BLE001
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="d", choices=sorted(CONFIGS))
    ap.add_argument("--data", default="synthetic", choices=["synthetic", "clustered"],
                    help="synthetic: counter-hash corpus/queries (exact in the storage dtype); clustered: "
                         "unit-norm rows around one direction, fp32 queries")
    ap.add_argument("--nq", type=int, default=0, help="override query batch")
    ap.add_argument("--rows", type=int, default=0, help="override corpus rows (testing)")
    ap.add_argument("--recall-queries", type=int, default=0,
                    help="oracle recall sample (0: per config, RECALL_QUERIES: d 1000, b 1000, e 256)")
    ap.add_argument("--cpu-rows", type=int, default=1_000_000)
    ap.add_argument("--cpu-queries", type=int, default=0, help="fixed CPU sample (0: auto-size)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU baseline sample time")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline / recall leg")
    ap.add_argument("--latency-calls", type=int, default=200, help="single-query host calls of the latency_nq1 leg")
    ap.add_argument("--ranks-check", action="store_true", help=argparse.SUPPRESS)  # tests: report the rank, exit
    args = ap.parse_args()

    plan = launch_plan(args.gpus, os.environ)
    if plan.startswith("error"):
        log(f"[bench] {plan}")
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.ranks_check:  # before any GPU work: which rank of which world this process is
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": int(os.environ.get("WORLD_SIZE", "1")),
                          "gpus": args.gpus}), flush=True)
        return

    global torch, dist, fx
    import torch as _torch  # before the HIP library: one runtime per process
    import torch.distributed as _dist
    torch, dist = _torch, _dist
    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd import faiss as _fx
    fx = _fx
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=device)

    n_total, d, dtype, nq, k = CONFIGS[args.config]
    if not args.recall_queries:
        args.recall_queries = RECALL_QUERIES[args.config]
    if args.nq:
        nq = args.nq
    if args.rows:
        n_total = args.rows

    t0 = time.time()
    ix = fx.IndexFlatL2(d, dtype=dtype, device=local)
    lo, hi = build_shard(ix, rank, world, n_total, d, dtype, device, args.data)
    n_local = hi - lo
    xq = make_queries(nq, d, dtype, device, args.data)
    six = ShardedIndexFlatL2(d, n_total, local_index=ix)
    torch.cuda.synchronize()
    log(f"[rank {rank}] shard rows [{lo}, {hi}) built in {time.time() - t0:.1f}s")

    for _ in range(args.warmup):
        one_step(six, xq, k)
    ix.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D, I = one_step(six, xq, k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    scan_ms, merge_ms, launches = ix.profile_read()
    ix.profile(False)
    fallbacks = ix.last_fallbacks()
    try:
        exact_fb = ix.last_exact_fallbacks()
    except AttributeError:  # an older library under FX_INDEX_LIB (same-box A/B)
        exact_fb = None
    try:  # candidate-list integrity: ids outside [0, ntotal) the refine had to drop (0 unless broken)
        dropped = ix.last_dropped_candidates()
    except AttributeError:
        dropped = None
    if world > 1:
        t = torch.tensor([elapsed, scan_ms / max(launches, 1), float(fallbacks), float(dropped or 0)],
                         dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, scan_avg_ms = float(t[0].item()), float(t[1].item())
        fallbacks = int(t[2].item())
        dropped = None if dropped is None else int(t[3].item())
    else:
        scan_avg_ms = scan_ms / max(launches, 1)

    value = nq * args.steps / elapsed
    # roofline of the dominant kernel (the fused scan): algorithmic work per launch
    flops = 2.0 * nq * n_local * d
    esize = 4 if dtype == "float32" else 2
    alg_bytes = n_local * d * esize + nq * d * esize + nq * k * 12
    t_scan = scan_avg_ms / 1e3
    mfma_tf = flops / t_scan / 1e12
    peak = MFMA_PEAK[dtype]
    split = dtype == "float32" and os.environ.get("FX_F32_SPLIT", "1") != "0"
    if split:  # fp32 index scanned as 3 bf16 products per term (fx_scan.hip F32S)
        peak = MFMA_PEAK["bfloat16"] / 3.0
    ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    if flops / alg_bytes >= ridge:
        roof = {"bound": "mfma", "achieved": round(mfma_tf, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(mfma_tf / peak, 4)}
    else:
        gbs = alg_bytes / t_scan / 1e9
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4)}
    # the committed PMC pass measured the default scan: no traffic figure for an opt-in variant
    variant = os.environ.get("FX_F32_SPLIT", "1") == "0"
    roof["traffic"], roof["traffic_source"] = (None, None) if variant else \
        read_pmc_traffic(args.config, n_local, nq, args.data)
    plan = ix.last_scan_plan()  # the timed searches' scan kernel (k_scan_v5: 64-row tiles)
    roof["kernel"] = ("k_scan_v5" if plan["tile_rows"] == 64 else "k_scan_v4") + \
        (" F32S (fp32 as 3 bf16 MFMA products)" if split else "") + \
        " (fused MFMA distance GEMM + top-k select)"
    roof["scan_plan"] = plan
    roof["kernel_ms_avg"] = round(scan_avg_ms, 4)
    roof["launches"] = launches
    roof["merge_refine_ms_avg"] = round(merge_ms / max(launches, 1), 4)

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": SHORT_DT[dtype],
        "data": ("synthetic: counter-hash corpus/queries generated on the GPU (exact in bf16/fp16/fp32)"
                 if args.data == "synthetic" else
                 f"synthetic clustered: unit-norm rows base + {CLUSTER_SPREAD} N(0, I/d) generated on the GPU, "
                 f"stored as {SHORT_DT[dtype]}; fp32 queries of the same distribution (inexact in {SHORT_DT[dtype]})"),
        "config": {
            "workload": (f"{n_total} x {d} {SHORT_DT[dtype]} flat L2 index, {nq}-query batch, top-{k}, "
                         + (f"row-sharded over {world} GPUs, one RCCL all_gather + on-device merge"
                            if world > 1 else "1 GPU")),
            "baseline_config": args.config, "corpus_rows": n_total, "dim": d, "nq": nq, "k": k,
            "rows_per_gpu": n_local, "parallelism": f"row-shard x{world}",
        },
        "build": {"csrc_digest": source_digest(), "lib": _lib_path().name,
                  "lib_digest": _lib_digest()},
        "fallback_queries_last_step": fallbacks,
        "exact_fallback_queries_last_step": exact_fb,
        "dropped_candidate_ids_last_step": dropped,
        "roofline": roof,
    }
    if world == 1:
        # the reference's call form: host float32 queries in, host D / I out
        # (PCIe both ways), same index -- reported beside `value`, never as it
        try:
            xq_h = xq.float().cpu().numpy()  # (fp32: exact for 16-bit synthetic queries)
            ix.search(xq_h, k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                Dh, Ih = ix.search(xq_h, k)
            t_h = (time.perf_counter() - t0) / 3
            out["pcie_inclusive"] = {
                "value": round(nq / t_h, 2), "unit": "queries/s", "ms_per_step": round(t_h * 1e3, 3),
                "form": "numpy float32 queries -> host D/I (H2D + search + D2H), 3 steps",
                "ids_match_device_path": bool((Ih == I.cpu().numpy()).all()),
            }
        except Exception as e:  # noqa: BLE001 -- a side measurement never breaks the bench line
            log("pcie-inclusive leg failed:", e)
        try:
            if args.latency_calls > 0:  # 0: skip (profiling runs keep only the bench's own launches)
                out["latency_nq1"] = latency_nq1(ix, xq, I, k, args.latency_calls)
        except Exception as e:  # noqa: BLE001
            log("latency_nq1 leg failed:", e)
        try:
            if args.latency_calls > 0:
                out["latency_nq1_f32"] = latency_nq1_f32(args.latency_calls, device)
        except Exception as e:  # noqa: BLE001
            log("latency_nq1_f32 leg failed:", e)
    if rank == 0 and not args.no_cpu:
        nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
        with Heartbeat("cpu leg (recall oracle, CPU baseline) running"):
            extra = cpu_baseline_and_recall(args, n_total, d, dtype, k, D, I, xq, nthreads, device)
        if world > 1:
            extra.pop("cpu_baseline", None)
        out.update(extra)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
