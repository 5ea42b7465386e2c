"""Multi-process (world_size 2, gloo, CPU) coverage of the row-sharded search
path: ownership split, global id offsets, the all_gather exchange and the
(D, id) merge.  The per-rank index and the merge are oracle-backed test
doubles here (the GPU kernels are covered by test_gpu_parity.py); the
orchestration code under test is rag_faiss_embedding_amd.sharded."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import flat_l2 as F


class _OracleShard:
    def __init__(self, d, offset):
        self.d = d
        self.offset = offset
        self.xb = np.zeros((0, d), dtype=np.float32)

    @property
    def ntotal(self):
        return self.xb.shape[0]

    def add(self, x):
        self.xb = np.vstack([self.xb, np.asarray(x, dtype=np.float32)])

    def search(self, xq, k):
        D, I = F.knn_exact(xq, self.xb, k)
        return D, np.where(I >= 0, I + self.offset, -1)


def _oracle_merge(Dg, Ig, k):
    return F.merge_topk(list(Dg.numpy()), list(Ig.numpy()), k)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd.sharded import ShardedIndexFlatL2, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        n, d = 2501, 24
        xb = rng.standard_normal((n, d)).astype(np.float32)
        # duplicates straddling the shard boundary: ties must break to the smaller id
        lo1, _ = shard_bounds(n, world, 1)
        xb[lo1 - 1] = xb[lo1] = xb[7]
        xq = np.vstack([xb[7:8] + 0.01, rng.standard_normal((20, d)).astype(np.float32)])
        lo, _ = shard_bounds(n, world, rank)
        ix = ShardedIndexFlatL2(d, n, local_index=_OracleShard(d, lo), merge_fn=_oracle_merge)
        # every rank is handed the full corpus in two blocks; each keeps its rows
        ix.add(xb[:1000], row0=0)
        ix.add(xb[1000:], row0=1000)
        assert ix.ntotal == n
        D, I = ix.search(xq, 10)
        Dr, Ir = F.knn_exact(xq, xb, 10)
        ok = bool((I == Ir).all() and (D == Dr).all())
        q.put((rank, ok, I[0].tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_search_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok, _ in res), res
    assert all(r[2] == res[0][2] for r in res)


def test_shard_bounds_cover_rows():
    from rag_faiss_embedding_amd.sharded import shard_bounds
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
