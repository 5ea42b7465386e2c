"""Multi-process (world_size 2, gloo, CPU) coverage of the row-sharded search
path: ownership split, global id offsets, the all_gather exchange and the
(D, id) merge.  The per-rank index and the merge are oracle-backed test
doubles here (the GPU kernels are covered by test_gpu_parity.py); the
orchestration code under test is rag_faiss_embedding_amd.sharded."""
import os
import socket

import numpy as np
import pytest
import torch
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


class _DevShard(_OracleShard):
    device = 3  # the rank's GPU ordinal (read by comm_device)


def _fake_gather(calls, world):
    def gather(out, inp, group=None):
        calls.append(inp.device)
        # rank r's lists: the same entries with ids shifted by r * 1000
        parts = []
        for r in range(world):
            p = inp.clone()
            ids = p[:, :, 1:].contiguous().view(torch.int64) + r * 1000
            p[:, :, 1:] = ids.view(torch.int32).view(p.shape[0], p.shape[1], 2)
            parts.append(p)
        out.copy_(torch.cat(parts))
    return gather



def test_exchange_buffers_follow_the_backend(monkeypatch):
    """Under RCCL (backend "nccl") the all_gather must see device tensors even
    when the local search returned host numpy (the reference's call form,
    faiss_store.py:61-64); under gloo the host tensors are used as they are.
    The device decision is comm_device(); the GPU suite runs the real RCCL
    exchange (test_sharded_gpu.py::test_exchange_under_rccl_host_inputs)."""
    from rag_faiss_embedding_amd.sharded import ShardedIndexFlatL2
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda g=None: 2)
    monkeypatch.setattr(dist, "get_rank", lambda g=None: 0)
    ix = ShardedIndexFlatL2(8, 100, local_index=_DevShard(8, 0), merge_fn=_oracle_merge)
    host = torch.zeros(2, 2)
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "nccl")
    assert ix.comm_device(host) == torch.device("cuda", 3)
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "gloo")
    assert ix.comm_device(host) == host.device
    # the gloo exchange of host lists: numpy in, numpy out, merged across ranks
    calls = []
    monkeypatch.setattr(dist, "all_gather_into_tensor", _fake_gather(calls, 2))
    D = np.array([[0.5, 1.0, 2.0]], dtype=np.float32)
    I = np.array([[7, 3, 9]], dtype=np.int64)
    Dm, Im = ix.exchange(D, I, 3)
    assert calls == [torch.device("cpu")]
    assert isinstance(Dm, np.ndarray) and isinstance(Im, np.ndarray)
    assert Im.tolist() == [[7, 1007, 3]] and Dm.tolist() == [[0.5, 0.5, 1.0]]


def test_host_queries_under_rccl_stay_on_the_device(monkeypatch):
    """Host (numpy) queries under the nccl backend: the local search is handed
    the queries as a tensor on the exchange's device (not numpy), the
    all_gather and the merge run there, and the merged lists are converted to
    numpy once at the end (no host round trip of the local lists).  The
    comm device is the CPU here; the GPU suite's RCCL tests run it for real."""
    from rag_faiss_embedding_amd.sharded import ShardedIndexFlatL2
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda g=None: 2)
    monkeypatch.setattr(dist, "get_rank", lambda g=None: 0)
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "nccl")
    monkeypatch.setattr(ShardedIndexFlatL2, "comm_device", lambda self, like: torch.device("cpu"))
    seen = []

    class _TensorShard(_OracleShard):
        def search(self, xq, k):
            seen.append(type(xq))
            D, I = super().search(xq.numpy(), k)
            return torch.from_numpy(D), torch.from_numpy(I)

    def merge(Dg, Ig, k):
        assert isinstance(Dg, torch.Tensor) and isinstance(Ig, torch.Tensor)
        Dm, Im = F.merge_topk(list(Dg.numpy()), list(Ig.numpy()), k)
        return torch.from_numpy(Dm), torch.from_numpy(Im)

    rng = np.random.default_rng(3)
    xb = rng.standard_normal((50, 8)).astype(np.float32)
    ix = ShardedIndexFlatL2(8, 100, local_index=_TensorShard(8, 0), merge_fn=merge)
    ix.add(xb)
    calls = []
    monkeypatch.setattr(dist, "all_gather_into_tensor", _fake_gather(calls, 2))
    monkeypatch.setattr(dist, "all_reduce", lambda t, op=None, group=None: None)  # the integrity flag: 0
    xq = rng.standard_normal((4, 8))  # float64: converted like faiss (float32)
    D, I = ix.search(xq, 5)
    assert seen == [torch.Tensor] and len(calls) == 1
    assert isinstance(D, np.ndarray) and isinstance(I, np.ndarray)
    Dr, Ir = F.knn_exact(xq.astype(np.float32), xb, 5)
    # rank 1's lists are rank 0's with ids + 1000 (the fake gather): ties at
    # equal distance keep the smaller id
    assert (I[:, 0] == Ir[:, 0]).all() and (D[:, 0] == Dr[:, 0]).all()


def test_host_queries_under_rccl_fail_on_dropped_candidates(monkeypatch):
    """The sharded host-in path reports a corrupted local scan (candidate ids
    outside [0, ntotal)) as an error, like the single-index host search's
    FX_E_INTEGRITY, instead of returning a thinner top-k."""
    from rag_faiss_embedding_amd._lib import FxError
    from rag_faiss_embedding_amd.sharded import ShardedIndexFlatL2
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda g=None: 2)
    monkeypatch.setattr(dist, "get_rank", lambda g=None: 0)
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "nccl")
    monkeypatch.setattr(ShardedIndexFlatL2, "comm_device", lambda self, like: torch.device("cpu"))

    class _BadShard(_OracleShard):
        def search(self, xq, k):
            D, I = super().search(xq.numpy(), k)
            return torch.from_numpy(D), torch.from_numpy(I)

        def last_dropped_candidates(self):
            return 3

    def merge(Dg, Ig, k):
        Dm, Im = F.merge_topk(list(Dg.numpy()), list(Ig.numpy()), k)
        return torch.from_numpy(Dm), torch.from_numpy(Im)

    rng = np.random.default_rng(4)
    ix = ShardedIndexFlatL2(8, 100, local_index=_BadShard(8, 0), merge_fn=merge)
    ix.add(rng.standard_normal((50, 8)).astype(np.float32))
    gathers, reduces = [], []
    monkeypatch.setattr(dist, "all_gather_into_tensor", _fake_gather(gathers, 2))
    monkeypatch.setattr(dist, "all_reduce", lambda t, op=None, group=None: reduces.append(float(t.item())))
    with pytest.raises(FxError, match="dropped 3"):
        ix.search(rng.standard_normal((4, 8)).astype(np.float32), 5)
    # the flag was agreed on BEFORE the exchange: no all_gather with a bad list
    assert reduces == [1.0] and gathers == []


def _fail_worker(rank, world, port, q, mode):
    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd._lib import FxError
    from rag_faiss_embedding_amd.sharded import ShardedIndexFlatL2, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _Shard(_OracleShard):
        def search(self, xq, k):
            if rank == world - 1:  # only the last rank's local search fails
                raise FxError("search: 2 candidate row ids outside [0, n) were dropped (corrupted scan list)")
            return super().search(xq, k)

    try:
        rng = np.random.default_rng(5)
        n, d = 300, 8
        xb = rng.standard_normal((n, d)).astype(np.float32)
        lo, _ = shard_bounds(n, world, rank)
        ix = ShardedIndexFlatL2(d, n, local_index=_Shard(d, lo), merge_fn=_oracle_merge)
        ix.add(xb)
        outcome = "ok"
        try:
            ix.search(xb[:4], 5)
        except FxError as e:
            outcome = "raised" + (" own" if "dropped" in str(e) else " peer")
        # the group is still in step: one more collective completes on every rank
        t = torch.ones(1)
        dist.all_reduce(t)
        q.put((rank, outcome, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank_local_failure_raises_on_every_rank(world):
    """a host-input search whose local scan fails on ONE rank makes
    every rank raise (after one flag all_reduce), and the group stays usable."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q, "host")) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert [r[1] for r in res] == ["raised peer"] * (world - 1) + ["raised own"], res
    assert all(r[2] == float(world) for r in res)
