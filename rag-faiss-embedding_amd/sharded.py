"""Row-sharded flat index over the GPUs of one node (one process per GPU).

The reference is single-process; the multi-GPU layout
is this build's own: the corpus is split into contiguous row blocks, rank r
holding global rows [offset_r, offset_r + n_r).  A search runs the local
fused scan on every rank (local top-k with GLOBAL ids), exchanges the
(nq x k) result lists with ONE all_gather over RCCL/xGMI (the only data-path
collective), and merges them on the device (``fx_merge_shards``).  Because the
offsets are monotone in rank, "ties -> smaller id" survives the merge.

Works with any ``torch.distributed`` process group: ``nccl`` (= RCCL) in
production -- host (numpy) queries and results included: the exchange stages
them on the rank's GPU, RCCL's only memory -- and ``gloo`` with host tensors
in the CPU tests, where ``local_index`` / ``merge_fn`` can be test doubles.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, near-equal row block of ``rank`` (same rule as bench.py)."""
    return n_total * rank // world, n_total * (rank + 1) // world


class ShardedIndexFlatL2:
    """``IndexFlatL2`` semantics over a process group.

    add(x_global_block, row0): every rank is handed a block of global rows
    starting at ``row0`` (the same block on every rank, or only its own part)
    and keeps the rows it owns; ``n_total`` fixes the ownership split.
    """

    def __init__(self, d: int, n_total: int, dtype: str = "float32", group=None, device: Optional[int] = None,
                 local_index=None, merge_fn: Optional[Callable] = None):
        self.d = int(d)
        self.n_total = int(n_total)
        self.group = group
        ready = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if ready else 1
        self.rank = dist.get_rank(group) if ready else 0
        self.lo, self.hi = shard_bounds(self.n_total, self.world, self.rank)
        if local_index is None:
            from . import faiss as fx
            local_index = fx.IndexFlatL2(d, dtype=dtype, device=device if device is not None else 0)
            local_index.set_id_offset(self.lo)
        self._merge = merge_fn if merge_fn is not None else self._device_merge
        self.local = local_index

    def _device_merge(self, Dg, Ig, k):
        """fx_merge_shards on the local index's GPU; gathered host tensors (a
        gloo group) go there and come back."""
        from . import faiss as fx
        dev = torch.device("cuda", self.local.device)
        on_host = not Dg.is_cuda
        Dm, Im = fx.merge_shards(self.local.metric_type, Dg.to(dev), Ig.to(dev), k)
        return (Dm.cpu(), Im.cpu()) if on_host else (Dm, Im)

    @property
    def ntotal(self) -> int:
        if self.world == 1:
            return self.local.ntotal
        t = torch.tensor([self.local.ntotal], dtype=torch.int64)
        if dist.get_backend(self.group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def add(self, x, row0: int = 0) -> None:
        """Keep the rows of ``x`` (global rows row0 .. row0+len(x)-1) that
        fall in this rank's block."""
        n = x.shape[0]
        a = max(self.lo, row0)
        b = min(self.hi, row0 + n)
        if b > a:
            self.local.add(x[a - row0:b - row0])

    def comm_device(self, like: "torch.Tensor") -> "torch.device":
        """Where the exchange's buffers live.  RCCL (backend ``nccl``) moves
        device memory only, so host results (the reference's numpy call form,
        faiss_store.py:61-64) go to this rank's GPU first; gloo takes the
        tensors where they are."""
        if dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", int(getattr(self.local, "device", 0)))
        return like.device

    def exchange(self, D, I, k: int):
        """ONE all_gather of the packed local (D, I) lists (nq*k*12 B per
        rank) -> merge into the global top-k.  Host (numpy) lists come back
        as numpy, device tensors stay on the device."""
        is_np = isinstance(D, np.ndarray)
        Dt = torch.from_numpy(np.ascontiguousarray(D)) if is_np else D
        It = torch.from_numpy(np.ascontiguousarray(I)) if is_np else I
        dev = self.comm_device(Dt)
        Dt, It = Dt.to(dev), It.to(dev)
        nq = Dt.shape[0]
        # pack each (D f32, I i64) entry as 3 int32 words: one collective per batch
        mine = torch.empty((nq, k, 3), dtype=torch.int32, device=dev)
        mine[:, :, 0] = Dt.contiguous().view(torch.int32)
        mine[:, :, 1:] = It.contiguous().view(torch.int32).view(nq, k, 2)
        allg = torch.empty((self.world * nq, k, 3), dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(allg, mine, group=self.group)
        allg = allg.view(self.world, nq, k, 3)
        Dg = allg[..., 0].contiguous().view(torch.float32)
        Ig = allg[..., 1:].contiguous().view(torch.int64).view(self.world, nq, k)
        Dm, Im = self._merge(Dg, Ig, k)
        if is_np:
            as_np = lambda t: t.cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)  # noqa: E731
            return as_np(Dm), as_np(Im)
        return Dm, Im

    def search(self, xq, k: int):
        """Global top-k: local scan -> exchange (one all_gather + merge).

        Host queries under RCCL (the reference's numpy call form,
        faiss_store.py:61-64): the queries go to this rank's GPU once, the
        local scan, the all_gather and the merge stay on the device, and the
        merged lists come back in ONE device-to-host copy (numpy in -> numpy
        out, a host tensor -> host tensors).

        A host-input search fails on EVERY rank when one rank's local search
        failed or dropped corrupted candidate ids (one flag all_reduce before
        the exchange), so the ranks' collectives stay in step."""
        if self.world == 1:
            return self.local.search(xq, k)
        host_in = not (isinstance(xq, torch.Tensor) and xq.is_cuda)
        if host_in and dist.get_backend(self.group) == "nccl":
            return self.search_host_on_device(xq, k)
        if not host_in:  # device lists: the caller reads the integrity count
            D, I = self.local.search(xq, k)
            return self.exchange(D, I, k)
        D = I = None
        why = None
        try:
            D, I = self.local.search(xq, k)  # host output: raises FX_E_INTEGRITY itself
        except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
            why = f"{type(e).__name__}: {e}"
        self._agree(why, torch.zeros(1))
        return self.exchange(D, I, k)

    def search_host_on_device(self, xq, k: int):
        """search() of host queries under RCCL: H2D of the queries, local
        scan, all_gather and merge on the exchange device, ONE D2H of the
        merged lists (numpy in -> numpy out, a host tensor -> host tensors)."""
        is_np = not isinstance(xq, torch.Tensor)
        xt = torch.from_numpy(np.ascontiguousarray(xq, dtype=np.float32)) if is_np else xq
        dev = self.comm_device(xt)
        D = I = None
        why = None
        try:
            D, I = self.local.search(xt.to(dev), k)
            why = self._integrity_problem()
        except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
            why = f"{type(e).__name__}: {e}"
        self._agree(why, xt.new_zeros(1).to(dev))
        Dm, Im = self.exchange(D, I, k)
        Dm, Im = Dm.cpu(), Im.cpu()
        return (Dm.numpy(), Im.numpy()) if is_np else (Dm, Im)

    def _integrity_problem(self) -> Optional[str]:
        """A host-output search fails when the local scan's candidate lists
        held row ids outside [0, ntotal), as the single-index host search does
        (FX_E_INTEGRITY, fx_index.h): the local search here ran with device
        outputs (stream-ordered), so its dropped count is read (a stream sync)
        before the exchange.  Device-output callers read
        ``local.last_dropped_candidates()`` themselves."""
        dropped = getattr(self.local, "last_dropped_candidates", None)
        n = dropped() if dropped is not None else 0
        if n > 0:
            return f"local search dropped {n} corrupted candidate ids: its top-k may be missing rows"
        return None

    def _agree(self, why: Optional[str], like: "torch.Tensor") -> None:
        """All ranks learn whether any rank's local search failed (one MAX
        all_reduce of a flag on the exchange device) and then all raise
        FxError together -- never only the failing rank, whose peers would
        otherwise wait in the next collective."""
        flag = torch.tensor([1.0 if why else 0.0], dtype=torch.float32, device=self.comm_device(like))
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        if float(flag.item()) > 0:
            from ._lib import FxError
            raise FxError(why if why else "the local search failed on another rank of the group")
