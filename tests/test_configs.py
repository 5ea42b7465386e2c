"""GPU parity at the BASELINE.json workload shapes ("next round" 1).

* (e) 100M x 384 fp16, 10k-query batch: the whole 100M-row index on one GPU,
  and one eighth of it (a 12.5M-row shard, the per-GPU share at 8 GPUs), each
  with the full 10k batch;
* (d) 10M x 768 bf16, 10k-query batch: the 1.25M-row shard of one GPU at 8
  GPUs, and the whole 10M corpus as 8 row shards (global id offsets) merged by
  fx_merge_shards -- the on-device step after the RCCL all_gather -- checked
  against one 10M-row index and the streaming oracle;
* (c) encoder -> index hand-off: the device tensor path equals the host numpy
  path (the reference's ``.cpu().numpy()`` form, vectorization.py:44 ->
  faiss_store.py:46) and the oracle.

Oracle: the exact streaming restatement of faiss IndexFlatL2 (oracle/flat_l2.c,
rows regenerated from the shared counter-hash generator), on a query subset;
every query of the batch is checked for sortedness / id range / no fallback.
Bar: ids bit-exact, |dD| <= 1e-5 max(1, |D|) (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

from oracle import cpu as C
from oracle import flat_l2 as F
from tests.test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu

CSEED, QSEED = 1234, 4321


@pytest.fixture(scope="module")
def fx():
    from rag_faiss_embedding_amd import _lib, faiss
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return faiss


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _synth_index(fx, torch, n, d, dtype, row0=0, chunk=1 << 21):
    tdt = getattr(torch, dtype)
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.reserve(n)
    buf = torch.empty((min(chunk, n), d), dtype=tdt, device="cuda")
    for r0 in range(0, n, chunk):
        part = buf[:min(chunk, n - r0)]
        fx.synth_fill(part, row0 + r0, CSEED)
        ix.add(part)
    ix.set_id_offset(row0)
    return ix


def _queries(fx, torch, nq, d, dtype):
    xq = torch.empty((nq, d), dtype=getattr(torch, dtype), device="cuda")
    fx.synth_fill(xq, 0, QSEED)
    return xq


def _check_batch(D, I, n_lo, n_hi):
    D = D.cpu().numpy()
    I = I.cpu().numpy()
    assert (np.diff(D, axis=1) >= 0).all()
    assert (I >= n_lo).all() and (I < n_hi).all()
    return D, I


# oracle sample (>= 1,000 queries where the oracle allows): the
# streaming oracle costs ~0.03 s per query on the (d) shard, ~0.15 s on (e)
@pytest.mark.timeout(400)
@pytest.mark.parametrize("cfg,n,d,dtype,nsub", [
    ("e", 12_500_000, 384, "float16", 512),    # 100M x 384 fp16 / 8
    ("d", 1_250_000, 768, "bfloat16", 1000),   # 10M x 768 bf16 / 8
])
def test_config_shard_full_batch(fx, torch_cuda, cfg, n, d, dtype, nsub):
    torch = torch_cuda
    ix = _synth_index(fx, torch, n, d, dtype)
    xq = _queries(fx, torch, 10_000, d, dtype)
    D, I = ix.search(xq, 10)
    assert ix.last_fallbacks() == 0
    D, I = _check_batch(D, I, 0, n)
    sub = np.linspace(0, 9_999, nsub).astype(np.int64)
    Dr, Ir = C.knn_exact_synth(CSEED, n, d, F.synth(QSEED, 0, 10_000, d)[sub], 10)
    assert_parity(D[sub], I[sub], Dr, Ir)
    # self-retrieval at the shard's edges
    rows = np.array([0, 1, n // 3, n - 2, n - 1])
    Ds, Is = ix.search(np.concatenate([F.synth(CSEED, int(r), 1, d) for r in rows]), 2)
    assert (Is[:, 0] == rows).all() and (Ds[:, 0] == 0).all()


@pytest.mark.timeout(600)
def test_config_d_eight_shards_merged(fx, torch_cuda):
    """Config (d) end to end at N=8 on one GPU: 8 contiguous row shards with
    global id offsets (sharded.shard_bounds), each searched with the full 10k
    batch, then the [8][nq][k] lists merged on the device."""
    torch = torch_cuda
    from rag_faiss_embedding_amd.sharded import shard_bounds
    n, d, nq, k = 10_000_000, 768, 10_000, 10
    xq = _queries(fx, torch, nq, d, "bfloat16")
    Ds, Is = [], []
    for g in range(8):
        lo, hi = shard_bounds(n, 8, g)
        ix = _synth_index(fx, torch, hi - lo, d, "bfloat16", row0=lo)
        D, I = ix.search(xq, k)
        assert ix.last_fallbacks() == 0
        _check_batch(D, I, lo, hi)
        Ds.append(D)
        Is.append(I)
        del ix
    Dm, Im = fx.merge_shards(fx.METRIC_L2, torch.stack(Ds), torch.stack(Is), k)
    Dm, Im = _check_batch(Dm, Im, 0, n)
    del Ds, Is
    # the same corpus as ONE index: identical lists
    ix = _synth_index(fx, torch, n, d, "bfloat16")
    D1, I1 = ix.search(xq, k)
    np.testing.assert_array_equal(I1.cpu().numpy(), Im)
    np.testing.assert_array_equal(D1.cpu().numpy(), Dm)
    # 1,000 oracle queries over the full 10M rows (the streaming oracle's
    # integer path: ~30-60 s on the box's host cores)
    sub = np.linspace(0, nq - 1, 1000).astype(np.int64)
    Dr, Ir = C.knn_exact_synth(CSEED, n, d, F.synth(QSEED, 0, nq, d)[sub], k)
    assert_parity(Dm[sub], Im[sub], Dr, Ir)


@pytest.mark.timeout(600)
def test_config_e_full_index(fx, torch_cuda):
    """Config (e) at its stated size on one GPU: ONE 100M x 384 fp16 index
    (76.8 GB of codes, the north star's HBM-bound point) searched with the
    full 10k batch.  Properties on every query (sorted lists, ids in range,
    no fallback, self-retrieval at the index's edges); the streaming oracle
    over all 100M rows on a 128-query subset."""
    torch = torch_cuda
    n, d, nq, k = 100_000_000, 384, 10_000, 10
    ix = _synth_index(fx, torch, n, d, "float16")
    assert ix.ntotal == n
    xq = _queries(fx, torch, nq, d, "float16")
    D, I = ix.search(xq, k)
    assert ix.last_fallbacks() == 0 and ix.last_exact_fallbacks() == 0
    D, I = _check_batch(D, I, 0, n)
    rows = np.array([0, 1, n // 2, n - 129, n - 128, n - 2, n - 1])
    Ds, Is = ix.search(np.concatenate([F.synth(CSEED, int(r), 1, d) for r in rows]), 2)
    assert (Is[:, 0] == rows).all() and (Ds[:, 0] == 0).all()
    sub = np.linspace(0, nq - 1, 128).astype(np.int64)
    Dr, Ir = C.knn_exact_synth(CSEED, n, d, F.synth(QSEED, 0, nq, d)[sub], k)
    assert_parity(D[sub], I[sub], Dr, Ir)


def _tokens(torch, n, lo, hi, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(lo, hi + 1, (n,), generator=g)
    ids = torch.randint(1000, 30522, (n, hi), generator=g)
    ids = torch.where(torch.arange(hi)[None, :] < lens[:, None], ids, torch.zeros_like(ids))
    ids[:, 0] = 101
    ids[torch.arange(n), lens - 1] = 102
    return ids, lens


def test_config_c_device_handoff_equals_host_path(fx, torch_cuda):
    """Config (c) at its stated size (BASELINE.json: 100k encoded chunks,
    initialize_rag.py:57-61 -> vectorization.py:25-44 -> faiss_store.py:46)
    with 1,000 encoded queries: encoder embeddings handed to the index on the
    device give the same results as the reference's host hand-off, and the
    oracle's on every query."""
    torch = torch_cuda
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    pipe = VectorizationPipeline(device="cuda", precision="fp32", seed=0, allow_random_init=True)
    ids, lens = _tokens(torch, 100_000, 16, 128, 11)
    qids, qlens = _tokens(torch, 1000, 8, 48, 12)
    emb = pipe.encode_lengths(ids.cuda(), lens, 256)
    qemb = pipe.encode_lengths(qids.cuda(), qlens, 256)
    assert emb.dtype == torch.float32 and emb.is_cuda
    dev = fx.IndexFlatL2(384)
    dev.add(emb)
    Dd, Id = dev.search(qemb, 10)
    host = fx.IndexFlatL2(384)
    xb = emb.cpu().numpy()
    host.add(xb)
    xq = qemb.cpu().numpy()
    Dh, Ih = host.search(xq, 10)
    np.testing.assert_array_equal(Id.cpu().numpy(), Ih)
    np.testing.assert_array_equal(Dd.cpu().numpy(), Dh)
    assert dev.last_fallbacks() == 0 and host.last_fallbacks() == 0
    Dr, Ir = C.knn_exact(xq, xb, 10)
    assert_parity(Dh, Ih, Dr, Ir)
