"""k > 32, the device-decided exact fallback and the stream-ordered device
search (faiss_store.py:49,64 pass the caller's k to IndexFlatL2.search, which
has no cap in faiss; the reference's results never wait on anything but the
search itself).

Parity bar as in test_gpu_parity.py: ids bit-exact, |dD| <= 1e-5 max(1, |D|).
k > 32 takes k_refine_big (block top-K re-rank of the splits' candidate
lists, scan without the shared threshold); FX_FORCE_FALLBACK=1 flags every
query so the device-gated exact fallback (k_fb_scan / k_fb_merge) produces
every result.  k > 1024 (FX_MAX_K) takes the exact sort path (fx_hugek.hip):
exact keys of every (query, row) pair and one radix sort per query -- a
segmented sort per batch up to 65,536 rows, a device-wide sort per query
above -- so its results must equal the oracle's at any k.
"""
import numpy as np
import pytest

from oracle import cpu as C
from oracle import flat_l2 as F
from tests.test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


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


@pytest.fixture(scope="module")
def gauss():
    rng = np.random.default_rng(33)
    xb = rng.standard_normal((200_000, 384)).astype(np.float32)
    xq = rng.standard_normal((24, 384)).astype(np.float32)
    return xb, xq


@pytest.mark.parametrize("k", [33, 100, 256, 1024])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_big_k_parity(fx, gauss, k, dtype):
    xb, xq = gauss
    ix = fx.IndexFlatL2(384, dtype=dtype)
    ix.add(xb)
    D, I = ix.search(xq, k)
    Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, xb.shape[0]), k)
    assert_parity(D, I, Dr, Ir)
    print(f"k={k} {dtype}: fallbacks {ix.last_fallbacks()} of {len(xq)}")
    assert ix.last_fallbacks() <= len(xq) // 4


def test_big_k_inner_product(fx, gauss):
    xb, xq = gauss
    ix = fx.IndexFlatIP(384)
    ix.add(xb[:50_000])
    D, I = ix.search(xq, 100)
    Dr, Ir = F.knn_inner_product(xq, xb[:50_000], 100)
    assert_parity(D, I, Dr, Ir)


def test_big_k_1m_bf16(fx, torch_cuda):
    """k = 100 on a 1M x 768 bf16 corpus (the config (d) shard dtype)."""
    torch = torch_cuda
    n, d = 1_000_000, 768
    xb = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
    fx.synth_fill(xb, 0, 1234)
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    ix.add(xb)
    del xb
    xq = torch.empty((256, d), dtype=torch.bfloat16, device="cuda")
    fx.synth_fill(xq, 0, 4321)
    D, I = ix.search(xq, 100)
    D, I = D.cpu().numpy(), I.cpu().numpy()
    assert (np.diff(D, axis=1) >= 0).all() and (I >= 0).all() and (I < n).all()
    assert all(len(set(r)) == 100 for r in I.tolist())
    sub = np.arange(0, 256, 16)
    Dr, Ir = C.knn_exact_synth(1234, n, d, F.synth(4321, 0, 256, d)[sub], 100)
    assert_parity(D[sub], I[sub], Dr, Ir)
    print(f"1M x 768 bf16, k=100: fallbacks {ix.last_fallbacks()} of 256")


def test_k_beyond_ntotal_pads(fx):
    rng = np.random.default_rng(5)
    xb = rng.standard_normal((50, 32)).astype(np.float32)
    xq = rng.standard_normal((3, 32)).astype(np.float32)
    ix = fx.IndexFlatL2(32)
    ix.add(xb)
    D, I = ix.search(xq, 100)
    Dr, Ir = C.knn_exact(xq, xb, 50)
    assert_parity(D[:, :50], I[:, :50], Dr, Ir)
    assert (I[:, 50:] == -1).all() and (D[:, 50:] == np.float32(3.4028234663852886e38)).all()


@pytest.mark.parametrize("k", [10, 100])
def test_forced_fallback_is_exact(diag_fx, gauss, monkeypatch, k):
    """Every query through the device-gated exact fallback (force_fallback 2:
    past the re-scan too; a hook of the diagnostic build): same results."""
    xb, xq = gauss
    ix = diag_fx.IndexFlatL2(384)
    ix.add(xb[:100_000])
    ix.set_option("force_fallback", 2)
    D, I = ix.search(xq, k)
    assert ix.last_fallbacks() == len(xq) and ix.last_exact_fallbacks() == len(xq)
    Dr, Ir = C.knn_exact(xq, xb[:100_000], k)
    assert_parity(D, I, Dr, Ir)


def test_forced_fallback_many_queries(diag_fx, monkeypatch):
    """More flagged queries than the fallback's work-item budget splits for
    (fbs shrinks as nf grows): 5000 flagged queries on a small corpus."""
    rng = np.random.default_rng(6)
    xb = rng.standard_normal((3000, 64)).astype(np.float32)
    xq = rng.standard_normal((5000, 64)).astype(np.float32)
    ix = diag_fx.IndexFlatL2(64)
    ix.add(xb)
    ix.set_option("force_fallback", 2)
    D, I = ix.search(xq, 7)
    assert ix.last_fallbacks() == 5000 and ix.last_exact_fallbacks() == 5000
    Dr, Ir = C.knn_exact(xq, xb, 7)
    assert_parity(D, I, Dr, Ir)


@pytest.mark.stream_ordered
def test_device_search_is_stream_ordered(fx, torch_cuda):
    """FX_MEM_DEVICE search enqueues and returns: queued behind a ~0.1 s spin
    kernel on the same stream, the call comes back while that stream is still
    busy (a host sync inside would have waited for the spin to finish)."""
    torch = torch_cuda
    n, d, nq = 200_000, 768, 512
    xb = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
    fx.synth_fill(xb, 0, 99)
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    ix.add(xb)
    xq = torch.empty((nq, d), dtype=torch.bfloat16, device="cuda")
    fx.synth_fill(xq, 0, 98)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ix.search(xq, 10)            # sizes the workspace (may allocate)
        s.synchronize()
        torch.cuda._sleep(200_000_000)
        D, I = ix.search(xq, 10)     # the measured call: nothing to allocate
        pending = not s.query()
    s.synchronize()
    assert pending, "device search returned only after the stream had drained"
    Dh, Ih = ix.search(xq[:64].float().cpu().numpy(), 10)
    assert (I[:64].cpu().numpy() == Ih).all()
    assert ix.last_fallbacks() == 0


def test_device_add_is_stream_ordered(fx, torch_cuda):
    torch = torch_cuda
    n, d = 100_000, 384
    x = torch.empty((n, d), dtype=torch.float16, device="cuda")
    fx.synth_fill(x, 0, 7)
    ix = fx.IndexFlatL2(d, dtype="float16")
    ix.reserve(2 * n)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        torch.cuda._sleep(200_000_000)
        ix.add(x)
        pending = not s.query()
        ix.add(x)
    s.synchronize()
    assert pending, "device add returned only after the stream had drained"
    assert ix.ntotal == 2 * n
    q = F.synth(7, 123, 1, d)
    Ds, Is = ix.search(q, 2)
    assert sorted(Is[0].tolist()) == [123, n + 123] and (Ds[0] == 0).all()


def test_merge_shards_big_k(fx, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(9)
    xb = rng.standard_normal((6000, 40)).astype(np.float32)
    xq = rng.standard_normal((30, 40)).astype(np.float32)
    bounds = [0, 1500, 2600, 4800, 6000]
    Ds, Is = [], []
    for g in range(4):
        ix = fx.IndexFlatL2(40)
        ix.add(xb[bounds[g]:bounds[g + 1]])
        ix.set_id_offset(bounds[g])
        D, I = ix.search(xq, 150)
        Ds.append(D)
        Is.append(I)
    Dm, Im = fx.merge_shards(fx.METRIC_L2, torch.tensor(np.stack(Ds), device="cuda"),
                             torch.tensor(np.stack(Is), device="cuda"), 150)
    Dr, Ir = C.knn_exact(xq, xb, 150)
    assert_parity(Dm.cpu().numpy(), Im.cpu().numpy(), Dr, Ir)


@pytest.mark.parametrize("n", [20_000, 100_000])   # segmented sort / device-wide sort per query
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_huge_k_parity(fx, n, dtype):
    """k > FX_MAX_K: faiss takes any k (faiss_store.py:49,64)."""
    rng = np.random.default_rng(41)
    xb = rng.standard_normal((n, 96)).astype(np.float32)
    xq = rng.standard_normal((20, 96)).astype(np.float32)
    ix = fx.IndexFlatL2(96, dtype=dtype)
    ix.add(xb)
    for k in (1025, 3000):
        D, I = ix.search(xq, k)
        Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, n), k)
        assert_parity(D, I, Dr, Ir)
        assert ix.last_fallbacks() == 0


def test_huge_k_ties_and_padding(fx, torch_cuda):
    """Duplicate rows (equal distances -> smaller id first), k past ntotal
    (I = -1, D = FLT_MAX), device-resident queries and results, IP order."""
    torch = torch_cuda
    rng = np.random.default_rng(42)
    base = rng.standard_normal((700, 48)).astype(np.float32)
    xb = np.concatenate([base, base[::-1], base[:300]])          # 1700 rows, many exact ties
    xq = np.concatenate([base[:4], rng.standard_normal((6, 48)).astype(np.float32)])
    k = 2500
    ix = fx.IndexFlatL2(48)
    ix.add(xb)
    D, I = ix.search(torch.tensor(xq, device="cuda"), k)
    D, I = D.cpu().numpy(), I.cpu().numpy()
    Dr, Ir = C.knn_exact(xq, xb, xb.shape[0])
    assert_parity(D[:, :1700], I[:, :1700], Dr, Ir)
    assert (I[:, 1700:] == -1).all() and (D[:, 1700:] == np.float32(3.4028234663852886e38)).all()
    ip = fx.IndexFlatIP(48)
    ip.add(xb)
    D, I = ip.search(xq, 1200)
    Dr, Ir = F.knn_inner_product(xq, xb, 1200)
    assert_parity(D, I, Dr, Ir)


def test_merge_shards_huge_k(fx, torch_cuda):
    """fx_merge_shards with k > FX_MAX_K (sort by id, then stably by D)."""
    torch = torch_cuda
    rng = np.random.default_rng(43)
    xb = rng.standard_normal((5000, 24)).astype(np.float32)
    xb[4000:4400] = xb[100:500]                                   # ties across shards
    xq = rng.standard_normal((12, 24)).astype(np.float32)
    bounds = [0, 1100, 2300, 4100, 5000]
    k = 1300
    Ds, Is = [], []
    for g in range(4):
        ix = fx.IndexFlatL2(24)
        ix.add(xb[bounds[g]:bounds[g + 1]])
        ix.set_id_offset(bounds[g])
        D, I = ix.search(xq, k)
        Ds.append(D)
        Is.append(I)
    Dm, Im = fx.merge_shards(fx.METRIC_L2, torch.tensor(np.stack(Ds), device="cuda"),
                             torch.tensor(np.stack(Is), device="cuda"), k)
    Dr, Ir = C.knn_exact(xq, xb, k)
    assert_parity(Dm.cpu().numpy(), Im.cpu().numpy(), Dr, Ir)


def test_store_huge_k(fx):
    """FAISSVectorStore.search with k > 1024 returns results (no silent ([], []))."""
    from rag_faiss_embedding_amd.faiss_store import FAISSVectorStore
    rng = np.random.default_rng(44)
    xb = rng.standard_normal((3000, 32)).astype(np.float32)
    FAISSVectorStore._instance = None
    st = FAISSVectorStore(dimension=32)
    st.add_vectors(xb, list(range(100, 3100)))
    dist, ids = st.search(xb[7], k=2000)
    Dr, Ir = C.knn_exact(xb[7:8], xb, 2000)
    assert ids == [int(i) + 100 for i in Ir[0]]
    assert np.allclose(dist, Dr[0], rtol=1e-5, atol=1e-5)
    FAISSVectorStore._instance = None


def test_output_buffer_checks(fx, torch_cuda):
    torch = torch_cuda
    ix = fx.IndexFlatL2(16)
    ix.add(np.ones((10, 16), np.float32))
    q = np.zeros((2, 16), np.float32)
    with pytest.raises(AssertionError):
        ix.search(q, 3, D=np.empty((2, 3), np.float64))
    with pytest.raises(AssertionError):
        ix.search(q, 3, I=np.empty((3, 2), np.int64))
    qt = torch.zeros((2, 16), device="cuda")
    with pytest.raises(AssertionError):
        ix.search(qt, 3, D=torch.empty((2, 3), device="cuda")[:, :2])
