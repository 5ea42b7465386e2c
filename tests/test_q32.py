"""Small-batch scan (FX_SCAN_Q32=1, k_scan_q32): nq <= 32, the reference's
own call shape (faiss_store.py:61 searches one query at a time).

Same bar as every search: ids bit-exact with the oracle, distances within
RTOL; plus the scan's key matrix against a float64 restatement, as in
test_scan_keys.py.
"""
import numpy as np
import pytest
import torch

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


@pytest.mark.parametrize("dtype,d", [("float32", 128), ("float32", 384), ("bfloat16", 768), ("float16", 384)])
@pytest.mark.parametrize("nq", [1, 7, 32])
@pytest.mark.parametrize("metric", ["L2", "IP"])
def test_q32_search_parity(fx, monkeypatch, dtype, d, nq, metric):
    monkeypatch.setenv("FX_SCAN_Q32", "1")
    rng = np.random.default_rng(d + nq)
    n = 20_000 + 77                                   # many splits, a ragged last tile
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xb = torch.from_numpy(xb).to(getattr(torch, dtype)).float().numpy()   # exact in the storage dtype
    xb[n - 1] = xb[5]                                 # duplicate across the corpus: tie -> smaller id
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    xq = torch.from_numpy(xq).to(getattr(torch, dtype)).float().numpy()
    xq[0] = xb[5]
    ix = (fx.IndexFlatL2 if metric == "L2" else fx.IndexFlatIP)(d, dtype=dtype)
    ix.add(xb)
    D, I = ix.search(xq, 10)
    Dr, Ir = C.knn_exact(xq, xb, 10) if metric == "L2" else F.knn_inner_product(xq, xb, 10)
    assert_parity(D, I, Dr, Ir)


@pytest.mark.parametrize("split", ["0", "1"])
def test_q32_keys(fx, tmp_path, monkeypatch, split):
    monkeypatch.setenv("FX_SCAN_Q32", "1")
    monkeypatch.setenv("FX_F32_SPLIT", split)
    monkeypatch.setenv("FX_CENTER", "0")  # uncentred keys (test_f32_split pins the centred ones)
    monkeypatch.setenv("FX_SCAN_DBG", "32")
    path = tmp_path / "keys.bin"
    monkeypatch.setenv("FX_SCAN_KEYS", str(path))
    rng = np.random.default_rng(3)
    d, n, nq = 384, 3000, 20
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    ix = fx.IndexFlatL2(d)
    ix.add(xb)
    ix.search(xq, 10)
    ld = (n + 127) // 128 * 128
    kv = np.fromfile(path, dtype=np.float32).reshape(-1, ld)[:nq, :n].astype(np.float64)
    y, x = xb.astype(np.float64), xq.astype(np.float64)
    ny = (y ** 2).sum(1)[None, :]
    nx = np.sqrt((x ** 2).sum(1))[:, None]
    ref = ny - 2 * x @ y.T
    u = 2.0 ** -24
    K = 3 * d + 1 if split == "1" else d
    g = K * u / (1 - K * u)
    bound = (2 * g + u) * (ny + 2 * nx * np.sqrt(ny))
    if split == "1":
        bound += 2 * 4.73e-5 * nx * np.sqrt(ny)
    assert np.isfinite(kv).all()
    assert (np.abs(kv - ref) <= bound + 1e-30).all()


def test_q32_single_query_store(fx, monkeypatch):
    """FAISSVectorStore-style single-query calls, one after another."""
    monkeypatch.setenv("FX_SCAN_Q32", "1")
    rng = np.random.default_rng(4)
    xb = rng.standard_normal((5000, 384)).astype(np.float32)
    ix = fx.IndexFlatL2(384)
    ix.add(xb)
    for r in (0, 1, 2499, 4999):
        D, I = ix.search(xb[r:r + 1], 5)
        Dr, Ir = C.knn_exact(xb[r:r + 1], xb, 5)
        assert_parity(D, I, Dr, Ir)
        assert I[0, 0] == r and D[0, 0] == 0
