"""The wide-tile scan k_scan_w (fx_scan_w.hip; 192 queries per workgroup, 64-row
corpus tiles), forced on with FX_SCAN_W=1 at sizes the oracle checks quickly.

* its whole key matrix (FX_SCAN_DBG=32) against the float64 restatement of the
  same operands within the certification bound (as test_scan_keys.py does for
  k_scan_v4);
* search parity against the oracle: ragged query tiles (nq not a multiple of
  192), a ragged last corpus tile, k > KP, inner product, split fp32;
* identical results to k_scan_v4 on a 1M-row synthetic corpus.
"""
import numpy as np
import pytest

from oracle import cpu as C
from oracle import flat_l2 as F
from tests.test_gpu_parity import assert_parity
from tests.test_scan_keys import _round

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx():
    from rag_faiss_embedding_amd import _lib, faiss
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return faiss


@pytest.mark.parametrize("dtype,d", [("bfloat16", 384), ("bfloat16", 512), ("bfloat16", 768),
                                     ("float16", 384), ("float16", 768)])
@pytest.mark.parametrize("metric", ["L2", "IP"])
def test_scan_w_keys(fx, tmp_path, monkeypatch, dtype, d, metric):
    monkeypatch.setenv("FX_SCAN_W", "1")
    path = tmp_path / "keys.bin"
    monkeypatch.setenv("FX_SCAN_DBG", "32")
    monkeypatch.setenv("FX_SCAN_KEYS", str(path))
    rng = np.random.default_rng(3 * d + (metric == "IP"))
    n, nq = 1500 + d, 450           # ragged last 64-row tile; 3 wide tiles, the last ragged
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    ix = (fx.IndexFlatL2 if metric == "L2" else fx.IndexFlatIP)(d, dtype=dtype)
    ix.add(xb)
    ix.search(xq, 10)
    ld = (n + 127) // 128 * 128
    kv = np.fromfile(path, dtype=np.float32).reshape(-1, ld)[:nq, :n].astype(np.float64)
    yb = ix.reconstruct_n(0, n).astype(np.float64)
    xr = _round(xq, dtype)
    dot = xr @ yb.T
    ny = (yb ** 2).sum(1)
    ref = ny[None, :] - 2 * dot if metric == "L2" else -dot
    u = 2.0 ** -24
    g = d * u / (1 - d * u)
    nx = np.sqrt((xr ** 2).sum(1))[:, None]
    bound = (2 * g + u) * (ny[None, :] + 2 * nx * np.sqrt(ny)[None, :]) + 1e-30
    err = np.abs(kv - ref)
    assert np.isfinite(kv).all()
    assert (err <= bound).all(), f"max err/bound {np.max(err / bound):.3g}"


@pytest.mark.parametrize("dtype,n,d,nq,k,metric", [
    ("bfloat16", 20_000, 768, 1000, 10, "L2"),
    ("float16", 50_001, 384, 2000, 10, "L2"),
    ("float32", 30_000, 384, 1500, 10, "L2"),   # split fp32 (F32S), centred
    ("float32", 30_000, 256, 1100, 5, "L2"),
    ("bfloat16", 20_000, 768, 500, 100, "L2"),  # k > KP: no cross-split pruning
    ("bfloat16", 9_000, 512, 700, 10, "IP"),
    ("float32", 9_000, 384, 700, 10, "IP"),     # F32S, uncentred (IP)
])
def test_scan_w_parity(fx, monkeypatch, dtype, n, d, nq, k, metric):
    monkeypatch.setenv("FX_SCAN_W", "1")
    rng = np.random.default_rng(n + d + nq)
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xb[n - 1] = xb[5]                 # an exact duplicate: tie -> smaller id
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    xq[3] = xb[5]
    ix = (fx.IndexFlatL2 if metric == "L2" else fx.IndexFlatIP)(d, dtype=dtype)
    ix.add(xb)
    D, I = ix.search(xq, k)
    assert ix.last_fallbacks() == 0
    yb = xb if dtype == "float32" else ix.reconstruct_n(0, n)
    sub = np.unique(np.concatenate([np.arange(0, nq, max(1, nq // 40)), [3, nq - 1]]))
    if metric == "L2":
        Dr, Ir = C.knn_exact(xq[sub], yb, k)
    else:
        Dr, Ir = F.knn_inner_product(xq[sub], yb, k)
    assert_parity(D[sub], I[sub], Dr, Ir)


def test_scan_w_equals_v4(fx, monkeypatch):
    import torch
    n, d, nq = 1_000_000, 768, 2000
    xb = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
    fx.synth_fill(xb, 0, 1234)
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    ix.add(xb)
    del xb
    xq = torch.empty((nq, d), dtype=torch.bfloat16, device="cuda")
    fx.synth_fill(xq, 0, 4321)
    res = {}
    for w in ("0", "1"):
        monkeypatch.setenv("FX_SCAN_W", w)
        D, I = ix.search(xq, 10)
        assert ix.last_fallbacks() == 0
        res[w] = (D.cpu().numpy(), I.cpu().numpy())
    np.testing.assert_array_equal(res["0"][1], res["1"][1])
    np.testing.assert_array_equal(res["0"][0], res["1"][0])
