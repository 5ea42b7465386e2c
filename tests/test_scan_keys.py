"""Scan-level parity: every approximate key the fused MFMA scan computes.

The search results are exact even when a scan key is wrong: the refine
recomputes distances exactly and an uncertified query falls back to the exact
scan (fx_index.cpp do_search).  So end-to-end parity alone cannot pin the scan
kernel.  Here the scan's whole key matrix is dumped (FX_SCAN_DBG=32 ->
FX_SCAN_KEYS) and compared with a float64 restatement of the same operands:

    L2: key = |y|^2 - 2 x.y      IP: key = -x.y

with y the stored (storage-dtype) rows, x the query rounded to the storage
dtype, |y|^2 the index's fp32 row norm.  Tolerance: the certification bound of
DESIGN.md 3.2 for fp32 accumulation over K terms,
(2 gamma_K + u) (|y|^2 + 2 |x| |y|) with gamma_K = K u / (1 - K u), u = 2^-24.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx(diag_fx):
    # the scan's key matrix is dumped by the diagnostic build (FX_SCAN_DBG=32 -> FX_SCAN_KEYS)
    return diag_fx


def _round(a, dtype):
    return torch.from_numpy(a).to(getattr(torch, dtype)).to(torch.float32).numpy().astype(np.float64)


def _scan_keys(fx, tmp_path, monkeypatch, cls, xb, xq, dtype):
    path = tmp_path / "keys.bin"
    monkeypatch.setenv("FX_SCAN_DBG", "32")
    monkeypatch.setenv("FX_SCAN_KEYS", str(path))
    monkeypatch.setenv("FX_F32_SPLIT", "0")  # fp32 rows: pin the fp32-MFMA scan (test_f32_split pins F32S)
    d = xb.shape[1]
    ix = cls(d, dtype=dtype)
    ix.add(xb)
    ix.search(xq, 10)
    n, nq = xb.shape[0], xq.shape[0]
    ld = (n + 127) // 128 * 128
    kv = np.fromfile(path, dtype=np.float32).reshape(-1, ld)[:nq, :n].astype(np.float64)
    return ix, kv


# every row width the MFMA scan has a kernel for (row_bytes / 64 in {8,12,16,24})
CASES = [("float32", 128), ("float32", 192), ("float32", 256), ("float32", 384),
         ("bfloat16", 256), ("bfloat16", 384), ("bfloat16", 512), ("bfloat16", 768),
         ("float16", 384), ("float16", 768)]


@pytest.mark.parametrize("dtype,d", CASES)
@pytest.mark.parametrize("metric", ["L2", "IP"])
def test_scan_keys_match(fx, tmp_path, monkeypatch, dtype, d, metric):
    rng = np.random.default_rng(d + (0 if metric == "L2" else 1))
    n, nq = 1500 + d, 150          # several tiles, a ragged last tile, two query tiles
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    cls = fx.IndexFlatL2 if metric == "L2" else fx.IndexFlatIP
    ix, kv = _scan_keys(fx, tmp_path, monkeypatch, cls, xb, xq, dtype)
    yb = ix.reconstruct_n(0, n).astype(np.float64)       # stored values
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
