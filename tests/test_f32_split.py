"""Split-fp32 scan (the default for fp32 indexes): an fp32 index scanned through its
[hi | lo] bf16 image with 3 bf16 MFMA products per term (fx_scan.hip, F32S).

The scan key changes, the contract does not: results must equal the oracle's
(ids bit-exact, distances within RTOL) because the refine recomputes the
candidates' distances from the fp32 rows and certifies them against the
scan's error bound, which for F32S adds the dropped lo*lo and residual terms:
    |key - exact| <= (2 gamma_{3K+1} + u)(|y|^2 + 2|x||y|) + 2 * 4.73e-5 |x||y|   (L2)
    |key - exact| <= (gamma_{3K+1} + u)|x||y| + 4.73e-5 |x||y|                    (IP)

(FX_F32_SPLIT=0 selects the fp32-MFMA scan instead; test_scan_keys pins that.)
"""
import numpy as np
import pytest

from oracle import cpu as C
from oracle import flat_l2 as F
from tests.test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx(diag_fx):
    # the scan's key matrix is dumped by the diagnostic build (FX_SCAN_DBG=32 -> FX_SCAN_KEYS)
    return diag_fx


@pytest.mark.parametrize("d", [128, 192, 256, 384])
@pytest.mark.parametrize("metric,centre", [("L2", False), ("L2", True), ("IP", False)])
def test_split_scan_keys(fx, tmp_path, monkeypatch, d, metric, centre):
    """Raw F32S scan keys against the fp64 model within the certification
    bound.  L2 images are centred by default (FX_CENTER): keys are then
    |y - mu|^2 - 2 (x - mu).(y - mu), mu = the fp32 mean of the rows (all of
    them below MU_SAMPLE), and the bound takes the centred norms + 3u."""
    monkeypatch.setenv("FX_F32_SPLIT", "1")
    monkeypatch.setenv("FX_CENTER", "1" if centre else "0")
    monkeypatch.setenv("FX_SCAN_DBG", "32")
    path = tmp_path / "keys.bin"
    monkeypatch.setenv("FX_SCAN_KEYS", str(path))
    rng = np.random.default_rng(100 + d)
    n, nq = 1500 + d, 150
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    if centre:  # a common offset: the case centring is for
        off = (3.0 * rng.standard_normal(d)).astype(np.float32)
        xb += off
        xq += off
    ix = (fx.IndexFlatL2 if metric == "L2" else fx.IndexFlatIP)(d)
    ix.add(xb)
    ix.search(xq, 10)
    ld = (n + 127) // 128 * 128
    kv = np.fromfile(path, dtype=np.float32).reshape(-1, ld)[:nq, :n].astype(np.float64)
    y = xb.astype(np.float64)
    x = xq.astype(np.float64)
    cu = 0.0
    if centre:
        mu = y.mean(0).astype(np.float32).astype(np.float64)
        y = (xb - mu.astype(np.float32)).astype(np.float64)
        x = (xq - mu.astype(np.float32)).astype(np.float64)
        cu = 3 * 2.0 ** -24
    dot = x @ y.T
    ny = (y ** 2).sum(1)[None, :]
    nx = np.sqrt((x ** 2).sum(1))[:, None]
    u = 2.0 ** -24
    K = 3 * d + 1                            # kdim == d for these widths
    g = K * u / (1 - K * u)
    if metric == "L2":
        ref = ny - 2 * dot
        bound = (2 * g + u + cu) * (ny + 2 * nx * np.sqrt(ny)) + 2 * 4.73e-5 * nx * np.sqrt(ny)
    else:
        ref = -dot
        bound = (g + u) * nx * np.sqrt(ny) + 4.73e-5 * nx * np.sqrt(ny)
    err = np.abs(kv - ref)
    assert np.isfinite(kv).all()
    assert (err <= bound + 1e-30).all(), f"max err/bound {np.max(err / bound):.3g}"


@pytest.mark.parametrize("d", [100, 128, 192, 256, 384])
@pytest.mark.parametrize("metric", ["L2", "IP"])
def test_split_search_parity(fx, monkeypatch, d, metric):
    monkeypatch.setenv("FX_F32_SPLIT", "1")
    rng = np.random.default_rng(7 * d + (metric == "IP"))
    n, nq = 5000, 300
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xb[4000] = xb[17]                       # an exact duplicate: tie -> smaller id
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    xq[0] = xb[17]
    ix = (fx.IndexFlatL2 if metric == "L2" else fx.IndexFlatIP)(d)
    ix.add(xb[:3000])
    ix.search(xq[:5], 10)                   # builds the split image of the first 3000 rows
    ix.add(xb[3000:])                       # ... which the next search extends
    D, I = ix.search(xq, 10)
    Dr, Ir = C.knn_exact(xq, xb, 10) if metric == "L2" else F.knn_inner_product(xq, xb, 10)
    assert_parity(D, I, Dr, Ir)
    assert ix.last_fallbacks() <= nq // 10
    ix.reset()
    ix.add(xb[:700])
    D, I = ix.search(xq[:50], 5)
    Dr, Ir = C.knn_exact(xq[:50], xb[:700], 5) if metric == "L2" else F.knn_inner_product(xq[:50], xb[:700], 5)
    assert_parity(D, I, Dr, Ir)
