"""k_scan_v5 (fx_scan5.hip: 64-row tiles, 3 or 4 query blocks of 16 per
wave, 192 / 256 queries per workgroup) against the oracle on the edges its
shape adds to k_scan_v4's: query counts that are not whole 192 / 256-query
tiles, an index whose last 64-row tile is partial (and indexes smaller than
one tile), inner product, k above the fused lists' 32 (no cross-split
pruning), the cold-start bound, and the re-scan of uncertified queries (the
diagnostic build's force_fallback).  The option scan_v5 = 2 takes v5 wherever
it has the row width (the plan alone takes it only where it adds no padding
work); scan_v5 = 0 gives k_scan_v4 on the same index, whose results must be
identical.  Bar: ids bit-exact, |dD| <= 1e-5 max(1, |D|) (test_gpu_parity)."""
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


def _data(n, d, nq, seed, kind="gauss"):
    rng = np.random.default_rng(seed)
    if kind == "clustered":
        base = rng.standard_normal(d)
        xb = base / np.linalg.norm(base) + 0.05 * rng.standard_normal((n, d)) / np.sqrt(d)
        xq = base / np.linalg.norm(base) + 0.05 * rng.standard_normal((nq, d)) / np.sqrt(d)
        return xb.astype(np.float32), xq.astype(np.float32)
    return rng.standard_normal((n, d)).astype(np.float32), rng.standard_normal((nq, d)).astype(np.float32)


def _check(fx, ix, xq, ref, k, ip=False):
    out = {}
    for v in (2, 0):
        ix.set_option("scan_v5", v)
        D, I = ix.search(xq, k)
        out[v] = (D, I)
    Dr, Ir = F.knn_inner_product(xq, ref, k) if ip else C.knn_exact(xq, ref, k)
    assert_parity(out[2][0], out[2][1], Dr, Ir)
    np.testing.assert_array_equal(out[2][1], out[0][1])
    np.testing.assert_array_equal(out[2][0], out[0][0])
    return out[2]


@pytest.mark.parametrize("dtype,d", [("bfloat16", 768), ("float16", 384), ("bfloat16", 256), ("float16", 768)])
@pytest.mark.parametrize("nq", [1, 191, 257, 1000])
def test_v5_query_tiles_and_ragged_rows(fx, dtype, d, nq):
    n = 70_001  # the last 64-row tile holds 17 rows
    xb, xq = _data(n, d, nq, 5)
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    _check(fx, ix, xq, ix.reconstruct_n(0, n), 10)
    assert ix.last_fallbacks() <= max(1, nq // 100)


@pytest.mark.parametrize("n", [1, 50, 64, 65, 200])
def test_v5_tiny_indexes(fx, n):
    d, nq = 384, 300
    xb, xq = _data(n, d, nq, 6)
    ix = fx.IndexFlatL2(d, dtype="float16")
    ix.add(xb)
    _check(fx, ix, xq, ix.reconstruct_n(0, n), min(10, n) if n > 1 else 5)


@pytest.mark.parametrize("dtype,d", [("bfloat16", 768), ("float16", 384)])
@pytest.mark.parametrize("anti", [False, True])
def test_v5_inner_product(fx, dtype, d, anti):
    n, nq = 30_017, 400
    rng = np.random.default_rng(7)
    base = np.abs(rng.standard_normal(d)) + 0.5
    xb = (base + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    xq = (rng.standard_normal((nq, d)) * 0.3 - (base if anti else 0.0)).astype(np.float32)
    ix = fx.IndexFlatIP(d, dtype=dtype)
    ix.add(xb)
    for cold in (-1, 1):
        ix.set_option("cold_bound", cold)
        _check(fx, ix, xq, ix.reconstruct_n(0, n), 10, ip=True)


@pytest.mark.parametrize("k", [1, 32, 33, 100, 1024])
def test_v5_any_k(fx, k):
    n, d, nq = 40_000, 768, 300
    xb, xq = _data(n, d, nq, 8)
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    ix.add(xb)
    _check(fx, ix, xq, ix.reconstruct_n(0, n), k)


@pytest.mark.parametrize("dtype,d", [("bfloat16", 768), ("float16", 384)])
def test_v5_clustered_certifies(fx, dtype, d):
    """Clustered unit-norm rows with fp32 queries inexact in the storage
    dtype (the certification's hard case) through v5: <= 1 % re-scanned."""
    n, nq = 200_000, 1024
    xb, xq = _data(n, d, nq, 9, kind="clustered")
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    _check(fx, ix, xq, ix.reconstruct_n(0, n), 10)
    ix.set_option("scan_v5", 2)
    ix.search(xq, 10)
    assert ix.last_fallbacks() <= nq // 100


def test_v5_rescan_path(diag_fx):
    """Every query forced through the device-gated re-scan (k_scan_v5's
    RESCAN instance over the gathered queries) and through the exact scan."""
    n, d, nq = 50_000, 768, 500
    xb, xq = _data(n, d, nq, 10)
    for mode in (1, 2):
        ix = diag_fx.IndexFlatL2(d, dtype="bfloat16")
        ix.add(xb)
        ix.set_option("scan_v5", 2)
        ix.set_option("force_fallback", mode)
        D, I = ix.search(xq, 10)
        Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, n), 10)
        assert_parity(D, I, Dr, Ir)
        assert ix.last_fallbacks() == nq


def test_scan_plan_reports_the_kernel(fx):
    """fx_index_last_scan_plan names the scan the plan took (bench.py labels
    its roofline line with it): v5 (64-row tiles, 192 queries per workgroup
    for 1,536-B rows) for a whole-tile bf16 768 batch, v4 (128-row tiles, 128
    queries) with scan_v5 = 0 and for one query."""
    n, d = 20_000, 768
    xb, xq = _data(n, d, 192 * 4, 11)
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    assert ix.last_scan_plan() == {"tile_rows": 0, "query_tile": 0, "splits": 0}
    ix.add(xb)
    ix.search(xq, 10)
    p = ix.last_scan_plan()
    assert (p["tile_rows"], p["query_tile"]) == (64, 192) and p["splits"] >= 1
    ix.search(xq[:1], 10)
    assert ix.last_scan_plan()["tile_rows"] == 128
    ix.set_option("scan_v5", 0)
    ix.search(xq, 10)
    assert (ix.last_scan_plan()["tile_rows"], ix.last_scan_plan()["query_tile"]) == (128, 128)


def test_v5_convoy_start_repeated(fx):
    """The convoy start (option convoy, ScanParams.conv): a block begins its
    split where the split's other blocks published they are.  A first version
    let every wave read the word itself; a store landing between two waves'
    reads made one stage hold two tiles' rows, which lost rows of that split
    about one search in three on this case.  Six searches against the oracle,
    and identical to the plain start."""
    n, d, nq = 200_000, 768, 1024
    xb, xq = _data(n, d, nq, 9, kind="clustered")
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    ix.add(xb)
    Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, n), 10)
    ix.set_option("scan_v5", 2)
    ix.set_option("convoy", 0)
    D0, I0 = ix.search(xq, 10)
    ix.set_option("convoy", 1)
    for _ in range(6):
        D, I = ix.search(xq, 10)
        assert_parity(D, I, Dr, Ir)
        np.testing.assert_array_equal(I, I0)
        np.testing.assert_array_equal(D, D0)


def test_v4_convoy_start_repeated(fx):
    """The convoy start in k_scan_v4 (fp32 storage: the split-fp32 scan) on a
    grid of four dispatch rounds: four searches against the oracle, identical
    to the plain start (option convoy 0)."""
    n, d, nq = 200_000, 384, 2048
    xb, xq = _data(n, d, nq, 12, kind="clustered")
    ix = fx.IndexFlatL2(d)
    ix.add(xb)
    Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, n), 10)
    ix.set_option("convoy", 0)
    D0, I0 = ix.search(xq, 10)
    assert ix.last_scan_plan()["tile_rows"] == 128
    assert_parity(D0, I0, Dr, Ir)
    ix.set_option("convoy", 1)
    for _ in range(4):
        D, I = ix.search(xq, 10)
        assert_parity(D, I, Dr, Ir)
        np.testing.assert_array_equal(I, I0)
        np.testing.assert_array_equal(D, D0)
