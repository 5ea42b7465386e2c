"""The scan's list-maintenance options (fx_scan_common.h compact_regs) keep
results exact whatever their value: the compaction trigger `compact_at`
(a list is compacted to its KP best once it holds that many entries, 33..64)
and the union-bound window `union_w` (16, 32 or 64 splits, each contributing
its first 256 / union_w published keys), and whether a compaction's union
bound is waited for in place or fetched by LDS-DMA and bounded a tile later
(`union_defer`), and the re-bounding of a list's threshold between
compactions (`tight_at`: a bisection over the list's keys for its rank-th),
and an empty list's first bound from the tile's group minima (`cold_bound`),
and how many lists of one compaction call take the union bound in place
(`union_inplace`).
All only change how fast the
pruning threshold falls; every dropped row still lies above the final shared
threshold that the refine certifies against.  Checked against the oracle on
a batch that runs many splits (short splits: cold lists, frequent
compactions), on uniform and clustered rows."""
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


def rows(kind, n, d, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        return rng.standard_normal((n, d)).astype(np.float32)
    base = rng.standard_normal(d)
    x = base / np.linalg.norm(base) + 0.05 * rng.standard_normal((n, d)) / np.sqrt(d)
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("kind", ["uniform", "clustered"])
# float16 at d = 384: the fp16 12-K-step scan instance of config (e)
@pytest.mark.parametrize("dtype,d", [("bfloat16", 256), ("float32", 256), ("float16", 384)])
def test_compaction_and_union_options_exact(fx, kind, dtype, d):
    n, nq, k = 300_000, 300, 10
    xb = rows(kind, n, d, 11)
    xq = rows(kind, nq, d, 12)
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    ref = xb if dtype == "float32" else ix.reconstruct_n(0, n)
    Dr, Ir = C.knn_exact(xq, ref, k)
    for compact_at, union_w, defer, tight, cold, inplace in [
            (64, 16, 1, 0, 0, -1), (40, 16, 0, 0, 0, -1), (48, 64, 1, 0, 0, 64), (33, 32, 0, 0, 0, 4),
            (64, 64, 0, 0, 0, 0), (0, 0, 0, 0, 0, -1), (0, 0, 1, 0, 0, 8), (64, 16, 1, 33, 0, -1),
            (48, 0, 1, 36, 1, 64), (64, 64, 0, 40, 1, -1), (0, 0, 1, 0, 1, 0), (0, 0, 1, -1, -1, -1)]:
        ix.set_option("compact_at", compact_at)
        ix.set_option("union_w", union_w)
        ix.set_option("union_defer", defer)
        ix.set_option("union_inplace", inplace)
        ix.set_option("tight_at", tight)
        ix.set_option("cold_bound", cold)
        D, I = ix.search(xq, k)
        assert_parity(D, I, Dr, Ir)
        print(f"\n[scan-options] {kind} {dtype} compact_at={compact_at} union_w={union_w} "
              f"union_defer={defer} tight_at={tight} cold_bound={cold} union_inplace={inplace}: fallbacks {ix.last_fallbacks()}/{nq}")


# --------------------------------------------------------------------------
# Inner product and the index's padded edge tile: IP keys of
# the zero padding rows are 0, not +inf, so a cold list whose first record tile
# is the index's last tile must not count padding groups as rows when it
# bounds its threshold from the tile's group minima (cold_bound).  Queries
# anti-correlated to every row have no positive inner product at all: every
# real key is > 0 = a padding key, which is the case the bound got wrong.

def ip_rows(n, d, nq, seed, anti):
    rng = np.random.default_rng(seed)
    base = np.abs(rng.standard_normal(d)) + 0.5
    xb = (base + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    xq = (rng.standard_normal((nq, d)) * 0.3 - (base if anti else 0.0)).astype(np.float32)
    return xb, xq


@pytest.mark.parametrize("n", [50, 127, 10_016, 70_001])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("cold", [-1, 1])
def test_inner_product_edge_tile_cold_bound(fx, n, dtype, cold):
    d, nq, k = 64, 96, 10
    xb, xq = ip_rows(n, d, nq, 31, anti=True)
    ix = fx.IndexFlatIP(d, dtype=dtype)
    ix.add(xb)
    ix.set_option("cold_bound", cold)
    ref = xb if dtype == "float32" else ix.reconstruct_n(0, n)
    assert (xq.astype(np.float64) @ ref.astype(np.float64).T < 0).all()  # no positive inner product
    D, I = ix.search(xq, k)
    Dr, Ir = F.knn_inner_product(xq, ref, k)
    assert (I >= 0).all()
    assert_parity(D, I, Dr, Ir)


@pytest.mark.parametrize("anti", [False, True])
def test_inner_product_options_exact(fx, anti):
    """The option sweep above on IndexFlatIP (300k rows: many short splits)."""
    n, d, nq, k = 300_000, 256, 300, 10
    xb, xq = ip_rows(n, d, nq, 13, anti)
    ix = fx.IndexFlatIP(d, dtype="bfloat16")
    ix.add(xb)
    ref = ix.reconstruct_n(0, n)
    Dr, Ir = F.knn_inner_product(xq, ref, k)
    for compact_at, union_w, defer, tight, cold, inplace in [
            (0, 0, 1, -1, -1, -1), (0, 0, 1, 0, 1, 0), (48, 64, 1, 0, 1, 3), (64, 16, 0, 33, 1, -1),
            (40, 32, 1, 0, 0, 5)]:
        ix.set_option("compact_at", compact_at)
        ix.set_option("union_w", union_w)
        ix.set_option("union_defer", defer)
        ix.set_option("union_inplace", inplace)
        ix.set_option("tight_at", tight)
        ix.set_option("cold_bound", cold)
        D, I = ix.search(xq, k)
        assert_parity(D, I, Dr, Ir)
