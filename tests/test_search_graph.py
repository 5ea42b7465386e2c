"""Replayed small-batch search (FX_SEARCH_GRAPH=1): host queries in, host
results out -- the reference's FAISSVectorStore.search call form
(faiss_store.py:57-77) -- through one captured hipGraph per shape.

Every replay must equal the oracle; the graph must be rebuilt whenever the
index or the shape changes (add, reset, another k or nq).  The graph holds
the H2D copy, the three kernels and the packed D2H; a replay whose copy
reports uncertified queries runs their fallback chain eagerly right after
(FX_FORCE_FALLBACK=1 case).
"""
import numpy as np
import pytest

from oracle import cpu as C
from tests.test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx():
    from rag_faiss_embedding_amd import _lib, faiss
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return faiss


def test_eager_small_search_equals_graph(fx, monkeypatch):
    """The eager path (FX_SEARCH_GRAPH=0, the default since round 6) and the
    replay return the same results exactly."""
    rng = np.random.default_rng(12)
    xb = rng.standard_normal((10_000, 384)).astype(np.float32)
    q = rng.standard_normal((3, 384)).astype(np.float32)
    out = {}
    for g in ("0", "1"):
        monkeypatch.setenv("FX_SEARCH_GRAPH", g)
        ix = fx.IndexFlatL2(384)
        ix.add(xb)
        out[g] = [ix.search(q[i:i + 1], 5) for i in range(3)] + [ix.search(q, 5)]
    Dr, Ir = C.knn_exact(q, xb, 5)
    assert_parity(out["1"][3][0], out["1"][3][1], Dr, Ir)
    for (De, Ie), (Dg, Ig) in zip(out["0"], out["1"]):
        assert np.array_equal(Ie, Ig) and np.array_equal(De, Dg)


def test_graph_replay_matches_oracle(fx, monkeypatch):
    monkeypatch.setenv("FX_SEARCH_GRAPH", "1")
    rng = np.random.default_rng(11)
    xb = rng.standard_normal((20_000, 384)).astype(np.float32)
    ix = fx.IndexFlatL2(384)
    ix.add(xb[:15_000])
    for r in (3, 77, 14_999, 5, 3):                   # capture, then replays with new query values
        D, I = ix.search(xb[r:r + 1], 5)
        Dr, Ir = C.knn_exact(xb[r:r + 1], xb[:15_000], 5)
        assert_parity(D, I, Dr, Ir)
    ix.add(xb[15_000:])                               # ntotal changed: re-capture
    q = rng.standard_normal((1, 384)).astype(np.float32)
    for _ in range(2):
        D, I = ix.search(q, 5)
        Dr, Ir = C.knn_exact(q, xb, 5)
        assert_parity(D, I, Dr, Ir)
    for k in (1, 10, 32):                             # another shape each time
        D, I = ix.search(q, k)
        Dr, Ir = C.knn_exact(q, xb, k)
        assert_parity(D, I, Dr, Ir)
    qs = rng.standard_normal((17, 384)).astype(np.float32)
    for _ in range(2):
        D, I = ix.search(qs, 10)
        Dr, Ir = C.knn_exact(qs, xb, 10)
        assert_parity(D, I, Dr, Ir)
    ix.reset()
    ix.add(xb[:100])
    D, I = ix.search(q, 5)
    Dr, Ir = C.knn_exact(q, xb[:100], 5)
    assert_parity(D, I, Dr, Ir)


def test_graph_store_single_queries(fx, monkeypatch):
    """FAISSVectorStore-style loop: many single-query calls on one index."""
    monkeypatch.setenv("FX_SEARCH_GRAPH", "1")
    rng = np.random.default_rng(12)
    xb = rng.standard_normal((5000, 128)).astype(np.float32)
    ix = fx.IndexFlatIP(128)
    ix.add(xb)
    from oracle import flat_l2 as F
    for r in range(0, 5000, 500):
        D, I = ix.search(xb[r:r + 1], 5)
        Dr, Ir = F.knn_inner_product(xb[r:r + 1], xb, 5)
        assert_parity(D, I, Dr, Ir)


@pytest.mark.parametrize("k", [5, 100])
def test_graph_replays_the_fallback(diag_fx, monkeypatch, k):
    """The captured graph holds the device-gated exact fallback: with every
    query flagged (FX_FORCE_FALLBACK=1) each replay is still exact."""
    monkeypatch.setenv("FX_SEARCH_GRAPH", "1")
    monkeypatch.setenv("FX_FORCE_FALLBACK", "1")
    rng = np.random.default_rng(13)
    xb = rng.standard_normal((8000, 64)).astype(np.float32)
    ix = diag_fx.IndexFlatL2(64)
    ix.add(xb)
    for r in (1, 2, 4000, 7999):
        D, I = ix.search(xb[r:r + 1] + 0.01, k)
        Dr, Ir = C.knn_exact(xb[r:r + 1] + 0.01, xb, k)
        assert_parity(D, I, Dr, Ir)
        assert ix.last_fallbacks() == 1
