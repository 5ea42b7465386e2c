"""Certification stress: tightly clustered, near-duplicate embeddings (VERDICT
r1/r2, "parity sampling"), the shape of real sentence embeddings (one dominant
common direction) where the scan's rounding margin is
largest relative to the gaps between neighbours.

Uncertified queries are re-ranked by the exact fallback, so ids stay
bit-exact either way; what these tests pin is that the fallback stays rare
(the search does not silently degrade to a full exact rescan per query) for
every storage dtype, with fp32 queries that are NOT representable in the
storage dtype (the encoder -> bf16 index case): the 16-bit indexes scan
x - mu against |y - mu|^2 and certify with the query's own rounding residual
(DESIGN.md 3.3).
"""
import time

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


def clustered(n, d, spread, seed, unit=True, scale=1.0):
    """n rows around one common direction: (base + spread * noise), unit norm
    (or scaled) -- pairwise cosine ~ 1 - spread^2."""
    rng = np.random.default_rng(seed)
    base = rng.standard_normal(d)
    base /= np.linalg.norm(base)
    x = base[None, :] + spread * rng.standard_normal((n, d)) / np.sqrt(d)
    if unit:
        x /= np.linalg.norm(x, axis=1, keepdims=True)
    return (x * scale).astype(np.float32)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
@pytest.mark.parametrize("spread,scale", [(0.1, 1.0), (0.1, 20.0), (0.02, 1.0)])
def test_clustered_embeddings(fx, dtype, spread, scale):
    n, d, nq = 200_000, 384, 512
    xb = clustered(n, d, spread, 1, scale=scale)
    xq = clustered(nq, d, spread, 1, scale=scale)[::-1].copy() + np.float32(1e-3 * scale)
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    ix.search(xq[:8], 10)
    t0 = time.perf_counter()
    D, I = ix.search(xq, 10)
    dt = time.perf_counter() - t0
    nfb = ix.last_fallbacks()
    print(f"\n[cert-stress] {dtype} spread={spread} scale={scale}: fallbacks {nfb}/{nq}, search {dt * 1e3:.2f} ms")
    # the oracle on the stored values (bf16 / fp16 rows upcast; the query stays fp32)
    ref = xb if dtype == "float32" else ix.reconstruct_n(0, n)
    sub = np.arange(0, nq, 8)
    Dr, Ir = C.knn_exact(xq[sub], ref, 10)
    assert_parity(D[sub], I[sub], Dr, Ir)
    assert nfb <= nq // 100, f"{nfb}/{nq} queries fell back to the exact scan"


def test_recentre_after_growth(fx):
    """The image's centre follows the data: a few rows of one cluster first
    (centre there), then the index grows past twice that size around another
    centre -- the image is re-centred and rebuilt, and searches before and
    after stay exact (the fallback count depends on the global max row norm,
    which the far first cluster keeps large: reported, not asserted)."""
    d = 256
    a = clustered(500, d, 0.1, 5, scale=10.0)
    b = clustered(60_000, d, 0.1, 6, scale=10.0)
    for dtype in ("float32", "bfloat16"):
        ix = fx.IndexFlatL2(d, dtype=dtype)
        ix.add(a)
        ra = a if dtype == "float32" else ix.reconstruct_n(0, len(a))
        xq = np.concatenate([a[:8], b[:56]]) + np.float32(0.01)
        D, I = ix.search(xq, 10)
        Dr, Ir = C.knn_exact(xq, ra, 10)
        assert_parity(D, I, Dr, Ir)
        ix.add(b)
        xb = np.concatenate([a, b]) if dtype == "float32" else ix.reconstruct_n(0, len(a) + len(b))
        D, I = ix.search(xq, 10)
        Dr, Ir = C.knn_exact(xq, xb, 10)
        assert_parity(D, I, Dr, Ir)
        print(f"\n[recentre] {dtype}: fallbacks {ix.last_fallbacks()}/{len(xq)}")


@pytest.mark.timeout(400)
def test_clustered_bf16_d_shard(fx):
    """Config (d)'s per-GPU shard at 8 GPUs (1.25M x 768 bf16, 10k-query
    batch) holding clustered fp32 embeddings (spread 0.1, unit norm) stored as
    bf16, with fp32 queries: fallback count asserted (<= 1 %), ids oracle-exact
    on a 1,000-query sample, time reported."""
    import torch
    n, d, nq, k = 1_250_000, 768, 10_000, 10
    g = torch.Generator(device="cuda").manual_seed(7)
    base = torch.randn(d, device="cuda", generator=g)
    base /= base.norm()
    ix = fx.IndexFlatL2(d, dtype="bfloat16")
    ix.reserve(n)
    chunk = 1 << 18
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        x = base[None, :] + 0.1 * torch.randn((m, d), device="cuda", generator=g) / d ** 0.5
        ix.add(x / x.norm(dim=1, keepdim=True))
    xq = base[None, :] + 0.1 * torch.randn((nq, d), device="cuda", generator=g) / d ** 0.5
    xq = (xq / xq.norm(dim=1, keepdim=True)).contiguous()
    ix.search(xq[:256], k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    D, I = ix.search(xq, k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nfb = ix.last_fallbacks()
    print(f"\n[cert-stress d-shard] bf16 1.25M x 768 clustered, nq {nq}: fallbacks {nfb}/{nq}, "
          f"search {dt * 1e3:.1f} ms ({nq / dt:.0f} qps)")
    # the oracle over >= 1,000 queries of the batch
    sub = np.linspace(0, nq - 1, 1000).astype(np.int64)
    ref = ix.reconstruct_n(0, n)
    Dr, Ir = C.knn_exact(xq[sub].cpu().numpy(), ref, k)
    assert_parity(D[sub].cpu().numpy(), I[sub].cpu().numpy(), Dr, Ir)
    assert nfb <= nq // 100, f"{nfb}/{nq} queries fell back to the exact scan"
