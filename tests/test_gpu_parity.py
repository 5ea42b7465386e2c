"""GPU parity: the HIP index (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): returned ids bit-exact; distances
within |dD| <= 1e-5 * max(1, |D_ref|) of the oracle's exact fp32 distance
(scale-relative reading of "within 1e-5 fp32").  In practice the refine makes
them identical; the tolerance is what is asserted.
"""
import json
import shutil

import numpy as np
import pytest

from oracle import cpu as C
from oracle import flat_l2 as F
from tests._data import gaussian_small

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def assert_parity(D, I, Dr, Ir):
    D = np.asarray(D)
    I = np.asarray(I)
    np.testing.assert_array_equal(I, Ir)
    valid = Ir >= 0
    tol = RTOL * np.maximum(1.0, np.abs(Dr[valid].astype(np.float64)))
    assert (np.abs(D[valid].astype(np.float64) - Dr[valid]) <= tol).all()
    assert (D[~valid] == Dr[~valid]).all()


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


# --------------------------------------------------------------------------
# reference fixtures
# --------------------------------------------------------------------------

@pytest.mark.parametrize("k", [1, 5, 10, 23, 30])
def test_shipped_index_all_rows(fx, golden_dir, k):
    z = np.load(golden_dir / "shipped_knn.npz")
    xb = z["xb"]
    ix = fx.IndexFlatL2(384)
    ix.add(xb)
    D, I = ix.search(xb, k)
    assert_parity(D, I, z[f"D_k{k}"], z[f"I_k{k}"])
    assert ix.last_fallbacks() == 0
    # single-query calls as FAISSVectorStore makes them (faiss_store.py:61)
    for i in range(0, 23, 5):
        D1, I1 = ix.search(xb[i:i + 1], k)
        assert_parity(D1, I1, z[f"D_k{k}"][i:i + 1], z[f"I_k{k}"][i:i + 1])


def test_read_write_shipped_index(fx, golden_dir, tmp_path):
    ix = fx.read_index(str(golden_dir / "shipped_index.bin"))
    assert ix.ntotal == 23 and ix.d == 384
    out = tmp_path / "rt.bin"
    fx.write_index(ix, str(out))
    assert out.read_bytes() == (golden_dir / "shipped_index.bin").read_bytes()
    with pytest.raises(RuntimeError):
        fx.read_index(str(tmp_path / "missing.bin"))


def test_store_golden_on_gpu(fx, golden_dir, tmp_path, monkeypatch):
    from rag_faiss_embedding_amd import _mapping, faiss_store
    G = json.loads((golden_dir / "wrapper_golden.json").read_text())
    xb = np.load(golden_dir / "shipped_knn.npz")["xb"]
    (tmp_path / "data").mkdir()
    shutil.copy(golden_dir / "shipped_index.bin", tmp_path / "data" / "faiss_index.bin")
    ids = json.loads((golden_dir / "shipped_ids.json").read_text())["mapping_ids"]
    (tmp_path / "data" / "faiss_index.bin.mapping").write_bytes(_mapping.dumps_ids(ids))
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(faiss_store.FAISSVectorStore, "_instance", None)
    monkeypatch.setattr(faiss_store.FAISSVectorStore, "_initialized", False)
    store = faiss_store.FAISSVectorStore()
    assert store.doc_ids == G["load"]["doc_ids"] and store.index.ntotal == 23
    for i, res in enumerate(G["search_k5"]):
        D, got = store.search(xb[i], 5)
        assert got == res["ids"]
        np.testing.assert_allclose(D, np.float32(res["D"]), rtol=RTOL, atol=RTOL)
    D, got = store.search(list(map(float, xb[3])), 30)
    assert got == G["search_list_k30"]["ids"]
    D, got = store.search(xb[0][:100], 5)
    assert got == [] and D.size == 0
    store.save_index(str(tmp_path / "out" / "ix.bin"))
    assert (tmp_path / "out" / "ix.bin").read_bytes() == (golden_dir / "shipped_index.bin").read_bytes()
    assert (tmp_path / "out" / "ix.bin.mapping").read_bytes().hex() == G["save_mapping_hex"]
    store.reset()
    store.add_vectors(xb[5], [105])
    store.add_vectors([list(map(float, r)) for r in xb[6:9]], [106, 107, 108])
    store.add_vectors(xb[9:12], [109, 110, 111])
    assert store.doc_ids == G["after_add"]["doc_ids"] and store.index.ntotal == 7
    D, got = store.search(xb[7], 3)
    assert got == G["after_add_search"]["ids"]
    monkeypatch.setattr(faiss_store.FAISSVectorStore, "_instance", None)
    monkeypatch.setattr(faiss_store.FAISSVectorStore, "_initialized", False)


# --------------------------------------------------------------------------
# seeded corpora
# --------------------------------------------------------------------------

def test_gaussian_fp32_golden(fx, golden_dir):
    z = np.load(golden_dir / "synth_small.npz")
    xb, xq = gaussian_small()
    ix = fx.IndexFlatL2(384)
    ix.add(xb)
    D, I = ix.search(xq, 10)
    assert_parity(D, I, z["g_D"], z["g_I"])


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
def test_synth_grid_golden(fx, golden_dir, dtype):
    z = np.load(golden_dir / "synth_small.npz")
    xb = F.synth(11, 0, 3000, 768)
    xq = F.synth(12, 0, 32, 768)
    ix = fx.IndexFlatL2(768, dtype=dtype)
    ix.add(xb)
    D, I = ix.search(xq, 10)
    assert_parity(D, I, z["s_D"], z["s_I"])
    assert ix.last_fallbacks() == 0


@pytest.mark.parametrize("n,d,nq,k", [(1, 16, 3, 4), (129, 100, 7, 8), (5000, 64, 300, 32),
                                      (40000, 384, 129, 10), (3, 8, 2, 32)])
def test_shapes_fp32(fx, n, d, nq, k):
    rng = np.random.default_rng(n * 7 + d)
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    ix = fx.IndexFlatL2(d)
    ix.add(xb)
    D, I = ix.search(xq, k)
    Dr, Ir = C.knn_exact(xq, xb, k)
    assert_parity(D, I, Dr, Ir)


def test_incremental_add_and_reset(fx):
    rng = np.random.default_rng(5)
    xb = rng.standard_normal((3000, 128)).astype(np.float32)
    xq = rng.standard_normal((40, 128)).astype(np.float32)
    ix = fx.IndexFlatL2(128)
    for lo in range(0, 3000, 700):
        ix.add(xb[lo:lo + 700])
    assert ix.ntotal == 3000
    D, I = ix.search(xq, 10)
    Dr, Ir = C.knn_exact(xq, xb, 10)
    assert_parity(D, I, Dr, Ir)
    ix.reset()
    assert ix.ntotal == 0
    D, I = ix.search(xq, 5)
    assert (I == -1).all() and (D == np.float32(3.4028235e38)).all()
    ix.add(xb[:10])
    D, I = ix.search(xq, 12)
    Dr, Ir = C.knn_exact(xq, xb[:10], 12)
    assert_parity(D, I, Dr, Ir)


def test_duplicates_and_ties(fx):
    # many identical rows: ties must resolve to the smaller id
    base = np.random.default_rng(9).standard_normal((50, 32)).astype(np.float32)
    xb = np.repeat(base, 40, axis=0)  # each row 40 times
    xq = base[:9] + np.float32(0.25)
    ix = fx.IndexFlatL2(32)
    ix.add(xb)
    D, I = ix.search(xq, 32)
    Dr, Ir = C.knn_exact(xq, xb, 32)
    assert_parity(D, I, Dr, Ir)


def test_inner_product(fx):
    rng = np.random.default_rng(2)
    xb = rng.standard_normal((7000, 96)).astype(np.float32)
    xq = rng.standard_normal((50, 96)).astype(np.float32)
    ix = fx.IndexFlatIP(96)
    ix.add(xb)
    D, I = ix.search(xq, 10)
    Dr, Ir = F.knn_inner_product(xq, xb, 10)
    assert_parity(D, I, Dr, Ir)


def test_normalize_mode(fx):
    rng = np.random.default_rng(4)
    xb = (rng.standard_normal((2000, 64)) * 3).astype(np.float32)
    xq = rng.standard_normal((20, 64)).astype(np.float32)
    ix = fx.IndexFlatL2(64, normalize=True)
    ix.add(xb)
    xbn = xb / np.linalg.norm(xb.astype(np.float64), axis=1, keepdims=True).astype(np.float32)
    D, I = ix.search(xq, 10)
    Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, 2000), 10)
    assert_parity(D, I, Dr, Ir)
    np.testing.assert_allclose(ix.reconstruct_n(0, 2000), xbn, rtol=1e-6, atol=1e-6)


def test_device_tensors_roundtrip(fx, torch_cuda):
    torch = torch_cuda
    for dt, tdt in (("bfloat16", torch.bfloat16), ("float16", torch.float16), ("float32", torch.float32)):
        xb = torch.empty((20000, 256), dtype=tdt, device="cuda")
        fx.synth_fill(xb, 0, 21)
        xq = torch.empty((300, 256), dtype=tdt, device="cuda")
        fx.synth_fill(xq, 0, 22)
        np.testing.assert_array_equal(xb.float().cpu().numpy(), F.synth(21, 0, 20000, 256))
        ix = fx.IndexFlatL2(256, dtype=dt)
        ix.add(xb)
        D, I = ix.search(xq, 10)
        assert D.is_cuda and I.is_cuda
        Dr, Ir = C.knn_exact(xq.float().cpu().numpy(), xb.float().cpu().numpy(), 10)
        assert_parity(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)


def test_merge_shards_kernel(fx, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(8)
    xb = rng.standard_normal((4000, 48)).astype(np.float32)
    xq = rng.standard_normal((70, 48)).astype(np.float32)
    bounds = [0, 1000, 1700, 3100, 4000]
    Ds, Is = [], []
    for g in range(4):
        ix = fx.IndexFlatL2(48)
        ix.add(xb[bounds[g]:bounds[g + 1]])
        ix.set_id_offset(bounds[g])
        D, I = ix.search(xq, 10)
        Ds.append(D)
        Is.append(I)
    Dg = torch.tensor(np.stack(Ds), device="cuda")
    Ig = torch.tensor(np.stack(Is), device="cuda")
    Dm, Im = fx.merge_shards(fx.METRIC_L2, Dg, Ig, 10)
    Dr, Ir = C.knn_exact(xq, xb, 10)
    assert_parity(Dm.cpu().numpy(), Im.cpu().numpy(), Dr, Ir)


# --------------------------------------------------------------------------
# larger sizes: oracle on a query subset, size-independent properties
# --------------------------------------------------------------------------

@pytest.mark.parametrize("dtype,n,d", [("float32", 1_000_000, 384), ("bfloat16", 1_000_000, 768)])
def test_large_synth_subset(fx, torch_cuda, dtype, n, d):
    torch = torch_cuda
    tdt = {"float32": torch.float32, "bfloat16": torch.bfloat16}[dtype]
    xb = torch.empty((n, d), dtype=tdt, device="cuda")
    fx.synth_fill(xb, 0, 1234)
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    del xb
    xq = torch.empty((1000, d), dtype=tdt, device="cuda")
    fx.synth_fill(xq, 0, 4321)
    D, I = ix.search(xq, 10)
    D = D.cpu().numpy()
    I = I.cpu().numpy()
    assert ix.last_fallbacks() == 0
    # sortedness / validity over every query
    assert (np.diff(D, axis=1) >= 0).all() and (I >= 0).all() and (I < n).all()
    # every one of the 1,000 queries against the exact oracle over the whole
    # corpus (>= 1,000 where the oracle allows; ~10-25 s of
    # host fp64 on the box's cores)
    Dr, Ir = C.knn_exact_synth(1234, n, d, F.synth(4321, 0, 1000, d), 10)
    assert_parity(D, I, Dr, Ir)
    # self-retrieval: corpus rows as queries find themselves at D = 0
    rows = np.array([0, 17, n // 2, n - 1])
    qs = np.concatenate([F.synth(1234, int(r), 1, d) for r in rows])
    Ds, Is = ix.search(qs, 3)
    assert (Is[:, 0] == rows).all() and (Ds[:, 0] == 0).all()
