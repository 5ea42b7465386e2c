"""The CPU oracle (test infrastructure) pinned against the reference's own
artefacts and known answers."""
import json

import numpy as np
import pytest

from oracle import cpu as C
from oracle import flat_l2 as F
from tests._data import gaussian_small


def test_ixf2_roundtrip_shipped_index_byte_exact(golden_dir):
    # data/faiss_index.bin of the reference (faiss.write_index output)
    buf = (golden_dir / "shipped_index.bin").read_bytes()
    xb = F.read_ixf2_bytes(buf)
    assert xb.shape == (23, 384)
    assert F.write_ixf2_bytes(xb) == buf


def test_ixf2_rejects_malformed(golden_dir):
    buf = (golden_dir / "shipped_index.bin").read_bytes()
    with pytest.raises(RuntimeError):
        F.read_ixf2_bytes(b"IxFI" + buf[4:])
    with pytest.raises(RuntimeError):
        F.read_ixf2_bytes(buf[:-4])
    with pytest.raises(RuntimeError):
        F.read_ixf2_bytes(buf[:20])


def test_shipped_mapping_matches_documents_json(golden_dir):
    ids = json.loads((golden_dir / "shipped_ids.json").read_text())
    # rag_datastore_manager.py:189 writes [doc["id"] for doc in documents]
    assert ids["mapping_ids"] == ids["documents_json_ids"]
    assert sorted(ids["mapping_ids"]) == list(range(1, 24))


def test_self_retrieval_known_answer(golden_dir):
    z = np.load(golden_dir / "shipped_knn.npz")
    xb = z["xb"]
    D, I = F.knn_exact(xb, xb, 1)
    assert (I[:, 0] == np.arange(23)).all()
    assert (D[:, 0] == 0).all()


@pytest.mark.parametrize("k", [1, 5, 10, 23, 30])
def test_oracle_shipped_knn_fixture(golden_dir, k):
    z = np.load(golden_dir / "shipped_knn.npz")
    xb = z["xb"]
    D, I = F.knn_exact(xb, xb, k)
    np.testing.assert_array_equal(I, z[f"I_k{k}"])
    np.testing.assert_array_equal(D, z[f"D_k{k}"])
    # C restatement agrees bit for bit
    D2, I2 = C.knn_exact(xb, xb, k)
    np.testing.assert_array_equal(I2, I)
    np.testing.assert_array_equal(D2, D)
    if k > 23:  # faiss padding for k > ntotal
        assert (I[:, 23:] == -1).all() and (D[:, 23:] == np.float32(3.4028235e38)).all()


def test_wrapper_golden_search_matches_oracle(golden_dir):
    """wrapper_golden.json was produced by the reference faiss_store.py itself
    (tests/golden/make_golden.py); its row->doc-id mapping of the oracle's
    answers is what FAISSVectorStore.search returns."""
    G = json.loads((golden_dir / "wrapper_golden.json").read_text())
    z = np.load(golden_dir / "shipped_knn.npz")
    doc_ids = G["load"]["doc_ids"]
    for i, res in enumerate(G["search_k5"]):
        assert res["ids"] == [doc_ids[j] for j in z["I_k5"][i]]
        np.testing.assert_array_equal(np.float32(res["D"]), z["D_k5"][i])
    assert G["search_k5"][0]["ids"] == [9, 11, 14, 21, 8]
    assert G["search_list_k30"]["ids"].__len__() == 23
    assert G["search_wrong_d"] == {"D": [], "ids": [], "D_dtype": "float64"}


def test_gaussian_fixture(golden_dir):
    z = np.load(golden_dir / "synth_small.npz")
    xb, xq = gaussian_small()
    D, I = C.knn_exact(xq, xb, 10)
    np.testing.assert_array_equal(I, z["g_I"])
    np.testing.assert_array_equal(D, z["g_D"])


def test_synth_grid_fixture_and_generators_agree(golden_dir):
    z = np.load(golden_dir / "synth_small.npz")
    xb = F.synth(11, 0, 3000, 768)
    np.testing.assert_array_equal(xb, C.synth(11, 0, 3000, 768))
    xq = F.synth(12, 0, 32, 768)
    D, I = C.knn_exact_synth(11, 3000, 768, xq, 10)
    np.testing.assert_array_equal(I, z["s_I"])
    np.testing.assert_array_equal(D, z["s_D"])
    # exactly representable in bf16 (8 significant bits) and fp16
    num = xb * 64
    assert (num == np.round(num)).all() and np.abs(num).max() <= 255


def test_blas_path_is_close_but_not_exact(golden_dir):
    """FAISS's own BLAS path (nq >= 20) deviates from exact on the shipped
    vectors: the reason the parity key is the exact oracle."""
    z = np.load(golden_dir / "shipped_knn.npz")
    xb = z["xb"]
    D, I = F.knn_exact(xb, xb, 10)
    Db, Ib = C.knn_blas(xb, xb, 10)
    np.testing.assert_array_equal(Ib, I)
    err = np.abs(Db.astype(np.float64) - D)
    assert err.max() < 1e-3


def test_tie_breaks_to_smaller_id():
    xb = np.zeros((6, 4), dtype=np.float32)
    xb[[1, 3, 4]] = 1.0
    xq = np.ones((1, 4), dtype=np.float32)
    for fn in (F.knn_exact, C.knn_exact, C.knn_blas):
        D, I = fn(xq, xb, 4)
        assert I[0].tolist() == [1, 3, 4, 0]


def test_mapping_parser_rejects_non_list():
    import pickle
    with pytest.raises(ValueError):
        F.parse_id_mapping(pickle.dumps({"a": 1}, protocol=4))
    assert F.parse_id_mapping(pickle.dumps(list(range(2500)), protocol=4)) == list(range(2500))


def test_merge_topk_matches_global():
    rng = np.random.default_rng(3)
    xb = rng.standard_normal((900, 32)).astype(np.float32)
    xq = rng.standard_normal((7, 32)).astype(np.float32)
    D, I = F.knn_exact(xq, xb, 10)
    parts = []
    for lo, hi in ((0, 300), (300, 650), (650, 900)):
        d, i = F.knn_exact(xq, xb[lo:hi], 10)
        parts.append((d, np.where(i >= 0, i + lo, -1)))
    Dm, Im = F.merge_topk([p[0] for p in parts], [p[1] for p in parts], 10)
    np.testing.assert_array_equal(Im, I)
    np.testing.assert_array_equal(Dm, D)


@pytest.mark.parametrize("d,nb,nq", [(768, 20_000, 9), (384, 30_001, 13), (100, 5_003, 7), (7, 1_000, 3)])
def test_synth_oracle_integer_path_is_exact(d, nb, nq):
    """flat_l2.c fxo_knn_exact_synth: grid-valued queries take the integer
    path (exact 4096 * sum (x - y)^2, rounded to fp32 once); it must equal the
    fp64 restatement bit for bit (ids and distances), including the
    zero-padded tails of d not a multiple of 16 and partial 4-row blocks."""
    xq = F.synth(4321, 0, nq, d)
    D1, I1 = C.knn_exact_synth(1234, nb, d, xq, 10)
    D2, I2 = C.knn_exact_synth(1234, nb, d, xq, 10, f64=True)
    np.testing.assert_array_equal(I1, I2)
    np.testing.assert_array_equal(D1, D2)
    # and against the numpy restatement on the materialised rows
    Dr, Ir = F.knn_exact(xq, F.synth(1234, 0, nb, d), 10)
    np.testing.assert_array_equal(I1, Ir)
    np.testing.assert_array_equal(D1, Dr)


def test_synth_oracle_off_grid_queries_take_fp64():
    xq = F.synth(4321, 0, 5, 64) + np.float32(1e-3)  # not multiples of 1/64
    D1, I1 = C.knn_exact_synth(1234, 3_000, 64, xq, 10)
    D2, I2 = C.knn_exact_synth(1234, 3_000, 64, xq, 10, f64=True)
    np.testing.assert_array_equal(I1, I2)
    np.testing.assert_array_equal(D1, D2)
