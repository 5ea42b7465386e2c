"""Retrieval callers on CPU: the reference's two
search front ends -- RAGDatabaseManager.search_similar_documents
(rag_datastore_manager.py:211-238) and QueryEngine.search (query.py:21-55) --
restated per query from the reference's own steps (one faiss search per
query, pickled mapping, one SQLite row fetch per hit) and compared with the
batched counterparts in rag_faiss_embedding_amd.retrieval.  The index is the
CPU oracle standing in for the HIP index (a test double: the caller logic is
what is under test here; tests/test_gpu_parity.py covers the index)."""
import sqlite3

import numpy as np
import pytest

from oracle import flat_l2 as F
from rag_faiss_embedding_amd import retrieval as R


class _OracleIndex:
    def __init__(self, xb):
        self.xb = np.ascontiguousarray(xb, dtype=np.float32)

    def search(self, x, k):
        x = np.atleast_2d(np.asarray(x, dtype=np.float32))
        k_eff = min(k, self.xb.shape[0])
        D, I = F.knn_exact(x, self.xb, k_eff)
        if k_eff < k:  # faiss pads with -1 / FLT_MAX
            D = np.hstack([D, np.full((x.shape[0], k - k_eff), np.float32(3.4028235e38))])
            I = np.hstack([I, np.full((x.shape[0], k - k_eff), -1)])
        return D, I


def _db(n, schema_a=True):
    conn = sqlite3.connect(":memory:")
    if schema_a:
        conn.execute("CREATE TABLE documents (id INTEGER PRIMARY KEY, url TEXT UNIQUE, title TEXT, content TEXT,"
                     " created_at TEXT, updated_at TEXT)")
        conn.executemany("INSERT INTO documents VALUES (?,?,?,?,?,?)",
                         [(i, f"u{i}", f"t{i}", f"c{i}", "2024", "2024") for i in range(1, n + 1)])
    else:
        conn.execute("CREATE TABLE documents (id INTEGER PRIMARY KEY AUTOINCREMENT, url TEXT UNIQUE, title TEXT,"
                     " content TEXT)")
        conn.executemany("INSERT INTO documents VALUES (?,?,?,?)", [(i, f"u{i}", f"t{i}", f"c{i}")
                                                                     for i in range(1, n + 1)])
    return conn


def _fetch(conn, doc_id, cols):
    row = conn.execute(f"SELECT {', '.join(cols)} FROM documents WHERE id = ?", (doc_id,)).fetchone()
    return dict(zip(cols, row)) if row else None


def _ref_search_similar(index, doc_ids, conn, q, k):
    # rag_datastore_manager.py:215-234, one query
    D, I = index.search(q.reshape(1, -1), k)
    out = []
    for idx, dist in zip(I[0], D[0]):
        doc_id = doc_ids[idx]            # note: idx = -1 -> doc_ids[-1] in the reference (:228)
        doc = _fetch(conn, doc_id, R._COLS_A)
        if doc:
            doc["distance"] = float(dist)
            out.append(doc)
    return out


def _ref_query_engine(index, doc_ids, conn, q, k):
    # faiss_store.py:61-77 then query.py:36-43
    D, I = index.search(q.reshape(1, -1), k)
    valid_d, valid_ids = [], []
    for idx, dist in zip(I[0], D[0]):
        if idx != -1 and idx < len(doc_ids):
            valid_d.append(dist)
            valid_ids.append(doc_ids[idx])
    out = []
    for idx, dist in zip(valid_ids, valid_d):
        doc = _fetch(conn, int(idx) + 1, R._COLS_B)
        if doc:
            # python float + np.float32 scalar is float64 under the reference's
            # pinned numpy 1.24.3 (requirements.txt:8; numpy 2 would stay float32)
            doc["score"] = float(1.0 / (1.0 + np.float64(dist)))
            out.append(doc)
    return out


@pytest.fixture
def corpus():
    rng = np.random.default_rng(3)
    xb = rng.standard_normal((60, 32)).astype(np.float32)
    xq = rng.standard_normal((9, 32)).astype(np.float32)
    doc_ids = list(rng.permutation(np.arange(1, 61)))   # row -> doc id, as the .mapping file
    return xb, xq, [int(i) for i in doc_ids]


def test_batched_search_similar_matches_reference(corpus):
    xb, xq, doc_ids = corpus
    conn = _db(60)
    index = _OracleIndex(xb)
    got = R.search_similar_documents(index, doc_ids, R.DocumentStore(conn), xq, 5)
    assert len(got) == xq.shape[0]
    for qi in range(xq.shape[0]):
        assert got[qi] == _ref_search_similar(index, doc_ids, conn, xq[qi], 5)


def test_query_engine_matches_reference_off_by_one(corpus):
    xb, xq, doc_ids = corpus
    conn = _db(61, schema_a=False)

    class _Store:
        pass
    st = _Store()
    st.index, st.doc_ids = _OracleIndex(xb), doc_ids
    got = R.query_engine_search(st, R.DocumentStore(conn, R._COLS_B), xq, 5)
    for qi in range(xq.shape[0]):
        assert got[qi] == _ref_query_engine(st.index, doc_ids, conn, xq[qi], 5)
    fixed = R.query_engine_search(st, R.DocumentStore(conn, R._COLS_B), xq, 5, id_shift=0)
    D, I = st.index.search(xq, 5)
    assert [d["id"] for d in fixed[0]] == [doc_ids[i] for i in I[0]]


def test_minus_one_slots_are_dropped_not_wrapped():
    # k > ntotal: faiss pads I with -1; the reference's Stack A maps -1 to the
    # LAST document (rag_datastore_manager.py:228), this counterpart drops it
    xb = np.eye(3, 8, dtype=np.float32)
    conn = _db(3)
    got = R.search_similar_documents(_OracleIndex(xb), [1, 2, 3], R.DocumentStore(conn), xb[:1], 5)
    assert [d["id"] for d in got[0]] == [1, 2, 3]
    assert got[0][0]["distance"] == 0.0


def test_errors_give_empty_lists(corpus):
    xb, xq, doc_ids = corpus

    class _Broken:
        def search(self, x, k):
            raise RuntimeError("device lost")
    got = R.search_similar_documents(_Broken(), doc_ids, R.DocumentStore(_db(3)), xq, 5)
    assert got == [[] for _ in range(xq.shape[0])]


def test_similarity_and_batched_sql_lookup():
    assert R.similarity(0.0) == 1.0 and abs(R.similarity(3.0) - 0.25) < 1e-12
    conn = _db(2500)
    docs = R.DocumentStore(conn).fetch_many(range(1, 2001))   # > SQLite's parameter limit per query
    assert len(docs) == 2000 and docs[1999]["title"] == "t1999"
    assert R.DocumentStore(conn).count() == 2500


def test_engine_with_stub_encoder(corpus):
    xb, xq, doc_ids = corpus

    class _Enc:
        def generate_embeddings(self, texts):
            return np.stack([xq[int(t)] for t in texts])
    eng = R.RetrievalEngine(_Enc(), _OracleIndex(xb), doc_ids, R.DocumentStore(_db(60)))
    res = eng.search(["0", "4"], 3)
    assert [d["id"] for d in res[1]] == [d["id"] for d in eng.search_one("4", 3)]
    assert eng.search([], 3) == []


@pytest.mark.gpu
def test_batched_callers_on_hip_index(golden_dir):
    """The same callers over the HIP index, on the shipped 23-row corpus and
    its shipped row -> doc-id mapping (tests/golden/shipped_ids.json)."""
    import json

    from rag_faiss_embedding_amd import _lib, faiss
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    xb = np.load(golden_dir / "shipped_knn.npz")["xb"]
    doc_ids = json.loads((golden_dir / "shipped_ids.json").read_text())
    doc_ids = doc_ids["mapping_ids"]
    ix = faiss.IndexFlatL2(xb.shape[1])
    ix.add(xb)
    conn = _db(max(doc_ids) + 1)
    got = R.search_similar_documents(ix, doc_ids, R.DocumentStore(conn), xb, 5)
    ref = R.search_similar_documents(_OracleIndex(xb), doc_ids, R.DocumentStore(conn), xb, 5)
    assert [[d["id"] for d in r] for r in got] == [[d["id"] for d in r] for r in ref]
    for g, r in zip(got, ref):
        for dg, dr in zip(g, r):
            assert abs(dg["distance"] - dr["distance"]) <= 1e-5 * max(1.0, abs(dr["distance"]))
