"""Retrieval callers over the MI355X index.

The reference runs its two retrieval callers one query at a time, each with a
device round trip and a CPU faiss scan:

* ``RAGDatabaseManager.search_similar_documents(query, k=5)``
  (rag_datastore_manager.py:211-238, Stack A): encode -> ``faiss_index.search``
  -> re-read the pickled row->doc-id mapping from disk on EVERY query (:221-223)
  -> ``doc_ids[idx]`` (no -1 filter: a missing slot silently maps to the last
  document, :228) -> ``Database.fetch_document`` one row at a time (:229) ->
  ``doc['distance'] = float(d)``.  Any error -> ``[]`` (:236-238).
* ``QueryEngine.search(query, top_k=5)`` (query.py:21-55, Stack B): encode ->
  ``FAISSVectorStore.search`` (already maps rows to doc ids and drops -1,
  faiss_store.py:70-74) -> ``Database.get_document_by_id(int(idx) + 1)``
  (query.py:40 -- an off-by-one on ids that are already document ids) ->
  ``doc['score'] = 1 / (1 + distance)`` (query.py:42).  Any error -> ``[]``.

Here both take a BATCH of queries: one encoder pass (device-resident, no
per-batch ``.cpu()``), one fused scan for all queries, one SQLite ``IN``
lookup for all hits.  Result dictionaries keep the reference's keys and
order.  Deliberate differences, in this counterpart only:

* ``search_similar_documents`` drops ``I = -1`` slots instead of mapping them
  to ``doc_ids[-1]`` ("fix -1 handling in the build's own
  counterpart only"), and reads the mapping once, not per query;
* ``query_engine_search`` reproduces the ``+1`` of query.py:40 by default
  (``id_shift=1``) so a switched caller returns the same rows; pass
  ``id_shift=0`` for the corrected join.
"""
from __future__ import annotations

import logging
import sqlite3
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

logger = logging.getLogger("rag_faiss_embedding_amd.retrieval")

# column sets of the two reference schemas
_COLS_A = ("id", "url", "title", "content", "created_at", "updated_at")  # rag_datastore_manager.py:33-42
_COLS_B = ("id", "url", "title", "content")                             # database.py:60-72 row -> dict


def similarity(distance: float) -> float:
    """The score both reference front ends show: 1 / (1 + d)
    (query.py:42, 2-cli-rag-search.py:48)."""
    return float(1.0 / (1.0 + distance))


class DocumentStore:
    """Read side of the reference's SQLite ``documents`` table
    (rag_datastore_manager.py:22-97 / database.py:10-104), batched: one
    ``SELECT ... WHERE id IN (...)`` per search batch instead of one query
    per hit."""

    def __init__(self, conn_or_path, columns: Sequence[str] = _COLS_A):
        self.conn = conn_or_path if isinstance(conn_or_path, sqlite3.Connection) else sqlite3.connect(conn_or_path)
        self.columns = tuple(columns)

    def fetch_many(self, ids: Iterable[int]) -> Dict[int, Dict]:
        ids = sorted({int(i) for i in ids})
        out: Dict[int, Dict] = {}
        cols = ", ".join(self.columns)
        for lo in range(0, len(ids), 900):  # SQLite's bound-parameter limit
            chunk = ids[lo:lo + 900]
            q = f"SELECT {cols} FROM documents WHERE id IN ({','.join('?' * len(chunk))})"
            for row in self.conn.execute(q, chunk):
                out[int(row[0])] = dict(zip(self.columns, row))
        return out

    def count(self) -> int:
        return int(self.conn.execute("SELECT COUNT(*) FROM documents").fetchone()[0])


def _to_numpy(x) -> np.ndarray:
    if hasattr(x, "detach"):  # torch tensor (device results of a device search)
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def search_similar_documents(index, doc_ids: Sequence[int], store: DocumentStore, query_embeddings,
                             k: int = 5) -> List[List[Dict]]:
    """Batched ``RAGDatabaseManager.search_similar_documents``
    (rag_datastore_manager.py:211-238): for every query row, the documents
    of its k nearest index rows, nearest first, each with ``distance`` (the
    squared L2 distance the index returned).  ``doc_ids`` is the row -> doc
    id mapping (faiss_index.bin.mapping).  Errors are logged and give empty
    lists, as the reference's blanket ``except`` does."""
    try:
        D, I = index.search(query_embeddings, int(k))
        D, I = _to_numpy(D), _to_numpy(I)
        ids = np.asarray(doc_ids, dtype=np.int64)
        valid = (I >= 0) & (I < len(ids))
        docs = store.fetch_many(ids[I[valid]].tolist())
        results: List[List[Dict]] = []
        for qi in range(I.shape[0]):
            row: List[Dict] = []
            for idx, dist in zip(I[qi], D[qi]):
                if idx < 0 or idx >= len(ids):
                    continue  # faiss pads missing slots with -1 (see module note)
                doc = docs.get(int(ids[idx]))
                if doc is not None:
                    d = dict(doc)
                    d["distance"] = float(dist)
                    row.append(d)
            results.append(row)
        return results
    except Exception as e:  # noqa: BLE001 -- reference contract (rag_datastore_manager.py:236-238)
        logger.error("Error searching documents: %s", e)
        n = getattr(query_embeddings, "shape", [1])[0] if hasattr(query_embeddings, "shape") else 1
        return [[] for _ in range(n)]


def query_engine_search(store_index, store: DocumentStore, query_embeddings, top_k: int = 5,
                        id_shift: int = 1) -> List[List[Dict]]:
    """Batched ``QueryEngine.search`` (query.py:21-55) over a
    ``FAISSVectorStore``-like object (``.index`` + ``.doc_ids``): vector
    search, the join ``get_document_by_id(doc_id + id_shift)`` (query.py:40
    uses +1) and ``score = 1 / (1 + distance)``.  Returns one list per query;
    errors give empty lists (query.py:53-55)."""
    try:
        D, I = store_index.index.search(query_embeddings, int(top_k))
        D, I = _to_numpy(D), _to_numpy(I)
        ids = np.asarray(store_index.doc_ids, dtype=np.int64)
        valid = (I >= 0) & (I < len(ids))          # faiss_store.py:70-73
        docs = store.fetch_many((ids[I[valid]] + id_shift).tolist())
        results: List[List[Dict]] = []
        for qi in range(I.shape[0]):
            row: List[Dict] = []
            for idx, dist in zip(I[qi], D[qi]):
                if idx < 0 or idx >= len(ids):
                    continue
                doc = docs.get(int(ids[idx]) + id_shift)
                if doc is not None:
                    d = dict(doc)
                    d["score"] = similarity(float(dist))
                    row.append(d)
            results.append(row)
        return results
    except Exception as e:  # noqa: BLE001 -- reference contract
        logger.exception("Search error: %s", e)
        n = query_embeddings.shape[0] if hasattr(query_embeddings, "shape") else 1
        return [[] for _ in range(n)]


class RetrievalEngine:
    """Encoder + index + document store: the retrieval half of the
    reference's CLI / QueryEngine, batched.  ``search(texts, k)`` encodes all
    texts in one device-resident pass and scans the index once."""

    def __init__(self, vectorizer, index, doc_ids: Sequence[int], store: DocumentStore):
        self.vectorizer = vectorizer
        self.index = index
        self.doc_ids = list(doc_ids)
        self.store = store

    def embed(self, texts: List[str]):
        if hasattr(self.vectorizer, "generate_embeddings_device"):
            return self.vectorizer.generate_embeddings_device(texts)
        return np.asarray(self.vectorizer.generate_embeddings(texts), dtype=np.float32)

    def search(self, texts: List[str], k: int = 5) -> List[List[Dict]]:
        if not texts:
            return []
        return search_similar_documents(self.index, self.doc_ids, self.store, self.embed(texts), k)

    def search_one(self, text: str, k: int = 5) -> List[Dict]:
        """The reference's single-query call shape (rag_datastore_manager.py:211)."""
        out = self.search([text], k)
        return out[0] if out else []


def load_store_and_mapping(db_path: str, mapping_path: str, columns: Optional[Sequence[str]] = None):
    """(DocumentStore, doc_ids) from the reference's on-disk artefacts:
    ``data/documents.db`` and ``data/faiss_index.bin.mapping`` (parsed
    without unpickling, see _mapping.py)."""
    from pathlib import Path

    from ._mapping import loads_ids
    return DocumentStore(db_path, columns or _COLS_A), loads_ids(Path(mapping_path).read_bytes())
