"""``FAISSVectorStore`` on the MI355X flat index.

Same class, methods, attributes and error behaviour as the reference
``faiss_store.py:10-128``; only the engine underneath changes (the HIP index
of :mod:`.faiss` instead of faiss-cpu).  Logging uses the stdlib instead of
loguru.  The mapping sidecar is read without unpickling (:mod:`._mapping`).

Extensions (keyword-only, defaults reproduce the reference): ``dtype`` of the
HBM codes ("float32" like the reference, or "bfloat16"/"float16") and the
GPU ``device``.  ``add_vectors``/``search`` also accept torch tensors that
already live on the GPU (encoder hand-off without ``.cpu().numpy()``).
"""
from __future__ import annotations

import logging
import os
from typing import List, Optional, Tuple

import numpy as np

from . import _mapping
from . import faiss as _fx

logger = logging.getLogger("rag_faiss_embedding_amd.faiss_store")


class FAISSVectorStore:
    """One store per process (faiss_store.py:14-17): later constructions
    return the first instance and ignore their arguments (:21-22)."""

    _instance = None
    _initialized = False

    def __new__(cls, *args, **kwargs):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self, dimension: int = 384, index_path: str = "data/faiss_index.bin", *,
                 dtype: str = "float32", device: int = 0):
        if self._initialized:
            return
        self.dimension, self.index_path = dimension, index_path
        self.dtype, self.device = dtype, device
        self.doc_ids: List[int] = []
        self.index = _fx.IndexFlatL2(dimension, dtype=dtype, device=device)
        if os.path.exists(index_path):
            self.load_index()
        logger.info("store ready: d=%d, %s on cuda:%d", dimension, dtype, device)
        self._initialized = True

    @staticmethod
    def _as_rows(x):
        """list -> float32 array; a single vector -> one row (:38-42)."""
        if isinstance(x, list):
            x = np.array(x, dtype=np.float32)
        return x.reshape(1, -1) if len(x.shape) == 1 else x

    def add_vectors(self, vectors, ids: List[int]):
        """faiss_store.py:36-47.  The ids are recorded before the rows go in,
        and their count is not checked against the rows (as there)."""
        rows = self._as_rows(vectors)
        self.doc_ids.extend(ids)
        self.index.add(rows)
        logger.info("add: %d ids -> ntotal %d", len(ids), self.index.ntotal)

    def search(self, query_vector, k: int = 5) -> Tuple[np.ndarray, List[int]]:
        """faiss_store.py:49-81: one query; index rows map to document ids,
        -1 and rows past the id list are dropped; on any error the result is
        ``(np.array([]), [])``.  Any k, as faiss (k > ``FX_MAX_K`` = 1024
        takes the index's exact sort path)."""
        try:
            q = query_vector
            if isinstance(q, list):
                q = np.array(q, dtype=np.float32)
            dist, rows = self.index.search(q.reshape(1, -1), k)
            if not isinstance(dist, np.ndarray):  # device tensors -> host
                dist, rows = dist.cpu().numpy(), rows.cpu().numpy()
            n_ids = len(self.doc_ids)
            keep = [(float(dv), int(r)) for dv, r in zip(dist[0], rows[0]) if r != -1 and r < n_ids]
            found = [self.doc_ids[r] for _, r in keep]
            logger.info("search k=%d over %d rows -> %s", k, self.index.ntotal, found)
            return np.array([dv for dv, _ in keep], dtype=np.float32) if keep else np.array([]), found
        except Exception as e:  # noqa: BLE001 -- the reference swallows every error here
            logger.error("search failed: %s", e)
            return np.array([]), []

    def save_index(self, filepath: Optional[str] = None):
        """faiss_store.py:83-97: IxF2 index file + pickle-protocol-4 id list
        at ``<path>.mapping``."""
        path = filepath or self.index_path
        os.makedirs(os.path.dirname(path), exist_ok=True)
        _fx.write_index(self.index, path)
        with open(path + ".mapping", "wb") as f:
            f.write(_mapping.dumps_ids(self.doc_ids))
        logger.info("saved %d rows to %s", self.index.ntotal, path)

    def load_index(self, filepath: Optional[str] = None):
        """faiss_store.py:99-122: without a mapping file the ids are the row
        numbers; errors are logged and raised again."""
        path = filepath or self.index_path
        try:
            self.index = _fx.read_index(path, dtype=self.dtype, device=self.device)
            if os.path.exists(path + ".mapping"):
                with open(path + ".mapping", "rb") as f:
                    self.doc_ids = _mapping.loads_ids(f.read())
            else:
                self.doc_ids = list(range(self.index.ntotal))
                logger.warning("%s.mapping missing: ids are the row numbers", path)
            logger.info("loaded %d rows, %d ids from %s", self.index.ntotal, len(self.doc_ids), path)
        except Exception as e:
            logger.error("load of %s failed: %s", path, e)
            raise

    def reset(self):
        """faiss_store.py:124-128: a fresh empty index, no ids."""
        self.index = _fx.IndexFlatL2(self.dimension, dtype=self.dtype, device=self.device)
        self.doc_ids = []
        logger.info("reset")
