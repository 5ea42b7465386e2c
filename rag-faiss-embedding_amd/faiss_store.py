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
    _instance = None
    _initialized = False

    def __new__(cls, *args, **kwargs):  # process-wide singleton (faiss_store.py:14-17)
        if cls._instance is None:
            cls._instance = super(FAISSVectorStore, cls).__new__(cls)
        return cls._instance

    def __init__(self, dimension: int = 384, index_path: str = "data/faiss_index.bin", *,
                 dtype: str = "float32", device: int = 0):
        if self._initialized:  # later constructions ignore their arguments (:21-22)
            return
        self.dimension = dimension
        self.index_path = index_path
        self.dtype = dtype
        self.device = device
        self.doc_ids: List[int] = []
        self.index = _fx.IndexFlatL2(dimension, dtype=dtype, device=device)
        if os.path.exists(index_path):
            self.load_index()
        logger.info(f"Initialized FAISS index with dimension {dimension}")
        self._initialized = True

    def add_vectors(self, vectors, ids: List[int]):
        """faiss_store.py:36-47: ids are recorded before the rows are added."""
        if isinstance(vectors, list):
            vectors = np.array(vectors, dtype=np.float32)
        if len(vectors.shape) == 1:
            vectors = vectors.reshape(1, -1)
        self.doc_ids.extend(ids)
        self.index.add(vectors)
        logger.info(f"Added {len(ids)} vectors to FAISS index with IDs: {ids}")

    def search(self, query_vector, k: int = 5) -> Tuple[np.ndarray, List[int]]:
        """faiss_store.py:49-81: single query, row -> document id, drop -1 and
        out-of-range rows; any exception -> ``(np.array([]), [])``."""
        try:
            logger.info(f"Searching FAISS index with k={k}")
            logger.info(f"Index contains {self.index.ntotal} vectors")
            if isinstance(query_vector, list):
                query_vector = np.array(query_vector, dtype=np.float32)
            query_vector = query_vector.reshape(1, -1)
            distances, indices = self.index.search(query_vector, k)
            if not isinstance(distances, np.ndarray):  # device tensors -> host
                distances = distances.cpu().numpy()
                indices = indices.cpu().numpy()
            logger.info(f"Raw FAISS results - distances: {distances}, indices: {indices[0]}")
            doc_ids = []
            valid_distances = []
            for i, idx in enumerate(indices[0]):
                if idx != -1 and idx < len(self.doc_ids):
                    doc_ids.append(self.doc_ids[idx])
                    valid_distances.append(distances[0][i])
            logger.info(f"Mapped to document IDs: {doc_ids}")
            return np.array(valid_distances), doc_ids
        except Exception as e:  # noqa: BLE001 -- reference swallows every error
            logger.error(f"Error during FAISS search: {e}")
            return np.array([]), []

    def save_index(self, filepath: Optional[str] = None):
        """faiss_store.py:83-97: IxF2 index + pickle protocol-4 id mapping."""
        save_path = filepath or self.index_path
        mapping_path = save_path + ".mapping"
        os.makedirs(os.path.dirname(save_path), exist_ok=True)
        _fx.write_index(self.index, save_path)
        with open(mapping_path, "wb") as f:
            f.write(_mapping.dumps_ids(self.doc_ids))
        logger.info(f"Saved FAISS index and mapping to {save_path}")

    def load_index(self, filepath: Optional[str] = None):
        """faiss_store.py:99-122: errors are logged and re-raised."""
        load_path = filepath or self.index_path
        mapping_path = load_path + ".mapping"
        try:
            self.index = _fx.read_index(load_path, dtype=self.dtype, device=self.device)
            if os.path.exists(mapping_path):
                with open(mapping_path, "rb") as f:
                    self.doc_ids = _mapping.loads_ids(f.read())
                logger.info(f"Loaded ID mapping for {len(self.doc_ids)} documents")
            else:
                self.doc_ids = list(range(self.index.ntotal))
                logger.warning(f"No mapping file found. Created sequential IDs: {self.doc_ids}")
            logger.info(f"Loaded FAISS index from {load_path}")
        except Exception as e:
            logger.error(f"Error loading FAISS index: {e}")
            raise

    def reset(self):
        """faiss_store.py:124-128."""
        self.index = _fx.IndexFlatL2(self.dimension, dtype=self.dtype, device=self.device)
        self.doc_ids = []
        logger.info("Reset FAISS index")
