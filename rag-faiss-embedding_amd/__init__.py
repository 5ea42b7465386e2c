"""MI355X-native drop-in for the dense-retrieval hot path of
luzbetak/rag-faiss-embedding.

Surfaces (each mirrors the reference interface it replaces):

* :mod:`.faiss`          -- ``IndexFlatL2`` / ``IndexFlatIP`` / ``write_index`` /
                            ``read_index`` (faiss-cpu as called at
                            faiss_store.py:29-126, rag_datastore_manager.py:138-218)
* :mod:`.faiss_store`    -- ``FAISSVectorStore`` (faiss_store.py:10-128)
* :mod:`.vectorization`  -- ``VectorizationPipeline`` (vectorization.py:10-47)
* :mod:`.sharded`        -- row-sharded multi-GPU index (one process per GPU,
                            RCCL allgather merge)
* :mod:`.retrieval`      -- batched callers: ``search_similar_documents``
                            (rag_datastore_manager.py:211-238) and
                            ``QueryEngine.search`` (query.py:21-55) over the
                            index + the SQLite document table

Importing a submodule that touches the GPU path loads ``libfx_index.so``
(HIP, gfx950) and fails loudly when it is absent.  The directory name is not a
Python identifier; import it through the repo-root shim ``amd_fx``:

    import amd_fx                       # registers rag_faiss_embedding_amd
    from rag_faiss_embedding_amd import faiss
"""
__all__ = ["faiss", "faiss_store", "vectorization", "sharded", "retrieval"]
