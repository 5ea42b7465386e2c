"""Import shim for the package directory ``rag-faiss-embedding_amd/``.

The directory name (fixed by the project layout) is not a valid Python
identifier, so it is registered here under ``rag_faiss_embedding_amd``::

    import amd_fx
    from rag_faiss_embedding_amd import faiss, faiss_store
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

PKG_NAME = "rag_faiss_embedding_amd"
PKG_DIR = Path(__file__).resolve().parent / "rag-faiss-embedding_amd"


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(PKG_NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod


load()
