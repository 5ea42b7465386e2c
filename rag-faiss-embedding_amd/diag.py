"""Indexes bound to the diagnostic build of the library (tests only).

``libfx_index_diag.so`` is ``libfx_index.so``'s kernels with the host side
compiled under ``-DFX_DIAG`` (``make -C csrc diag``): its option table adds
the test hooks the product library does not carry -- ``force_fallback``
(1: every query through the device-gated re-scan, 2: through the exact fp64
scan) and ``scan_dbg`` 32 (the scan's whole key matrix dumped to
``FX_SCAN_KEYS``) -- plus the FX_SCAN_TRACE / _CAND dumps.  The classes here
are the faiss.py ones with every call going to that build.
"""
from __future__ import annotations

import ctypes

from . import _lib
from . import faiss as _faiss

if not _lib.DIAG_PATH.exists():
    raise ImportError(f"{_lib.DIAG_PATH} not found: build it with `make -C {_lib._HERE / 'csrc'} diag`")

lib = _lib.bind(_lib.DIAG_PATH)


class IndexFlatL2(_faiss.IndexFlatL2):
    _lib = lib


class IndexFlatIP(_faiss.IndexFlatIP):
    _lib = lib


def read_index(path: str, dtype: str = "float32", device: int = 0) -> IndexFlatL2:
    h = ctypes.c_void_p()
    _lib.check(lib.fx_index_read(str(path).encode(), _faiss._DTYPES[dtype], int(device), ctypes.byref(h)), lib)
    return IndexFlatL2(0, dtype=dtype, device=device, _handle=h)
