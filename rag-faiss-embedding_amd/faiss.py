"""faiss-compatible surface over the MI355X flat index.

Mirrors the slice of the faiss Python API the reference uses
(faiss_store.py:29,46,64,91,106,126; rag_datastore_manager.py:138,173,186,
205,218) so a caller can switch with ``import rag_faiss_embedding_amd.faiss
as faiss``:

* ``IndexFlatL2(d)`` / ``IndexFlatIP(d)`` with ``.d``, ``.ntotal``,
  ``.metric_type``, ``.is_trained``, ``.add(x)``, ``.search(x, k) -> (D, I)``,
  ``.reset()``, ``.reconstruct_n(i0, n)``;
* ``write_index(index, path)`` / ``read_index(path)`` on the IxF2 format.

Inputs may be numpy arrays (as in the reference: host fp32, results returned
as numpy) or torch tensors already resident on the GPU (fp32/bf16/fp16;
results returned as device tensors, no host round trip) -- the latter is the
device-resident hand-off from the encoder.

Errors follow faiss: a dimension mismatch raises ``AssertionError`` (the
SWIG wrapper's ``assert d == self.d``); library failures raise
``RuntimeError``.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import check, lib

METRIC_INNER_PRODUCT = _lib.METRIC_INNER_PRODUCT
METRIC_L2 = _lib.METRIC_L2

_DTYPES = {"float32": _lib.F32, "bfloat16": _lib.BF16, "float16": _lib.F16}
_DTYPE_NAMES = {v: k for k, v in _DTYPES.items()}
_UNBOUND = object()  # no stream bound yet by this Python object


def _torch():
    try:
        import torch  # noqa: F401
        return torch
    except Exception:  # pragma: no cover - torch is in the image
        return None


def _is_device_tensor(x) -> bool:
    t = _torch()
    return t is not None and isinstance(x, t.Tensor) and x.is_cuda


def _tensor_dtype(x) -> int:
    t = _torch()
    m = {t.float32: _lib.F32, t.bfloat16: _lib.BF16, t.float16: _lib.F16}
    if x.dtype not in m:
        raise TypeError(f"unsupported tensor dtype {x.dtype}")
    return m[x.dtype]


class _FlatIndex:
    """Common implementation of IndexFlatL2 / IndexFlatIP."""

    metric_type: int = METRIC_L2
    _lib = lib  # the ctypes build this index lives in (the diagnostic build: diag.py)

    def _check(self, rc: int) -> None:
        check(rc, self._lib)

    def __init__(self, d: int, dtype: str = "float32", device: int = 0, normalize: bool = False,
                 _handle: Optional[ctypes.c_void_p] = None):
        if dtype not in _DTYPES:
            raise ValueError(f"dtype must be one of {sorted(_DTYPES)}")
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            self._check(self._lib.fx_index_create(int(d), _DTYPES[dtype], self.metric_type, int(device),
                                                  ctypes.byref(self._h)))
        self.device = int(device)
        self.storage_dtype = dtype
        self.is_trained = True
        self.verbose = False
        if normalize:
            self._check(self._lib.fx_index_set_normalize(self._h, 1))

    # -- faiss attributes ------------------------------------------------------
    @property
    def d(self) -> int:
        v = ctypes.c_int(0)
        self._check(self._lib.fx_index_dim(self._h, ctypes.byref(v)))
        return v.value

    @property
    def ntotal(self) -> int:
        v = ctypes.c_int64(0)
        self._check(self._lib.fx_index_ntotal(self._h, ctypes.byref(v)))
        return v.value

    # -- stream plumbing --------------------------------------------------------
    def _bind_stream(self, use_torch: bool) -> None:
        s = _torch().cuda.current_stream(self.device).cuda_stream if use_torch else None
        if getattr(self, "_bound", _UNBOUND) == s:  # (one C call less per search on the latency-bound path)
            return
        self._check(self._lib.fx_index_set_stream(self._h, ctypes.c_void_p(s) if s is not None else None))
        self._bound = s

    # -- add / search --------------------------------------------------------------
    def add(self, x) -> None:
        """``IndexFlat.add`` (faiss_store.py:46): append rows of ``x``."""
        if _is_device_tensor(x):
            assert x.dim() == 2 and x.shape[1] == self.d, "dimension mismatch"
            assert x.device.index == self.device, f"tensor on cuda:{x.device.index}, index on cuda:{self.device}"
            x = x.contiguous()
            self._bind_stream(True)
            self._check(self._lib.fx_index_add(self._h, x.shape[0], ctypes.c_void_p(x.data_ptr()),
                                               _tensor_dtype(x), _lib.MEM_DEVICE))
            return
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.ndim == 2 and x.shape[1] == self.d, "dimension mismatch"
        self._bind_stream(False)
        self._check(self._lib.fx_index_add(self._h, x.shape[0], x.ctypes.data_as(ctypes.c_void_p), _lib.F32,
                                           _lib.MEM_HOST))

    def search(self, x, k: int, *, D=None, I=None) -> Tuple:
        """``IndexFlat.search`` (faiss_store.py:64): k nearest rows of every
        query row.  Returns ``(D, I)`` shaped ``(nq, k)``.  Any k, as faiss:
        k <= ``MAX_K`` runs the fused scan, larger k the exact sort path;
        slots past ntotal hold I = -1, D = +-FLT_MAX."""
        k = int(k)
        if k <= 0:
            raise AssertionError("k must be positive")
        if _is_device_tensor(x):
            t = _torch()
            assert x.dim() == 2 and x.shape[1] == self.d, "dimension mismatch"
            assert x.device.index == self.device, f"queries on cuda:{x.device.index}, index on cuda:{self.device}"
            x = x.contiguous()
            nq = x.shape[0]
            if D is None:
                D = t.empty((nq, k), dtype=t.float32, device=x.device)
            if I is None:
                I = t.empty((nq, k), dtype=t.int64, device=x.device)
            for name, a, dt in (("D", D, t.float32), ("I", I, t.int64)):
                # the C side writes nq*k elements through the raw pointer
                assert _is_device_tensor(a) and a.device == x.device, f"{name} must be on {x.device}"
                assert a.dtype == dt and tuple(a.shape) == (nq, k) and a.is_contiguous(), \
                    f"{name} must be a contiguous {dt} tensor of shape ({nq}, {k})"
            self._bind_stream(True)
            self._check(self._lib.fx_index_search(self._h, nq, ctypes.c_void_p(x.data_ptr()), _tensor_dtype(x),
                                                  _lib.MEM_DEVICE, k, ctypes.c_void_p(D.data_ptr()),
                                                  ctypes.c_void_p(I.data_ptr()), _lib.MEM_DEVICE))
            return D, I
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.ndim == 2 and x.shape[1] == self.d, "dimension mismatch"
        nq = x.shape[0]
        Dh = np.empty((nq, k), dtype=np.float32) if D is None else D
        Ih = np.empty((nq, k), dtype=np.int64) if I is None else I
        for name, a, dt in (("D", Dh, np.float32), ("I", Ih, np.int64)):
            # the C side writes nq*k elements through the raw pointer
            assert isinstance(a, np.ndarray) and a.dtype == dt and a.shape == (nq, k) and \
                a.flags.c_contiguous and a.flags.writeable, \
                f"{name} must be a writeable C-contiguous {np.dtype(dt).name} array of shape ({nq}, {k})"
        self._bind_stream(False)
        # (raw addresses: .ctypes.data is an int, much cheaper per call than data_as)
        self._check(self._lib.fx_index_search(self._h, nq, x.ctypes.data, _lib.F32, _lib.MEM_HOST, k,
                                              Dh.ctypes.data, Ih.ctypes.data, _lib.MEM_HOST))
        return Dh, Ih

    def last_fallbacks(self) -> int:
        """Queries of the last search whose top-k the scan's candidates could
        not certify (re-scanned with a wide candidate set)."""
        v = ctypes.c_int64(0)
        self._check(self._lib.fx_index_last_fallbacks(self._h, ctypes.byref(v)))
        return v.value

    def last_exact_fallbacks(self) -> int:
        """Of those, the queries the re-scan could not certify either,
        re-ranked by the exact fp64 scan of every row."""
        v = ctypes.c_int64(0)
        self._check(self._lib.fx_index_last_exact_fallbacks(self._h, ctypes.byref(v)))
        return v.value

    def last_scan_plan(self) -> dict:
        """The last search's scan plan: tile_rows (128 = k_scan_v4, 64 =
        k_scan_v5), query_tile (queries per workgroup), splits."""
        v = [ctypes.c_int(0) for _ in range(3)]
        self._check(self._lib.fx_index_last_scan_plan(self._h, *(ctypes.byref(x) for x in v)))
        return {"tile_rows": v[0].value, "query_tile": v[1].value, "splits": v[2].value}

    def last_dropped_candidates(self) -> int:
        """Candidate entries the last search's exact re-rank dropped for a row
        id outside [0, ntotal): 0 unless a scan list was corrupted (then the
        top-k may miss rows; treat it as an error)."""
        v = ctypes.c_int64(0)
        self._check(self._lib.fx_index_last_dropped_candidates(self._h, ctypes.byref(v)))
        return v.value

    def reset(self) -> None:
        self._check(self._lib.fx_index_reset(self._h))

    def reserve(self, n: int) -> None:
        self._check(self._lib.fx_index_reserve(self._h, int(n)))

    def reconstruct_n(self, i0: int, n: int) -> np.ndarray:
        out = np.empty((int(n), self.d), dtype=np.float32)
        self._check(self._lib.fx_index_reconstruct_n(self._h, int(i0), int(n),
                                                     out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def set_id_offset(self, offset: int) -> None:
        self._check(self._lib.fx_index_set_id_offset(self._h, int(offset)))

    def set_option(self, name: str, value: int) -> None:
        """Per-index tuning / diagnostic option (include/fx_index.h
        ``fx_index_set_option``; defaults from the FX_* environment at creation)."""
        self._check(self._lib.fx_index_set_option(self._h, name.encode(), int(value)))

    # -- profiling (bench roofline) -------------------------------------------------
    def profile(self, enable: bool = True) -> None:
        self._check(self._lib.fx_index_profile(self._h, 1 if enable else 0))

    def profile_read(self) -> Tuple[float, float, int]:
        a, b, n = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0)
        self._check(self._lib.fx_index_profile_read(self._h, ctypes.byref(a), ctypes.byref(b),
                                                    ctypes.byref(n)))
        return a.value, b.value, n.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.fx_index_free(h)
            self._h = ctypes.c_void_p()


class IndexFlatL2(_FlatIndex):
    """``faiss.IndexFlatL2`` (faiss_store.py:29): exact squared-L2 search."""

    metric_type = METRIC_L2


class IndexFlatIP(_FlatIndex):
    """``faiss.IndexFlatIP`` (the ``FAISS_INDEX_TYPE = "IP"`` option of
    config.py:30): exact maximum inner product search."""

    metric_type = METRIC_INNER_PRODUCT


def write_index(index: _FlatIndex, path: str) -> None:
    """``faiss.write_index`` (faiss_store.py:91): IxF2 file, fp32 codes."""
    check(index._lib.fx_index_write(index._h, str(path).encode()), index._lib)


def read_index(path: str, dtype: str = "float32", device: int = 0) -> IndexFlatL2:
    """``faiss.read_index`` (faiss_store.py:106): IxF2 file -> HBM index."""
    h = ctypes.c_void_p()
    rc = lib.fx_index_read(str(path).encode(), _DTYPES[dtype], int(device), ctypes.byref(h))
    check(rc)
    return IndexFlatL2(0, dtype=dtype, device=device, _handle=h)


def synth_fill(out, row0: int, seed: int) -> None:
    """Fill a 2-D device tensor with rows ``row0..`` of the synthetic corpus
    (definition shared with oracle/flat_l2.py ``synth``)."""
    t = _torch()
    assert _is_device_tensor(out) and out.dim() == 2 and out.is_contiguous()
    s = t.cuda.current_stream(out.device).cuda_stream
    check(lib.fx_synth_fill(ctypes.c_void_p(out.data_ptr()), int(row0), out.shape[0], out.shape[1],
                            _tensor_dtype(out), int(seed), out.device.index, ctypes.c_void_p(s)))


def merge_shards(metric: int, Dg, Ig, k: int, D_out=None, I_out=None):
    """Merge gathered per-shard results ``Dg``/``Ig`` shaped (G, nq, k) (device
    tensors) into the global top-k (the step after the RCCL allgather)."""
    t = _torch()
    G, nq, kk = Dg.shape
    assert kk == k and Ig.shape == Dg.shape
    if D_out is None:
        D_out = t.empty((nq, k), dtype=t.float32, device=Dg.device)
    if I_out is None:
        I_out = t.empty((nq, k), dtype=t.int64, device=Dg.device)
    s = t.cuda.current_stream(Dg.device).cuda_stream
    check(lib.fx_merge_shards(int(metric), G, nq, k, ctypes.c_void_p(Dg.data_ptr()), ctypes.c_void_p(Ig.data_ptr()),
                              ctypes.c_void_p(D_out.data_ptr()), ctypes.c_void_p(I_out.data_ptr()),
                              Dg.device.index, ctypes.c_void_p(s)))
    return D_out, I_out
