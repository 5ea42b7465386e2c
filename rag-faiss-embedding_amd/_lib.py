"""ctypes binding of libfx_index.so (include/fx_index.h).

The product path has no CPU fallback: if the HIP library is missing or has
not been built, importing this module raises immediately.  Build it with
``make -C rag-faiss-embedding_amd/csrc`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("FX_INDEX_LIB", _HERE / "libfx_index.so"))

if not LIB_PATH.exists():
    raise ImportError(
        f"{LIB_PATH} not found: the MI355X HIP library is required (build it with "
        f"`make -C {_HERE / 'csrc'}`); there is no CPU fallback")

# One HIP runtime per process: torch ships its own libamdhip64 (SONAME
# libamdhip64.so.7, like /opt/rocm's).  Loaded first, torch's copy satisfies
# our NEEDED entry and both share it; loaded second, torch would pull a second
# runtime that sees no device.  So bring torch in first when it is installed.
try:  # pragma: no cover - torch is part of the image
    import torch  # noqa: F401
except Exception:  # noqa: BLE001
    pass

F32, BF16, F16 = 0, 1, 2
METRIC_INNER_PRODUCT, METRIC_L2 = 0, 1
MEM_HOST, MEM_DEVICE = 0, 1
MAX_K = 1024  # == FX_MAX_K (include/fx_index.h): largest k of the fused scan path (larger k: exact sort path)

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i = ctypes.c_int
_pp = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); every symbol declared in include/fx_index.h
SIGNATURES = {
    "fx_last_error": (ctypes.c_char_p, []),
    "fx_device_count": (_i, [ctypes.POINTER(_i)]),
    "fx_index_create": (_i, [_i, _i, _i, _i, _pp]),
    "fx_index_free": (None, [_vp]),
    "fx_index_set_normalize": (_i, [_vp, _i]),
    "fx_index_set_stream": (_i, [_vp, _vp]),
    "fx_index_set_id_offset": (_i, [_vp, _i64]),
    "fx_index_set_option": (_i, [_vp, ctypes.c_char_p, _i64]),
    "fx_index_dim": (_i, [_vp, ctypes.POINTER(_i)]),
    "fx_index_ntotal": (_i, [_vp, ctypes.POINTER(_i64)]),
    "fx_index_storage_dtype": (_i, [_vp, ctypes.POINTER(_i)]),
    "fx_index_metric": (_i, [_vp, ctypes.POINTER(_i)]),
    "fx_index_reserve": (_i, [_vp, _i64]),
    "fx_index_add": (_i, [_vp, _i64, _vp, _i, _i]),
    "fx_index_search": (_i, [_vp, _i64, _vp, _i, _i, _i, _vp, _vp, _i]),
    "fx_index_last_fallbacks": (_i, [_vp, ctypes.POINTER(_i64)]),
    "fx_index_last_scan_plan": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "fx_index_last_exact_fallbacks": (_i, [_vp, ctypes.POINTER(_i64)]),
    "fx_index_last_dropped_candidates": (_i, [_vp, ctypes.POINTER(_i64)]),
    "fx_index_reset": (_i, [_vp]),
    "fx_index_reconstruct_n": (_i, [_vp, _i64, _i64, _vp]),
    "fx_index_write": (_i, [_vp, ctypes.c_char_p]),
    "fx_index_read": (_i, [ctypes.c_char_p, _i, _i, _pp]),
    "fx_merge_shards": (_i, [_i, _i, _i64, _i, _vp, _vp, _vp, _vp, _i, _vp]),
    "fx_synth_fill": (_i, [_vp, _i64, _i64, _i, _i, ctypes.c_uint64, _i, _vp]),
    "fx_index_profile": (_i, [_vp, _i]),
    "fx_index_profile_read": (_i, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(_i64)]),
}


def bind(path: Path, ab_build: bool = False) -> ctypes.CDLL:
    """Load one build of the library and declare every signature.  An A/B
    build (FX_INDEX_LIB: an older library on the same box) may predate a
    symbol, which is then left unbound; any other build must export all."""
    so = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(so, name)
        except AttributeError:
            if not ab_build:
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    return so


lib = bind(LIB_PATH, ab_build="FX_INDEX_LIB" in os.environ)

# The diagnostic build (make -C csrc diag): the same kernels with test hooks
# (force_fallback, the scan's key dump) in its option table.  Loaded only by
# rag_faiss_embedding_amd.diag (tests); the product never touches it.
DIAG_PATH = _HERE / "libfx_index_diag.so"


class FxError(RuntimeError):
    """A failure reported by the HIP library (faiss raises RuntimeError)."""


def last_error(so: ctypes.CDLL = None) -> str:
    msg = (so or lib).fx_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int, so: ctypes.CDLL = None) -> None:
    """Raise the library's thread-local message (of the build `so` that
    returned rc; default the product library) when rc != 0."""
    if rc != 0:
        raise FxError(last_error(so) or f"fx error {rc}")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib.fx_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0
