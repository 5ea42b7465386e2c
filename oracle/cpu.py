"""ctypes binding of oracle/flat_l2.c.  TEST INFRASTRUCTURE ONLY (see
oracle/flat_l2.py header): used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker or the timed CPU baseline."""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "_build" / "libfx_oracle.so"
_lib: Optional[ctypes.CDLL] = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build(arch: Optional[str] = None, out_dir: Optional[Path] = None) -> Path:
    """Compile flat_l2.c (``make -C oracle``); ``arch`` overrides -march."""
    env = dict(os.environ)
    args = ["make", "-s", "-C", str(_HERE)]
    if arch:
        args.append(f"ARCH={arch}")
    if out_dir is not None:
        args.append(f"OUT={out_dir}")
    subprocess.run(args, check=True, env=env)
    return (Path(out_dir) if out_dir else _HERE / "_build") / "libfx_oracle.so"


def load(path: Optional[Path] = None) -> ctypes.CDLL:
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else _LIB_PATH
    if not p.exists():
        build()
    lib = ctypes.CDLL(str(p))
    lib.fxo_synth_fill.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, _f32p, ctypes.c_int]
    lib.fxo_synth_fill.restype = None
    for name in ("fxo_knn_exact", "fxo_knn_blas"):
        fn = getattr(lib, name)
        fn.argtypes = [_f32p, ctypes.c_int64, _f32p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _f32p, _i64p, ctypes.c_int]
        fn.restype = None
    for name in ("fxo_knn_exact_synth", "fxo_knn_exact_synth_f64"):
        fn = getattr(lib, name)
        fn.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, _f32p, ctypes.c_int64, ctypes.c_int, _f32p,
                       _i64p, ctypes.c_int]
        fn.restype = None
    lib.fxo_max_threads.restype = ctypes.c_int
    if path is None:
        _lib = lib
    return lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def _ip(a: np.ndarray):
    return a.ctypes.data_as(_i64p)


def synth(seed: int, row0: int, nrows: int, d: int, nthreads: int = 0) -> np.ndarray:
    out = np.empty((nrows, d), dtype=np.float32)
    load().fxo_synth_fill(seed, row0, nrows, d, _fp(out), nthreads)
    return out


def knn_exact(xq: np.ndarray, xb: np.ndarray, k: int, nthreads: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    nq, d = xq.shape
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    load().fxo_knn_exact(_fp(xq), nq, _fp(xb), xb.shape[0], d, k, _fp(D), _ip(I), nthreads)
    return D, I


def knn_blas(xq: np.ndarray, xb: np.ndarray, k: int, nthreads: int = 0,
             lib: Optional[ctypes.CDLL] = None) -> Tuple[np.ndarray, np.ndarray]:
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    nq, d = xq.shape
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    (lib or load()).fxo_knn_blas(_fp(xq), nq, _fp(xb), xb.shape[0], d, k, _fp(D), _ip(I), nthreads)
    return D, I


def knn_exact_synth(cseed: int, nb: int, d: int, xq: np.ndarray, k: int,
                    nthreads: int = 0, f64: bool = False) -> Tuple[np.ndarray, np.ndarray]:
    """Exact k-NN against synthetic corpus rows [0, nb) (streamed, never
    materialised).  Grid-valued queries take the integer path (flat_l2.c:
    the same exact sums); f64=True forces the fp64 restatement (its check)."""
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    nq = xq.shape[0]
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    fn = load().fxo_knn_exact_synth_f64 if f64 else load().fxo_knn_exact_synth
    fn(cseed, nb, d, _fp(xq), nq, k, _fp(D), _ip(I), nthreads)
    return D, I


def max_threads() -> int:
    return int(load().fxo_max_threads())
