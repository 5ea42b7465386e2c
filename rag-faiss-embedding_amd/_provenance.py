"""Which build a measurement belongs to.

``source_digest()`` hashes the sources the HIP library is compiled from
(``csrc/*.hip|*.h|*.cpp``, the Makefile and ``include/fx_index.h``), so a
committed rocprofv3 summary (``profiles/pmc_scan_<cfg>.json``, written by
tools/summarize_profile.py) can say which kernels it profiled, and bench.py
can refuse to quote a traffic figure measured on other kernels than the ones
it runs.  Works without git (the GPU box gets the tree without ``.git``) and
without the library (no GPU, no import of ``_lib``).
"""
from __future__ import annotations

import hashlib
from pathlib import Path

_PKG = Path(__file__).resolve().parent
_ROOT = _PKG.parent


def source_files():
    csrc = _PKG / "csrc"
    files = sorted(p for p in csrc.iterdir() if p.is_file() and (p.suffix in (".hip", ".h", ".cpp") or
                                                               p.name == "Makefile"))
    return files + [_ROOT / "include" / "fx_index.h"]


def source_digest() -> str:
    """sha256 (first 16 hex digits) over the library's source files, by name
    and content."""
    h = hashlib.sha256()
    for p in source_files():
        h.update(p.name.encode() + b"\0")
        h.update(p.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:16]


def file_digest(path) -> str:
    """sha256 (first 16 hex digits) of one built file (the library a run loaded)."""
    return hashlib.sha256(Path(path).read_bytes()).hexdigest()[:16]
