"""CPU oracle for the flat squared-L2 k-NN path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the *checker*.  The product path
(``rag-faiss-embedding_amd/``) never imports it and has no CPU fallback.

What it restates
----------------
The reference does all hot-path arithmetic inside the un-vendored
``faiss-cpu`` dependency (``requirements.txt:13``, unpinned; not installed in
this image, no source available).  Call sites of that dependency:

* ``faiss.IndexFlatL2(d)``            -- ``faiss_store.py:29,126``; ``rag_datastore_manager.py:138``
* ``IndexFlatL2.add(x)``              -- ``faiss_store.py:46``; ``rag_datastore_manager.py:173``
* ``IndexFlatL2.search(x, k)``        -- ``faiss_store.py:64``; ``rag_datastore_manager.py:218``
* ``faiss.write_index / read_index``  -- ``faiss_store.py:91,106``; ``rag_datastore_manager.py:186,205``

This module restates FAISS's *published* ``IndexFlatL2`` semantics
(``faiss/IndexFlat.cpp`` / ``faiss/utils/distances.cpp::knn_L2sqr`` upstream):

* distances are SQUARED L2, no sqrt, no normalisation (:func:`knn_exact`);
* results per query sorted ascending by distance; ties resolve to the
  smaller row id (max-heap ``CMax<float, idx_t>`` replacement rule);
* missing slots (k > ntotal) are ``I = -1`` and ``D = FLT_MAX``;
* for ``nq >= 20`` FAISS uses the BLAS expansion ``|x|^2 + |y|^2 - 2 x.y`` in
  fp32 with negatives clamped to 0 (:func:`knn_blas` emulates that order of
  operations so tests can show how far FAISS itself is from exact).

Pinning (see ``tests/test_oracle.py``): the IxF2 reader/writer round-trips the
reference's own shipped index ``data/faiss_index.bin`` byte-exactly, the
shipped mapping decodes to the ids of ``data/documents.json`` in file order
(``rag_datastore_manager.py:189``), every shipped row retrieves itself at
D = 0, and the wrapper-level golden JSON in ``tests/golden/`` was produced by
running the reference ``faiss_store.py`` itself with this module standing in
for ``faiss`` (``tests/golden/make_golden.py``).  Nothing pins FAISS's
arithmetic beyond that: the distance semantics are "parity unpinned" by any
reference test, exactly as recorded in SURVEY.md section 8c.
"""
from __future__ import annotations

import struct
from typing import List, Sequence, Tuple

import numpy as np

FLT_MAX = np.float32(3.4028234663852886e38)

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1


# ----------------------------------------------------------------------------
# k-NN restatements
# ----------------------------------------------------------------------------

def _topk_rows(dist: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Per-row k smallest of ``dist`` (fp64 or fp32) ordered by (D, id).

    Mirrors the heap replacement order of FAISS ``CMax`` heaps: a candidate
    with an equal distance never displaces a smaller id.
    """
    nq, nb = dist.shape
    D = np.full((nq, k), FLT_MAX, dtype=np.float32)
    I = np.full((nq, k), -1, dtype=np.int64)
    if nb == 0 or k == 0:
        return D, I
    kk = min(k, nb)
    ids = np.arange(nb, dtype=np.int64)
    for i in range(nq):
        row = dist[i]
        # lexsort: primary key distance, secondary key id (stable by id)
        order = np.lexsort((ids, row))[:kk]
        D[i, :kk] = row[order].astype(np.float32)
        I[i, :kk] = order
    return D, I


def knn_exact(xq: np.ndarray, xb: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Exact squared-L2 k-NN: D[i,j] = sum_t (x_it - y_jt)^2 evaluated in fp64,
    rounded once to fp32 (the value FAISS's fp32 kernels approximate).

    Follows ``IndexFlatL2.search`` as called at ``faiss_store.py:64``.
    Ordering and padding as in :func:`_topk_rows`.
    """
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    assert xq.ndim == 2 and xb.ndim == 2 and xq.shape[1] == xb.shape[1]
    q = xq.astype(np.float64)
    b = xb.astype(np.float64)
    # exact per-pair differences (no expansion: no cancellation)
    dist = np.empty((q.shape[0], b.shape[0]), dtype=np.float64)
    step = max(1, 4_000_000 // max(1, b.size))
    for i0 in range(0, q.shape[0], step):
        diff = q[i0:i0 + step, None, :] - b[None, :, :]
        dist[i0:i0 + step] = np.einsum("qnd,qnd->qn", diff, diff)
    # rank on the fp32-rounded value: that is the value returned, and ties in
    # the returned value must order by id (FAISS heap order).
    return _topk_rows(dist.astype(np.float32), k)


def knn_blas(xq: np.ndarray, xb: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Emulation of FAISS's BLAS path (``knn_L2sqr`` for nq >= 20): fp32
    ``|x|^2 + |y|^2 - 2 x.y`` with negatives clamped to 0.  Used to measure how
    far CPU FAISS itself sits from :func:`knn_exact`, never as the parity key.
    """
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xn = np.einsum("ij,ij->i", xq, xq, dtype=np.float32)
    yn = np.einsum("ij,ij->i", xb, xb, dtype=np.float32)
    ip = xq @ xb.T
    dist = (xn[:, None] + yn[None, :]) - np.float32(2) * ip
    np.maximum(dist, np.float32(0), out=dist)
    return _topk_rows(dist.astype(np.float32), k)


def knn_inner_product(xq: np.ndarray, xb: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Exact max-inner-product k-NN (``IndexFlatIP`` semantics, ``config.py:30``
    "IP" option): results sorted by DEScending similarity, ties to smaller id,
    padding ``I=-1`` / ``D=-FLT_MAX``."""
    xq = np.ascontiguousarray(xq, dtype=np.float32).astype(np.float64)
    xb = np.ascontiguousarray(xb, dtype=np.float32).astype(np.float64)
    sim = (xq @ xb.T).astype(np.float32)
    D, I = _topk_rows(-sim, k)
    D = np.where(I >= 0, -D, -FLT_MAX).astype(np.float32)
    return D, I


def merge_topk(Ds: Sequence[np.ndarray], Is: Sequence[np.ndarray], k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Merge per-shard (D, I) lists (global ids) into the global top-k under the
    (D asc, id asc) order -- the result-merge FAISS applies across shards
    (``IndexShards`` / ``merge_knn_results``)."""
    D = np.concatenate(Ds, axis=1)
    I = np.concatenate(Is, axis=1)
    nq = D.shape[0]
    outD = np.full((nq, k), FLT_MAX, dtype=np.float32)
    outI = np.full((nq, k), -1, dtype=np.int64)
    for i in range(nq):
        valid = I[i] >= 0
        d, ids = D[i][valid], I[i][valid]
        order = np.lexsort((ids, d))[:k]
        outD[i, :len(order)] = d[order]
        outI[i, :len(order)] = ids[order]
    return outD, outI


# ----------------------------------------------------------------------------
# On-disk formats (faiss_store.py:83-122, rag_datastore_manager.py:182-209)
# ----------------------------------------------------------------------------

IXF2_HEADER = struct.Struct("<4siqqqBiq")  # 45 bytes


def write_ixf2_bytes(xb: np.ndarray) -> bytes:
    """Serialise an IndexFlatL2 the way ``faiss.write_index`` does (fourcc
    ``IxF2``): i32 d, i64 ntotal, i64 dummy (1<<20) x2, u8 is_trained, i32
    metric_type (1 = L2), i64 count-of-floats, f32 codes."""
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    n, d = xb.shape
    hdr = IXF2_HEADER.pack(b"IxF2", d, n, 1 << 20, 1 << 20, 1, METRIC_L2, n * d)
    return hdr + xb.astype("<f4").tobytes()


def read_ixf2_bytes(buf: bytes) -> np.ndarray:
    """Inverse of :func:`write_ixf2_bytes`; raises ``RuntimeError`` on any
    malformed field (as ``faiss.read_index`` raises ``RuntimeError``)."""
    if len(buf) < IXF2_HEADER.size:
        raise RuntimeError("IxF2: truncated header")
    fourcc, d, n, _d1, _d2, trained, metric, count = IXF2_HEADER.unpack_from(buf, 0)
    if fourcc != b"IxF2":
        raise RuntimeError(f"IxF2: unsupported fourcc {fourcc!r}")
    if metric != METRIC_L2 or d <= 0 or n < 0 or count != n * d:
        raise RuntimeError("IxF2: inconsistent header")
    body = buf[IXF2_HEADER.size:]
    if len(body) != 4 * count:
        raise RuntimeError("IxF2: truncated codes")
    return np.frombuffer(body, dtype="<f4").reshape(n, d).astype(np.float32)


def parse_id_mapping(buf: bytes) -> List[int]:
    """Decode the ``.mapping`` sidecar (``faiss_store.py:94-95``: a pickled
    ``list[int]``) WITHOUT unpickling: only the opcodes a protocol 2-5 pickle
    of a flat list of Python ints uses are accepted; anything else raises."""
    out: List[int] = []
    pos = 0
    n = len(buf)
    stack_marks = 0
    pending: List[int] = []
    have_list = False

    def need(m: int) -> None:
        if pos + m > n:
            raise ValueError("mapping: truncated")

    while True:
        need(1)
        op = buf[pos]
        pos += 1
        if op == 0x80:  # PROTO
            need(1); pos += 1
        elif op == 0x95:  # FRAME
            need(8); pos += 8
        elif op == 0x5D:  # EMPTY_LIST
            if have_list:
                raise ValueError("mapping: nested list")
            have_list = True
        elif op == 0x94:  # MEMOIZE
            pass
        elif op == 0x71:  # BINPUT
            need(1); pos += 1
        elif op == 0x28:  # MARK
            stack_marks += 1
        elif op == 0x4B:  # BININT1
            need(1); pending.append(buf[pos]); pos += 1
        elif op == 0x4D:  # BININT2
            need(2); pending.append(int.from_bytes(buf[pos:pos + 2], "little")); pos += 2
        elif op == 0x4A:  # BININT
            need(4); pending.append(int.from_bytes(buf[pos:pos + 4], "little", signed=True)); pos += 4
        elif op == 0x8A:  # LONG1
            need(1); m = buf[pos]; pos += 1; need(m)
            pending.append(int.from_bytes(buf[pos:pos + m], "little", signed=True)); pos += m
        elif op == 0x61:  # APPEND
            if not have_list or len(pending) != 1:
                raise ValueError("mapping: bad APPEND")
            out.extend(pending); pending = []
        elif op == 0x65:  # APPENDS
            if not have_list or stack_marks != 1:
                raise ValueError("mapping: bad APPENDS")
            out.extend(pending); pending = []; stack_marks = 0
        elif op == 0x2E:  # STOP
            if not have_list or pending or stack_marks:
                raise ValueError("mapping: not a flat list of ints")
            return out
        else:
            raise ValueError(f"mapping: opcode 0x{op:02x} not allowed")


# ----------------------------------------------------------------------------
# Synthetic corpora (shared definition with oracle/flat_l2.c and the HIP
# generator in rag-faiss-embedding_amd/csrc/fx_index.hip)
# ----------------------------------------------------------------------------

_M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def synth(seed: int, row0: int, nrows: int, d: int) -> np.ndarray:
    """Rows ``row0 .. row0+nrows-1`` of the counter-based synthetic corpus.

    element(row, col) = (b0 + b1 - 255) / 64 with b0, b1 the two low bytes of
    splitmix64(seed * GOLDEN + row * d + col).  Every value is a multiple of
    1/64 with |numerator| <= 255, so it is exact in fp32, bf16 and fp16: a
    bf16/fp16 index and the fp32 CPU oracle see identical inputs.
    """
    rows = np.arange(row0, row0 + nrows, dtype=np.uint64)[:, None]
    cols = np.arange(d, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        z = (np.uint64((seed * GOLDEN) & _M64) + rows * np.uint64(d) + cols)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b0 = (z & np.uint64(0xFF)).astype(np.int32)
    b1 = ((z >> np.uint64(8)) & np.uint64(0xFF)).astype(np.int32)
    return ((b0 + b1 - 255).astype(np.float32) / np.float32(64.0))
