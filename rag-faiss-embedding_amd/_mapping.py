"""The ``.mapping`` sidecar of a saved index (faiss_store.py:86,94-95,109-116):
a pickled ``list[int]`` of document ids, one per index row.

Reading never unpickles: only the opcodes a protocol 2-5 pickle of a flat
list of Python ints uses are accepted, so a mapping file cannot execute code.
Writing uses ``pickle`` protocol 4 -- byte-identical to what the reference's
``pickle.dump(self.doc_ids, f)`` produces on Python 3.8-3.13.
"""
from __future__ import annotations

import pickle
from typing import Iterable, List


def dumps_ids(ids: Iterable[int]) -> bytes:
    return pickle.dumps([int(i) for i in ids], protocol=4)


def loads_ids(buf: bytes) -> List[int]:
    out: List[int] = []
    pending: List[int] = []
    pos, n, marks, have_list = 0, len(buf), 0, False

    def take(m: int) -> bytes:
        nonlocal pos
        if pos + m > n:
            raise ValueError("mapping: truncated")
        b = buf[pos:pos + m]
        pos += m
        return b

    while True:
        op = take(1)[0]
        if op == 0x80:            # PROTO
            take(1)
        elif op == 0x95:          # FRAME
            take(8)
        elif op == 0x5D:          # EMPTY_LIST
            if have_list:
                raise ValueError("mapping: nested list")
            have_list = True
        elif op == 0x94:          # MEMOIZE
            pass
        elif op == 0x71:          # BINPUT
            take(1)
        elif op == 0x28:          # MARK
            marks += 1
        elif op == 0x4B:          # BININT1
            pending.append(take(1)[0])
        elif op == 0x4D:          # BININT2
            pending.append(int.from_bytes(take(2), "little"))
        elif op == 0x4A:          # BININT
            pending.append(int.from_bytes(take(4), "little", signed=True))
        elif op == 0x8A:          # LONG1
            m = take(1)[0]
            pending.append(int.from_bytes(take(m), "little", signed=True))
        elif op == 0x61:          # APPEND
            if not have_list or len(pending) != 1:
                raise ValueError("mapping: bad APPEND")
            out.extend(pending)
            pending = []
        elif op == 0x65:          # APPENDS
            if not have_list or marks != 1:
                raise ValueError("mapping: bad APPENDS")
            out.extend(pending)
            pending, marks = [], 0
        elif op == 0x2E:          # STOP
            if not have_list or pending or marks:
                raise ValueError("mapping: not a flat list of ints")
            return out
        else:
            raise ValueError(f"mapping: opcode 0x{op:02x} not allowed (not a list of ints)")
