"""CPU model of the scan's packed-key bitonic sort (fx_scan_common.h
sort64_packed / cmpx_packed): 64 lanes each hold one (key, row) entry packed
as a 64-bit value; step (S, size) takes the partner lane ^ S's value where
(partner < mine) == up_mask(S, size) bit of the lane.  The network must sort
ascending for any input, duplicates included (empty list slots are all
(+inf, INT_MAX))."""
import numpy as np


def up_mask(S, size):
    return np.array([((l & S) == 0) == ((l & size) == 0) for l in range(64)])


def sort64_packed(v):
    x = v.copy()
    for L in range(6):
        size = 2 << L
        for T in range(L + 1):
            S = (size >> 1) >> T
            o = x[np.arange(64) ^ S]
            x = np.where(~((o < x) ^ up_mask(S, size)), o, x)
    return x


def f2ord(f):
    u = np.asarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, ~u & 0xFFFFFFFF, u | 0x80000000)


def test_network_sorts_any_input():
    rng = np.random.default_rng(1)
    for trial in range(500):
        v = rng.integers(0, 50, 64).astype(np.uint64) * 1000 + rng.permutation(64).astype(np.uint64)
        if trial % 3 == 0:
            v[rng.random(64) < 0.3] = np.uint64(2 ** 63)
        np.testing.assert_array_equal(sort64_packed(v), np.sort(v))


def test_packed_order_is_key_then_row():
    """(key asc, row asc) for keys of either sign, as the lists are ordered."""
    rng = np.random.default_rng(2)
    keys = rng.standard_normal(64).astype(np.float32)
    keys[:8] = keys[8]                      # ties: the smaller row first
    rows = rng.permutation(1000)[:64].astype(np.uint64)
    packed = (f2ord(keys) << np.uint64(32)) | rows
    out = sort64_packed(packed)
    order = np.lexsort((rows, keys))
    np.testing.assert_array_equal(out, packed[order])
