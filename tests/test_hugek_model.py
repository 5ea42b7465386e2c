"""CPU model of the k > FX_MAX_K sort path's key arithmetic (fx_hugek.hip).

The GPU path packs key = ord(D') << idbits | row (D' = D for L2, -D for IP,
-0 folded into +0) and radix-sorts it; the shard merge sorts (id, D) pairs by
id and then stably by ord(D').  Both must reproduce faiss's result order --
ascending D (L2) / descending D (IP), ties to the smaller id -- which the
oracle (oracle/flat_l2.py) defines.  Here the same packing is restated in
numpy and sorted with numpy's stable sort, against the oracle's ordering on
inputs with exact ties, signed zeros and padding.
"""
import numpy as np

from oracle import flat_l2 as F


def f2ord(f):
    u = np.asarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)


def ord2f(o):
    o = np.asarray(o, dtype=np.uint64)
    u = np.where(o & 0x80000000, o & 0x7FFFFFFF, (~o) & 0xFFFFFFFF).astype(np.uint32)
    return u.view(np.float32)


def id_bits(n):
    b = 1
    while b < 32 and (1 << b) < n:
        b += 1
    return b


def hugek_select(dist, k, metric="L2"):
    """fx_hugek.hip: pack, sort, unpack the first k (padding past ntotal)."""
    n = dist.shape[1]
    ib = id_bits(n)
    key_f = (dist if metric == "L2" else -dist).astype(np.float32) + np.float32(0.0)
    keys = (f2ord(key_f) << np.uint64(ib)) | np.arange(n, dtype=np.uint64)[None, :]
    keys = np.sort(keys, axis=1)[:, :k]
    D = ord2f(keys >> np.uint64(ib))
    D = D if metric == "L2" else -D
    I = (keys & np.uint64((1 << ib) - 1)).astype(np.int64)
    pad = k - D.shape[1]
    if pad > 0:
        fill = np.float32(3.4028234663852886e38) if metric == "L2" else np.float32(-3.4028234663852886e38)
        D = np.concatenate([D, np.full((D.shape[0], pad), fill, np.float32)], axis=1)
        I = np.concatenate([I, np.full((I.shape[0], pad), -1, np.int64)], axis=1)
    return D.astype(np.float32), I


def test_ord_roundtrip_and_order():
    v = np.array([-np.inf, -3.5, -1e-30, -0.0, 0.0, 1e-30, 2.0, np.inf], np.float32)
    o = f2ord(v)
    assert (ord2f(o) == v).all()
    assert (np.diff(o.astype(np.int64)) >= 0).all()


def test_l2_select_matches_oracle_with_ties():
    rng = np.random.default_rng(1)
    base = rng.standard_normal((300, 16)).astype(np.float32)
    xb = np.concatenate([base, base[::-1], base[:50]])   # exact duplicate rows -> tied distances
    xq = np.concatenate([base[:3], rng.standard_normal((4, 16)).astype(np.float32)])
    dist = ((xq.astype(np.float64)[:, None, :] - xb.astype(np.float64)[None]) ** 2).sum(-1).astype(np.float32)
    for k in (100, 650, 900):
        D, I = hugek_select(dist, k)
        Dr, Ir = F.knn_exact(xq, xb, k)
        assert (I == Ir).all()
        assert (D[Ir >= 0] == Dr[Ir >= 0]).all()


def test_ip_select_matches_oracle_and_signed_zero():
    rng = np.random.default_rng(2)
    xb = rng.standard_normal((400, 8)).astype(np.float32)
    xb[10] = 0.0
    xb[20] = 0.0                                            # IP = +-0 with any query
    xq = rng.standard_normal((5, 8)).astype(np.float32)
    dist = (xq.astype(np.float64) @ xb.astype(np.float64).T).astype(np.float32)
    D, I = hugek_select(dist, 400, metric="IP")
    Dr, Ir = F.knn_inner_product(xq, xb, 400)
    assert (I == Ir).all()
    assert (D == Dr).all()


def test_merge_two_pass_equals_single_key_order():
    """Shard merge: stable sort by id, then stable sort by ord(D) == (D, id) order."""
    rng = np.random.default_rng(3)
    G, k = 4, 50
    d = rng.integers(0, 20, size=(G, k)).astype(np.float32)   # many equal distances
    ids = rng.permutation(10_000)[: G * k].reshape(G, k).astype(np.int64)
    ids[1, -5:] = -1                                          # missing entries go last
    d[1, -5:] = np.float32(3.4028234663852886e38)
    dk = np.where(ids < 0, np.uint64(0xFFFFFFFF), f2ord(d)).ravel()
    idk = np.where(ids < 0, np.uint64(2**64 - 1), ids.astype(np.uint64)).ravel()
    o1 = np.argsort(idk, kind="stable")
    o2 = np.argsort(dk[o1], kind="stable")
    order = o1[o2][:k]
    got = list(zip(d.ravel()[order].tolist(), ids.ravel()[order].tolist()))
    valid = [(float(a), int(b)) for a, b in zip(d.ravel(), ids.ravel()) if b >= 0]
    assert got == sorted(valid)[:k]
