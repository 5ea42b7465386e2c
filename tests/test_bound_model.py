"""CPU model of the 16-bit scan's error bound and of the certification that
uses it (fx_kernels.hip k_prep_queries mode "L2, scan dtype BF16 / F16" and
`certified`).

The scan key of row y for query x is, with mu the image centre and op =
rn16(fl32(x - mu)) the query operand,

    a(y) = fl_chain(|y - mu|^2 ; y_k * (-2 op_k), k = 0..K-1)

(an fp32 accumulation of exact 16-bit products onto srcC).  k_prep_queries
claims, with r = (x - mu) - op (exact), rho = |r|, s_q = |x|^2 - |mu|^2 - 2 r.x,

    |a(y) + s_q - D(y)| <= 2 rho sqrt(D(y)) + E,
    E = u Smax + gamma_{K+1} (Smax + 2 M |op|)   (x 1.0625 in the kernel)

for every row (D = the exact squared distance of the fp32 query to the stored
row).  Here the fp32 chain is emulated in numpy (each step one fp32 rounding;
bf16 x bf16 products are exact in fp32), in two accumulation orders, on
clustered and isotropic data, and the claim is checked row by row; then the
certification rule is checked on adversarial keys that use the whole bound.
"""
import numpy as np
import pytest

U = 2.0 ** -24


def rn_bf16(x):
    """round-to-nearest-even fp32 -> bf16 -> fp32 (f2bf in fx_device.h)."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def rn16(x, dt):
    return rn_bf16(x) if dt == "bf16" else np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def prep(x, mu, M, Smax, K, dt):
    """k_prep_queries, L2 16-bit mode (restated)."""
    xc = (x - mu).astype(np.float32)
    op = rn16(xc, dt)
    r = (x.astype(np.float64) - mu.astype(np.float64)) - op.astype(np.float64)
    rho = np.sqrt(np.sum(r * r))
    shift = np.sum(x.astype(np.float64) ** 2) - np.sum(mu.astype(np.float64) ** 2) - 2.0 * np.dot(r, x)
    gamma = (K + 1) * U / (1 - (K + 1) * U)
    on = np.sqrt(np.sum(op.astype(np.float64) ** 2))
    E = U * Smax * 1.01 + gamma * (Smax * 1.01 + 2.0 * M * on)
    return op, rho, shift, E


def scan_keys(Y, mu, op, order):
    """The MFMA scan restated: srcC = fl32(|y - mu|^2), then one fp32 rounding
    per exact product y_k * (-2 op_k), in the given k order."""
    S = np.sum((Y.astype(np.float64) - mu.astype(np.float64)) ** 2, axis=1).astype(np.float32)
    acc = S.copy()
    B = (-2.0 * op).astype(np.float32)
    for k in order:
        acc = (acc.astype(np.float64) + Y[:, k].astype(np.float64) * np.float64(B[k])).astype(np.float32)
    return acc, S


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("kind", ["clustered", "isotropic", "offset"])
def test_scan_key_bound_holds(dt, kind):
    rng = np.random.default_rng(3 if kind == "clustered" else 4)
    n, d = 3000, 96
    if kind == "clustered":
        base = rng.standard_normal(d)
        base /= np.linalg.norm(base)
        Y = base + 0.05 * rng.standard_normal((n, d)) / np.sqrt(d)
        Y /= np.linalg.norm(Y, axis=1, keepdims=True)
        Xq = base + 0.05 * rng.standard_normal((16, d)) / np.sqrt(d)
    elif kind == "isotropic":
        Y = rng.standard_normal((n, d))
        Xq = rng.standard_normal((16, d))
    else:  # large common offset, small spread: the worst cancellation
        Y = 30.0 + 0.01 * rng.standard_normal((n, d))
        Xq = 30.0 + 0.01 * rng.standard_normal((16, d))
    Y = rn16(Y.astype(np.float32), dt)                      # the stored rows
    Xq = Xq.astype(np.float32)                                # fp32 queries, inexact in 16 bits
    mu = Y[:: max(1, n // 512)].astype(np.float64).mean(axis=0).astype(np.float32)
    M = float(np.sqrt(np.max(np.sum(Y.astype(np.float64) ** 2, axis=1))))
    worst = 0.0
    for order in (np.arange(d), np.arange(d)[::-1]):
        for x in Xq:
            op, rho, shift, E = prep(x, mu, M, 0.0, d, dt)  # op only (Smax comes from the keys)
            a, S = scan_keys(Y, mu, op, order)
            Smax = float(S.max())
            op, rho, shift, E = prep(x, mu, M, Smax, d, dt)
            D = np.sum((x.astype(np.float64) - Y.astype(np.float64)) ** 2, axis=1)
            err = np.abs(a.astype(np.float64) + shift - D)
            bound = 2.0 * rho * np.sqrt(D) + E
            assert (err <= bound).all(), (kind, float((err - bound).max()))
            worst = max(worst, float((err / bound).max()))
    print(f"\n[bound-model] {dt} {kind}: max |err| / bound = {worst:.3f}")


def certified(kth, tb, shift, E, rho):
    """fx_kernels.hip `certified` restated."""
    T = tb + shift - E
    if rho > 0:
        t = max(T, 0.0)
        sd = t / (np.sqrt(rho * rho + t) + rho)
        dmin = sd * sd * (1 - 1e-12)
    else:
        dmin = T
    return kth + abs(kth) * 2.384185791015625e-7 < dmin


@pytest.mark.parametrize("seed", range(30))
def test_certification_with_rho_is_sound(seed):
    """Keys that use the whole bound adversarially: a(y) = D - shift + e(y),
    |e| <= 2 rho sqrt(D) + E.  The refine keeps the KP smallest keys, re-ranks
    them exactly, and certifies against tb = the KP-th key; a certified top-k
    must equal the exact one."""
    rng = np.random.default_rng(seed)
    KP, k = 32, int(rng.integers(1, 11))
    n = int(rng.integers(100, 4000))
    D = np.abs(rng.standard_normal(n)) * rng.choice([1e-3, 1.0, 400.0]) + rng.choice([0.0, 0.01, 5.0])
    D[rng.integers(0, n, n // 20)] = D[rng.integers(0, n, n // 20)]    # exact ties
    rho = float(rng.choice([0.0, 1e-5, 1e-3, 0.05])) * np.sqrt(np.median(D))
    E = float(rng.choice([1e-9, 1e-6, 1e-3])) * np.median(D)
    shift = float(rng.standard_normal()) * 10
    e = (rng.uniform(-1, 1, n)) * (2 * rho * np.sqrt(D) + E)
    a = D - shift + e
    order = np.lexsort((np.arange(n), a))
    top = order[:KP]
    tb = a[order[KP - 1]] if n > KP else np.inf
    ranked = sorted((D[i], i) for i in top)
    got = [i for _, i in ranked[:k]]
    want = [i for _, i in sorted((D[i], i) for i in range(n))[:k]]
    if n <= KP or certified(ranked[k - 1][0], tb, shift, E, rho):
        assert got == want
