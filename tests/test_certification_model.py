"""Model test of the search's exactness argument, on the CPU.

The GPU scan computes approximate keys (|approx - exact| <= eps), keeps per
corpus split a top-KP list under a threshold shared by all splits (gtau), and
the refine merges the splits' lists, re-ranks the KP best exactly and
certifies the top-k.  This test restates that pipeline in numpy, with the
scan's tile order, list capacity, compaction and shared-threshold updates
(fx_scan.hip epilogue / compact_wave; fx_kernels.hip k_refine), feeds it
adversarial keys (ties, duplicates, noise up to the bound, splits visited in
random interleaved order) and checks: every certified query's top-k equals
the exact top-k under the (D, id) order.
"""
import numpy as np
import pytest

KP, CAP = 32, 64


def _scan_split_lists(keys, ids, splits, tile, rng):
    """Per-split candidate lists after a scan in random split interleaving,
    with the shared threshold (min over splits' published KP-th keys)."""
    n = keys.shape[0]
    bounds = np.linspace(0, n, splits + 1).astype(int)
    cursors = list(bounds[:-1])
    lists = [[] for _ in range(splits)]
    tau = [np.inf] * splits
    gtau = np.inf
    active = list(range(splits))
    while active:
        s = active[rng.integers(len(active))]
        lo = cursors[s]
        hi = min(lo + tile, bounds[s + 1])
        tn = min(tau[s], gtau)
        for r in range(lo, hi):
            if keys[r] <= tn:
                lists[s].append((keys[r], ids[r]))
                if len(lists[s]) >= CAP:                     # compaction: keep KP best, publish tau
                    lists[s].sort()
                    lists[s] = lists[s][:KP]
                    tau[s] = lists[s][-1][0]
                    gtau = min(gtau, tau[s])
                    tn = min(tau[s], gtau)
        cursors[s] = hi
        if hi >= bounds[s + 1]:
            active.remove(s)
    return [sorted(lst)[:KP] for lst in lists]


def _refine(lists, exact, k, eps):
    """k_refine: KP best approx over all lists -> exact re-rank -> certify."""
    cand = sorted(c for lst in lists for c in lst)
    nvalid = len(cand)
    top = cand[:KP]
    td = top[-1][0] if len(top) == KP else np.inf
    ranked = sorted((exact[i], i) for _, i in top)
    res = ranked[:k]
    kth = res[-1][0]
    certified = nvalid < KP or (kth + abs(kth) * 2.4e-7 < td - eps)
    return [i for _, i in res], certified


@pytest.mark.parametrize("seed", range(40))
def test_certified_results_are_exact(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(200, 3000))
    k = int(rng.integers(1, 11))
    exact = rng.standard_normal(n) * rng.choice([0.05, 1.0, 30.0])
    # duplicates and exact ties
    dup = rng.integers(0, n, size=n // 10)
    exact[dup] = exact[rng.integers(0, n, size=dup.size)]
    eps = float(rng.choice([1e-6, 1e-3, 0.05]))
    approx = exact + rng.uniform(-eps, eps, n)              # the scan's bounded error
    ids = np.arange(n)
    splits = int(rng.integers(1, 9))
    tile = int(rng.choice([8, 32, 128]))
    lists = _scan_split_lists(approx, ids, splits, tile, rng)
    got, cert = _refine(lists, exact, k, eps)
    want = [i for _, i in sorted((exact[i], i) for i in range(n))[:k]]
    if cert:
        assert got == want
    # and it certifies whenever the exact k-th and KP-th keys are > 2 eps apart
    # (plus the 2-ulp slack): the bound is not vacuous
    s = np.sort(exact)
    if s[KP - 1] - s[k - 1] > 2 * eps + 3e-7 * abs(s[k - 1]) + 1e-12:
        assert cert
