"""CPU check of the split-fp32 scan's error constant (fx_kernels.hip
k_prep_queries, F32S).

The scan keeps hi*hi + hi*lo + lo*hi of every product, with hi = rn_bf16(v)
and lo = rn_bf16(v - hi) for both operands (bf16 products are exact in fp32).
The certification margin charges the dropped part with
    delta_s = 4.73e-5  per unit of sum_k |x_k||y_k|.
Here the dropped part is measured in float64 over operands with a wide
dynamic range, and v - hi is checked to be exact in fp32.
"""
import numpy as np
import torch

DELTA_S = 4.73e-5


def _split(v32: np.ndarray):
    t = torch.from_numpy(v32)
    hi = t.to(torch.bfloat16).to(torch.float32)
    rest = t - hi                                    # fp32 subtraction, as on the device
    lo = rest.to(torch.bfloat16).to(torch.float32)
    return hi.numpy().astype(np.float64), lo.numpy().astype(np.float64), rest.numpy().astype(np.float64)


def test_split_residual_exact_and_bounded():
    rng = np.random.default_rng(5)
    for scale in (1e-30, 1e-3, 1.0, 7.5, 1e4, 1e30):
        v = (rng.standard_normal(200_000) * scale).astype(np.float32)
        hi, lo, rest = _split(v)
        v64 = v.astype(np.float64)
        np.testing.assert_array_equal(rest, v64 - hi)           # v - hi exact in fp32
        assert np.all(np.abs(v64 - hi) <= 2.0 ** -8 * np.abs(v64))
        assert np.all(np.abs(v64 - hi - lo) <= 2.0 ** -16 * np.abs(v64) + 1e-45)


def test_split_dot_error_within_delta_s():
    rng = np.random.default_rng(6)
    worst = 0.0
    for d in (96, 384, 768):
        for scale in (1.0, 1e-2, 3e3):
            x = (rng.standard_normal((64, d)) * scale).astype(np.float32)
            # L2 operand: -2 x (exact power-of-two scaling), as k_prep_queries does
            xs = (-2.0 * x).astype(np.float32)
            y = (rng.standard_normal((257, d)) * rng.uniform(0.1, 10, (257, 1))).astype(np.float32)
            xh, xl, _ = _split(xs)
            yh, yl, _ = _split(y)
            approx = xh @ yh.T + xh @ yl.T + xl @ yh.T          # float64: the products, exactly
            exact = xs.astype(np.float64) @ y.astype(np.float64).T
            mag = np.abs(xs.astype(np.float64)) @ np.abs(y.astype(np.float64)).T
            ratio = np.abs(approx - exact) / mag
            worst = max(worst, float(ratio.max()))
    assert worst <= DELTA_S, worst
    # the constant is not loose by orders of magnitude either (sanity)
    assert worst > DELTA_S / 1000


def test_split_key_within_certification_margin():
    """The whole scan key of the split path, emulated with sequential fp32
    accumulation (a worst case for the MFMA chain: every product rounded into
    a running fp32 sum), against k_prep_queries' margin for F32S:
    eps = (2 gamma_{3K+1} + u)(M^2 + 2|x|M) + 2 delta_s |x| M,  times 1.0625."""
    rng = np.random.default_rng(8)
    u = 2.0 ** -24
    for d in (128, 384):
        y = rng.standard_normal((64, d)).astype(np.float32) * np.float32(3.0)
        x = rng.standard_normal((8, d)).astype(np.float32)
        xs = (-2.0 * x).astype(np.float32)
        xh, xl, _ = _split(xs)
        yh, yl, _ = _split(y)
        ny = np.add.accumulate((y.astype(np.float32) ** 2), axis=1, dtype=np.float32)[:, -1]   # fp32 norms
        M = float(np.sqrt(ny.astype(np.float64).max()))
        K = 3 * d + 1
        g = K * u / (1 - K * u)
        for qi in range(x.shape[0]):
            terms = np.concatenate([xh[qi] * yh, xl[qi] * yh, xh[qi] * yl], axis=1).astype(np.float32)  # exact products
            acc = ny.copy()
            for c in range(terms.shape[1]):                       # sequential fp32 chain, srcC = |y|^2
                acc = (acc + terms[:, c]).astype(np.float32)
            exact = (y.astype(np.float64) ** 2).sum(1) - 2 * y.astype(np.float64) @ x[qi].astype(np.float64)
            xn = float(np.linalg.norm(x[qi].astype(np.float64)))
            eps = ((2 * g + u) * (M * M + 2 * xn * M) + 2 * DELTA_S * xn * M) * 1.0625
            assert np.abs(acc.astype(np.float64) - exact).max() <= eps
