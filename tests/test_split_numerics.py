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
