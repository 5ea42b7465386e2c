"""Seeded test inputs shared by tests/ and tests/golden/make_golden.py."""
import numpy as np


def gaussian_small():
    """fp32 gaussian corpus (4096 x 384) and queries (64 x 384); the answers are
    committed in tests/golden/synth_small.npz."""
    rng = np.random.default_rng(20241220)
    xb = rng.standard_normal((4096, 384)).astype(np.float32)
    xq = rng.standard_normal((64, 384)).astype(np.float32)
    return xb, xq
