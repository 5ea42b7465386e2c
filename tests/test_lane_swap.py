"""gfx950 cross-lane helpers of the scan's list pushes (fx_scan_common.h
lane_xor16 / lane_xor32 / quad_prefix, built on v_permlane16_swap and
v_permlane32_swap): checked on the device against their definition, through a
small probe kernel compiled with the same header (hipcc, gfx950)."""
import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "rag-faiss-embedding_amd" / "csrc"
PROBE = ROOT / "tests" / "native" / "lane_probe.hip"
LIB = ROOT / "tests" / "native" / "_build" / "liblane_probe.so"


def build_probe():
    LIB.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    f"-I{CSRC}", "-o", str(LIB), str(PROBE)], check=True)


def test_probe_builds():
    """CPU: the probe compiles for gfx950 (the driver's GPU run loads it)."""
    build_probe()
    assert LIB.exists()


@pytest.mark.gpu
def test_lane_swaps_on_device():
    import torch  # noqa: F401  (one HIP runtime per process)
    if not LIB.exists():
        pytest.fail(f"{LIB} missing: build it on the CPU first (tests/test_lane_swap.py::test_probe_builds)")
    lib = ctypes.CDLL(str(LIB))
    out = np.zeros((4, 64), dtype=np.int32)
    rc = lib.lane_probe(out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    x = (np.arange(64) * 7 + 3) % 11
    lane = np.arange(64)
    assert (out[0] == x[lane ^ 16]).all(), out[0]
    assert (out[1] == x[lane ^ 32]).all(), out[1]
    # quad prefix over lanes l & 15 + 16 j, j = 0..3
    ex = np.array([x[[(l & 15) + 16 * j for j in range(l >> 4)]].sum() for l in lane])
    tot = np.array([x[[(l & 15) + 16 * j for j in range(4)]].sum() for l in lane])
    assert (out[2] == ex).all(), out[2]
    assert (out[3] == tot).all(), out[3]
