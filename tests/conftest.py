import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import amd_fx  # noqa: E402,F401  (registers rag_faiss_embedding_amd)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "stream_ordered: device searches must not synchronise inside the test "
                                       "(their candidate-integrity count is read at teardown)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def diag_fx():
    """Indexes bound to the diagnostic build libfx_index_diag.so (the same
    kernels; test hooks force_fallback / scan_dbg in its option table)."""
    from rag_faiss_embedding_amd import _lib
    if _lib.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    from rag_faiss_embedding_amd import diag
    return diag


@pytest.fixture(autouse=True)
def _candidate_lists_intact(request, monkeypatch):
    """In every -m gpu test, every search through the Python API must report
    0 candidate entries dropped for an out-of-range row id
    (fx_index_last_dropped_candidates): a corrupted scan list fails the test
    even when the top-k it left happened to match the oracle."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from rag_faiss_embedding_amd import faiss
    orig = faiss._FlatIndex.search
    dropped, pending = [], {}

    defer = request.node.get_closest_marker("stream_ordered") is not None

    def search(self, x, *a, **kw):
        out = orig(self, x, *a, **kw)
        if defer and faiss._is_device_tensor(x):
            # a test of stream ordering: reading the count would synchronise
            # inside it; read at teardown, for the index's last search
            pending[id(self)] = self
        else:  # every other search: its own count (a device search syncs here)
            dropped.append(self.last_dropped_candidates())
        return out

    monkeypatch.setattr(faiss._FlatIndex, "search", search)
    yield
    dropped.extend(ix.last_dropped_candidates() for ix in pending.values())
    assert not any(dropped), f"searches dropped corrupted candidate ids: {dropped}"
