"""k_scan_v5 with and without the convoy start on the clustered certification case
(tests/test_scan_v5.py::test_v5_clustered_certifies) against the oracle."""
import sys
import numpy as np
sys.path.insert(0, ".")
import amd_fx  # noqa: F401
from oracle import cpu as C
from rag_faiss_embedding_amd import faiss as fx
from tests.test_scan_v5 import _data

for dtype, d in (("bfloat16", 768), ("float16", 384)):
    n, nq = 200_000, 1024
    xb, xq = _data(n, d, nq, 9, kind="clustered")
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    ref = ix.reconstruct_n(0, n).astype(np.float64)
    Dr, Ir = C.knn_exact(xq, ix.reconstruct_n(0, n), 10)
    for conv in (0, 1, 0, 1, 1):
        ix.set_option("scan_v5", 2)
        ix.set_option("convoy", conv)
        D, I = ix.search(xq, 10)
        bad = np.nonzero((I != Ir).any(axis=1))[0]
        print(dtype, "convoy", conv, "queries with id mismatches", len(bad), "fallbacks", ix.last_fallbacks(),
              "plan", ix.last_scan_plan(), flush=True)
        for q in bad[:4]:
            x = xq[q].astype(np.float64)
            ex_got = ((ref[I[q]] - x) ** 2).sum(1)
            ex_ref = ((ref[Ir[q]] - x) ** 2).sum(1)
            print("  q", q, "got", I[q].tolist(), "\n   ref", Ir[q].tolist(), "\n   exact got", ex_got.tolist(),
                  "\n   exact ref", ex_ref.tolist(), "\n   D", D[q].tolist(), flush=True)
