"""Small batches (nq <= 16) through k_scan_v4 / k_scan_v5 against the oracle.  Round 6 used it to
find the removed small-batch instance's wrong neighbours (option small_scan 1 vs 0)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import amd_fx  # noqa: F401  (registers rag_faiss_embedding_amd)
from oracle import cpu as C
from rag_faiss_embedding_amd import faiss as fx

cases = [("bfloat16", 768, 70_001, 1, 5), ("bfloat16", 768, 70_001, 4, 5), ("float16", 384, 70_001, 1, 5),
         ("float32", 384, 70_001, 1, 5), ("bfloat16", 768, 20_000, 1, 3), ("float16", 768, 70_001, 16, 5)]
for dtype, d, n, nq, seed in cases:
    rng = np.random.default_rng(seed)
    xb = rng.standard_normal((n, d)).astype(np.float32)
    xq = rng.standard_normal((nq, d)).astype(np.float32)
    ix = fx.IndexFlatL2(d, dtype=dtype)
    ix.add(xb)
    ref = ix.reconstruct_n(0, n)
    Dr, Ir = C.knn_exact(xq, ref, 10)
    for ss in (0, 2):
        ix.set_option("scan_v5", ss)
        D, I = ix.search(xq, 10)
        bad = int((I != Ir).sum())
        print(dtype, d, n, nq, "scan_v5", ss, "id mismatches", bad, "fallbacks", ix.last_fallbacks(), flush=True)
        if bad:
            for q in range(nq):
                miss = sorted(set(Ir[q]) - set(I[q]))
                if miss:
                    print("  q", q, "missing", miss, "true D", [float(Dr[q][list(Ir[q]).index(m)]) for m in miss],
                          "got D", D[q].tolist(), flush=True)
