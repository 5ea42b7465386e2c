#!/usr/bin/env python3
"""Regenerate the committed golden fixtures in tests/golden/.

Run in the build container (it reads /root/reference, which does not exist on
the GPU box):   python tests/golden/make_golden.py

Outputs (all data, no reference source):
  shipped_index.bin          byte copy of the reference's data/faiss_index.bin
                             (IxF2, 23 x 384 fp32 CLS embeddings)
  shipped_ids.json           ids decoded from data/faiss_index.bin.mapping by
                             the non-unpickling parser, and the ids of
                             data/documents.json in file order
  shipped_knn.npz            oracle exact k-NN, all 23 rows as queries, k in
                             {1, 5, 10, 23, 30}
  wrapper_golden.json        behaviour of the reference faiss_store.py
                             (FAISSVectorStore) itself, executed with the
                             oracle standing in for the absent faiss-cpu
                             package and a no-op loguru stand-in.
  synth_small.npz            small seeded corpora + oracle answers used by the
                             GPU parity tests (fp32 gaussian / bf16-exact grid)

The reference's pickled mapping is never unpickled: the wrapper run uses a
mapping file written by this script from the safely parsed id list.
"""
from __future__ import annotations

import importlib
import json
import shutil
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(REPO))

from oracle import flat_l2 as F  # noqa: E402


def _standin_faiss() -> types.ModuleType:
    """Minimal ``faiss`` module backed by the oracle (only what faiss_store.py
    touches: IndexFlatL2(d), .add, .search, .ntotal, write_index, read_index)."""
    m = types.ModuleType("faiss")

    class IndexFlatL2:
        def __init__(self, d):
            self.d = int(d)
            self.xb = np.zeros((0, self.d), dtype=np.float32)

        @property
        def ntotal(self):
            return self.xb.shape[0]

        def add(self, x):
            x = np.ascontiguousarray(x, dtype=np.float32)
            assert x.shape[1] == self.d
            self.xb = np.vstack([self.xb, x])

        def search(self, x, k):
            x = np.ascontiguousarray(x, dtype=np.float32)
            assert x.shape[1] == self.d
            return F.knn_exact(x, self.xb, k)

    def write_index(index, path):
        Path(path).write_bytes(F.write_ixf2_bytes(index.xb))

    def read_index(path):
        xb = F.read_ixf2_bytes(Path(path).read_bytes())
        ix = IndexFlatL2(xb.shape[1])
        ix.xb = xb
        return ix

    m.IndexFlatL2 = IndexFlatL2
    m.write_index = write_index
    m.read_index = read_index
    return m


def _standin_loguru() -> types.ModuleType:
    m = types.ModuleType("loguru")

    class _L:
        def __getattr__(self, name):
            return lambda *a, **k: None

    m.logger = _L()
    return m


def _jsonable(x):
    if isinstance(x, np.ndarray):
        return [_jsonable(v) for v in x.tolist()]
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    return x


def shipped_fixtures() -> tuple:
    idx = (REF / "data" / "faiss_index.bin").read_bytes()
    (HERE / "shipped_index.bin").write_bytes(idx)
    mapping_ids = F.parse_id_mapping((REF / "data" / "faiss_index.bin.mapping").read_bytes())
    docs = json.loads((REF / "data" / "documents.json").read_text())
    (HERE / "shipped_ids.json").write_text(json.dumps({
        "mapping_ids": mapping_ids,
        "documents_json_ids": [d["id"] for d in docs],
        "source": "reference data/faiss_index.bin.mapping (parsed without unpickling) "
                  "and data/documents.json (rag_datastore_manager.py:189)",
    }, indent=1))
    xb = F.read_ixf2_bytes(idx)
    out = {}
    for k in (1, 5, 10, 23, 30):
        D, I = F.knn_exact(xb, xb, k)
        out[f"D_k{k}"] = D
        out[f"I_k{k}"] = I
    np.savez_compressed(HERE / "shipped_knn.npz", xb=xb, **out)
    return xb, mapping_ids


def wrapper_golden(xb: np.ndarray, mapping_ids) -> dict:
    """Run the reference FAISSVectorStore (faiss_store.py:10-128)."""
    sys.modules["faiss"] = _standin_faiss()
    sys.modules["loguru"] = _standin_loguru()
    tmp = Path(tempfile.mkdtemp(prefix="fx_golden_"))
    try:
        data = tmp / "data"
        data.mkdir()
        shutil.copy(HERE / "shipped_index.bin", data / "faiss_index.bin")
        import pickle  # writing our own file only
        with open(data / "faiss_index.bin.mapping", "wb") as f:
            pickle.dump(list(mapping_ids), f, protocol=4)
        sys.path.insert(0, str(REF))
        import os
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            fs = importlib.import_module("faiss_store")
            G: dict = {}
            store = fs.FAISSVectorStore()  # loads data/faiss_index.bin (:30-31)
            G["load"] = {"ntotal": store.index.ntotal, "doc_ids": list(store.doc_ids),
                         "dimension": store.dimension, "index_path": store.index_path}
            # singleton: new ctor args are ignored (:14-22)
            again = fs.FAISSVectorStore(dimension=7, index_path="other.bin")
            G["singleton"] = {"same_object": again is store, "dimension": again.dimension,
                              "index_path": again.index_path}
            G["search_k5"] = []
            for i in range(xb.shape[0]):
                D, ids = store.search(xb[i], 5)
                G["search_k5"].append({"D": _jsonable(D), "ids": _jsonable(ids)})
            D, ids = store.search(list(map(float, xb[3])), 30)  # list input, k > ntotal
            G["search_list_k30"] = {"D": _jsonable(D), "ids": _jsonable(ids)}
            D, ids = store.search(xb[0][:100], 5)  # wrong d -> swallowed (:79-81)
            G["search_wrong_d"] = {"D": _jsonable(D), "ids": _jsonable(ids), "D_dtype": str(np.asarray(D).dtype)}
            D, ids = store.search(xb[0], 1)
            G["search_k1"] = {"D": _jsonable(D), "ids": _jsonable(ids), "D_dtype": str(np.asarray(D).dtype)}
            # save -> bytes identical to the shipped file; mapping written by pickle p4
            store.save_index(str(tmp / "out" / "ix.bin"))
            G["save_roundtrip_bytes_equal"] = (tmp / "out" / "ix.bin").read_bytes() == (HERE / "shipped_index.bin").read_bytes()
            G["save_mapping_hex"] = (tmp / "out" / "ix.bin.mapping").read_bytes().hex()
            # reset + add (1-D vector reshaped :41-42; ids extended before add :45-46)
            store.reset()
            G["reset"] = {"ntotal": store.index.ntotal, "doc_ids": list(store.doc_ids)}
            store.add_vectors(xb[5], [105])
            store.add_vectors([list(map(float, r)) for r in xb[6:9]], [106, 107, 108])
            store.add_vectors(xb[9:12], [109, 110, 111])
            G["after_add"] = {"ntotal": store.index.ntotal, "doc_ids": list(store.doc_ids)}
            D, ids = store.search(xb[7], 3)
            G["after_add_search"] = {"D": _jsonable(D), "ids": _jsonable(ids)}
            # load without mapping -> sequential ids (:113-116)
            shutil.copy(tmp / "out" / "ix.bin", tmp / "nomap.bin")
            store.load_index(str(tmp / "nomap.bin"))
            G["load_nomapping"] = {"ntotal": store.index.ntotal, "doc_ids": list(store.doc_ids)}
            # load of a missing file re-raises (:120-122)
            try:
                store.load_index(str(tmp / "missing.bin"))
                G["load_missing_raises"] = False
            except Exception as e:  # noqa: BLE001
                G["load_missing_raises"] = type(e).__name__
            return G
        finally:
            os.chdir(cwd)
            sys.path.remove(str(REF))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def synth_small() -> None:
    from tests._data import gaussian_small
    out = {}
    xb, xq = gaussian_small()
    # fp32 gaussian (real-valued, rounding-sensitive)
    D, I = F.knn_exact(xq, xb, 10)
    out.update(g_D=D, g_I=I)  # inputs: regenerate from the seed (tests/_data.py)
    # bf16/fp16-exact grid corpus (the bench generator), d = 768
    xb2 = F.synth(11, 0, 3000, 768)
    xq2 = F.synth(12, 0, 32, 768)
    D2, I2 = F.knn_exact(xq2, xb2, 10)
    out.update(s_D=D2, s_I=I2)
    np.savez_compressed(HERE / "synth_small.npz", **out)


def main() -> None:
    xb, mapping_ids = shipped_fixtures()
    G = wrapper_golden(xb, mapping_ids)
    (HERE / "wrapper_golden.json").write_text(json.dumps(G, indent=1))
    synth_small()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
