"""Encoder surface (vectorization.py:10-47 contract).  Parity against the real
all-MiniLM-L6-v2 checkpoint is unpinned offline (no weights): the tests opt in
to the seeded random-weight stand-in, and the GPU path is checked against the
same seeded model run in fp32 on the CPU.

Tolerances (stated here, asserted below):
* fp32 on the GPU (the default, the reference's arithmetic) vs fp32 on the
  CPU: max |diff| <= 1e-4 * max |ref| -- only summation order differs;
* bf16 autocast (opt-in): max |diff| <= 2e-2 * max |ref|; retrieval-level
  check on 30 query embeddings over a 300-text corpus: the nearest neighbour
  equals the fp32 encoder's for every query and >= 90 % of the top-5 ids do."""
import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def cpu_pipe():
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    return VectorizationPipeline(device="cpu", precision="fp32", seed=0, allow_random_init=True)


def _corpus(n=300, seed=0):
    rng = np.random.default_rng(seed)
    words = ["gpu", "index", "vector", "search", "faiss", "embedding", "query", "document", "retrieval", "model",
             "flat", "matrix", "kernel", "memory", "corpus", "token", "batch", "shard", "merge", "distance"]
    return [" ".join(rng.choice(words, size=int(rng.integers(5, 30)))) for _ in range(n)]


TEXTS = ["FAISS flat index on MI355X", "retrieval augmented generation", "a", "x " * 300,
         "Vector databases store embeddings for similarity search."]


def test_missing_checkpoint_raises(monkeypatch):
    """The reference's from_pretrained failure propagates (vectorization.py:12-13);
    the random-weight stand-in is never chosen silently."""
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    monkeypatch.delenv("FX_ALLOW_RANDOM_ENCODER", raising=False)
    with pytest.raises(Exception):
        VectorizationPipeline("no-such-org/no-such-model", device="cpu")
    with pytest.raises(ValueError):
        VectorizationPipeline(device="cpu", precision="fp16", allow_random_init=True)


def test_default_precision_is_fp32():
    import inspect
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    assert inspect.signature(VectorizationPipeline).parameters["precision"].default == "fp32"


def test_contract_shapes(cpu_pipe):
    e = cpu_pipe.generate_embeddings(TEXTS, batch_size=2)
    assert e.shape == (len(TEXTS), 384) and e.dtype == np.float32
    assert np.array(cpu_pipe.generate_embeddings([])).shape == (0,)
    # order preserved despite length bucketing; batch size does not change values
    e1 = cpu_pipe.generate_embeddings(TEXTS, batch_size=1)
    np.testing.assert_allclose(e, e1, rtol=1e-4, atol=1e-4)


def test_cls_pooling_no_normalisation(cpu_pipe):
    enc = cpu_pipe.tokenizer(TEXTS[:2], padding=True, truncation=True, max_length=512, return_tensors="pt")
    with torch.no_grad():
        ref = cpu_pipe.model(**enc).last_hidden_state[:, 0].numpy()
    np.testing.assert_allclose(cpu_pipe.generate_embeddings(TEXTS[:2]), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_gpu_encoder_matches_cpu_and_hands_off(cpu_pipe):
    import amd_fx  # noqa: F401
    from rag_faiss_embedding_amd import faiss
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    g = VectorizationPipeline(device="cuda", seed=0, allow_random_init=True)  # default: fp32
    assert g.precision == "fp32"
    ref = cpu_pipe.generate_embeddings(TEXTS)
    dev = g.generate_embeddings_device(TEXTS)
    assert dev.is_cuda
    err = np.abs(dev.cpu().numpy() - ref).max() / np.abs(ref).max()
    print(f"fp32 GPU vs CPU: max rel diff {err:.3e}")
    assert err <= 1e-4, err
    # device-resident hand-off into the index: no host round trip
    ix = faiss.IndexFlatL2(384)
    ix.add(dev)
    D, I = ix.search(dev, 2)
    assert (I[:, 0].cpu().numpy() == np.arange(len(TEXTS))).all()


@pytest.mark.gpu
def test_bf16_encoder_tolerance_and_retrieval(cpu_pipe):
    """bf16 autocast is opt-in: stated value tolerance, and the same nearest
    neighbours as the fp32 encoder on a 300-text corpus."""
    import amd_fx  # noqa: F401
    from oracle import cpu as C
    from rag_faiss_embedding_amd.vectorization import VectorizationPipeline
    texts = _corpus()
    g32 = VectorizationPipeline(device="cuda", seed=0, allow_random_init=True)
    gb = VectorizationPipeline(device="cuda", precision="bf16", seed=0, allow_random_init=True)
    e32 = g32.generate_embeddings(texts)
    eb = gb.generate_embeddings(texts)
    err = np.abs(eb - e32).max() / np.abs(e32).max()
    print(f"bf16 vs fp32: max rel diff {err:.3e}")
    assert err <= 2e-2, err
    _, I32 = C.knn_exact(e32[:30], e32, 5)
    _, Ib = C.knn_exact(eb[:30], eb, 5)
    assert (I32[:, 0] == Ib[:, 0]).all()
    assert (I32 == Ib).mean() >= 0.9


def test_encode_lengths_matches_unpadded_rows(cpu_pipe):
    """Length-bucketed ragged batches give each row's own unpadded CLS vector,
    in input order (padding is masked out of attention)."""
    g = torch.Generator().manual_seed(7)
    lens = [5, 40, 12, 3, 33, 17, 9, 26]
    ids = torch.zeros((len(lens), 48), dtype=torch.long)
    for i, L in enumerate(lens):
        ids[i, :L] = torch.randint(1000, 30522, (L,), generator=g)
        ids[i, 0], ids[i, L - 1] = 101, 102
    got = cpu_pipe.encode_lengths(ids, lens, batch_size=3).numpy()
    for i, L in enumerate(lens):
        one = cpu_pipe.encode_token_batches(ids[i:i + 1, :L], torch.ones((1, L), dtype=torch.long)).numpy()
        np.testing.assert_allclose(got[i], one[0], rtol=1e-4, atol=1e-4)
    assert cpu_pipe.encode_lengths(ids[:0], [], batch_size=3).shape == (0, 384)
