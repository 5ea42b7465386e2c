"""``VectorizationPipeline`` on PyTorch-ROCm (reference: vectorization.py:10-47,
twin rag_datastore_manager.py:99-132).

Same constructor and ``generate_embeddings(texts, batch_size=32)`` contract:
tokenise (pad to the batch's longest, truncate at 512), BERT forward, CLS-row
pooling ``last_hidden_state[:, 0]`` with NO normalisation, float32
``np.ndarray[n, hidden]``; an empty input gives ``np.array([])``.

MI355X changes:
* ``generate_embeddings_device`` returns the embeddings as one device tensor
  (no per-batch ``.cpu().numpy()`` sync at vectorization.py:44) so they can be
  handed straight to ``IndexFlatL2.add`` / ``FAISSVectorStore.add_vectors``;
* batches are length-bucketed (sorted by token count).  The default
  ``precision="fp32"`` keeps the reference arithmetic (vectorization.py:41-44
  runs the fp32 forward); ``precision="bf16"`` (bf16 autocast) is opt-in.

Checkpoint loading follows the reference: ``from_pretrained`` failing raises
(vectorization.py:12-13 let the exception propagate).  The checkpoint
``sentence-transformers/all-MiniLM-L6-v2`` cannot be downloaded in this
environment, so benches and tests opt in to a stand-in with
``allow_random_init=True`` (or ``FX_ALLOW_RANDOM_ENCODER=1``): the same
architecture (BertModel: 6 layers, hidden 384, 12 heads, FFN 1536, vocab
30522) with seeded random weights and a deterministic hashing tokenizer, so
throughput and the device hand-off are faithful while embedding VALUES are not
the checkpoint's ("parity unpinned").  A WARNING is logged whenever
the stand-in is active.
"""
from __future__ import annotations

import hashlib
import logging
import os
import re
from typing import Dict, List, Optional

import numpy as np
import torch

logger = logging.getLogger("rag_faiss_embedding_amd.vectorization")

MINILM_CONFIG = dict(vocab_size=30522, hidden_size=384, num_hidden_layers=6, num_attention_heads=12,
                     intermediate_size=1536, max_position_embeddings=512, type_vocab_size=2,
                     hidden_act="gelu", layer_norm_eps=1e-12)


class HashingTokenizer:
    """Deterministic stand-in for the WordPiece tokenizer (vocab unavailable
    offline): lower-case word pieces hashed into the BERT vocab range, [CLS]
    / [SEP] / [PAD] ids as in bert-base-uncased, HF-style batch output."""

    cls_id, sep_id, pad_id = 101, 102, 0

    def __init__(self, vocab_size: int = 30522):
        self.vocab_size = vocab_size

    def _ids(self, text: str, max_length: int) -> List[int]:
        words = re.findall(r"[a-z0-9]+|[^\sa-z0-9]", text.lower())
        ids = [self.cls_id]
        for w in words[: max_length - 2]:
            h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=4).digest(), "little")
            ids.append(1000 + h % (self.vocab_size - 1000))
        ids.append(self.sep_id)
        return ids

    def __call__(self, texts, padding=True, truncation=True, max_length=512, return_tensors="pt"):
        seqs = [self._ids(t, max_length if truncation else 10 ** 9) for t in texts]
        L = max(len(s) for s in seqs)
        ids = torch.full((len(seqs), L), self.pad_id, dtype=torch.long)
        mask = torch.zeros((len(seqs), L), dtype=torch.long)
        for i, s in enumerate(seqs):
            ids[i, :len(s)] = torch.tensor(s)
            mask[i, :len(s)] = 1
        return {"input_ids": ids, "token_type_ids": torch.zeros_like(ids), "attention_mask": mask}


def random_init_allowed(flag: Optional[bool] = None) -> bool:
    if flag is not None:
        return bool(flag)
    return os.environ.get("FX_ALLOW_RANDOM_ENCODER", "0") not in ("", "0")


def build_encoder(model_name: str, seed: int = 0, allow_random_init: Optional[bool] = None):
    """(tokenizer, model, pretrained?) -- the checkpoint from the local HF
    cache.  If it cannot be loaded the error propagates, as in the reference,
    unless the seeded random-weight stand-in was asked for explicitly."""
    from transformers import AutoModel, AutoTokenizer, BertConfig, BertModel
    try:
        tok = AutoTokenizer.from_pretrained(model_name, local_files_only=True)
        model = AutoModel.from_pretrained(model_name, local_files_only=True)
        return tok, model, True
    except Exception as e:  # noqa: BLE001
        if not random_init_allowed(allow_random_init):
            raise
        logger.warning("checkpoint %s unavailable (%s: %s); using the seeded random-weight MiniLM stand-in "
                       "(embedding values are NOT the checkpoint's)", model_name, type(e).__name__, e)
        torch.manual_seed(seed)
        cfg = BertConfig(**MINILM_CONFIG)
        try:
            model = BertModel(cfg, add_pooling_layer=False, attn_implementation="sdpa")
        except TypeError:
            model = BertModel(cfg, add_pooling_layer=False)
        return HashingTokenizer(cfg.vocab_size), model, False


class VectorizationPipeline:
    def __init__(self, model_name: str = "sentence-transformers/all-MiniLM-L6-v2", *, device: Optional[str] = None,
                 precision: str = "fp32", seed: int = 0, allow_random_init: Optional[bool] = None):
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        self.tokenizer, self.model, self.pretrained = build_encoder(model_name, seed, allow_random_init)
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.model.to(self.device).eval()
        self.precision = precision if self.device.type == "cuda" else "fp32"
        logger.info("Initialized vectorization pipeline (%s, pretrained=%s)", self.device, self.pretrained)

    @torch.no_grad()
    def _forward_cls(self, encoded: Dict[str, torch.Tensor]) -> torch.Tensor:
        encoded = {k: v.to(self.device, non_blocking=True) for k, v in encoded.items()}
        if self.precision == "bf16":
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
                out = self.model(**encoded)
        else:
            out = self.model(**encoded)
        return out.last_hidden_state[:, 0].float()  # CLS pooling, no normalisation

    @torch.no_grad()
    def generate_embeddings_device(self, texts: List[str], batch_size: int = 32) -> torch.Tensor:
        """[n, hidden] float32 embeddings resident on ``self.device``, in input
        order (batches are length-bucketed internally)."""
        n = len(texts)
        hidden = self.model.config.hidden_size
        out = torch.empty((n, hidden), dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        lens = [len(t) for t in texts]
        order = sorted(range(n), key=lambda i: lens[i])
        for i in range(0, n, batch_size):
            idx = order[i:i + batch_size]
            enc = self.tokenizer([texts[j] for j in idx], padding=True, truncation=True, max_length=512,
                                 return_tensors="pt")
            out[torch.tensor(idx, device=self.device)] = self._forward_cls(enc)
        return out

    @torch.no_grad()
    def encode_token_batches(self, input_ids: torch.Tensor, attention_mask: torch.Tensor,
                             batch_size: int = 256) -> torch.Tensor:
        """Pre-tokenised path (bench config c): [n, L] ids -> [n, hidden] on device."""
        n = input_ids.shape[0]
        out = torch.empty((n, self.model.config.hidden_size), dtype=torch.float32, device=self.device)
        for i in range(0, n, batch_size):
            enc = {"input_ids": input_ids[i:i + batch_size], "attention_mask": attention_mask[i:i + batch_size],
                   "token_type_ids": torch.zeros_like(input_ids[i:i + batch_size])}
            out[i:i + batch_size] = self._forward_cls(enc)
        return out

    @torch.no_grad()
    def encode_lengths(self, input_ids: torch.Tensor, lengths, batch_size: int = 256) -> torch.Tensor:
        """Ragged pre-tokenised path (bench config c): row i of ``input_ids``
        [n, Lmax] holds ``lengths[i]`` valid tokens.  Rows are sorted by
        length and every batch is cut to its own longest row (the reference
        pads per batch, vectorization.py:29-35, but in input order).  Returns
        [n, hidden] float32 on ``self.device`` in input order.  ``lengths``
        is read on the host, so the loop never waits on the device."""
        n = input_ids.shape[0]
        out = torch.empty((n, self.model.config.hidden_size), dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        lens = torch.as_tensor(lengths, dtype=torch.long).cpu()
        assert lens.shape[0] == n and int(lens.min()) >= 1 and int(lens.max()) <= input_ids.shape[1], "bad lengths"
        order = torch.argsort(lens, stable=True)
        lens_sorted = lens[order]
        ids = input_ids.to(self.device, non_blocking=True)
        lens_dev = lens.to(self.device, non_blocking=True)
        pos = torch.arange(input_ids.shape[1], device=self.device)
        for i in range(0, n, batch_size):
            idx = order[i:i + batch_size].to(self.device, non_blocking=True)
            L = int(lens_sorted[min(i + batch_size, n) - 1])
            b_ids = ids[idx, :L]
            mask = (pos[None, :L] < lens_dev[idx][:, None]).to(torch.long)
            out[idx] = self._forward_cls({"input_ids": b_ids, "attention_mask": mask,
                                          "token_type_ids": torch.zeros_like(b_ids)})
        return out

    def generate_embeddings(self, texts: List[str], batch_size: int = 32) -> np.ndarray:
        """vectorization.py:18-47: np.ndarray[n, hidden] float32 (np.array([])
        for no texts)."""
        logger.info("Generating embeddings for %d texts", len(texts))
        if len(texts) == 0:
            return np.array([])
        return self.generate_embeddings_device(texts, batch_size).cpu().numpy()
