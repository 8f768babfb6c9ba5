"""Embedding providers for the memory tier (``internal/memory/embedding.go:36-105``).

* :class:`LocalModelEmbedder` -- the MI355X path: a Llama-shaped encoder forward
  on the in-node engine kernels (paged prefill attention, fused norms, hipBLASLt
  GEMMs) followed by the K17 mean-pool + L2 kernel.  Sequences are packed into
  one variable-length batch (no padding), each given contiguous scratch KV pages.
* :class:`HashEmbedder` -- deterministic feature-hashing embedder (unigrams +
  bigrams, signed hashing); CPU fallback for tests and GPU-less data planes.
* :class:`HTTPEmbedder` -- OpenAI-compatible ``/v1/embeddings`` or Ollama
  ``/api/embed`` (the reference's Provider CRD embedding role,
  ``api/v1alpha1/provider_types.go:107-124``; dimensions capped at 4096).
"""
from __future__ import annotations

import asyncio
import hashlib
import math
import re
import threading

import numpy as np

MAX_DIMENSIONS = 4096


class Embedder:
    dim: int = 0
    model: str = ""

    async def embed(self, texts: list[str]) -> list[list[float]]:  # pragma: no cover
        raise NotImplementedError

    def embed_sync(self, texts: list[str]) -> list[list[float]]:
        return asyncio.run(self.embed(texts))


_WORD = re.compile(r"\w+", re.UNICODE)


def _stem(w: str) -> str:
    for suf in ("ingly", "edly", "ing", "ed", "es", "s", "ly"):
        if len(w) > len(suf) + 2 and w.endswith(suf):
            return w[: -len(suf)]
    return w


class HashEmbedder(Embedder):
    def __init__(self, dim: int = 384, model: str = "hash-v1"):
        self.dim = dim
        self.model = model

    def _vec(self, text: str) -> list[float]:
        words = [_stem(w.lower()) for w in _WORD.findall(text or "")]
        feats = words + [a + "_" + b for a, b in zip(words, words[1:])]
        v = np.zeros(self.dim, dtype=np.float32)
        for f in feats:
            h = hashlib.blake2b(f.encode(), digest_size=8).digest()
            idx = int.from_bytes(h[:4], "little") % self.dim
            v[idx] += 1.0 if h[4] & 1 else -1.0
        n = float(np.linalg.norm(v))
        return (v / n).tolist() if n > 0 else v.tolist()

    async def embed(self, texts):
        return [self._vec(t) for t in texts]


class LocalModelEmbedder(Embedder):
    """Encoder forward + K17 pooling on the GPU (CPU reference path otherwise)."""

    def __init__(self, model: str = "omnia-embed-1b", device: str | None = None,
                 max_tokens_per_batch: int = 16384, max_seq_len: int = 512, seed: int = 0,
                 weights: dict | None = None, tokenizer=None):
        import torch

        from ..models.config import resolve
        from ..models.llama import KVCache, LlamaModel

        self.cfg = resolve(model)
        self.model = self.cfg.name
        self.dim = self.cfg.hidden_size
        if self.dim > MAX_DIMENSIONS:
            raise ValueError("embedding dimensions capped at 4096")
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.net = LlamaModel(self.cfg, device=self.device, seed=seed, weights=weights)
        self.bs = 32
        self.max_tokens = max_tokens_per_batch
        self.max_seq = min(max_seq_len, max_tokens_per_batch)
        self.max_seqs = 256  # sequences per packed batch
        # every sequence wastes < 1 page; block 0 is never handed out
        nblocks = (max_tokens_per_batch + self.bs - 1) // self.bs + self.max_seqs + 1
        self.kv = KVCache.allocate(self.cfg, nblocks, self.bs, self.device)
        if tokenizer is None:
            from ..engine.tokenizer import SyntheticTokenizer

            tokenizer = SyntheticTokenizer(self.cfg.vocab_size, self.cfg.bos_token_id,
                                           self.cfg.eos_token_ids)
        self.tok = tokenizer
        self._lock = threading.Lock()  # one forward at a time on the scratch KV

    def _batches(self, toks: list[list[int]]):
        cur, n = [], 0
        for i, t in enumerate(toks):
            if cur and (n + len(t) > self.max_tokens or len(cur) >= self.max_seqs):
                yield cur
                cur, n = [], 0
            cur.append(i)
            n += len(t)
        if cur:
            yield cur

    def _forward(self, seqs: list[list[int]]):
        import torch

        from .. import ops
        from ..models.llama import ForwardBatch

        bs = self.bs
        ids, pos, slots, qsl, lens, tables = [], [], [], [0], [], []
        nb = 1  # block 0 stays scratch-free
        for t in seqs:
            need = (len(t) + bs - 1) // bs
            blocks = list(range(nb, nb + need))
            nb += need
            ids.extend(t)
            pos.extend(range(len(t)))
            slots.extend(blocks[p // bs] * bs + p % bs for p in range(len(t)))
            qsl.append(qsl[-1] + len(t))
            lens.append(len(t))
            tables.append(blocks)
        maxb = max(len(b) for b in tables)
        bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
        for i, b in enumerate(tables):
            bt[i, :len(b)] = torch.tensor(b, dtype=torch.int32)
        tseq, tq0 = ops.prefill_tiles(lens)
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        fb = ForwardBatch(
            input_ids=torch.tensor(ids, **i32), positions=torch.tensor(pos, **i32),
            slots=torch.tensor(slots, dtype=torch.int64, device=dev), block_tables=bt.to(dev),
            seq_lens=torch.tensor(lens, **i32), logits_indices=None, is_decode=False,
            q_start_loc=torch.tensor(qsl, **i32), tile_seq=torch.tensor(tseq, **i32),
            tile_q0=torch.tensor(tq0, **i32), num_seqs=len(seqs))
        h = self.net.hidden_states(fb, self.kv)
        return ops.mean_pool_l2(h, fb.q_start_loc)

    def embed_tokens(self, toks: list[list[int]]):
        import torch

        toks = [(t or [self.cfg.bos_token_id])[: self.max_seq] for t in toks]
        out = [None] * len(toks)
        with self._lock, torch.inference_mode():
            for idx in self._batches(toks):
                v = self._forward([toks[i] for i in idx]).float().cpu()
                for j, i in enumerate(idx):
                    out[i] = v[j]
        return torch.stack(out) if out else torch.empty(0, self.dim)

    async def embed(self, texts):
        toks = [[self.cfg.bos_token_id] + self.tok.encode(t or "") for t in texts]
        v = await asyncio.to_thread(self.embed_tokens, toks)
        return v.tolist()


class HTTPEmbedder(Embedder):
    def __init__(self, base_url: str, model: str, dim: int = 0, api_key: str = "",
                 flavor: str = "openai", timeout: float = 30.0):
        self.base = base_url.rstrip("/")
        self.model = model
        self.dim = dim
        self.key = api_key
        self.flavor = flavor
        self.timeout = timeout

    async def embed(self, texts):
        import aiohttp

        headers = {"Content-Type": "application/json"}
        if self.key:
            headers["Authorization"] = f"Bearer {self.key}"
        if self.flavor == "ollama":
            url, body = f"{self.base}/api/embed", {"model": self.model, "input": texts}
        else:
            url, body = f"{self.base}/v1/embeddings", {"model": self.model, "input": texts}
            if self.dim:
                body["dimensions"] = self.dim
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout)) as s:
            async with s.post(url, json=body, headers=headers) as r:
                if r.status >= 400:
                    raise RuntimeError(f"embedding provider HTTP {r.status}: {await r.text()}")
                data = await r.json()
        if self.flavor == "ollama":
            vecs = data.get("embeddings") or []
        else:
            vecs = [d["embedding"] for d in sorted(data.get("data", []),
                                                   key=lambda d: d.get("index", 0))]
        out = []
        for v in vecs:
            n = math.sqrt(sum(x * x for x in v)) or 1.0
            out.append([x / n for x in v])
        if out and not self.dim:
            self.dim = len(out[0])
        return out


def build_embedder(spec: dict | None) -> Embedder | None:
    """Provider-CRD-shaped spec -> embedder.  ``{"type": "local", "model": ...}``,
    ``{"type": "hash", "dimensions": 384}``, ``{"type": "openai"|"ollama",
    "baseURL": ..., "model": ..., "dimensions": N}``."""
    if not spec:
        return None
    t = (spec.get("type") or "hash").lower()
    dims = int(spec.get("dimensions") or 0)
    if dims > MAX_DIMENSIONS:
        raise ValueError("dimensions must be <= 4096")
    if t == "hash":
        return HashEmbedder(dims or 384)
    if t in ("local", "engine"):
        return LocalModelEmbedder(spec.get("model") or "omnia-embed-1b",
                                  device=spec.get("device"))
    if t in ("openai", "vllm", "ollama"):
        return HTTPEmbedder(spec.get("baseURL") or spec.get("base_url") or "",
                            spec.get("model") or "", dims, spec.get("apiKey", ""),
                            "ollama" if t == "ollama" else "openai")
    raise ValueError(f"unknown embedding provider type {t!r}")
