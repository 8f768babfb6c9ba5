"""Tokenizers for the in-node engine.

* :class:`SyntheticTokenizer` -- byte-level encoder for random-init models (no
  checkpoints or tokenizer files are fetchable offline).  ids 0..255 are raw
  bytes; the model's special ids are named; every other id decodes to a
  deterministic pseudo-word so streamed output is printable and stable.
* :class:`HFTokenizer` -- wraps a ``tokenizer.json`` via the ``tokenizers``
  package when the Provider points at one.

Both implement incremental detokenisation for streaming (``Detokenizer``):
UTF-8 fragments split across byte tokens are held back until complete.
"""
from __future__ import annotations

import os

_SYLL = ["ka", "lo", "mi", "ne", "ru", "ta", "vo", "shi", "el", "an", "or", "is", "um", "pe",
         "di", "ga"]


class SyntheticTokenizer:
    def __init__(self, vocab_size: int, bos_id: int, eos_ids, special: dict | None = None):
        self.vocab_size = vocab_size
        self.bos_id = bos_id
        self.eos_ids = tuple(eos_ids)
        # llama-3 style chat specials (mapped into the top of the vocab when it is large enough)
        names = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>",
                 "<|end_header_id|>", "<|eot_id|>", "<|python_tag|>"]
        self.special: dict[str, int] = dict(special or {})
        if not self.special:
            base = bos_id
            if vocab_size >= 128256 and base == 128000:
                ids = [128000, 128001, 128006, 128007, 128009, 128010]
            else:
                ids = [min(vocab_size - 1, base + i) for i in range(len(names))]
                ids[1] = self.eos_ids[0]
            self.special = dict(zip(names, ids))
        self.inv_special = {v: k for k, v in self.special.items()}

    @property
    def eos_token_ids(self):
        return self.eos_ids

    def encode(self, text: str, add_bos: bool = False, allow_special: bool = True) -> list[int]:
        ids: list[int] = [self.bos_id] if add_bos else []
        if allow_special and "<|" in text:
            i = 0
            while i < len(text):
                j = text.find("<|", i)
                if j < 0:
                    ids.extend(text[i:].encode("utf-8"))
                    break
                ids.extend(text[i:j].encode("utf-8"))
                k = text.find("|>", j)
                tok = text[j:k + 2] if k >= 0 else None
                if tok in self.special:
                    ids.append(self.special[tok])
                    i = k + 2
                else:
                    ids.extend(b"<|")
                    i = j + 2
            return ids
        ids.extend(text.encode("utf-8"))
        return ids

    def token_bytes(self, tid: int) -> bytes:
        if 0 <= tid < 256:
            return bytes([tid])
        if tid in self.inv_special:
            return b""
        # deterministic printable pseudo-word for random-init ids
        x = tid
        s = []
        for _ in range(2):
            s.append(_SYLL[x & 15])
            x >>= 4
        return (" " + "".join(s)).encode()

    def decode(self, ids, skip_special: bool = True) -> str:
        out = bytearray()
        for t in ids:
            if not skip_special and t in self.inv_special:
                out.extend(self.inv_special[t].encode())
            else:
                out.extend(self.token_bytes(int(t)))
        return out.decode("utf-8", errors="replace")


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.tk = Tokenizer.from_file(path)
        self.vocab_size = self.tk.get_vocab_size()
        vocab = self.tk.get_vocab()
        self.bos_id = vocab.get("<|begin_of_text|>", vocab.get("<s>", 0))
        eos = [vocab[t] for t in ("<|end_of_text|>", "<|eot_id|>", "</s>") if t in vocab]
        self.eos_ids = tuple(eos) or (0,)
        self.special = {t: i for t, i in vocab.items() if t.startswith("<|") and t.endswith("|>")}

    @property
    def eos_token_ids(self):
        return self.eos_ids

    def encode(self, text: str, add_bos: bool = False, allow_special: bool = True) -> list[int]:
        ids = self.tk.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] if add_bos else []) + ids

    def token_bytes(self, tid: int) -> bytes:
        return self.tk.decode([tid], skip_special_tokens=True).encode()

    def decode(self, ids, skip_special: bool = True) -> str:
        return self.tk.decode(list(ids), skip_special_tokens=skip_special)


def _token_bytes_cached(tok, tid: int) -> bytes:
    cache = tok.__dict__.setdefault("_tb_cache", {})
    b = cache.get(tid)
    if b is None:
        b = cache[tid] = tok.token_bytes(tid)
    return b


class Detokenizer:
    """Incremental UTF-8-safe streaming detokeniser for one sequence.

    Incomplete multi-byte sequences are held until they complete; bytes that
    can never become valid UTF-8 are emitted as U+FFFD at once (Python's
    incremental decoder, ``errors="replace"``), so a run of invalid byte tokens
    -- e.g. a random-init model repeating a lone lead byte -- still streams one
    character per token instead of stalling the stream until the end."""

    def __init__(self, tok):
        import codecs

        self.tok = tok
        self.dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
        self.held = False  # the decoder holds an incomplete sequence

    def push(self, tid: int) -> str:
        b = _token_bytes_cached(self.tok, tid)
        if not self.held:
            # fast path: a token that is complete UTF-8 on its own (the common case)
            try:
                return b.decode("utf-8")
            except UnicodeDecodeError:
                pass
        s = self.dec.decode(b)
        self.held = bool(self.dec.getstate()[0])
        return s

    def flush(self) -> str:
        s = self.dec.decode(b"", final=True)
        self.held = False
        return s


def make_tokenizer(cfg, path: str | None = None):
    path = path or os.environ.get("OMNIA_TOKENIZER")
    if path and os.path.exists(path):
        return HFTokenizer(path)
    return SyntheticTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_ids)
