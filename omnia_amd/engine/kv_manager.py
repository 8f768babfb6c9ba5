"""Paged KV block manager with per-session prefix retention and tiering.

The reference drops the conversation at the end of every Converse stream and
re-sends the whole history to the remote provider on the next turn
(``internal/runtime/server.go:719-725``, ``conversation.go:260-276``).  Here the
engine keeps each session's KV pages resident in HBM after its turn, keyed by
``session_id``; the next turn re-uses the longest common token prefix and
prefills only the delta (SURVEY §0.7 / §5.4 design).

Tiers (the KV analogue of Omnia's hot/warm/cold session "compaction",
``internal/compaction/engine.go:85-129``):
  * hot   -- pages in HBM (this pool).
  * warm  -- pages copied to pinned host DRAM on eviction (``SwapSpace``), copied
             back on the next turn instead of re-prefilling.
  * cold  -- nothing: the transcript in the runtime's context store is the source
             of truth and the next turn re-prefills ("cache empty != definitive").
Block 0 is a reserved null page used by padded rows of captured decode graphs.

Cross-session prefix sharing (``share_prefix``): every full page of a computed
prompt is published under a chain hash of its tokens and all the tokens before
it.  A new sequence whose session holds no pages maps the longest published run
of its prompt's leading pages instead of prefilling them: the agents of one
deployment all start from the same PromptPack system prompt and tool schemas.
Shared pages are reference-counted (the table holds one reference).  A sequence
never writes into one: only full pages are shared, and a hit always leaves the
page that holds the prompt's last token private.  Once only the table holds a
page, an allocation that needs it reclaims it, before any idle session.

Isolation (a shared page is attention input for every later mapper, so a forged
match is KV-cache poisoning, and a hit is observable through cached_tokens and
TTFT):
  * the chain hash is a keyed BLAKE2b (128-bit digest, per-process random key),
    not Python's ``hash``: a client cannot craft a page whose key collides with
    a published one; each shared page also keeps its tokens and parent digest,
    compared on every lookup;
  * ``salt`` (``SamplingParams.cache_salt``) seeds the chain: pages published
    under one salt are invisible under another (per tenant / workspace scope);
  * ``limit`` (``SamplingParams.share_limit``) bounds what a prompt publishes:
    the runtime passes the length of the rendered system prompt + tool schemas
    (``runtime/chat.py shared_prefix_len``), so no user's conversation pages are
    ever published, only the deployment's PromptPack prefix.
"""
from __future__ import annotations

import hashlib
import os
import time
from array import array
from collections import OrderedDict
from dataclasses import dataclass, field


class OutOfBlocks(Exception):
    pass


@dataclass
class SessionKV:
    session_id: str
    blocks: list[int]
    tokens: list[int]  # token ids whose KV is stored (len <= len(blocks)*BS)
    last_used: float = field(default_factory=time.monotonic)
    in_use: bool = False
    swapped: object = None  # host-tier handle when evicted to DRAM


def common_prefix(a: list[int], b: list[int]) -> int:
    n = min(len(a), len(b))
    i = 0
    # chunked compare is much faster than a python loop for long prompts
    step = 256
    while i + step <= n and a[i:i + step] == b[i:i + step]:
        i += step
    while i < n and a[i] == b[i]:
        i += 1
    return i


class BlockManager:
    CHAIN_SEED = b"\x00" * 16  # chain digest of the empty prefix (no salt)

    def __init__(self, num_blocks: int, block_size: int, swap=None, share_prefix: bool = False,
                 max_shared: int | None = None):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks")
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.free: list[int] = list(range(num_blocks - 1, 0, -1))  # block 0 reserved
        self.sessions: "OrderedDict[str, SessionKV]" = OrderedDict()
        self.idle_blocks = 0  # private pages held by parked (evictable) sessions
        self.swap = swap
        self.share_prefix = share_prefix
        self.max_shared = max_shared if max_shared is not None else max(1, num_blocks // 4)
        self._key = os.urandom(32)  # BLAKE2b key of the chain digests
        self.table: dict[bytes, int] = {}  # chain digest -> shared page
        self.key_of: dict[int, bytes] = {}  # shared page -> chain digest
        self.page_of: dict[int, tuple] = {}  # shared page -> (parent digest, its tokens)
        self.ref: dict[int, int] = {}  # shared page -> holders, the table included
        self.evictable: "OrderedDict[int, None]" = OrderedDict()  # shared pages only the table holds
        self.stats = {"prefix_hit_tokens": 0, "prefix_miss_tokens": 0, "evictions": 0,
                      "swap_out": 0, "swap_in": 0, "shared_hit_tokens": 0,
                      "shared_pages": 0, "shared_evictions": 0}

    # -------------------------------------------------------------- pool
    @property
    def num_free(self) -> int:
        return len(self.free)

    @property
    def num_available(self) -> int:
        """Free pages plus pages an allocation may reclaim: idle sessions' private
        pages and shared pages only the table holds.  (A lower bound: evicting a
        session can also leave its shared pages to the table alone.)"""
        return len(self.free) + self.idle_blocks + len(self.evictable)

    def _n_private(self, blocks: list[int]) -> int:
        if not self.ref:
            return len(blocks)
        return sum(1 for b in blocks if b not in self.ref)

    def utilization(self) -> float:
        return 1.0 - len(self.free) / (self.num_blocks - 1)

    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    def _evict_one(self) -> bool:
        # first the shared pages nobody maps: a prompt page that matters to many
        # sessions (the system prompt) is held by a live sequence or a parked
        # session, so what sits here is mostly a finished one-off prompt's page,
        # worth less than a parked session's whole conversation
        if self.evictable:
            b, _ = self.evictable.popitem(last=False)
            del self.table[self.key_of.pop(b)]
            self.page_of.pop(b, None)
            del self.ref[b]
            self.free.append(b)
            self.stats["shared_evictions"] += 1
            return True
        for sid, s in self.sessions.items():  # LRU order
            if not s.in_use:
                self.sessions.pop(sid)
                self.idle_blocks -= self._n_private(s.blocks)
                if self.swap is not None and s.tokens and self.swap.can_hold(len(s.blocks)):
                    s.swapped = self.swap.swap_out(s.blocks)
                    self.swap.park(sid, s)
                    self.stats["swap_out"] += 1
                self.release(s.blocks)
                self.stats["evictions"] += 1
                return True
        return False

    def allocate(self, n: int) -> list[int]:
        while len(self.free) < n:
            if not self._evict_one():
                raise OutOfBlocks(f"need {n} blocks, {len(self.free)} free")
        out = [self.free.pop() for _ in range(n)]
        return out

    def can_allocate(self, n: int) -> bool:
        return self.num_available >= n

    def release(self, blocks: list[int]) -> None:
        if not self.ref:
            self.free.extend(blocks)
            return
        for b in blocks:
            r = self.ref.get(b)
            if r is None:
                self.free.append(b)
            elif r == 1:  # the last holder of a page the table let go of
                del self.ref[b]
                self.free.append(b)
            else:
                self.ref[b] = r - 1
                if r == 2 and b in self.key_of:
                    self.evictable[b] = None  # only the table holds it now

    def _incref(self, b: int) -> None:
        r = self.ref[b]
        if r == 1:
            self.evictable.pop(b, None)
        self.ref[b] = r + 1

    def reset_shared(self) -> None:
        """Forget every published page (engine-fault recovery: a page may be
        half-written).  Pages still mapped stay counted until their holders
        release them."""
        for b in list(self.key_of):
            if self.ref[b] == 1:
                del self.ref[b]
                self.free.append(b)
            else:
                self.ref[b] -= 1
        self.table.clear()
        self.key_of.clear()
        self.page_of.clear()
        self.evictable.clear()

    # -------------------------------------------------------------- sharing
    def seed(self, salt: str | None) -> bytes:
        """Chain digest of the empty prefix in the scope ``salt``."""
        if not salt:
            return self.CHAIN_SEED
        return hashlib.blake2b(salt.encode(), key=self._key, digest_size=16,
                               person=b"omnia-salt").digest()

    def _chain(self, h: bytes, tokens: list[int], i: int) -> bytes:
        bs = self.block_size
        page = array("q", tokens[i * bs:(i + 1) * bs]).tobytes()
        return hashlib.blake2b(h + page, key=self._key, digest_size=16).digest()

    def _acquire_shared(self, prompt: list[int], salt: str | None = None
                        ) -> tuple[list[int], int]:
        """Map the longest published run of ``prompt``'s leading full pages,
        stopping before the page that holds its last token."""
        blocks: list[int] = []
        h = self.seed(salt)
        bs = self.block_size
        for i in range((len(prompt) - 1) // bs):
            parent = h
            h = self._chain(h, prompt, i)
            b = self.table.get(h)
            if b is None or self.page_of.get(b) != (parent, tuple(prompt[i * bs:(i + 1) * bs])):
                break
            self._incref(b)
            blocks.append(b)
        n = len(blocks) * bs
        self.stats["shared_hit_tokens"] += n
        return blocks, n

    def publish(self, tokens: list[int], blocks: list[int], n_computed: int, done: int = 0,
                h: bytes | None = None, salt: str | None = None,
                limit: int | None = None) -> tuple[int, bytes]:
        """Publish the full pages among the first ``n_computed`` tokens of
        ``tokens`` (a prompt whose KV is in ``blocks``), from page ``done`` on
        (``h``: chain digest up to it), none past ``limit`` tokens.  Returns the
        new ``(done, h)``."""
        h = self.seed(salt) if h is None else h
        if not self.share_prefix:
            return done, h
        n = min(n_computed, len(tokens))
        if limit is not None and limit >= 0:
            n = min(n, limit)
        full = n // self.block_size
        bs = self.block_size
        for i in range(done, full):
            parent = h
            h = self._chain(h, tokens, i)
            b = blocks[i]
            if h in self.table or b in self.ref:
                continue  # published already (this page, or an equal one)
            if len(self.table) >= self.max_shared:
                if not self.evictable:
                    continue
                old, _ = self.evictable.popitem(last=False)
                del self.table[self.key_of.pop(old)]
                self.page_of.pop(old, None)
                del self.ref[old]
                self.free.append(old)
                self.stats["shared_evictions"] += 1
            self.table[h] = b
            self.key_of[b] = h
            self.page_of[b] = (parent, tuple(tokens[i * bs:(i + 1) * bs]))
            self.ref[b] = 2  # the table and the sequence that computed it
            self.stats["shared_pages"] += 1
        return max(done, full), h

    # -------------------------------------------------------------- sessions
    def acquire_prefix(self, session_id: str | None, prompt: list[int],
                       share: bool = True, salt: str | None = None) -> tuple[list[int], int]:
        """Take ownership of the session's cached pages matching `prompt`.

        Returns (blocks, n_cached_tokens).  At least one prompt token is always
        left uncached so the step produces logits."""
        s = self.sessions.pop(session_id, None) if session_id else None
        if s is not None:
            self.idle_blocks -= self._n_private(s.blocks)
        elif self.swap is not None:
            s = self.swap.unpark(session_id)
            if s is not None:
                try:
                    blocks = self.allocate(len(s.blocks))
                except OutOfBlocks:
                    self.swap.drop(s.swapped)
                    s = None
                else:
                    self.swap.swap_in(s.swapped, blocks)
                    s.blocks = blocks
                    s.swapped = None
                    self.stats["swap_in"] += 1
        if s is None:
            blocks, n = (self._acquire_shared(prompt, salt) if (self.share_prefix and share)
                         else ([], 0))
            self.stats["prefix_hit_tokens"] += n
            self.stats["prefix_miss_tokens"] += len(prompt) - n
            return blocks, n
        n = common_prefix(s.tokens, prompt)
        n = min(n, len(prompt) - 1)
        keep = self.blocks_needed(n)
        if keep and n % self.block_size and s.blocks[keep - 1] in self.ref:
            keep -= 1  # the next write would land in a shared page: re-prefill it
            n = keep * self.block_size
        self.release(s.blocks[keep:])
        self.stats["prefix_hit_tokens"] += n
        self.stats["prefix_miss_tokens"] += len(prompt) - n
        return s.blocks[:keep], n

    def retain(self, session_id: str | None, blocks: list[int], tokens: list[int]) -> None:
        """Park a finished turn's pages under its session (or free them)."""
        if not session_id:
            self.release(blocks)
            return
        old = self.sessions.pop(session_id, None)
        if old is not None:
            self.idle_blocks -= self._n_private(old.blocks)
            self.release(old.blocks)
        need = self.blocks_needed(len(tokens))
        self.release(blocks[need:])
        self.sessions[session_id] = SessionKV(session_id, blocks[:need], list(tokens))
        self.idle_blocks += self._n_private(blocks[:need])

    def drop_session(self, session_id: str) -> bool:
        s = self.sessions.pop(session_id, None)
        if s is not None:
            self.idle_blocks -= self._n_private(s.blocks)
            self.release(s.blocks)
        if self.swap is not None:
            p = self.swap.unpark(session_id)
            if p is not None:
                self.swap.drop(p.swapped)
        return s is not None

    def has_session(self, session_id: str) -> bool:
        return session_id in self.sessions or (self.swap is not None
                                               and self.swap.has(session_id))

    def session_tokens(self, session_id: str) -> int:
        s = self.sessions.get(session_id)
        return len(s.tokens) if s else 0
