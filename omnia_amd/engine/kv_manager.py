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
"""
from __future__ import annotations

import time
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
    def __init__(self, num_blocks: int, block_size: int, swap=None):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks")
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.free: list[int] = list(range(num_blocks - 1, 0, -1))  # block 0 reserved
        self.sessions: "OrderedDict[str, SessionKV]" = OrderedDict()
        self.idle_blocks = 0  # pages held by parked (evictable) sessions
        self.swap = swap
        self.stats = {"prefix_hit_tokens": 0, "prefix_miss_tokens": 0, "evictions": 0,
                      "swap_out": 0, "swap_in": 0}

    # -------------------------------------------------------------- pool
    @property
    def num_free(self) -> int:
        return len(self.free)

    @property
    def num_available(self) -> int:
        """Free pages plus pages an allocation may reclaim from idle sessions."""
        return len(self.free) + self.idle_blocks

    def utilization(self) -> float:
        return 1.0 - len(self.free) / (self.num_blocks - 1)

    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    def _evict_one(self) -> bool:
        for sid, s in self.sessions.items():  # LRU order
            if not s.in_use:
                self.sessions.pop(sid)
                self.idle_blocks -= len(s.blocks)
                if self.swap is not None and s.tokens and self.swap.can_hold(len(s.blocks)):
                    s.swapped = self.swap.swap_out(s.blocks)
                    self.swap.park(sid, s)
                    self.stats["swap_out"] += 1
                self.free.extend(s.blocks)
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
        self.free.extend(blocks)

    # -------------------------------------------------------------- sessions
    def acquire_prefix(self, session_id: str | None, prompt: list[int]) -> tuple[list[int], int]:
        """Take ownership of the session's cached pages matching `prompt`.

        Returns (blocks, n_cached_tokens).  At least one prompt token is always
        left uncached so the step produces logits."""
        if not session_id:
            self.stats["prefix_miss_tokens"] += len(prompt)
            return [], 0
        s = self.sessions.pop(session_id, None)
        if s is not None:
            self.idle_blocks -= len(s.blocks)
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
            self.stats["prefix_miss_tokens"] += len(prompt)
            return [], 0
        n = common_prefix(s.tokens, prompt)
        n = min(n, len(prompt) - 1)
        keep = self.blocks_needed(n)
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
            self.idle_blocks -= len(old.blocks)
            self.release(old.blocks)
        need = self.blocks_needed(len(tokens))
        self.release(blocks[need:])
        self.sessions[session_id] = SessionKV(session_id, blocks[:need], list(tokens))
        self.idle_blocks += len(blocks[:need])

    def drop_session(self, session_id: str) -> bool:
        s = self.sessions.pop(session_id, None)
        if s is not None:
            self.idle_blocks -= len(s.blocks)
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
