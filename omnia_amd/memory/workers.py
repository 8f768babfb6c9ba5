"""Background workers of memory-api.

* :class:`ReembedWorker` -- backfills missing / stale-model embeddings in
  batches (``internal/memory/reembed_worker.go:81-148``); batching is what makes
  the in-node embedder efficient (one packed varlen forward per batch).
* :class:`RetentionWorker` -- TTL expiry + purge of forgotten rows
  (``internal/memory/retention.go``).
* :class:`CompactionWorker` -- LLM-summarises old observations of a scope into
  one ``summary`` memory that supersedes them
  (``internal/memory/compaction_worker.go:93-218``); the summariser is any
  async callable ``(texts) -> str`` (the local engine provider in-node).
"""
from __future__ import annotations

import asyncio
import logging

from ..observability import metrics as M
from .model import SCOPE_WORKSPACE, Memory

log = logging.getLogger("omnia.memory.workers")


class ReembedWorker:
    def __init__(self, svc, interval: float = 5.0, batch: int = 64):
        self.svc, self.interval, self.batch = svc, interval, batch

    async def run_once(self) -> int:
        total = 0
        while True:
            n = await self.svc.reembed(self.batch)
            total += n
            if n < self.batch:
                return total

    async def run(self):
        M.MEMORY_WORKER_RUNNING.labels("reembed").set(1)  # doctor liveness gauge
        try:
            while True:
                try:
                    await self.run_once()
                except Exception as e:  # noqa: BLE001
                    log.warning("reembed pass failed: %s", e)
                await asyncio.sleep(self.interval)
        finally:
            M.MEMORY_WORKER_RUNNING.labels("reembed").set(0)


class RetentionWorker:
    """``policy``: a MemoryPolicy spec (the operator's ``memory-policy-<name>``
    ConfigMap); its tier rules run first (:mod:`.retention`), then expiry and the
    purge of rows forgotten longer than the soft-delete grace."""

    def __init__(self, svc, interval: float = 300.0, forgotten_grace_s: float = 30 * 86400,
                 policy: dict | None = None):
        self.svc, self.interval, self.grace = svc, interval, forgotten_grace_s
        self.policy = policy
        self.last_stats: dict = {}
        if policy:
            from .retention import grace_seconds

            self.grace = grace_seconds(policy, forgotten_grace_s / 86400.0)

    def run_once(self) -> int:
        if self.policy:
            from .retention import apply_memory_policy

            self.last_stats = apply_memory_policy(self.svc.store, self.policy)
        obs = self.svc.store.expire() + self.svc.store.purge_forgotten(self.grace)
        self.svc._drop_vectors(obs)
        return len(obs)

    async def run(self):
        M.MEMORY_WORKER_RUNNING.labels("retention").set(1)  # doctor liveness gauge
        try:
            while True:
                try:
                    self.run_once()
                except Exception as e:  # noqa: BLE001
                    log.warning("retention pass failed: %s", e)
                await asyncio.sleep(self.interval)
        finally:
            M.MEMORY_WORKER_RUNNING.labels("retention").set(0)


def default_summarizer_prompt(texts: list[str]) -> str:
    joined = "\n".join(f"- {t}" for t in texts)
    return ("Consolidate these memories about the same subject into a short list of durable "
            "facts. Drop duplicates and superseded details.\n" + joined)


async def noop_summarizer(texts: list[str]) -> str:
    """Deterministic default summary (``compaction_worker.go`` NoopSummarizer):
    the originals are still superseded, so the retrieval surface shrinks even
    without an LLM summarizer."""
    if not texts:
        raise ValueError("noop summarizer called with no entries")
    return f"Summary of {len(texts)} observations. First: {texts[0][:80]}"


class CompactionWorker:
    """Temporal summarisation of old memories.  ``workspaces`` is a fixed list or
    a callable discovering them (the store's workspaces with live memories, as
    ``ListWorkspaceIDs``)."""

    def __init__(self, svc, summarize=None, workspaces=None, older_than_s: float = 30 * 86400,
                 min_count: int = 10, interval: float = 3600.0):
        self.svc, self.summarize = svc, summarize or noop_summarizer
        self.workspaces = workspaces if workspaces is not None else \
            svc.store.list_workspace_ids
        self.older_than_s, self.min_count, self.interval = older_than_s, min_count, interval
        self.passes = 0

    async def run_once(self) -> int:
        done = 0
        self.passes += 1
        wss = self.workspaces() if callable(self.workspaces) else self.workspaces
        for ws in wss:
            for cand in self.svc.store.compaction_candidates(ws, self.older_than_s,
                                                             self.min_count):
                texts = [e["content"] for e in cand["entries"]]
                try:
                    summary = await self.summarize(texts)
                except Exception as e:  # noqa: BLE001
                    log.warning("summarize failed for %s: %s", cand["scope"], e)
                    continue
                if not summary:
                    continue
                mem = Memory(type="summary", content=summary, confidence=0.8,
                             scope=dict(cand["scope"]),
                             metadata={"source_type": "system_generated",
                                       "compacted_from": len(texts)})
                await self.svc.supersede([e["id"] for e in cand["entries"]], mem)
                done += 1
        return done

    async def run(self):
        M.MEMORY_WORKER_RUNNING.labels("compaction").set(1)  # doctor liveness gauge
        try:
            while True:
                try:
                    await self.run_once()
                except Exception as e:  # noqa: BLE001
                    log.warning("compaction pass failed: %s", e)
                await asyncio.sleep(self.interval)
        finally:
            M.MEMORY_WORKER_RUNNING.labels("compaction").set(0)


class TombstoneWorker:
    """Prunes superseded / expired observation chains (``tombstone_worker.go``):
    every ``interval`` seconds, per workspace (a fixed list or the store's
    discoverer), ``store.tombstone_gc(min_age, min_inactive, keep_recent)``."""

    def __init__(self, svc, interval: float = 3600.0, workspaces=None,
                 min_age_s: float = 30 * 86400, min_inactive: int = 20, keep_recent: int = 5):
        if keep_recent >= min_inactive:
            raise ValueError("keep_recent must be less than min_inactive")
        self.svc, self.interval = svc, interval
        self.workspaces = workspaces if workspaces is not None else \
            svc.store.list_workspace_ids
        self.min_age_s, self.min_inactive, self.keep_recent = min_age_s, min_inactive, keep_recent
        self.deleted = 0

    def run_once(self) -> int:
        n = 0
        wss = self.workspaces() if callable(self.workspaces) else self.workspaces
        for ws in wss:
            try:
                n += self.svc.store.tombstone_gc(ws, self.min_age_s, self.min_inactive,
                                                 self.keep_recent)
            except Exception as e:  # noqa: BLE001 - one workspace never stops the pass
                log.warning("tombstone gc failed for %s: %s", ws, e)
        self.deleted += n
        return n

    async def run(self):
        M.MEMORY_WORKER_RUNNING.labels("tombstone_gc").set(1)
        try:
            while True:
                await asyncio.sleep(self.interval)
                try:
                    self.run_once()
                except Exception as e:  # noqa: BLE001
                    log.warning("tombstone pass failed: %s", e)
        finally:
            M.MEMORY_WORKER_RUNNING.labels("tombstone_gc").set(0)


__all__ = ["ReembedWorker", "RetentionWorker", "CompactionWorker", "TombstoneWorker",
           "SCOPE_WORKSPACE"]
