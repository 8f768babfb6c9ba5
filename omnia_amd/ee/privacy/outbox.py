"""Consent-revocation outbox + notifier (``ee/pkg/privacy/outbox_store.go``,
``consent_notifier.go``, ``ee/cmd/privacy-api/outbox_replay.go``).

A revocation and its outbox row are written in ONE transaction
(:meth:`Outbox.revoke_with_outbox`), so a crash between "consent removed" and
"memory-api told" cannot lose the notification.  The request path notifies at
once and marks the row delivered on success; :class:`OutboxReplayWorker`
re-sends whatever is still undelivered (rows younger than the retention
window), prunes delivered rows past it, and exports the count of rows stuck
longer than ``stuck_after_s`` (``omnia_privacy_outbox_stuck``).

:class:`MemoryAPINotifier` POSTs ``{"userId", "category"}`` to every configured
memory-api (one per service group) at ``/api/v1/memories/consent-events``
(``?workspace=`` when set); delivered only when every target answered 2xx.
"""
from __future__ import annotations

import asyncio
import logging
import time
import uuid

from ...observability import metrics as M

log = logging.getLogger("omnia.privacy.outbox")

SCHEMA = """
CREATE TABLE IF NOT EXISTS consent_revocation_outbox (
  id TEXT PRIMARY KEY, user_id TEXT NOT NULL, category TEXT NOT NULL,
  created_at REAL NOT NULL, delivered_at REAL, attempts INTEGER NOT NULL DEFAULT 0,
  last_error TEXT);
CREATE INDEX IF NOT EXISTS ix_outbox_pending ON consent_revocation_outbox(delivered_at, created_at);
"""


class Outbox:
    """Over a ``PrivacyStore`` (its SQLite connection and lock)."""

    def __init__(self, store):
        self.store = store
        with store.lock:
            store.db.executescript(SCHEMA)

    def revoke_with_outbox(self, user: str, category: str) -> str | None:
        """Record the revocation and its outbox row atomically; None when the
        category was not granted (nothing to notify) -- as
        ``RemoveConsentGrantWithOutbox``."""
        db = self.store.db
        with self.store.lock:
            db.execute("BEGIN IMMEDIATE")
            try:
                cur = db.execute("SELECT granted FROM consent WHERE user_id = ? AND category = ?",
                                 (user, category)).fetchone()
                from . import CATEGORIES

                was_granted = cur[0] == 1 if cur else not CATEGORIES.get(category, True)
                db.execute("INSERT OR REPLACE INTO consent VALUES (?,?,0,?)",
                           (user, category, time.time()))
                oid = None
                if was_granted:
                    oid = uuid.uuid4().hex
                    db.execute("INSERT INTO consent_revocation_outbox (id, user_id, category, "
                               "created_at) VALUES (?,?,?,?)", (oid, user, category, time.time()))
                db.execute("COMMIT")
            except BaseException:
                db.execute("ROLLBACK")
                raise
        return oid

    def mark_delivered(self, oid: str):
        self.store.q("UPDATE consent_revocation_outbox SET delivered_at = ? WHERE id = ?",
                     (time.time(), oid))

    def mark_failed(self, oid: str, err: str):
        self.store.q("UPDATE consent_revocation_outbox SET attempts = attempts + 1, "
                     "last_error = ? WHERE id = ?", (err[:500], oid))

    def undelivered(self, max_age_s: float, limit: int = 100) -> list[tuple[str, str, str]]:
        return self.store.q("SELECT id, user_id, category FROM consent_revocation_outbox WHERE "
                            "delivered_at IS NULL AND created_at > ? ORDER BY created_at LIMIT ?",
                            (time.time() - max_age_s, limit))

    def prune_delivered(self, ttl_s: float) -> int:
        with self.store.lock:
            return self.store.db.execute(
                "DELETE FROM consent_revocation_outbox WHERE delivered_at IS NOT NULL AND "
                "delivered_at < ?", (time.time() - ttl_s,)).rowcount

    def count_stuck(self, stuck_after_s: float) -> int:
        return self.store.q("SELECT count(*) FROM consent_revocation_outbox WHERE delivered_at "
                            "IS NULL AND created_at < ?", (time.time() - stuck_after_s,))[0][0]


class MemoryAPINotifier:
    def __init__(self, memory_urls: list[str], workspace: str = "", token: str = "",
                 timeout_s: float = 10.0):
        self.urls = [u.rstrip("/") for u in memory_urls if u]
        self.workspace = workspace
        self.token = token
        self.timeout_s = timeout_s

    async def notify_revocation(self, user: str, category: str) -> tuple[bool, str]:
        """(delivered to every target, first error)."""
        if not self.urls:
            return True, ""
        import aiohttp

        headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        params = {"workspace": self.workspace} if self.workspace else {}
        err = ""
        async with aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
            for base in self.urls:
                try:
                    async with s.post(f"{base}/api/v1/memories/consent-events", params=params,
                                      json={"userId": user, "category": category},
                                      headers=headers) as r:
                        if not 200 <= r.status < 300:
                            err = err or f"{base}: HTTP {r.status}"
                except Exception as e:  # noqa: BLE001
                    err = err or f"{base}: {e}"
        return not err, err


async def deliver(outbox: Outbox, notifier, oid: str, user: str, category: str) -> bool:
    ok, err = await notifier.notify_revocation(user, category)
    if ok:
        outbox.mark_delivered(oid)
    else:
        outbox.mark_failed(oid, err)
        log.warning("consent revocation notify failed (will replay): %s", err)
    return ok


class OutboxReplayWorker:
    def __init__(self, outbox: Outbox, notifier, interval_s: float = 30.0,
                 retention_s: float = 7 * 86400, stuck_after_s: float = 3600.0, batch: int = 100):
        self.outbox, self.notifier = outbox, notifier
        self.interval_s, self.retention_s = interval_s, retention_s
        self.stuck_after_s, self.batch = stuck_after_s, batch

    async def run_once(self) -> dict:
        sent = failed = 0
        for oid, user, cat in self.outbox.undelivered(self.retention_s, self.batch):
            if await deliver(self.outbox, self.notifier, oid, user, cat):
                sent += 1
            else:
                failed += 1
        pruned = self.outbox.prune_delivered(self.retention_s)
        stuck = self.outbox.count_stuck(self.stuck_after_s)
        M.PRIVACY_OUTBOX_STUCK.set(stuck)
        return {"sent": sent, "failed": failed, "pruned": pruned, "stuck": stuck}

    async def run(self):
        while True:
            try:
                await self.run_once()
            except Exception as e:  # noqa: BLE001
                log.warning("outbox replay pass failed: %s", e)
            await asyncio.sleep(self.interval_s)
