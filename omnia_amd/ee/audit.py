"""Audit log: buffered logger, query API, retention, forwarder (SURVEY §2.2 E6;
reference ``ee/pkg/audit/{types,logger,handler,forwarder}.go``).

* :class:`AuditLogger` -- ``log_event`` never blocks the caller: entries go to
  a bounded in-memory buffer (full -> dropped + counted, like the reference's
  non-blocking channel send) and a writer thread flushes them in batches
  (``batch_size`` or ``flush_interval_s``, whichever first) into SQLite
  (Postgres in the reference).  A retention pass deletes entries older than
  ``retention_days`` (0 = keep forever).
* :meth:`AuditLogger.query` -- filters by session / user / workspace / event
  types / time window with limit+offset paging and ``hasMore``.
* :func:`mount_routes` -- ``GET /api/v1/audit/sessions`` (the session-api's
  audit endpoint shape).
* :class:`Forwarder` -- drains rows not yet forwarded to the central privacy
  audit hub (``POST /api/v1/privacy/audit-events``) in id order, marks them
  forwarded only after a 2xx, retries the same batch on failure.
"""
from __future__ import annotations

import json
import queue
import sqlite3
import threading
import time
from dataclasses import asdict, dataclass, field

EVENT_TYPES = (
    "session_created", "session_accessed", "session_searched", "session_exported",
    "session_deleted", "pii_redacted", "memory_write_blocked", "decryption_requested",
    "memory_created", "memory_accessed", "memory_deleted", "memory_exported",
    "memory_consolidated",
)


@dataclass
class Entry:
    eventType: str
    timestamp: float = field(default_factory=time.time)
    sessionId: str = ""
    userId: str = ""
    workspace: str = ""
    agentName: str = ""
    namespace: str = ""
    query: str = ""
    resultCount: int = 0
    ipAddress: str = ""
    userAgent: str = ""
    reason: str = ""
    metadata: dict = field(default_factory=dict)
    id: int = 0


SCHEMA = """CREATE TABLE IF NOT EXISTS audit_log (
  id INTEGER PRIMARY KEY AUTOINCREMENT, timestamp REAL, event_type TEXT, session_id TEXT,
  user_id TEXT, workspace TEXT, agent_name TEXT, namespace TEXT, query TEXT,
  result_count INTEGER, ip_address TEXT, user_agent TEXT, reason TEXT, metadata TEXT,
  forwarded INTEGER DEFAULT 0);
CREATE INDEX IF NOT EXISTS audit_ts ON audit_log(timestamp);
CREATE INDEX IF NOT EXISTS audit_sess ON audit_log(session_id);"""

_COLS = ("timestamp", "event_type", "session_id", "user_id", "workspace", "agent_name",
         "namespace", "query", "result_count", "ip_address", "user_agent", "reason",
         "metadata")


def _row_to_entry(r) -> Entry:
    return Entry(id=r[0], timestamp=r[1], eventType=r[2], sessionId=r[3] or "",
                 userId=r[4] or "", workspace=r[5] or "", agentName=r[6] or "",
                 namespace=r[7] or "", query=r[8] or "", resultCount=r[9] or 0,
                 ipAddress=r[10] or "", userAgent=r[11] or "", reason=r[12] or "",
                 metadata=json.loads(r[13] or "{}"))


class AuditLogger:
    def __init__(self, db: str = ":memory:", buffer_size: int = 10000, batch_size: int = 100,
                 flush_interval_s: float = 1.0, retention_days: int = 0):
        self.db = sqlite3.connect(db, check_same_thread=False)
        self.db.executescript(SCHEMA)
        self.lock = threading.Lock()
        self.buf: queue.Queue = queue.Queue(maxsize=buffer_size)
        self.batch_size = batch_size
        self.flush_interval_s = flush_interval_s
        self.retention_days = retention_days
        self.dropped = 0
        self.written = 0
        self._stop = threading.Event()
        self._worker = threading.Thread(target=self._run, name="audit-writer", daemon=True)
        self._worker.start()

    # -- write path
    def log_event(self, e: Entry) -> bool:
        try:
            self.buf.put_nowait(e)
            return True
        except queue.Full:
            self.dropped += 1
            return False

    def _run(self):
        batch: list[Entry] = []
        deadline = time.monotonic() + self.flush_interval_s
        while not self._stop.is_set() or not self.buf.empty():
            try:
                batch.append(self.buf.get(timeout=max(0.0, deadline - time.monotonic())))
            except queue.Empty:
                pass
            if len(batch) >= self.batch_size or time.monotonic() >= deadline or \
                    (self._stop.is_set() and self.buf.empty()):
                if batch:
                    self._write(batch)
                    batch = []
                deadline = time.monotonic() + self.flush_interval_s
        if batch:
            self._write(batch)

    def _write(self, batch: list[Entry]):
        rows = [(e.timestamp, e.eventType, e.sessionId, e.userId, e.workspace, e.agentName,
                 e.namespace, e.query, e.resultCount, e.ipAddress, e.userAgent, e.reason,
                 json.dumps(e.metadata)) for e in batch]
        with self.lock:
            self.db.executemany(
                f"INSERT INTO audit_log ({','.join(_COLS)}) VALUES ({','.join('?' * len(_COLS))})",
                rows)
            self.db.commit()
        self.written += len(rows)

    def flush(self, timeout: float = 5.0) -> None:
        t_end = time.monotonic() + timeout
        while not self.buf.empty() and time.monotonic() < t_end:
            time.sleep(0.01)
        time.sleep(min(0.05, self.flush_interval_s) + 0.01)
        # whatever the worker holds in its batch is written at its next deadline
        while time.monotonic() < t_end:
            with self.lock:
                n = self.db.execute("SELECT count(*) FROM audit_log").fetchone()[0]
            if n >= self.written and self.buf.empty():
                break
            time.sleep(0.01)

    def close(self) -> None:
        self._stop.set()
        self._worker.join(10)

    # -- read path
    def query(self, session_id="", user_id="", workspace="", event_types=None,
              start: float | None = None, end: float | None = None, limit: int = 100,
              offset: int = 0) -> dict:
        where, args = [], []
        for col, v in (("session_id", session_id), ("user_id", user_id),
                       ("workspace", workspace)):
            if v:
                where.append(f"{col} = ?")
                args.append(v)
        if event_types:
            where.append(f"event_type IN ({','.join('?' * len(event_types))})")
            args += list(event_types)
        if start is not None:
            where.append("timestamp >= ?")
            args.append(start)
        if end is not None:
            where.append("timestamp <= ?")
            args.append(end)
        w = (" WHERE " + " AND ".join(where)) if where else ""
        limit = max(1, min(int(limit), 1000))
        with self.lock:
            total = self.db.execute(f"SELECT count(*) FROM audit_log{w}", args).fetchone()[0]
            rows = self.db.execute(
                f"SELECT id, {','.join(_COLS)} FROM audit_log{w} ORDER BY timestamp DESC, id DESC "
                "LIMIT ? OFFSET ?", args + [limit, offset]).fetchall()
        entries = [asdict(_row_to_entry(r)) for r in rows]
        return {"entries": entries, "total": total, "hasMore": offset + len(rows) < total}

    def delete_expired(self, now: float | None = None) -> int:
        if self.retention_days <= 0:
            return 0
        cutoff = (now or time.time()) - self.retention_days * 86400
        with self.lock:
            n = self.db.execute("DELETE FROM audit_log WHERE timestamp < ?", (cutoff,)).rowcount
            self.db.commit()
        return n

    # -- forwarder support
    def unforwarded(self, limit: int) -> list[Entry]:
        with self.lock:
            rows = self.db.execute(
                f"SELECT id, {','.join(_COLS)} FROM audit_log WHERE forwarded = 0 ORDER BY id "
                "LIMIT ?", (limit,)).fetchall()
        return [_row_to_entry(r) for r in rows]

    def mark_forwarded(self, ids: list[int]) -> None:
        if not ids:
            return
        with self.lock:
            self.db.execute(f"UPDATE audit_log SET forwarded = 1 WHERE id IN "
                            f"({','.join('?' * len(ids))})", ids)
            self.db.commit()


def mount_routes(app, logger: AuditLogger, prefix: str = "/api/v1/audit") -> None:
    from aiohttp import web

    async def list_events(request):
        q = request.query
        types = [t for t in q.get("eventTypes", "").split(",") if t]
        try:
            res = logger.query(q.get("sessionId", ""), q.get("userId", ""),
                               q.get("workspace", ""), types,
                               float(q["from"]) if "from" in q else None,
                               float(q["to"]) if "to" in q else None,
                               int(q.get("limit", 100)), int(q.get("offset", 0)))
        except ValueError as e:
            return web.json_response({"error": str(e)}, status=400)
        return web.json_response(res)

    app.router.add_get(prefix + "/sessions", list_events)


class Forwarder:
    """Ship local audit rows to the central audit hub (privacy-api)."""

    def __init__(self, logger: AuditLogger, hub_url: str, source: str = "session-api",
                 batch_size: int = 200, token: str | None = None, post=None):
        self.logger = logger
        self.url = hub_url.rstrip("/") + "/api/v1/privacy/audit-events"
        self.source = source
        self.batch_size = batch_size
        self.token = token
        self._post = post  # injectable async (url, json, headers) -> status
        self.forwarded = 0
        self.failures = 0

    async def _send(self, body: dict) -> int:
        if self._post is not None:
            return await self._post(self.url, body, self._headers())
        import aiohttp

        async with aiohttp.ClientSession() as s:
            async with s.post(self.url, json=body, headers=self._headers(),
                              timeout=aiohttp.ClientTimeout(total=10)) as r:
                return r.status

    def _headers(self) -> dict:
        return {"Authorization": f"Bearer {self.token}"} if self.token else {}

    async def drain_once(self) -> int:
        sent = 0
        while True:
            batch = self.logger.unforwarded(self.batch_size)
            if not batch:
                return sent
            body = {"source": self.source, "events": [
                {"type": e.eventType, "ts": e.timestamp, "user_id": e.userId,
                 "session_id": e.sessionId, "workspace": e.workspace, "reason": e.reason,
                 "metadata": e.metadata} for e in batch]}
            try:
                status = await self._send(body)
            except Exception:  # noqa: BLE001 - retried next drain
                status = 0
            if not 200 <= status < 300:
                self.failures += 1
                return sent
            self.logger.mark_forwarded([e.id for e in batch])
            sent += len(batch)
            self.forwarded += len(batch)
