"""Privacy API (``ee/cmd/privacy-api``, ``ee/pkg/privacy``).

* consent: per-user grants / revocations over the consent categories; categories
  that ``require an explicit grant`` (identity, location, health,
  analytics:aggregate) are denied until granted, the rest are granted by default
  (``consent.go:20-60``).  A revocation fans out to memory-api
  (``POST /api/v1/memories/consent-events``) so memories of that category go.
* opt-out: per-user (optionally per-agent) recording opt-out that the facade /
  session-api consult before recording (``handler.go``).
* DSAR erasure: ``POST /api/v1/privacy/deletion-request`` creates a request that
  a background eraser executes against session-api (delete the user's sessions)
  and memory-api (``DELETE /api/v1/memories?virtual_user_id=``), tracking
  progress / errors (``deletion.go``, ``fanout_eraser.go``).
* audit hub: ``POST /api/v1/privacy/audit-events`` ingests audit events from the
  other services (``audit_ingest_handler.go``); stats endpoints for the dashboard.

State is SQLite (Postgres in the reference).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import sqlite3
import threading
import time
import uuid

from aiohttp import web
from ...observability.logging import configure as configure_logging

log = logging.getLogger("omnia.privacy")

CATEGORIES = {"memory:preferences": False, "memory:context": False, "memory:history": False,
              "memory:identity": True, "memory:location": True, "memory:health": True,
              "analytics:aggregate": True}  # category -> requires explicit grant

SCHEMA = """
CREATE TABLE IF NOT EXISTS consent (user_id TEXT, category TEXT, granted INTEGER,
  updated_at REAL, PRIMARY KEY (user_id, category));
CREATE TABLE IF NOT EXISTS opt_out (user_id TEXT, scope TEXT, target TEXT, created_at REAL,
  PRIMARY KEY (user_id, scope, target));
CREATE TABLE IF NOT EXISTS deletion_requests (id TEXT PRIMARY KEY, body TEXT);
CREATE TABLE IF NOT EXISTS audit_events (id INTEGER PRIMARY KEY AUTOINCREMENT, ts REAL,
  source TEXT, type TEXT, user_id TEXT, body TEXT);
"""


class PrivacyStore:
    def __init__(self, path: str = ":memory:"):
        self.db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self.db.executescript(SCHEMA)
        self.lock = threading.RLock()

    def q(self, sql, args=()):
        with self.lock:
            return self.db.execute(sql, args).fetchall()

    # consent
    def set_consent(self, user: str, grants, revocations):
        bad = [c for c in list(grants) + list(revocations) if c not in CATEGORIES]
        if bad:
            raise ValueError(f"unknown consent categories: {bad}")
        now = time.time()
        with self.lock:
            for c in grants:
                self.db.execute("INSERT OR REPLACE INTO consent VALUES (?,?,1,?)", (user, c, now))
            for c in revocations:
                self.db.execute("INSERT OR REPLACE INTO consent VALUES (?,?,0,?)", (user, c, now))

    def consent(self, user: str) -> dict:
        rows = dict(self.q("SELECT category, granted FROM consent WHERE user_id = ?", (user,)))
        grants, defaults, denied = [], [], []
        for c, explicit in sorted(CATEGORIES.items()):
            if c in rows:
                (grants if rows[c] else denied).append(c)
            elif explicit:
                denied.append(c)
            else:
                defaults.append(c)
        return {"grants": grants, "defaults": defaults, "denied": denied}

    def allowed(self, user: str, category: str) -> bool:
        c = self.consent(user)
        return category in c["grants"] or category in c["defaults"]

    def consent_stats(self) -> dict:
        rows = self.q("SELECT category, granted, count(*) FROM consent GROUP BY 1, 2")
        out = {c: {"granted": 0, "revoked": 0} for c in CATEGORIES}
        for c, g, n in rows:
            out[c]["granted" if g else "revoked"] += n
        users = self.q("SELECT count(DISTINCT user_id) FROM consent")[0][0]
        return {"categories": out, "users": users}

    # opt-out
    def opt_out(self, user, scope="all", target=""):
        with self.lock:
            self.db.execute("INSERT OR REPLACE INTO opt_out VALUES (?,?,?,?)",
                            (user, scope, target or "", time.time()))

    def remove_opt_out(self, user, scope="all", target=""):
        with self.lock:
            return self.db.execute("DELETE FROM opt_out WHERE user_id = ? AND scope = ? AND "
                                   "target = ?", (user, scope, target or "")).rowcount

    def is_opted_out(self, user: str, agent: str = "") -> bool:
        return bool(self.q("SELECT 1 FROM opt_out WHERE user_id = ? AND (scope = 'all' OR "
                           "(scope = 'agent' AND target = ?))", (user, agent)))

    # deletion requests
    def put_request(self, r: dict):
        with self.lock:
            self.db.execute("INSERT OR REPLACE INTO deletion_requests VALUES (?, ?)",
                            (r["id"], json.dumps(r)))

    def get_request(self, rid: str):
        rows = self.q("SELECT body FROM deletion_requests WHERE id = ?", (rid,))
        return json.loads(rows[0][0]) if rows else None

    def list_requests(self, user: str | None = None):
        out = [json.loads(b) for (b,) in self.q("SELECT body FROM deletion_requests")]
        return [r for r in out if not user or r["virtualUserId"] == user]

    # audit
    def ingest(self, events: list[dict]) -> int:
        with self.lock:
            for e in events:
                self.db.execute("INSERT INTO audit_events (ts, source, type, user_id, body) "
                                "VALUES (?,?,?,?,?)", (e.get("timestamp") or time.time(),
                                                       e.get("source", ""), e.get("type", ""),
                                                       e.get("userId", ""), json.dumps(e)))
        return len(events)

    def audit(self, user: str | None = None, limit: int = 100):
        sql = "SELECT body FROM audit_events"
        args = []
        if user:
            sql += " WHERE user_id = ?"
            args.append(user)
        return [json.loads(b) for (b,) in self.q(sql + " ORDER BY id DESC LIMIT ?",
                                                 args + [limit])]


class FanoutEraser:
    """Executes a deletion request: every service group's session-api and
    memory-api through :class:`erasure.FanOutSubjectEraser`.  ``session_api`` /
    ``memory_api``: the default group; ``groups``: more :class:`GroupTarget` s."""

    def __init__(self, store: PrivacyStore, session_api: str = "", memory_api: str = "",
                 workspaces: list[str] | None = None, groups: list | None = None):
        from .erasure import FanOutSubjectEraser, GroupTarget

        self.store = store
        tg = list(groups or [])
        if session_api or memory_api:
            tg.insert(0, GroupTarget("default", session_api.rstrip("/"), memory_api.rstrip("/")))
        self.fanout = FanOutSubjectEraser(tg, workspaces or [])

    async def run(self, rid: str):
        r = self.store.get_request(rid)
        r.update(status="in_progress", startedAt=time.time())
        self.store.put_request(r)
        user = r["virtualUserId"]
        try:
            deleted, errors = await self.fanout.erase_subject(r)
        except Exception as e:  # noqa: BLE001
            deleted, errors = 0, [str(e)]
        r.update(status="completed" if not errors else "failed", completedAt=time.time(),
                 sessionsDeleted=deleted, errors=errors)
        self.store.put_request(r)
        self.store.ingest([{"source": "privacy-api", "type": "dsar.erasure", "userId": user,
                            "requestId": rid, "status": r["status"]}])
        return r


def build_app(store: PrivacyStore, eraser: FanoutEraser | None = None,
              memory_api: str = "", notifier=None) -> web.Application:
    """``notifier``: consent-revocation notifier (``outbox.MemoryAPINotifier``);
    when given, revocations go through the transactional outbox.  ``memory_api``
    alone builds a single-target notifier."""
    from .outbox import MemoryAPINotifier, Outbox, deliver

    eraser = eraser or FanoutEraser(store)
    if notifier is None and memory_api:
        notifier = MemoryAPINotifier([memory_api])
    outbox = Outbox(store)
    tasks: set = set()

    def bad(msg, code=400):
        return web.json_response({"error": msg}, status=code)

    async def set_consent(request):
        d = await request.json()
        user = request.match_info["userID"]
        revs = d.get("revocations") or []
        try:
            store.set_consent(user, d.get("grants") or [], [])
            bad_revs = [c for c in revs if c not in CATEGORIES]
            if bad_revs:
                raise ValueError(f"unknown consent categories: {bad_revs}")
        except ValueError as e:
            return bad(str(e))
        for c in revs:  # revocation + outbox row in one transaction, then notify
            oid = outbox.revoke_with_outbox(user, c)
            if oid is not None and notifier is not None:
                await deliver(outbox, notifier, oid, user, c)
        store.ingest([{"source": "privacy-api", "type": "consent.updated", "userId": user,
                       "grants": d.get("grants") or [], "revocations": d.get("revocations")
                       or []}])
        return web.json_response(store.consent(user))

    async def get_consent(request):
        return web.json_response(store.consent(request.match_info["userID"]))

    async def prefs(request):
        u = request.match_info["userID"]
        return web.json_response({"userId": u, "consent": store.consent(u),
                                  "optedOut": store.is_opted_out(u)})

    async def opt_out(request):
        d = await request.json()
        if not d.get("userId"):
            return bad("userId is required")
        store.opt_out(d["userId"], d.get("scope") or "all", d.get("target", ""))
        return web.json_response({"status": "opted_out"}, status=201)

    async def rm_opt_out(request):
        d = await request.json()
        n = store.remove_opt_out(d.get("userId", ""), d.get("scope") or "all",
                                 d.get("target", ""))
        return web.json_response({"removed": n})

    async def create_deletion(request):
        d = await request.json()
        if not d.get("virtualUserId"):
            return bad("virtualUserId is required")
        r = {"id": uuid.uuid4().hex, "virtualUserId": d["virtualUserId"],
             "reason": d.get("reason", ""), "scope": d.get("scope", "all"),
             "workspace": d.get("workspace", ""), "status": "pending",
             "createdAt": time.time(), "sessionsDeleted": 0, "errors": []}
        store.put_request(r)
        t = asyncio.create_task(eraser.run(r["id"]))
        tasks.add(t)
        t.add_done_callback(tasks.discard)
        return web.json_response(r, status=202)

    async def get_deletion(request):
        r = store.get_request(request.match_info["id"])
        return web.json_response(r) if r else bad("not found", 404)

    async def list_deletion(request):
        return web.json_response({"requests": store.list_requests(request.query.get("userId"))})

    async def audit_ingest(request):
        d = await request.json()
        events = d if isinstance(d, list) else d.get("events", [d])
        return web.json_response({"ingested": store.ingest(events)}, status=202)

    async def consent_stats(_):
        return web.json_response(store.consent_stats())

    async def enforcement_stats(_):
        rows = store.q("SELECT type, count(*) FROM audit_events GROUP BY type")
        return web.json_response({"events": dict(rows)})

    async def health(_):
        return web.json_response({"status": "ok"})

    app = web.Application()
    app["outbox"] = outbox
    r = app.router
    r.add_put("/api/v1/privacy/preferences/{userID}/consent", set_consent)
    r.add_get("/api/v1/privacy/preferences/{userID}/consent", get_consent)
    r.add_get("/api/v1/privacy/preferences/{userID}", prefs)
    r.add_post("/api/v1/privacy/opt-out", opt_out)
    r.add_delete("/api/v1/privacy/opt-out", rm_opt_out)
    r.add_post("/api/v1/privacy/deletion-request", create_deletion)
    r.add_get("/api/v1/privacy/deletion-request/{id}", get_deletion)
    r.add_get("/api/v1/privacy/deletion-requests", list_deletion)
    r.add_post("/api/v1/privacy/audit-events", audit_ingest)
    r.add_get("/api/v1/privacy/consent/stats", consent_stats)
    r.add_get("/api/v1/privacy/enforcement-stats", enforcement_stats)
    r.add_get("/healthz", health)
    r.add_get("/readyz", health)
    return app


def main(argv=None):
    ap = argparse.ArgumentParser(description="omnia privacy-api")
    ap.add_argument("--port", type=int, default=8085)
    ap.add_argument("--db", default=":memory:")
    ap.add_argument("--session-api", default="")
    ap.add_argument("--memory-api", default="")
    ap.add_argument("--workspaces", default="")
    ap.add_argument("--group", action="append", default=[],
                    help="extra service group NAME=SESSION_URL,MEMORY_URL (repeatable)")
    ap.add_argument("--outbox-replay-interval", type=float, default=30.0)
    ap.add_argument("--operator-url", default="",
                    help="watch SessionPrivacyPolicies through this API server")
    a = ap.parse_args(argv)
    from .erasure import GroupTarget
    from .outbox import MemoryAPINotifier, Outbox, OutboxReplayWorker

    store = PrivacyStore(a.db)
    groups = []
    for g in a.group:
        name, _, urls = g.partition("=")
        su, _, mu = urls.partition(",")
        groups.append(GroupTarget(name, su, mu))
    er = FanoutEraser(store, a.session_api, a.memory_api,
                      [w for w in a.workspaces.split(",") if w], groups)
    notifier = MemoryAPINotifier([a.memory_api] + [g.memory_url for g in groups])
    app = build_app(store, er, notifier=notifier)
    replay = OutboxReplayWorker(Outbox(store), notifier, a.outbox_replay_interval)

    async def start(app):
        app["replay"] = asyncio.create_task(replay.run())

    async def stop(app):
        app["replay"].cancel()

    app.on_startup.append(start)
    app.on_cleanup.append(stop)
    configure_logging()
    web.run_app(app, port=a.port)


if __name__ == "__main__":
    main()
