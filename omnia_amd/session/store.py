"""Tiered session storage: hot -> warm -> cold (``internal/session/providers``).

  hot   in-process LRU with TTL, or Redis (RESP) -- recent sessions + messages
  warm  SQL over a dialect (:mod:`.sqldialect`): SQLite in-process, or the
        reference's weekly-partitioned Postgres tables when a driver is present
  cold  Parquet files (pyarrow) in a blob store (local dir / memory), one file
        per archived batch plus a JSON manifest (``cold/provider.go``)

Reads fall through hot -> warm -> cold; a miss or an ERROR in an upper tier is
never treated as "does not exist" while a lower tier can still answer (the
reference's tiered-fallback matrix, CLAUDE.md:316-328): hit / miss / empty /
error / all-miss are all tested.
"""
from __future__ import annotations

import io
import json
import os
import sqlite3
import threading
import time
from collections import OrderedDict
from pathlib import Path

from ..utils import failpoints
from .model import (EvalResult, Message, ProviderCall, RuntimeEvent, Session, ToolCall,
                    STATUS_ACTIVE)


class TierError(Exception):
    pass


# ===================================================================== hot
class HotCache:
    def __init__(self, max_sessions: int = 10000, ttl_s: float = 3600, max_messages: int = 200):
        self.max_sessions = max_sessions
        self.ttl_s = ttl_s
        self.max_messages = max_messages
        self.d: "OrderedDict[str, tuple[float, Session, list]]" = OrderedDict()
        self.fail = False
        self.lock = threading.Lock()

    def _chk(self):
        if self.fail:
            raise TierError("hot tier unavailable")

    def get(self, sid: str):
        self._chk()
        with self.lock:
            v = self.d.get(sid)
            if v is None:
                return None
            if v[0] < time.time():
                self.d.pop(sid, None)
                return None
            self.d.move_to_end(sid)
            return v[1], list(v[2])

    def put(self, s: Session, msgs: list | None = None):
        self._chk()
        with self.lock:
            old = self.d.get(s.id)
            m = msgs if msgs is not None else (old[2] if old else [])
            self.d[s.id] = (time.time() + self.ttl_s, s, m[-self.max_messages:])
            self.d.move_to_end(s.id)
            while len(self.d) > self.max_sessions:
                self.d.popitem(last=False)

    def append(self, sid: str, msg: Message):
        self._chk()
        with self.lock:
            v = self.d.get(sid)
            if v is not None:
                v[2].append(msg)
                del v[2][:-self.max_messages]

    def invalidate(self, sid: str):
        with self.lock:
            self.d.pop(sid, None)


# ===================================================================== warm
class WarmStore:
    """The warm tier over a DB-API connection and a SQL dialect
    (:mod:`.sqldialect`): SQLite by default, Postgres with weekly partitions when
    a driver and DSN are given (:meth:`postgres`)."""

    def __init__(self, path: str = ":memory:", dialect=None, conn=None, schema_dialect=None):
        from .sqldialect import SQLiteDialect

        self.d = dialect or SQLiteDialect()
        self.db = conn if conn is not None else sqlite3.connect(path, check_same_thread=False)
        self.lock = threading.Lock()
        self.fail = False
        for stmt in (schema_dialect or self.d).schema():
            self._run(stmt, ())

    @classmethod
    def postgres(cls, dsn: str) -> "WarmStore":
        from .sqldialect import connect_postgres

        conn, dialect = connect_postgres(dsn)
        return cls(dialect=dialect, conn=conn)

    def _run(self, sql, args):
        cur = self.db.cursor()
        try:
            cur.execute(sql, tuple(args))
            rows = cur.fetchall() if cur.description else []
        finally:
            cur.close()
        self.db.commit()
        return rows

    def _x(self, sql, args=()):
        if self.fail:
            raise TierError("warm tier unavailable")
        with self.lock:
            return self._run(self.d.q(sql), args)

    def _upsert(self, table, args):
        if self.fail:
            raise TierError("warm tier unavailable")
        with self.lock:
            return self._run(self.d.upsert(table), args)

    def put_session(self, s: Session):
        self._upsert("sessions", (s.id, s.namespace, s.agent_name, s.workspace_name, s.status,
                                  s.created_at, s.updated_at, s.expires_at, s.virtual_user_id,
                                  json.dumps(s.to_json())))

    def get_session(self, sid: str) -> Session | None:
        r = self._x("SELECT doc FROM sessions WHERE id=?", (sid,))
        return Session.from_json(json.loads(r[0][0])) if r else None

    def add_message(self, sid: str, m: Message):
        self._upsert("messages", (m.id, sid, m.sequence_num, m.timestamp, m.role, m.content,
                                  json.dumps(m.to_json())))

    def scan_messages(self, after_id: str = "", limit: int = 100) -> list[tuple[str, str, dict]]:
        """(id, session_id, doc) of every message in id order after ``after_id``
        (the key-rotation re-encryption cursor)."""
        r = self._x("SELECT id, session_id, doc FROM messages WHERE id > ? ORDER BY id LIMIT ?",
                    (after_id, limit))
        return [(x[0], x[1], json.loads(x[2])) for x in r]

    def messages(self, sid: str, limit: int = 1000, offset: int = 0) -> list[Message]:
        r = self._x("SELECT doc FROM messages WHERE session_id=? ORDER BY seq, ts LIMIT ? "
                    "OFFSET ?", (sid, limit, offset))
        return [Message.from_json(json.loads(x[0])) for x in r]

    def add(self, table: str, obj, sid: str):
        d = obj.to_json()
        if table == "tool_calls":
            self._upsert("tool_calls", (obj.id, sid, obj.created_at, obj.name, obj.status,
                                        json.dumps(d)))
        elif table == "provider_calls":
            self._upsert("provider_calls", (obj.id, sid, obj.created_at, obj.provider,
                                            obj.model, obj.input_tokens, obj.output_tokens,
                                            obj.cost_usd, json.dumps(d)))
        elif table == "events":
            self._upsert("events", (obj.id, sid, obj.created_at, obj.type, json.dumps(d)))
        elif table == "eval_results":
            self._upsert("eval_results", (obj.id, sid, obj.created_at, obj.eval_id,
                                          int(obj.passed), obj.score, json.dumps(d)))

    def list_rows(self, table: str, sid: str) -> list[dict]:
        return [json.loads(x[0]) for x in self._x(
            f"SELECT doc FROM {table} WHERE session_id=? ORDER BY created", (sid,))]

    def list_eval_results(self, passed: bool | None = None, eval_id: str | None = None,
                          limit: int = 100, offset: int = 0) -> list[dict]:
        """Eval results across sessions, newest first (``ListEvalResults``)."""
        sql = "SELECT doc FROM eval_results WHERE 1=1"
        args: list = []
        if passed is not None:
            sql += " AND passed=?"
            args.append(int(bool(passed)))
        if eval_id:
            sql += " AND eval_id=?"
            args.append(eval_id)
        sql += " ORDER BY created DESC LIMIT ? OFFSET ?"
        args += [int(limit), int(offset)]
        return [json.loads(x[0]) for x in self._x(sql, args)]

    def list_sessions(self, namespace=None, agent=None, status=None, before=None, after=None,
                      user=None, limit=100, offset=0, q=None) -> list[Session]:
        sql = "SELECT doc FROM sessions WHERE 1=1"
        args: list = []
        for col, v in (("namespace", namespace), ("agent", agent), ("status", status),
                       ('"user"', user)):
            if v:
                sql += f" AND {col}=?"
                args.append(v)
        if before:
            sql += " AND created<?"
            args.append(before)
        if after:
            sql += " AND created>?"
            args.append(after)
        if q:
            sql += " AND id IN (SELECT session_id FROM messages WHERE content LIKE ?)"
            args.append(f"%{q}%")
        sql += " ORDER BY created DESC LIMIT ? OFFSET ?"
        args += [limit, offset]
        return [Session.from_json(json.loads(x[0])) for x in self._x(sql, args)]

    def delete_session(self, sid: str) -> bool:
        n = self._x("SELECT COUNT(*) FROM sessions WHERE id=?", (sid,))[0][0]
        for t in ("messages", "tool_calls", "provider_calls", "events", "eval_results"):
            self._x(f"DELETE FROM {t} WHERE session_id=?", (sid,))
        self._x("DELETE FROM sessions WHERE id=?", (sid,))
        return n > 0

    def sessions_older_than(self, ts: float, limit: int = 500) -> list[str]:
        return [x[0] for x in self._x("SELECT id FROM sessions WHERE updated<? ORDER BY updated "
                                      "LIMIT ?", (ts, limit))]

    def provider_usage(self, workspace: str, doc: dict):
        self._x("INSERT INTO provider_usage (workspace, created, doc) VALUES (?,?,?)",
                (workspace, time.time(), json.dumps(doc)))

    def aggregate_provider_calls(self, namespace=None, group_by="model") -> list[dict]:
        col = {"model": "model", "provider": "provider"}.get(group_by, "model")
        sql = (f"SELECT p.{col}, COUNT(*), SUM(p.input), SUM(p.output), SUM(p.cost) FROM "
               "provider_calls p JOIN sessions s ON s.id = p.session_id")
        args = []
        if namespace:
            sql += " WHERE s.namespace=?"
            args.append(namespace)
        sql += f" GROUP BY p.{col}"
        return [{group_by: r[0], "calls": r[1], "inputTokens": r[2] or 0,
                 "outputTokens": r[3] or 0, "costUsd": r[4] or 0.0} for r in self._x(sql, args)]

    def aggregate_evals(self, namespace=None) -> list[dict]:
        sql = ("SELECT e.eval_id, COUNT(*), SUM(e.passed), AVG(e.score) FROM eval_results e "
               "LEFT JOIN sessions s ON s.id = e.session_id")
        args = []
        if namespace:
            sql += " WHERE s.namespace=?"
            args.append(namespace)
        sql += " GROUP BY e.eval_id"
        return [{"evalId": r[0], "total": r[1], "passed": r[2] or 0,
                 "passRate": (r[2] or 0) / r[1] if r[1] else 0.0, "avgScore": r[3] or 0.0}
                for r in self._x(sql, args)]


# ===================================================================== cold
class LocalBlobStore:
    def __init__(self, root: str):
        self.root = Path(root)
        self.root.mkdir(parents=True, exist_ok=True)

    def put(self, key: str, data: bytes):
        p = self.root / key
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_suffix(p.suffix + ".tmp")
        tmp.write_bytes(data)
        os.replace(tmp, p)

    def get(self, key: str) -> bytes | None:
        p = self.root / key
        return p.read_bytes() if p.exists() else None

    def delete(self, key: str):
        p = self.root / key
        if p.exists():
            p.unlink()

    def list(self, prefix: str = "") -> list[str]:
        return sorted(str(p.relative_to(self.root)) for p in self.root.rglob("*")
                      if p.is_file() and str(p.relative_to(self.root)).startswith(prefix))


class MemoryBlobStore:
    def __init__(self):
        self.d: dict[str, bytes] = {}

    def put(self, key, data):
        self.d[key] = bytes(data)

    def get(self, key):
        return self.d.get(key)

    def delete(self, key):
        self.d.pop(key, None)

    def list(self, prefix=""):
        return sorted(k for k in self.d if k.startswith(prefix))


class ColdArchive:
    """Parquet batches + manifest {session_id: batch_key} (``cold/provider.go``, ``parquet.go``)."""

    MANIFEST = "manifest.json"

    def __init__(self, blob):
        self.blob = blob
        raw = blob.get(self.MANIFEST)
        self.manifest: dict = json.loads(raw) if raw else {"sessions": {}, "batches": {}}
        self.fail = False

    def _save(self):
        self.blob.put(self.MANIFEST, json.dumps(self.manifest).encode())

    def archive(self, items: list[tuple[Session, list[Message]]]) -> str:
        import pyarrow as pa
        import pyarrow.parquet as pq

        if self.fail:
            raise TierError("cold tier unavailable")
        key = f"batches/{int(time.time() * 1000)}-{os.urandom(4).hex()}.parquet"
        rows = {"session_id": [], "kind": [], "seq": [], "doc": []}
        for s, msgs in items:
            rows["session_id"].append(s.id)
            rows["kind"].append("session")
            rows["seq"].append(-1)
            rows["doc"].append(json.dumps(s.to_json()))
            for i, m in enumerate(msgs):
                rows["session_id"].append(s.id)
                rows["kind"].append("message")
                rows["seq"].append(m.sequence_num or i)
                rows["doc"].append(json.dumps(m.to_json()))
        buf = io.BytesIO()
        pq.write_table(pa.table(rows), buf, compression="zstd")
        self.blob.put(key, buf.getvalue())
        for s, _ in items:
            self.manifest["sessions"][s.id] = {"batch": key, "namespace": s.namespace,
                                               "created": s.created_at}
        self.manifest["batches"][key] = {"count": len(items), "created": time.time()}
        self._save()
        return key

    def get(self, sid: str):
        import pyarrow.parquet as pq

        if self.fail:
            raise TierError("cold tier unavailable")
        ent = self.manifest["sessions"].get(sid)
        if ent is None:
            return None
        raw = self.blob.get(ent["batch"])
        if raw is None:
            return None
        # one archive batch is small: decode it on this thread, not on arrow's
        # thread pool (a pooled read segfaulted once inside read_table during a
        # loaded parallel test run; single-threaded decode avoids the pool)
        t = pq.read_table(io.BytesIO(raw), use_threads=False).to_pydict()
        sess, msgs = None, []
        for i, s in enumerate(t["session_id"]):
            if s != sid:
                continue
            d = json.loads(t["doc"][i])
            if t["kind"][i] == "session":
                sess = Session.from_json(d)
            else:
                msgs.append(Message.from_json(d))
        msgs.sort(key=lambda m: (m.sequence_num, m.timestamp))
        return (sess, msgs) if sess else None

    def expire(self, older_than: float) -> int:
        """Drop whole batches older than the cold retention."""
        n = 0
        for key, meta in list(self.manifest["batches"].items()):
            if meta["created"] < older_than:
                self.blob.delete(key)
                self.manifest["batches"].pop(key)
                for sid in [s for s, e in self.manifest["sessions"].items() if e["batch"] == key]:
                    self.manifest["sessions"].pop(sid)
                    n += 1
        self._save()
        return n

    def delete_session(self, sid: str) -> bool:
        return self.manifest["sessions"].pop(sid, None) is not None


# ===================================================================== service
class TieredSessionService:
    def __init__(self, hot: HotCache | None = None, warm: WarmStore | None = None,
                 cold: ColdArchive | None = None, default_ttl_s: float = 24 * 3600,
                 publisher=None):
        self.hot = hot or HotCache()
        self.warm = warm or WarmStore()
        self.cold = cold
        self.default_ttl_s = default_ttl_s
        self.publisher = publisher  # async publish(namespace, event_dict)
        self.lock = threading.Lock()
        self.degraded_reads = 0
        # sessions whose hot copy may be stale: a write reached the warm tier while
        # the hot tier was unavailable; reads bypass the hot copy until refreshed
        self._stale: set = set()
        # ee/encryption.Encryptor when a SessionPrivacyPolicy enables encryption at
        # rest: message content / metadata are sealed before the warm tier and
        # opened on the way out (the hot cache holds plaintext in process memory)
        self.encryptor = None

    def _hot_put(self, s: Session, msgs: list | None = None, append: Message | None = None):
        """Write-through to the hot tier; a failure marks the session's hot copy
        stale (the warm tier, the source of truth, already has the write)."""
        try:
            self.hot.put(s, msgs)
            if append is not None:
                self.hot.append(s.id, append)
        except TierError:
            self._stale.add(s.id)

    # ------------------------------------------------------------ encryption
    def _seal(self, m: Message) -> Message:
        if self.encryptor is None:
            return m
        import dataclasses

        enc, _ = self.encryptor.encrypt_message({"content": m.content,
                                                 "metadata": dict(m.metadata or {})})
        return dataclasses.replace(m, content=enc.get("content", ""),
                                   metadata=enc.get("metadata") or {})

    def _unseal(self, m: Message) -> Message:
        from ..ee.encryption import META_KEY

        if self.encryptor is None or META_KEY not in (m.metadata or {}):
            return m
        import dataclasses

        dec = self.encryptor.decrypt_message({"content": m.content,
                                              "metadata": dict(m.metadata)})
        return dataclasses.replace(m, content=dec.get("content", ""),
                                   metadata=dec.get("metadata") or {})

    def reencrypt_batch(self, current_version: str, after_id: str = "", limit: int = 100
                        ) -> tuple[str, bool, int, int]:
        """Re-seal up to ``limit`` warm messages whose ``_encryption.keyVersion``
        is not ``current_version`` (``ee/pkg/encryption`` ``ReEncryptBatch``).
        Returns (last scanned id, more?, re-encrypted, errors)."""
        from ..ee.encryption import META_KEY

        rows = self.warm.scan_messages(after_id, limit)
        done = errors = 0
        last = after_id
        for mid, sid, doc in rows:
            last = mid
            m = Message.from_json(doc)
            rec = (m.metadata or {}).get(META_KEY)
            if rec is None:
                continue
            try:
                if json.loads(rec).get("keyVersion") == current_version:
                    continue
                self.warm.add_message(sid, self._seal(self._unseal(m)))
                done += 1
            except Exception:  # noqa: BLE001 - counted, the batch goes on
                errors += 1
        return last, len(rows) == limit, done, errors

    # ------------------------------------------------------------ writes
    def create(self, s: Session) -> Session:
        if not s.expires_at and self.default_ttl_s:
            s.expires_at = time.time() + self.default_ttl_s
        existing = self._get_session_only(s.id)
        if existing is not None:
            return existing  # idempotent ensure (facade EnsureSessionRecord)
        self.warm.put_session(s)
        self._hot_put(s, [])
        return s

    async def append_message(self, sid: str, m: Message) -> Message:
        failpoints.hit("session.write")
        s = self._get_session_only(sid)
        if s is None:
            raise KeyError(sid)
        with self.lock:
            m.sequence_num = s.message_count
            s.message_count += 1
            s.updated_at = time.time()
            s.total_input_tokens += m.input_tokens
            s.total_output_tokens += m.output_tokens
            s.estimated_cost_usd += m.cost_usd
            if m.content and self.encryptor is None:
                s.last_message_preview = m.content[:120]
        self.warm.add_message(sid, self._seal(m))
        self.warm.put_session(s)
        self._hot_put(s, append=m)
        if self.publisher is not None:
            await self.publisher({"type": "message.appended", "sessionId": sid,
                                  "namespace": s.namespace, "agentName": s.agent_name,
                                  "messageId": m.id, "role": m.role,
                                  "promptPackName": s.prompt_pack_name,
                                  "promptPackVersion": s.prompt_pack_version,
                                  "timestamp": time.time()})
        return m

    def record(self, table: str, sid: str, obj) -> None:
        s = self._get_session_only(sid)
        if s is None:
            raise KeyError(sid)
        self.warm.add(table, obj, sid)
        if table == "tool_calls":
            s.tool_call_count += 1
            s.updated_at = time.time()
            self.warm.put_session(s)
            self._hot_put(s)

    def _event(self, typ: str, s: Session) -> dict:
        return {"type": typ, "sessionId": s.id, "namespace": s.namespace,
                "agentName": s.agent_name, "promptPackName": s.prompt_pack_name,
                "promptPackVersion": s.prompt_pack_version, "timestamp": time.time()}

    async def publish_completed_if(self, prev: str, s: Session) -> None:
        """``session.completed`` on the transition into completed
        (``publishSessionCompleted``, service.go:413-446): the eval worker's
        on_session_complete trigger."""
        if self.publisher is not None and s.status == "completed" and prev != "completed":
            await self.publisher(self._event("session.completed", s))

    async def publish_evaluate(self, sid: str) -> Session:
        """``session.evaluate``: on-demand evaluation by the eval worker
        (``PublishEvaluateEvent``, service.go:655-679)."""
        s = self._get_session_only(sid)
        if s is None:
            raise KeyError(sid)
        if self.publisher is None:
            raise RuntimeError("event publisher not configured")
        if not s.agent_name:
            raise ValueError("session has no agent")
        await self.publisher(self._event("session.evaluate", s))
        return s

    def update_status(self, sid: str, status: str, ended_at: float | None = None) -> Session:
        s = self._get_session_only(sid)
        if s is None:
            raise KeyError(sid)
        s.status = status
        if ended_at or status != STATUS_ACTIVE:
            s.ended_at = ended_at or time.time()
        s.updated_at = time.time()
        self.warm.put_session(s)
        self._hot_put(s)
        return s

    def refresh_ttl(self, sid: str, ttl_s: float) -> Session:
        s = self._get_session_only(sid)
        if s is None:
            raise KeyError(sid)
        s.expires_at = time.time() + ttl_s
        self.warm.put_session(s)
        self._hot_put(s)
        return s

    def decorate(self, sid: str, tags=None, state=None) -> Session:
        s = self._get_session_only(sid)
        if s is None:
            raise KeyError(sid)
        if tags:
            s.tags = sorted(set(s.tags) | set(tags))
        if state:
            s.state.update(state)
        self.warm.put_session(s)
        self._hot_put(s)
        return s

    def delete(self, sid: str) -> bool:
        self.hot.invalidate(sid)
        self._stale.discard(sid)
        a = self.warm.delete_session(sid)
        b = self.cold.delete_session(sid) if self.cold else False
        return a or b

    # ------------------------------------------------------------ reads
    def _get_session_only(self, sid: str) -> Session | None:
        if sid not in self._stale:
            try:
                v = self.hot.get(sid)
                if v is not None:
                    return v[0]
            except TierError:
                self.degraded_reads += 1
        return self.warm.get_session(sid)

    def get(self, sid: str, with_messages: bool = True):
        """hot -> warm -> cold.  Returns (session, messages) or None.

        A miss is definitive only when the warm tier (source of truth) answered;
        if warm errored and cold has nothing, the read fails (TierError) rather
        than reporting "not found"."""
        warm_err = None
        if sid not in self._stale:
            try:
                v = self.hot.get(sid)
                # the hot copy keeps the last max_messages: it answers only when it
                # holds the whole history
                if v is not None and (not with_messages or len(v[1]) == v[0].message_count):
                    return v
            except TierError:
                self.degraded_reads += 1
        try:
            s = self.warm.get_session(sid)
            if s is not None:
                msgs = [self._unseal(m) for m in self.warm.messages(sid)] if with_messages \
                    else []
                try:
                    self.hot.put(s, msgs)
                    self._stale.discard(sid)
                except TierError:
                    pass
                return s, msgs
        except TierError as e:
            warm_err = e
            self.degraded_reads += 1
        if self.cold is not None:
            try:
                v = self.cold.get(sid)
                if v is not None:
                    return v[0], [self._unseal(m) for m in v[1]]
            except TierError as e:
                if warm_err is not None:
                    raise TierError("warm and cold tiers unavailable") from e
        if warm_err is not None:
            raise TierError("warm tier unavailable") from warm_err
        return None
