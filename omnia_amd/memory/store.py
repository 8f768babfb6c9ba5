"""Memory store: entities / observations / relations (``internal/memory/store*.go``).

Two SQL dialects (``sqldialect.py``): SQLite by default (an FTS5 table with the
porter stemmer for the ``search_vector`` tsvector column, bm25 for
``ts_rank_cd``, embeddings as float32 blobs) and Postgres + pgvector.  The store
(and every replica of the memory-api sharing it) is the vector source of truth:
embeddings live in the database and every change to them is appended to
``memory_vector_log``, which each replica tails to keep its device-resident
:class:`VectorIndex` in step.  Semantics kept from the reference:

* one entity carries a chain of observations; exactly the latest non-superseded,
  still-valid observation is "active" (``superseded_by IS NULL AND (valid_until IS
  NULL OR valid_until > now)``);
* ``about={kind,key}`` structured-key dedup upserts the entity and supersedes its
  prior observations (``store_write.go:88-140``);
* forget = soft delete (``forgotten``), DSAR delete-all / batch-delete are hard;
* multi-tier NULL-anchoring: a user-scoped request sees its own rows plus
  user-less rows, and likewise for agents (``retrieve_multi_tier.go:313-328``);
* reads bump ``accessed_at`` / ``access_count`` of the returned rows only.
"""
from __future__ import annotations

import json
import sqlite3
import threading
import time
from dataclasses import dataclass, field

import numpy as np

from . import retrieval as R
from .fts import to_fts5
from .sqldialect import (CONSENT_TABLE, EmbeddingDimConsentRequired, MemoryPostgres,
                         MemorySQLite, parse_vector_literal, vector_literal)
from .model import (META_ABOUT_KEY, META_ABOUT_KIND, META_CONSENT_CATEGORY, META_PURPOSE,
                    META_SOURCE_TYPE, META_TITLE, SCOPE_AGENT, SCOPE_USER, SCOPE_WORKSPACE,
                    SOURCE_TYPE_WEIGHT, Memory, Tier, derive_tier, new_id, normalize_scope)

SCHEMA = MemorySQLite().schema()  # the SQLite DDL (sqldialect.py)

_ACTIVE = "o.superseded_by IS NULL AND (o.valid_until IS NULL OR o.valid_until > ?)"
_ENT_COLS = ("e.id, e.kind, e.metadata, e.created_at, e.expires_at, e.title, e.virtual_user_id, "
             "e.agent_id, e.source_type, e.workspace_id")
_OBS_COLS = ("o.id, o.content, o.confidence, o.session_id, o.turn_range, o.observed_at, "
             "o.accessed_at, o.access_count, o.summary")


class NotFound(KeyError):
    pass


@dataclass
class MultiTierRequest:
    workspace_id: str
    user_id: str = ""
    agent_id: str = ""
    query: str = ""
    types: list = field(default_factory=list)
    purposes: list = field(default_factory=list)
    min_confidence: float = 0.0
    limit: int = R.DEFAULT_LIMIT
    tiers: list = field(default_factory=list)
    seed_entity_ids: list = field(default_factory=list)
    relation_types: list = field(default_factory=list)
    max_graph_hops: int = 1
    half_life: R.HalfLife = field(default_factory=R.HalfLife)
    ranker: R.TierRanker | None = None
    now: float = 0.0


def _f32(blob):
    return None if blob is None else np.frombuffer(blob, dtype=np.float32)


class AccessTouchBatcher:
    """Window-coalesced access bumps (``access_tracker.go``): ``add`` counts ids
    into the pending window; a daemon thread flushes every ``interval_s`` (or at
    once when ``cap`` distinct ids are pending) with ONE batched update carrying
    per-id increments; ``stop`` drains.  Flush failures are counted, never
    raised into the read path."""

    def __init__(self, execute, interval_s: float = 1.0, cap: int = 5000):
        self.execute = execute
        self.interval_s = interval_s
        self.cap = cap
        self.pending: dict[str, int] = {}
        self.mu = threading.Lock()
        self.wake = threading.Event()
        self.stopped = threading.Event()
        self.stats = {"flushes": 0, "rows": 0, "errors": 0}
        self.thread = threading.Thread(target=self._run, name="memory-access-touch",
                                       daemon=True)
        self.thread.start()

    def add(self, ids):
        with self.mu:
            for i in ids:
                if i:
                    self.pending[i] = self.pending.get(i, 0) + 1
            overflow = len(self.pending) >= self.cap
        if overflow:
            self.wake.set()

    def flush(self) -> int:
        with self.mu:
            if not self.pending:
                return 0
            batch, self.pending = self.pending, {}
        try:
            self.execute(list(batch), list(batch.values()))
            self.stats["flushes"] += 1
            self.stats["rows"] += len(batch)
        except Exception:  # noqa: BLE001 - best effort, like the reference's
            self.stats["errors"] += 1
        return len(batch)

    def _run(self):
        while not self.stopped.is_set():
            self.wake.wait(self.interval_s)
            self.wake.clear()
            self.flush()
        self.flush()

    def stop(self):
        self.stopped.set()
        self.wake.set()
        self.thread.join(timeout=5)


class _DB:
    """The store's connection: every statement passes through the dialect
    (placeholders) before it reaches SQLite or a DB-API Postgres connection."""

    def __init__(self, raw, dialect):
        self.raw, self.d = raw, dialect
        self.sqlite = isinstance(raw, sqlite3.Connection)

    def execute(self, sql: str, args=()):
        sql = self.d.q(sql)
        if self.sqlite:
            return self.raw.execute(sql, tuple(args))
        cur = self.raw.cursor()
        cur.execute(sql, tuple(args))
        return cur

    def executemany(self, sql: str, rows):
        sql = self.d.q(sql)
        if self.sqlite:
            return self.raw.executemany(sql, rows)
        cur = self.raw.cursor()
        cur.executemany(sql, rows)
        return cur


def default_dialect():
    """SQLite unless ``OMNIA_MEMORY_SQL_DIALECT=postgres-emulated`` (the Postgres
    DML on SQLite, as the dialect tests run it)."""
    import os

    if os.environ.get("OMNIA_MEMORY_SQL_DIALECT") == "postgres-emulated":
        return MemoryPostgres(emulate=True)
    return MemorySQLite()


class MemoryStore:
    """``path``: SQLite file (":memory:" default).  ``dialect``: MemorySQLite
    (default) or MemoryPostgres; ``conn``: an open Postgres DB-API connection
    (``sqldialect.connect_postgres``), otherwise SQLite at ``path``."""

    def __init__(self, path: str = ":memory:", dialect=None, conn=None):
        self.d = dialect or default_dialect()
        if conn is None:
            raw = sqlite3.connect(path, check_same_thread=False, isolation_level=None,
                                  timeout=30)
            raw.execute("PRAGMA journal_mode=WAL")
            raw.execute("PRAGMA synchronous=NORMAL")
        else:
            raw = conn
        self.db = _DB(raw, self.d)
        for stmt in self.d.schema():
            self.db.raw.execute(stmt) if self.db.sqlite else self.db.execute(stmt)
        self.lock = threading.RLock()
        self.touch_batcher: AccessTouchBatcher | None = None

    # ------------------------------------------------------------ helpers
    def _tx(self):
        store = self

        class _T:
            def __enter__(self_):
                store.lock.acquire()
                store.db.execute(store.d.begin())
                return store.db

            def __exit__(self_, et, ev, tb):
                try:
                    store.db.execute("ROLLBACK" if et else "COMMIT")
                finally:
                    store.lock.release()
                return False

        return _T()

    def _q(self, sql, args=()):
        with self.lock:
            return self.db.execute(sql, args).fetchall()

    @staticmethod
    def _row_to_memory(r) -> Memory:
        (eid, kind, meta, created, expires, title, uid, aid, stype, ws,
         oid, content, conf, sess, turns, observed, accessed, acount, summary) = r[:19]
        scope = {SCOPE_WORKSPACE: ws}
        if uid:
            scope[SCOPE_USER] = uid
        if aid:
            scope[SCOPE_AGENT] = aid
        m = Memory(id=eid, type=kind, content=content or "", confidence=conf if conf is not None
                   else 0.7, scope=scope, metadata=json.loads(meta or "{}"),
                   session_id=sess or "", turn_range=json.loads(turns) if turns else None,
                   created_at=created, accessed_at=accessed or 0.0, expires_at=expires,
                   observation_id=oid or "", observed_at=observed or 0.0,
                   access_count=acount or 0, title=title or "",
                   summary=summary or "")
        m.tier = derive_tier(scope)
        return m

    def _select_active(self, where: str, args: list, order: str = "o.observed_at DESC",
                       limit: int | None = None, extra_cols: str = "", join: str = ""):
        """Latest active observation per entity (DISTINCT ON e.id equivalent)."""
        now = time.time()
        sql = (f"SELECT {_ENT_COLS}, {_OBS_COLS}{extra_cols} FROM memory_entities e "
               f"JOIN memory_observations o ON o.entity_id = e.id AND {_ACTIVE} {join} "
               f"WHERE e.forgotten = 0 AND (e.expires_at IS NULL OR e.expires_at > ?) "
               f"AND o.observed_at = (SELECT max(o2.observed_at) FROM memory_observations o2 "
               f"WHERE o2.entity_id = e.id AND o2.superseded_by IS NULL AND "
               f"(o2.valid_until IS NULL OR o2.valid_until > ?)) AND {where} "
               f"ORDER BY {order}" + (f" LIMIT {int(limit)}" if limit else ""))
        return self._q(sql, [now, now, now] + list(args))

    @staticmethod
    def _scope_where(scope: dict, strict: bool = True) -> tuple[str, list]:
        """Single-tier strict scope match (``Retrieve``/``List``)."""
        ws = scope.get(SCOPE_WORKSPACE)
        if not ws:
            raise ValueError("workspace_id is required")
        parts, args = ["e.workspace_id = ?"], [ws]
        for col, key in (("e.virtual_user_id", SCOPE_USER), ("e.agent_id", SCOPE_AGENT)):
            v = scope.get(key)
            if v:
                parts.append(f"{col} = ?")
                args.append(v)
            elif strict:
                parts.append(f"{col} IS NULL")
        return " AND ".join(parts), args

    @staticmethod
    def _tier_where(req: MultiTierRequest) -> tuple[str, list]:
        if not req.workspace_id:
            raise ValueError("workspace_id is required")
        parts, args = ["e.workspace_id = ?"], [req.workspace_id]
        for col, v in (("e.virtual_user_id", req.user_id), ("e.agent_id", req.agent_id)):
            if v:
                parts.append(f"({col} IS NULL OR {col} = ?)")
                args.append(v)
            else:
                parts.append(f"{col} IS NULL")
        if req.types:
            parts.append("e.kind IN (%s)" % ",".join("?" * len(req.types)))
            args.extend(req.types)
        if req.purposes:
            parts.append("e.purpose IN (%s)" % ",".join("?" * len(req.purposes)))
            args.extend(req.purposes)
        if req.min_confidence > 0:
            parts.append("o.confidence >= ?")
            args.append(req.min_confidence)
        return " AND ".join(parts), args

    def _fts_ids(self, query: str, limit: int) -> dict[str, float]:
        """obs_id -> bm25 (lower = better) for a websearch-style query."""
        expr = to_fts5(query) if self.d.uses_fts_table else query.strip()
        if not expr:
            return {}
        sql, args = self.d.fts_search(expr, limit)
        try:
            rows = self._q(sql, args)
        except sqlite3.OperationalError:
            return {}
        return {r[0]: r[1] for r in rows}

    def touch(self, obs_ids: list[str]):
        """Reads bump ``accessed_at`` / ``access_count``: through the access-touch
        batcher when one is attached (``enable_touch_batching``), else at once."""
        if not obs_ids:
            return
        if self.touch_batcher is not None:
            self.touch_batcher.add(obs_ids)
            return
        self.apply_touches(list(dict.fromkeys(obs_ids)), None)

    def apply_touches(self, obs_ids: list[str], counts: list[int] | None):
        """One statement for a window of reads: each row gets its own increment."""
        now = time.time()
        counts = counts or [1] * len(obs_ids)
        with self.lock:
            self.db.executemany("UPDATE memory_observations SET accessed_at = ?, access_count = "
                                "access_count + ? WHERE id = ? AND superseded_by IS NULL",
                                [(now, c, i) for i, c in zip(obs_ids, counts)])

    def enable_touch_batching(self, interval_s: float = 1.0, cap: int = 5000):
        """Coalesce read-path access bumps (``internal/memory/access_tracker.go``):
        hot retrieval paths stop paying one UPDATE per read."""
        if self.touch_batcher is None:
            self.touch_batcher = AccessTouchBatcher(self.apply_touches, interval_s, cap)
        return self.touch_batcher

    # ------------------------------------------------------------ writes
    def save(self, mem: Memory, require_user: bool = True) -> dict:
        """``SaveWithResult``: returns {id, action, supersedes, supersede_reason}."""
        scope = normalize_scope(mem.scope)
        if not scope.get(SCOPE_WORKSPACE):
            raise ValueError("workspace_id is required")
        if require_user and not scope.get(SCOPE_USER):
            raise ValueError("virtual_user_id is required")
        mem.scope = scope
        meta = dict(mem.metadata or {})
        now = time.time()
        res = {"id": "", "action": "added"}
        about_kind, about_key = meta.get(META_ABOUT_KIND), meta.get(META_ABOUT_KEY)
        title = mem.title or meta.get(META_TITLE) or None
        with self._tx() as db:
            if not mem.id and about_kind and about_key:
                row = db.execute(
                    "SELECT id FROM memory_entities WHERE workspace_id = ? AND "
                    "coalesce(virtual_user_id,'') = ? AND coalesce(agent_id,'') = ? AND "
                    "about_kind = ? AND about_key = ? AND forgotten = 0",
                    (scope[SCOPE_WORKSPACE], scope.get(SCOPE_USER, ""), scope.get(SCOPE_AGENT, ""),
                     about_kind, about_key)).fetchone()
                if row:
                    mem.id = row[0]
                    db.execute("UPDATE memory_entities SET metadata = ?, updated_at = ?, title = "
                               "coalesce(?, title), kind = ? WHERE id = ?",
                               (json.dumps(meta), now, title, mem.type, mem.id))
                    sup = self._supersede_active(db, mem.id, None)
                    res.update(action="auto_superseded", supersedes=sup,
                               supersede_reason="structured_key")
                else:
                    self._insert_entity(db, mem, meta, title, now)
            elif not mem.id:
                self._insert_entity(db, mem, meta, title, now)
            else:
                n = db.execute("UPDATE memory_entities SET metadata = ?, updated_at = ?, kind = ?, "
                               "title = coalesce(?, title) WHERE id = ? AND forgotten = 0",
                               (json.dumps(meta), now, mem.type, title, mem.id)).rowcount
                if not n:
                    raise NotFound(mem.id)
            oid = self._insert_observation(db, mem, now)
            if res["action"] == "auto_superseded":
                self._log_vectors(db, "delete", res["supersedes"])
                db.execute("UPDATE memory_observations SET superseded_by = ? WHERE id IN (%s)"
                           % ",".join("?" * len(res["supersedes"])), [oid] + res["supersedes"]) \
                    if res["supersedes"] else None
        mem.observation_id = oid
        res["id"] = mem.id
        res["observation_id"] = oid
        return res

    def _insert_entity(self, db, mem: Memory, meta: dict, title, now):
        mem.id = mem.id or new_id()
        s = mem.scope
        db.execute(
            "INSERT INTO memory_entities (id, workspace_id, kind, metadata, created_at, "
            "updated_at, expires_at, title, virtual_user_id, agent_id, source_type, trust_model, "
            "purpose, consent_category, about_kind, about_key) VALUES "
            "(?,?,?,?,?,?,?,?,?,?,?,?,?,?,?,?)",
            (mem.id, s[SCOPE_WORKSPACE], mem.type or "fact", json.dumps(meta), now, now,
             mem.expires_at, title, s.get(SCOPE_USER), s.get(SCOPE_AGENT),
             meta.get(META_SOURCE_TYPE), meta.get("trust_model"), meta.get(META_PURPOSE),
             meta.get(META_CONSENT_CATEGORY), meta.get(META_ABOUT_KIND),
             meta.get(META_ABOUT_KEY)))
        mem.created_at = now

    def _insert_observation(self, db, mem: Memory, now) -> str:
        oid = new_id()
        db.execute(
            "INSERT INTO memory_observations (id, entity_id, content, confidence, session_id, "
            "turn_range, observed_at, summary, body_size_bytes) VALUES (?,?,?,?,?,?,?,?,?)",
            (oid, mem.id, mem.content, float(mem.confidence), mem.session_id or None,
             json.dumps(mem.turn_range) if mem.turn_range else None, now, mem.summary or None,
             len(mem.content.encode())))
        title = mem.title or (mem.metadata or {}).get(META_TITLE) or ""
        if self.d.uses_fts_table:  # Postgres: the generated search_vector column
            db.execute("INSERT INTO memory_fts (content, title, obs_id) VALUES (?,?,?)",
                       (mem.content, title, oid))
        return oid

    # ------------------------------------------------------------ vector log
    def _log_vectors(self, db, op: str, obs_ids: list[str], only_embedded: bool = True):
        """Append ``op`` ("upsert" / "delete") for these observations to the change
        log every replica's vector index tails (``vector_changes``)."""
        if not obs_ids:
            return
        ph = ",".join("?" * len(obs_ids))
        cond = " AND o.embedding IS NOT NULL" if only_embedded else ""
        db.execute(f"INSERT INTO memory_vector_log (obs_id, workspace_id, op, at) SELECT o.id, "
                   f"e.workspace_id, ?, ? FROM memory_observations o JOIN memory_entities e ON "
                   f"e.id = o.entity_id WHERE o.id IN ({ph}){cond}",
                   [op, time.time()] + list(obs_ids))

    def vector_changes(self, after_seq: int, limit: int = 10000) -> list[tuple]:
        """(seq, obs_id, workspace, op) after ``after_seq``, oldest first."""
        return self._q("SELECT seq, obs_id, workspace_id, op FROM memory_vector_log WHERE "
                       "seq > ? ORDER BY seq LIMIT ?", (after_seq, limit))

    def max_vector_seq(self) -> int:
        return int(self._q("SELECT coalesce(max(seq), 0) FROM memory_vector_log")[0][0])

    def embedding_of(self, obs_ids: list[str]) -> dict[str, np.ndarray]:
        if not obs_ids:
            return {}
        ph = ",".join("?" * len(obs_ids))
        return {r[0]: self._vec(r[1]) for r in self._q(
            f"SELECT o.id, {self.d.vec_select()} FROM memory_observations o WHERE o.id IN "
            f"({ph}) AND o.embedding IS NOT NULL", obs_ids)}

    @staticmethod
    def _vec(v):
        return parse_vector_literal(v) if isinstance(v, str) else _f32(v)

    def _supersede_active(self, db, entity_id: str, new_oid) -> list[str]:
        now = time.time()
        ids = [r[0] for r in db.execute(
            "SELECT id FROM memory_observations o WHERE entity_id = ? AND " + _ACTIVE,
            (entity_id, now)).fetchall()]
        if ids and new_oid:
            self._log_vectors(db, "delete", ids)
            db.execute("UPDATE memory_observations SET superseded_by = ? WHERE id IN (%s)"
                       % ",".join("?" * len(ids)), [new_oid] + ids)
        return ids

    def update(self, entity_id: str, content: str | None = None, metadata: dict | None = None,
               confidence: float | None = None) -> Memory:
        """PATCH: a new observation supersedes the active one (history kept)."""
        cur = self.get(entity_id)
        if cur is None:
            raise NotFound(entity_id)
        mem = Memory(id=entity_id, type=cur.type, content=content if content is not None
                     else cur.content, confidence=confidence if confidence is not None
                     else cur.confidence, scope=cur.scope,
                     metadata={**cur.metadata, **(metadata or {})}, title=cur.title)
        with self._tx() as db:
            db.execute("UPDATE memory_entities SET metadata = ?, updated_at = ? WHERE id = ?",
                       (json.dumps(mem.metadata), time.time(), entity_id))
            oid = self._insert_observation(db, mem, time.time())
            old = [r[0] for r in db.execute(
                "SELECT id FROM memory_observations WHERE entity_id = ? AND id != ? AND "
                "superseded_by IS NULL", (entity_id, oid)).fetchall()]
            self._log_vectors(db, "delete", old)
            db.execute("UPDATE memory_observations SET superseded_by = ? WHERE entity_id = ? "
                       "AND id != ? AND superseded_by IS NULL", (oid, entity_id, oid))
        mem.observation_id = oid
        return mem

    def supersede(self, source_ids: list[str], mem: Memory) -> dict:
        """Replace several entities with one consolidated memory."""
        res = self.save(mem, require_user=False)
        with self._tx() as db:
            ph = ",".join("?" * len(source_ids))
            old = [r[0] for r in db.execute(
                f"SELECT id FROM memory_observations WHERE entity_id IN ({ph}) AND "
                f"superseded_by IS NULL AND entity_id != ?",
                list(source_ids) + [res["id"]]).fetchall()]
            self._log_vectors(db, "delete", old)
            db.execute(f"UPDATE memory_observations SET superseded_by = ? WHERE entity_id IN "
                       f"({ph}) AND superseded_by IS NULL AND entity_id != ?",
                       [res["observation_id"]] + list(source_ids) + [res["id"]])
        res["supersedes"] = list(source_ids)
        return res

    def set_embedding(self, obs_id: str, vec, model: str):
        arr = None if vec is None else np.asarray(vec, dtype=np.float32)
        param = None if arr is None else self.d.vec_param(arr.tobytes(), vector_literal(arr))
        with self._tx() as db:
            if arr is None:
                self._log_vectors(db, "delete", [obs_id])
            db.execute("UPDATE memory_observations SET embedding = ?, embedding_model = ? "
                       "WHERE id = ?", (param, model, obs_id))
            if arr is not None:
                self._log_vectors(db, "upsert", [obs_id])

    def link(self, workspace: str, source: str, target: str, rtype: str,
             weight: float = 1.0) -> str:
        rid = new_id()
        with self.lock:
            for e in (source, target):
                if not self._q("SELECT 1 FROM memory_entities WHERE id = ? AND workspace_id = ?",
                               (e, workspace)):
                    raise NotFound(e)
            self.db.execute("INSERT INTO memory_relations VALUES (?,?,?,?,?,?,?)",
                            (rid, workspace, source, target, rtype, weight, time.time()))
        return rid

    # ------------------------------------------------------------ deletes
    def forget(self, entity_id: str, workspace: str | None = None) -> bool:
        sql = "UPDATE memory_entities SET forgotten = 1, updated_at = ? WHERE id = ?"
        args = [time.time(), entity_id]
        if workspace:
            sql += " AND workspace_id = ?"
            args.append(workspace)
        with self._tx() as db:
            n = db.execute(sql, args).rowcount
            if n:
                obs = [r[0] for r in db.execute("SELECT id FROM memory_observations WHERE "
                                                "entity_id = ?", (entity_id,)).fetchall()]
                self._log_vectors(db, "delete", obs)
            return n > 0

    def _hard_delete(self, db, entity_ids: list[str]) -> list[str]:
        if not entity_ids:
            return []
        ph = ",".join("?" * len(entity_ids))
        obs = [r[0] for r in db.execute(
            f"SELECT id FROM memory_observations WHERE entity_id IN ({ph})", entity_ids)]
        if obs:
            self._log_vectors(db, "delete", obs)
            if self.d.uses_fts_table:
                oph = ",".join("?" * len(obs))
                db.execute(f"DELETE FROM memory_fts WHERE obs_id IN ({oph})", obs)
        db.execute(f"DELETE FROM memory_observations WHERE entity_id IN ({ph})", entity_ids)
        db.execute(f"DELETE FROM memory_relations WHERE source_entity_id IN ({ph}) OR "
                   f"target_entity_id IN ({ph})", entity_ids + entity_ids)
        db.execute(f"DELETE FROM memory_entities WHERE id IN ({ph})", entity_ids)
        return obs

    def delete_all(self, scope: dict) -> tuple[int, list[str]]:
        """DSAR erasure of every row in the scope (all agents when no agent_id)."""
        where, args = self._scope_where(normalize_scope(scope), strict=False)
        with self._tx() as db:
            ids = [r[0] for r in db.execute(f"SELECT e.id FROM memory_entities e WHERE {where}",
                                            args)]
            obs = self._hard_delete(db, ids)
        return len(ids), obs

    def batch_delete(self, scope: dict, limit: int = 500) -> tuple[int, list[str]]:
        where, args = self._scope_where(normalize_scope(scope), strict=False)
        with self._tx() as db:
            ids = [r[0] for r in db.execute(
                f"SELECT e.id FROM memory_entities e WHERE {where} LIMIT ?", args + [limit])]
            obs = self._hard_delete(db, ids)
        return len(ids), obs

    def expire(self, now: float | None = None) -> list[str]:
        """Retention: hard-delete entities past expires_at; returns observation ids."""
        now = now or time.time()
        with self._tx() as db:
            ids = [r[0] for r in db.execute(
                "SELECT id FROM memory_entities WHERE expires_at IS NOT NULL AND expires_at <= ?",
                (now,))]
            return self._hard_delete(db, ids)

    def purge_forgotten(self, older_than_s: float = 0.0) -> list[str]:
        cutoff = time.time() - older_than_s
        with self._tx() as db:
            ids = [r[0] for r in db.execute(
                "SELECT id FROM memory_entities WHERE forgotten = 1 AND updated_at <= ?",
                (cutoff,))]
            return self._hard_delete(db, ids)

    def revoke_consent(self, workspace: str, user: str, category: str) -> list[str]:
        """Consent revocation: delete that user's memories of the category."""
        with self._tx() as db:
            db.execute(self.d.upsert("consent_revocations", ["workspace_id", "virtual_user_id",
                                                            "category", "revoked_at"]),
                       (workspace, user, category, time.time()))
            ids = [r[0] for r in db.execute(
                "SELECT id FROM memory_entities WHERE workspace_id = ? AND virtual_user_id = ? "
                "AND consent_category = ?", (workspace, user, category))]
            return self._hard_delete(db, ids)

    def is_revoked(self, workspace: str, user: str, category: str | None) -> bool:
        if not category or not user:
            return False
        return bool(self._q("SELECT 1 FROM consent_revocations WHERE workspace_id = ? AND "
                            "virtual_user_id = ? AND category = ?", (workspace, user, category)))

    # ------------------------------------------------------------ reads
    def get(self, entity_id: str, workspace: str | None = None, touch: bool = False):
        where, args = "e.id = ?", [entity_id]
        if workspace:
            where += " AND e.workspace_id = ?"
            args.append(workspace)
        rows = self._select_active(where, args, limit=1)
        if not rows:
            return None
        m = self._row_to_memory(rows[0])
        if touch:
            self.touch([m.observation_id])
        return m

    def list(self, scope: dict, types=None, limit: int = 50, offset: int = 0,
             strict: bool = True) -> list[Memory]:
        where, args = self._scope_where(normalize_scope(scope), strict)
        if types:
            where += " AND e.kind IN (%s)" % ",".join("?" * len(types))
            args += list(types)
        rows = self._select_active(where, args, limit=limit + offset)
        return [self._row_to_memory(r) for r in rows[offset:]]

    def count(self, scope: dict, strict: bool = True) -> int:
        where, args = self._scope_where(normalize_scope(scope), strict)
        return len(self._select_active(where, args))

    def search(self, scope: dict, query: str, limit: int = 10, strict: bool = True):
        """Keyword FTS within one scope (``Retrieve``)."""
        if not query.strip():
            return self.list(scope, limit=limit, strict=strict)
        hits = self._fts_ids(query, 1000)
        if not hits:
            return []
        where, args = self._scope_where(normalize_scope(scope), strict)
        ids = list(hits)
        where += " AND o.id IN (%s)" % ",".join("?" * len(ids))
        rows = self._select_active(where, args + ids)
        mems = [self._row_to_memory(r) for r in rows]
        mems.sort(key=lambda m: hits[m.observation_id])
        mems = mems[:limit]
        self.touch([m.observation_id for m in mems])
        return mems

    def export_all(self, scope: dict) -> list[Memory]:
        where, args = self._scope_where(normalize_scope(scope), strict=False)
        return [self._row_to_memory(r) for r in self._select_active(where, args)]

    def related(self, entity_ids: list[str]) -> dict[str, list[dict]]:
        if not entity_ids:
            return {}
        ph = ",".join("?" * len(entity_ids))
        out: dict[str, list[dict]] = {}
        for s, t, rt, w in self._q(f"SELECT source_entity_id, target_entity_id, relation_type, "
                                   f"weight FROM memory_relations WHERE source_entity_id IN "
                                   f"({ph})", entity_ids):
            out.setdefault(s, []).append({"source_entity_id": s, "target_entity_id": t,
                                          "relation_type": rt, "weight": w})
        return out

    def traverse(self, workspace: str, seeds: list[str], relation_types=None, max_hops: int = 1,
                 limit: int = R.CANDIDATE_POOL) -> list[Memory]:
        seen, frontier = set(seeds), list(seeds)
        found: list[str] = []
        for _ in range(max(1, max_hops)):
            if not frontier:
                break
            ph = ",".join("?" * len(frontier))
            sql = (f"SELECT target_entity_id FROM memory_relations WHERE workspace_id = ? AND "
                   f"source_entity_id IN ({ph})")
            args = [workspace] + frontier
            if relation_types:
                sql += " AND relation_type IN (%s)" % ",".join("?" * len(relation_types))
                args += list(relation_types)
            nxt = []
            for (t,) in self._q(sql, args):
                if t not in seen:
                    seen.add(t)
                    nxt.append(t)
                    found.append(t)
            frontier = nxt
        if not found:
            return []
        ph = ",".join("?" * len(found[:limit]))
        rows = self._select_active(f"e.id IN ({ph})", found[:limit])
        return [self._row_to_memory(r) for r in rows]

    def conflicts(self, workspace: str, user: str = "", limit: int = 50) -> list[dict]:
        """Entities holding more than one active observation."""
        now = time.time()
        sql = ("SELECT e.id, count(o.id) FROM memory_entities e JOIN memory_observations o ON "
               "o.entity_id = e.id AND " + _ACTIVE + " WHERE e.workspace_id = ? AND "
               "e.forgotten = 0")
        args = [now, workspace]
        if user:
            sql += " AND e.virtual_user_id = ?"
            args.append(user)
        sql += " GROUP BY e.id HAVING count(o.id) > 1 LIMIT ?"
        args.append(limit)
        out = []
        for eid, n in self._q(sql, args):
            obs = self._q("SELECT id, content, confidence, observed_at FROM memory_observations o "
                          "WHERE entity_id = ? AND " + _ACTIVE + " ORDER BY observed_at DESC",
                          (eid, now))
            out.append({"entity_id": eid, "active_observations": n,
                        "observations": [{"id": o[0], "content": o[1], "confidence": o[2],
                                          "observed_at": o[3]} for o in obs]})
        return out

    def aggregate(self, workspace: str, group_by: str = "category") -> list[dict]:
        col = {"category": "coalesce(e.consent_category, '')", "agent": "coalesce(e.agent_id, '')",
               "day": self.d.day_expr("e.created_at"),
               "tier": "CASE WHEN e.virtual_user_id IS NOT NULL THEN 'user' WHEN e.agent_id IS "
                       "NOT NULL THEN 'agent' ELSE 'institutional' END",
               "type": "e.kind"}.get(group_by)
        if col is None:
            raise ValueError(f"unsupported groupBy {group_by!r}")
        rows = self._q(f"SELECT {col} AS k, count(*) FROM memory_entities e WHERE "
                       f"e.workspace_id = ? AND e.forgotten = 0 GROUP BY k ORDER BY k",
                       (workspace,))
        return [{"key": k, "count": n} for k, n in rows]

    def stats(self, workspace: str, model: str = "") -> dict:
        now = time.time()
        live = self._q("SELECT count(*) FROM memory_entities WHERE workspace_id = ? AND "
                       "forgotten = 0", (workspace,))[0][0]
        emb = self._q("SELECT count(DISTINCT e.id) FROM memory_entities e JOIN "
                      "memory_observations o ON o.entity_id = e.id AND " + _ACTIVE +
                      " WHERE e.workspace_id = ? AND e.forgotten = 0 AND o.embedding IS NOT NULL",
                      (now, workspace))[0][0]
        backlog = len(self.reembed_backlog(workspace, model, limit=1_000_000)) if model else 0
        return {"entities": live, "embedded": emb,
                "embedding_coverage": (emb / live) if live else 1.0, "reembed_backlog": backlog}

    def reembed_backlog(self, workspace: str | None, model: str, limit: int = 256):
        now = time.time()
        sql = ("SELECT o.id, o.content, e.workspace_id FROM memory_observations o JOIN "
               "memory_entities e ON e.id = o.entity_id WHERE e.forgotten = 0 AND " + _ACTIVE +
               " AND (o.embedding IS NULL OR coalesce(o.embedding_model, '') != ?)")
        args = [now, model]
        if workspace:
            sql += " AND e.workspace_id = ?"
            args.append(workspace)
        return self._q(sql + " LIMIT ?", args + [limit])

    def embeddings(self, workspace: str | None = None, model: str | None = None):
        """(obs_id, workspace, vector) of active embedded observations -- index warm-up."""
        now = time.time()
        sql = (f"SELECT o.id, e.workspace_id, {self.d.vec_select()} FROM memory_observations o "
               "JOIN "
               "memory_entities e ON e.id = o.entity_id WHERE e.forgotten = 0 AND " + _ACTIVE +
               " AND o.embedding IS NOT NULL")
        args = [now]
        if workspace:
            sql += " AND e.workspace_id = ?"
            args.append(workspace)
        if model:
            sql += " AND o.embedding_model = ?"
            args.append(model)
        return [(r[0], r[1], self._vec(r[2])) for r in self._q(sql, args)]

    def observation_ids_of(self, entity_ids: list[str]) -> list[str]:
        if not entity_ids:
            return []
        ph = ",".join("?" * len(entity_ids))
        return [r[0] for r in self._q(f"SELECT id FROM memory_observations WHERE entity_id IN "
                                      f"({ph})", entity_ids)]

    def entity_of_observations(self, obs_ids: list[str]) -> dict[str, str]:
        if not obs_ids:
            return {}
        ph = ",".join("?" * len(obs_ids))
        return dict(self._q(f"SELECT id, entity_id FROM memory_observations WHERE id IN ({ph})",
                            obs_ids))

    def inactive_observation_ids(self, obs_ids: list[str]) -> set[str]:
        if not obs_ids:
            return set()
        now = time.time()
        ph = ",".join("?" * len(obs_ids))
        return {r[0] for r in self._q(
            f"SELECT o.id FROM memory_observations o JOIN memory_entities e ON e.id = o.entity_id "
            f"WHERE o.id IN ({ph}) AND (o.superseded_by IS NOT NULL OR (o.valid_until IS NOT NULL "
            f"AND o.valid_until <= ?) OR e.forgotten = 1)", list(obs_ids) + [now])}

    # ------------------------------------------------------------ multi-tier
    def _candidates(self, req: MultiTierRequest, obs_filter: list[str] | None = None,
                    limit: int | None = R.CANDIDATE_POOL):
        where, args = self._tier_where(req)
        if obs_filter is not None:
            if not obs_filter:
                return []
            where += " AND o.id IN (%s)" % ",".join("?" * len(obs_filter))
            args += list(obs_filter)
        extra = ", e.source_type"
        rows = self._select_active(where, args, limit=limit, extra_cols=extra)
        out = []
        for r in rows:
            m = self._row_to_memory(r)
            if r[19]:
                m.metadata.setdefault(META_SOURCE_TYPE, r[19])
            out.append(m)
        return out

    def _merge_multi_mode(self, req: MultiTierRequest, mems: list[Memory]) -> list[Memory]:
        if req.seed_entity_ids:
            seen = {m.id for m in mems}
            for m in self.traverse(req.workspace_id, req.seed_entity_ids, req.relation_types,
                                   req.max_graph_hops):
                if m.id not in seen:
                    seen.add(m.id)
                    m.access_count = 0
                    mems.append(m)
        return mems

    def retrieve_multi_tier(self, req: MultiTierRequest) -> list[Memory]:
        """FTS-only multi-tier retrieval + Go-side ranking (``retrieve_multi_tier.go:134``)."""
        if req.query.strip():
            hits = self._fts_ids(req.query, 5000)
            mems = self._candidates(req, list(hits))
        else:
            mems = self._candidates(req)
        mems = self._merge_multi_mode(req, mems)
        if req.tiers:
            mems = [m for m in mems if m.tier in req.tiers]
        now = req.now or time.time()
        ranker = req.ranker or R.TierRanker()
        for m in mems:
            ref = m.accessed_at or m.created_at
            base = R.compute_score(m.confidence, m.access_count, ref, now,
                                   req.half_life.for_tier(m.tier))
            m.score = ranker.adjust(base, m.tier)
        mems.sort(key=lambda m: -m.score)
        mems = mems[: req.limit or R.DEFAULT_LIMIT]
        self.touch([m.observation_id for m in mems])
        return mems

    def retrieve_multi_tier_hybrid(self, req: MultiTierRequest,
                                   ann: list[tuple[str, float]]) -> list[Memory]:
        """RRF(FTS rank, cosine rank) x source weight x confidence x recency
        (``retrieve_multi_tier_hybrid.go:57-175``).  ``ann``: (obs_id, cosine) from
        the vector index, already over-fetched x4 and sorted by similarity."""
        if not req.query.strip() or not ann:
            return self.retrieve_multi_tier(req)
        fan = R.HYBRID_FANOUT
        hits = self._fts_ids(req.query, 5000)
        fts_c = self._candidates(req, list(hits), limit=None)
        fts_c.sort(key=lambda m: hits[m.observation_id])
        fts_rank, seen = {}, set()
        for m in fts_c:
            if m.id not in seen and len(fts_rank) < fan:
                seen.add(m.id)
                fts_rank[m.id] = len(fts_rank) + 1
        ann_ids = [o for o, _ in ann]
        cos_c = {m.observation_id: m for m in self._candidates(req, ann_ids, limit=None)}
        cos_rank = {}
        for oid, _sim in ann:  # per-entity dedup keeps the nearest observation
            m = cos_c.get(oid)
            if m is not None and m.id not in cos_rank and len(cos_rank) < fan:
                cos_rank[m.id] = len(cos_rank) + 1
        fused = R.rrf_ranks(fts_rank, cos_rank)
        by_id = {m.id: m for m in fts_c}
        for m in cos_c.values():
            by_id.setdefault(m.id, m)
        now = req.now or time.time()
        mems = []
        for eid, rrf in fused.items():
            m = by_id[eid]
            sw = SOURCE_TYPE_WEIGHT.get(m.metadata.get(META_SOURCE_TYPE, ""), 0.7)
            rec = R.recency_decay(now - m.observed_at, req.half_life.for_tier(m.tier))
            m.score = rrf * sw * (m.confidence if m.confidence is not None else 0.7) * rec
            mems.append(m)
        mems = self._merge_multi_mode(req, mems)
        if req.tiers:
            mems = [m for m in mems if m.tier in req.tiers]
        ranker = req.ranker or R.TierRanker()
        for m in mems:
            m.score = ranker.adjust(m.score, m.tier)
        mems.sort(key=lambda m: -m.score)
        mems = mems[: req.limit or R.DEFAULT_LIMIT]
        self.touch([m.observation_id for m in mems])
        return mems

    # ------------------------------------------------------------ compaction / ingest
    def list_workspace_ids(self) -> list[str]:
        """Workspaces holding live (not forgotten) memories (``ListWorkspaceIDs``):
        the compaction worker's discoverer."""
        return [r[0] for r in self._q("SELECT DISTINCT workspace_id FROM memory_entities "
                                      "WHERE forgotten = 0 ORDER BY workspace_id")]

    def compaction_candidates(self, workspace: str, older_than_s: float, min_count: int = 10,
                              limit: int = 20) -> list[dict]:
        """Per (user, agent) scope: the old active observations to summarise."""
        cutoff = time.time() - older_than_s
        now = time.time()
        groups = self._q(
            "SELECT coalesce(e.virtual_user_id,''), coalesce(e.agent_id,''), count(*) FROM "
            "memory_entities e JOIN memory_observations o ON o.entity_id = e.id AND " + _ACTIVE +
            " WHERE e.workspace_id = ? AND e.forgotten = 0 AND o.observed_at < ? AND "
            "e.kind != 'summary' GROUP BY 1, 2 HAVING count(*) >= ? LIMIT ?",
            (now, workspace, cutoff, min_count, limit))
        out = []
        for user, agent, n in groups:
            rows = self._q(
                "SELECT e.id, o.content FROM memory_entities e JOIN memory_observations o ON "
                "o.entity_id = e.id AND " + _ACTIVE + " WHERE e.workspace_id = ? AND "
                "coalesce(e.virtual_user_id,'') = ? AND coalesce(e.agent_id,'') = ? AND "
                "e.forgotten = 0 AND o.observed_at < ? AND e.kind != 'summary' ORDER BY "
                "o.observed_at", (now, workspace, user, agent, cutoff))
            out.append({"scope": {k: v for k, v in ((SCOPE_WORKSPACE, workspace),
                                                   (SCOPE_USER, user), (SCOPE_AGENT, agent)) if v},
                        "count": n, "entries": [{"id": r[0], "content": r[1]} for r in rows]})
        return out


    # ------------------------------------------------------------ tombstones / dims
    def tombstone_gc(self, workspace: str, min_age_s: float = 30 * 86400,
                     min_inactive: int = 20, keep_recent: int = 5) -> int:
        """``RunTombstoneGC`` (``internal/memory/tombstone.go:76``): in entities whose
        chain holds more than ``min_inactive`` inactive (superseded or expired)
        observations older than ``min_age_s``, delete all but the ``keep_recent``
        newest inactive ones.  Active observations are never touched."""
        if not workspace:
            raise ValueError("workspace_id is required")
        if keep_recent >= min_inactive:
            raise ValueError(f"keep_recent ({keep_recent}) must be less than min_inactive "
                             f"({min_inactive})")
        now = time.time()
        inactive = "(o.superseded_by IS NOT NULL OR (o.valid_until IS NOT NULL AND " \
                   "o.valid_until <= ?))"
        with self._tx() as db:
            ids = [r[0] for r in db.execute(
                f"WITH chains AS (SELECT o.entity_id FROM memory_observations o JOIN "
                f"memory_entities e ON e.id = o.entity_id WHERE e.workspace_id = ? AND "
                f"{inactive} AND o.observed_at < ? GROUP BY o.entity_id HAVING count(*) > ?), "
                f"ranked AS (SELECT o.id, row_number() OVER (PARTITION BY o.entity_id ORDER BY "
                f"o.observed_at DESC) AS rn FROM memory_observations o JOIN chains c ON "
                f"c.entity_id = o.entity_id JOIN memory_entities e ON e.id = o.entity_id AND "
                f"e.workspace_id = ? WHERE {inactive}) SELECT id FROM ranked WHERE rn > ?",
                (workspace, now, now - min_age_s, min_inactive, workspace, now,
                 keep_recent)).fetchall()]
            if ids:
                ph = ",".join("?" * len(ids))
                self._log_vectors(db, "delete", ids)
                if self.d.uses_fts_table:
                    db.execute(f"DELETE FROM memory_fts WHERE obs_id IN ({ph})", ids)
                db.execute(f"DELETE FROM memory_observations WHERE id IN ({ph})", ids)
        return len(ids)

    def record_dim_consent(self, target_dim: int):
        with self.lock:
            self.db.execute(self.d.upsert(CONSENT_TABLE, ["id", "target_dim", "recorded_at"]),
                            (1, int(target_dim), time.time()))

    def ensure_embedding_dim(self, dim: int) -> dict:
        """Reconcile the stored embedding dimension with the embedder's
        (``EnsureEmbeddingSchema``).  Changing it while embeddings exist discards
        them, so it needs one-shot consent for exactly ``dim``; the consent is
        consumed and the re-embed worker backfills.  On a real Postgres the
        ``vector(D)`` column is reshaped in one transaction and the HNSW index
        is built after the commit on an autocommit connection
        (``internal/memory/postgres/embedding_schema.go``)."""
        consent = self._q(f"SELECT target_dim FROM {CONSENT_TABLE} WHERE id = 1")
        consent_dim = int(consent[0][0]) if consent else None
        if isinstance(self.d, MemoryPostgres) and not self.d.emulated:
            return self._ensure_embedding_dim_pg(dim, consent_dim)
        cur = self._q("SELECT value FROM memory_meta WHERE key = 'embedding_dim'")
        cur_dim = int(cur[0][0]) if cur else None
        has = bool(self._q("SELECT 1 FROM memory_observations WHERE embedding IS NOT NULL "
                           "LIMIT 1"))
        MemoryPostgres.embedding_schema(dim, cur_dim, has, consent_dim)  # consent rules
        stmts = [f"DELETE FROM {CONSENT_TABLE}"]  # SQLite blobs carry any dimension
        if cur_dim not in (None, dim) and has:
            stmts.insert(0, "UPDATE memory_observations SET embedding = NULL, "
                            "embedding_model = NULL")
        dropped = cur_dim not in (None, dim) and has
        with self._tx() as db:
            if dropped:
                ids = [r[0] for r in db.execute("SELECT id FROM memory_observations WHERE "
                                                "embedding IS NOT NULL").fetchall()]
                for i in range(0, len(ids), 500):
                    self._log_vectors(db, "delete", ids[i:i + 500])
            for st in stmts:
                db.execute(st)
            db.execute(self.d.upsert("memory_meta", ["key", "value"]), ("embedding_dim",
                                                                          str(dim)))
        return {"from": cur_dim, "to": dim, "dropped_embeddings": dropped}

    def _ensure_embedding_dim_pg(self, dim: int, consent_dim: int | None) -> dict:
        P = MemoryPostgres
        with self._tx() as db:
            db.execute(f"SELECT pg_advisory_xact_lock({P.SCHEMA_LOCK})")
            row = db.execute(P.CURRENT_DIM_SQL).fetchall()
            cur_dim = P.parse_dim(row[0][0]) if row else None
            has = cur_dim is not None and bool(db.execute(
                "SELECT 1 FROM memory_observations WHERE embedding IS NOT NULL LIMIT 1"
            ).fetchall())
            stmts = P.embedding_schema(dim, cur_dim, has, consent_dim)
            dropped = cur_dim not in (None, dim) and has
            if dropped:
                ids = [r[0] for r in db.execute("SELECT id FROM memory_observations WHERE "
                                                "embedding IS NOT NULL").fetchall()]
                for i in range(0, len(ids), 500):
                    self._log_vectors(db, "delete", ids[i:i + 500])
            for st in stmts[1:]:  # the xact lock is already held
                db.execute(st)
            db.execute(self.d.upsert("memory_meta", ["key", "value"]), ("embedding_dim",
                                                                          str(dim)))
        self._build_embedding_index()
        return {"from": cur_dim, "to": dim, "dropped_embeddings": dropped}

    def _build_embedding_index(self):
        """CONCURRENTLY builds cannot run in a transaction block: flip the DB-API
        connection to autocommit for them (psycopg / psycopg2 ``.autocommit``)."""
        P = MemoryPostgres
        with self.lock:
            raw = self.db.raw
            prev = getattr(raw, "autocommit", False)
            raw.autocommit = True
            try:
                row = self.db.execute(P.INVALID_INDEX_SQL).fetchall()
                invalid = bool(row and row[0][0])
                stmts = P.embedding_index_schema(invalid)
                try:
                    for st in stmts[:-1]:
                        self.db.execute(st)
                finally:
                    self.db.execute(stmts[-1])  # session advisory unlock
            finally:
                raw.autocommit = prev


__all__ = ["MemoryStore", "MultiTierRequest", "NotFound", "AccessTouchBatcher",
           "EmbeddingDimConsentRequired", "MemorySQLite", "MemoryPostgres"]
