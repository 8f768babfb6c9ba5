"""The memory store under the Postgres dialect (sqldialect.MemoryPostgres): every
test of test_memory.py re-runs with the Postgres DML ($n placeholders, ON
CONFLICT upserts, window-function tombstone GC) executing on SQLite, plus the
Postgres-only pieces checked as generated SQL (DDL with tsvector + pgvector,
websearch_to_tsquery / ts_rank_cd search, the embedding-dimension reconcile),
the tombstone GC, the multi-replica vector log and the dimension consent.
(No Postgres server or driver in this image: parity with a live pgvector is
unpinned.)"""
import asyncio
import os
import time

import numpy as np
import pytest

import test_memory as tm
from omnia_amd.memory import retrieval as R
from omnia_amd.memory import store as store_mod
from omnia_amd.memory.embedding import HashEmbedder
from omnia_amd.memory.model import Memory
from omnia_amd.memory.service import MemoryService
from omnia_amd.memory.sqldialect import (EmbeddingDimConsentRequired, MemoryPostgres,
                                         MemorySQLite, vector_literal)
from omnia_amd.memory.store import MemoryStore, MultiTierRequest

# re-collect the whole dialect-agnostic suite under the Postgres dialect
for _name in dir(tm):
    if _name.startswith("test_"):
        globals()[_name] = getattr(tm, _name)


@pytest.fixture(autouse=True)
def _postgres_dialect(monkeypatch):
    monkeypatch.setattr(store_mod, "default_dialect", lambda: MemoryPostgres(emulate=True))


def test_dialect_is_postgres_here():
    assert MemoryStore().d.name == "postgres"


def test_postgres_sql_generation():
    pg = MemoryPostgres()
    assert pg.q("SELECT a FROM t WHERE x = ? AND y = 'it''s ?' AND z IN (?,?)") == \
        "SELECT a FROM t WHERE x = $1 AND y = 'it''s ?' AND z IN ($2,$3)"
    assert MemoryPostgres(paramstyle="format").q("x = ? AND y = ?") == "x = %s AND y = %s"
    up = pg.upsert("consent_revocations", ["workspace_id", "virtual_user_id", "category",
                                           "revoked_at"])
    assert "ON CONFLICT (workspace_id, virtual_user_id, category) DO UPDATE SET revoked_at = " \
           "excluded.revoked_at" in up
    ddl = "\n".join(pg.schema())
    assert "search_vector tsvector GENERATED ALWAYS AS (to_tsvector('english'" in ddl
    assert "USING gin(search_vector)" in ddl and "BIGSERIAL" in ddl
    assert "CREATE EXTENSION IF NOT EXISTS vector" in ddl and "fts5" not in ddl
    sql, args = pg.fts_search("dark roast -decaf", 7)
    assert "websearch_to_tsquery('english', ?)" in sql and "ts_rank_cd" in sql
    assert args == ["dark roast -decaf", 7] and not pg.uses_fts_table
    assert pg.vec_param(b"x", "[1,2]") == "[1,2]" and pg.vec_select() == "o.embedding::text"
    assert vector_literal(np.array([0.5, -1.25], np.float32)) == "[0.5,-1.25]"
    assert MemorySQLite().upsert("memory_meta", ["key", "value"]).startswith(
        "INSERT OR REPLACE INTO memory_meta")


def test_embedding_schema_reconcile_rules():
    es = MemoryPostgres.embedding_schema
    fresh = es(384, None, False, None)
    assert "ALTER TABLE memory_observations ADD COLUMN embedding vector(384)" in fresh
    # the CONCURRENTLY index build is never part of the transactional list
    assert not any("CONCURRENTLY" in s or "hnsw" in s for s in fresh)
    idx = MemoryPostgres.embedding_index_schema(False)
    assert any("CREATE INDEX CONCURRENTLY" in s and "USING hnsw (embedding vector_cosine_ops)"
               in s for s in idx)
    assert idx[0].startswith("SELECT pg_advisory_lock(") and idx[-1].startswith(
        "SELECT pg_advisory_unlock(")
    assert any("DROP INDEX CONCURRENTLY" in s for s in MemoryPostgres.embedding_index_schema(True))
    assert not any("DROP COLUMN" in s for s in fresh)
    same = es(384, 384, True, None)
    assert not any("ALTER TABLE" in s for s in same)
    empty = es(768, 384, False, None)  # no data: reshape without consent
    assert any("DROP COLUMN embedding" in s for s in empty)
    with pytest.raises(EmbeddingDimConsentRequired):
        es(768, 384, True, None)
    with pytest.raises(EmbeddingDimConsentRequired):
        es(768, 384, True, 1024)  # consent for another target does not count
    ok = es(768, 384, True, 768)
    assert ok[-1].startswith("DELETE FROM memory_embedding_dim_change_consent")
    with pytest.raises(ValueError):
        es(4096, None, False, None)  # beyond the HNSW cap


class _FakePG:
    """DB-API stand-in for a real Postgres: records every statement with the
    connection's autocommit state and whether an explicit transaction is open;
    answers the catalog probes (column ``vector(384)`` with data, an invalid
    leftover index)."""

    def __init__(self, dim="vector(384)", has=True, consent=None, invalid=True):
        self.autocommit = False
        self.in_tx = False
        self.log = []
        self.dim, self.has, self.consent, self.invalid = dim, has, consent, invalid

    def cursor(self):
        return self

    def execute(self, sql, args=()):
        up = sql.strip().upper()
        if up.startswith("BEGIN"):
            self.in_tx = True
        self.log.append((sql, self.autocommit, self.in_tx))
        if up in ("COMMIT", "ROLLBACK"):
            self.in_tx = False
        if "format_type" in sql:
            self.rows = [(self.dim,)] if self.dim else []
        elif "embedding IS NOT NULL" in sql and "SELECT 1" in sql:
            self.rows = [(1,)] if self.has else []
        elif "SELECT id FROM memory_observations" in sql:
            self.rows = [("o1",), ("o2",)] if self.has else []
        elif "target_dim FROM" in sql:
            self.rows = [(self.consent,)] if self.consent else []
        elif "indisvalid" in sql:
            self.rows = [(True,)] if self.invalid else []
        else:
            self.rows = []

    def executemany(self, sql, rows):
        self.log.append((sql, self.autocommit, self.in_tx))

    def fetchall(self):
        return self.rows


def test_postgres_reshape_commits_before_concurrent_index_build():
    conn = _FakePG(consent=768)
    st = MemoryStore(dialect=MemoryPostgres(paramstyle="format"), conn=conn)
    conn.log.clear()
    out = st.ensure_embedding_dim(768)
    assert out == {"from": 384, "to": 768, "dropped_embeddings": True}
    sql = [s for s, _, _ in conn.log]
    # the dimension probe reads the catalog, never the (maybe absent) column
    probe = next(i for i, s in enumerate(sql) if "format_type" in s)
    assert not any("SELECT embedding" in s for s in sql[:probe])
    alter = [(s, ac, tx) for s, ac, tx in conn.log if s.startswith("ALTER TABLE")]
    assert [a[0].split()[3] for a in alter] == ["DROP", "ADD"]
    assert all(tx and not ac for _, ac, tx in alter)  # column change inside the tx
    commit = max(i for i, s in enumerate(sql) if s == "COMMIT")
    create = next(i for i, s in enumerate(sql) if "CREATE INDEX CONCURRENTLY" in s)
    drop = next(i for i, s in enumerate(sql) if "DROP INDEX CONCURRENTLY" in s)
    assert commit < drop < create  # after the commit, invalid leftover dropped first
    for i in (drop, create):
        _, ac, tx = conn.log[i]
        assert ac and not tx  # autocommit connection, no transaction block
    assert sql[-1].startswith("SELECT pg_advisory_unlock(")
    assert conn.autocommit is False  # restored
    # same dimension: no reshape, but the index is (idempotently) ensured
    conn2 = _FakePG(dim="vector(768)", invalid=False)
    st2 = MemoryStore(dialect=MemoryPostgres(paramstyle="format"), conn=conn2)
    conn2.log.clear()
    st2.ensure_embedding_dim(768)
    assert not any(s.startswith("ALTER TABLE") for s, _, _ in conn2.log)
    assert not any("DROP INDEX" in s for s, _, _ in conn2.log)
    # fresh database: no column yet -> add it, no consent needed
    conn3 = _FakePG(dim=None, has=False, invalid=False)
    st3 = MemoryStore(dialect=MemoryPostgres(paramstyle="format"), conn=conn3)
    assert st3.ensure_embedding_dim(384)["from"] is None
    # data present + no consent -> refused, nothing altered
    conn4 = _FakePG(consent=None)
    st4 = MemoryStore(dialect=MemoryPostgres(paramstyle="format"), conn=conn4)
    conn4.log.clear()
    with pytest.raises(EmbeddingDimConsentRequired, match="/admin/embedding-dimension-change"):
        st4.ensure_embedding_dim(768)
    assert not any(s.startswith("ALTER") or "CREATE INDEX" in s for s, _, _ in conn4.log)


def test_dimension_change_needs_consent_and_drops_embeddings(tmp_path):
    path = str(tmp_path / "m.db")

    async def go():
        svc = MemoryService(MemoryStore(path), HashEmbedder(32))
        await svc.save(tm.mem("coffee preference dark roast"))
        assert svc.store.stats(tm.WS)["embedded"] == 1
        with pytest.raises(EmbeddingDimConsentRequired):
            MemoryService(MemoryStore(path), HashEmbedder(64))
        st = MemoryStore(path)
        st.record_dim_consent(64)
        svc2 = MemoryService(st, HashEmbedder(64))
        assert st.stats(tm.WS)["embedded"] == 0  # dropped; the re-embed worker backfills
        assert await svc2.reembed() == 1 and st.stats(tm.WS)["embedded"] == 1
        # the consent was one-shot: a later change needs a fresh one
        with pytest.raises(EmbeddingDimConsentRequired):
            MemoryService(MemoryStore(path), HashEmbedder(32))

    asyncio.run(go())


def test_tombstone_gc_keeps_active_and_recent_inactive():
    st = MemoryStore()
    base = st.save(tm.mem("v0", metadata={"about_kind": "pref", "about_key": "coffee"}))
    eid = base["id"]
    for i in range(1, 30):  # 29 supersessions: 29 inactive + 1 active observation
        st.save(tm.mem(f"v{i}", metadata={"about_kind": "pref", "about_key": "coffee"}))
    old = time.time() - 40 * R.DAY
    with st.lock:
        st.db.execute("UPDATE memory_observations SET observed_at = observed_at - ? "
                      "WHERE superseded_by IS NOT NULL", (40 * R.DAY,))
    n = st.tombstone_gc(tm.WS, min_age_s=30 * R.DAY, min_inactive=20, keep_recent=5)
    assert n == 24
    left = st._q("SELECT superseded_by IS NULL FROM memory_observations WHERE entity_id = ?",
                 (eid,))
    assert sorted(r[0] for r in left) == [0] * 5 + [1]
    assert st.get(eid).content == "v29"  # the active observation untouched
    assert st.tombstone_gc(tm.WS, min_age_s=30 * R.DAY) == 0  # under the threshold now
    with pytest.raises(ValueError):
        st.tombstone_gc(tm.WS, min_inactive=5, keep_recent=5)
    assert old  # silence unused


def test_two_replicas_share_one_vector_source_of_truth(tmp_path):
    """Replica A writes; replica B's device index catches up from the store's
    vector log before its next ANN query (adds, supersessions, deletes)."""
    path = str(tmp_path / "shared.db")

    async def go():
        a = MemoryService(MemoryStore(path), HashEmbedder(64))
        b = MemoryService(MemoryStore(path), HashEmbedder(64))
        r = await a.save(tm.mem("the user loves hiking in the alps"))
        hits = await b.ann(tm.WS, "hiking in the alps", 5)
        assert [o for o, _ in hits] == [r["observation_id"]]
        up = await a.update(r["id"], content="the user now prefers sailing")
        hits = await b.ann(tm.WS, "sailing", 5)
        assert [o for o, _ in hits] == [up.observation_id]  # old vector gone on B too
        await a.delete_all({"workspace_id": tm.WS, "virtual_user_id": "u1"})
        assert await b.ann(tm.WS, "sailing", 5) == []
        assert b.vec_seq == b.store.max_vector_seq()

    asyncio.run(go())


@pytest.mark.parametrize("dialect", ["sqlite", "postgres"])
def test_tombstone_and_vector_log_on_both_dialects(dialect, monkeypatch):
    if dialect == "sqlite":
        monkeypatch.setattr(store_mod, "default_dialect", lambda: MemorySQLite())
    test_tombstone_gc_keeps_active_and_recent_inactive()


def test_redis_read_cache_hits_and_workspace_invalidation():
    """cache.go: list/search served from Redis until any write in the workspace
    bumps its version; a dead Redis degrades to the store."""
    from omnia_amd.memory.cache import CachedStore
    from omnia_amd.observability import metrics as M
    from omnia_amd.utils.resp import MiniRedis, RedisClient

    def count(op, res):
        return M.MEMORY_CACHE_LOOKUPS.labels(op, res)._value.get()

    async def go():
        r = MiniRedis()
        await r.start()
        svc = MemoryService(MemoryStore(), None)
        svc.cache = CachedStore(svc.store, RedisClient(r.url), ttl_s=60)
        scope = {"workspace_id": tm.WS, "virtual_user_id": "u1"}
        await svc.save(tm.mem("User prefers dark roast coffee"))
        h0, m0 = count("list", "hit"), count("list", "miss")
        a = await svc.list_cached(scope)
        b = await svc.list_cached(scope)
        assert [x.content for x in a] == [x.content for x in b]
        assert count("list", "miss") == m0 + 1 and count("list", "hit") == h0 + 1
        # another user's write in the same workspace invalidates every scope of it
        await svc.save(tm.mem("Another fact", user="u2"))
        await svc.list_cached(scope)
        assert count("list", "miss") == m0 + 2
        await svc.save(tm.mem("User lives in Chicago"))
        c = await svc.list_cached(scope)
        assert len(c) == 2  # fresh after the write
        s1 = await svc.search_cached(scope, "coffee")
        s2 = await svc.search_cached(scope, "coffee")
        assert [m.id for m in s1] == [m.id for m in s2] and s1
        await r.stop()
        # Redis unreachable: reads still answered by the store
        svc.cache = CachedStore(svc.store, RedisClient("redis://127.0.0.1:9/0", timeout=1.0),
                                ttl_s=60)
        d = await svc.list_cached(scope)
        assert len(d) == 2 and count("list", "error") >= 1

    asyncio.run(go())


def test_tombstone_worker_over_discovered_workspaces():
    from omnia_amd.memory.workers import TombstoneWorker

    st = MemoryStore()
    for i in range(8):
        st.save(tm.mem(f"v{i}", metadata={"about_kind": "k", "about_key": "x"}))
    with st.lock:
        st.db.execute("UPDATE memory_observations SET observed_at = observed_at - ? "
                      "WHERE superseded_by IS NOT NULL", (40 * R.DAY,))
    w = TombstoneWorker(MemoryService(st, None), min_inactive=3, keep_recent=1)
    assert w.run_once() == 6 and w.deleted == 6
    with pytest.raises(ValueError):
        TombstoneWorker(MemoryService(st, None), min_inactive=2, keep_recent=2)
