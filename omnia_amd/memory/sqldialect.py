"""SQL dialects of the memory store: SQLite (default, in-process) and Postgres
with pgvector (``internal/memory/postgres``: migrations, ``embedding_schema.go``).

The store writes every statement once, in qmark form; the dialect turns it into
the target's text:

* placeholders -- ``?`` -> ``$n`` (pgx / asyncpg style) or ``%s`` (DB-API
  ``format``), quoted literals left alone;
* upserts -- ``INSERT OR REPLACE`` (SQLite) vs ``INSERT .. ON CONFLICT (..) DO
  UPDATE SET .. = excluded..`` (Postgres; SQLite >= 3.24 runs it too);
* keyword search -- an FTS5 table with the porter stemmer and ``bm25`` (SQLite)
  vs the generated ``search_vector tsvector`` column + GIN index,
  ``websearch_to_tsquery`` and ``ts_rank_cd`` (Postgres);
* embeddings -- float32 blobs (SQLite) vs a ``vector(D)`` column with an HNSW
  ``vector_cosine_ops`` index (Postgres); :meth:`MemoryPostgres.embedding_schema`
  re-derives the reference's dimension reconcile: a reshape that would drop
  stored embeddings needs one-shot consent recorded for exactly that target
  dimension, and the consent is consumed by the migration; past 2,000
  dimensions pgvector cannot index, so the dimension is refused;
* the vector change log (``memory_vector_log``) every replica tails to keep its
  device-resident index in step with the shared store (BIGSERIAL vs
  AUTOINCREMENT).

No Postgres driver is importable in this image, so the Postgres dialect is
exercised two ways, as the session warm store's is: with ``emulate=True`` its
DML (``$n`` placeholders, ``ON CONFLICT`` upserts, window-function tombstone GC)
runs unchanged on SQLite under the same store tests, while the engine-specific
pieces (DDL, tsvector search, pgvector I/O, the dimension reconcile) are checked
as generated SQL.  With a DB-API driver present, :func:`connect_postgres` opens a
real connection (``paramstyle`` "format") and the same store code runs on it.
"""
from __future__ import annotations

import re

MAX_INDEXABLE_DIM = 2000  # pgvector HNSW cap (embedding_schema.go MaxIndexableEmbeddingDim)
CONSENT_TABLE = "memory_embedding_dim_change_consent"

_SQLITE_SCHEMA = """
CREATE TABLE IF NOT EXISTS memory_entities (
  id TEXT PRIMARY KEY, workspace_id TEXT NOT NULL, kind TEXT NOT NULL DEFAULT 'fact',
  metadata TEXT NOT NULL DEFAULT '{}', created_at REAL NOT NULL, updated_at REAL NOT NULL,
  expires_at REAL, title TEXT, virtual_user_id TEXT, agent_id TEXT,
  source_type TEXT, trust_model TEXT, purpose TEXT, consent_category TEXT,
  about_kind TEXT, about_key TEXT, forgotten INTEGER NOT NULL DEFAULT 0);
CREATE INDEX IF NOT EXISTS ix_ent_ws ON memory_entities(workspace_id, virtual_user_id, agent_id);
CREATE UNIQUE INDEX IF NOT EXISTS ux_ent_about ON memory_entities(
  workspace_id, coalesce(virtual_user_id, ''), coalesce(agent_id, ''), about_kind, about_key)
  WHERE about_kind IS NOT NULL AND forgotten = 0;
CREATE TABLE IF NOT EXISTS memory_observations (
  id TEXT PRIMARY KEY, entity_id TEXT NOT NULL, content TEXT NOT NULL,
  confidence REAL NOT NULL DEFAULT 0.7, session_id TEXT, turn_range TEXT,
  observed_at REAL NOT NULL, accessed_at REAL, access_count INTEGER NOT NULL DEFAULT 0,
  summary TEXT, body_size_bytes INTEGER, superseded_by TEXT, valid_until REAL,
  embedding BLOB, embedding_model TEXT);
CREATE INDEX IF NOT EXISTS ix_obs_ent ON memory_observations(entity_id, observed_at);
CREATE VIRTUAL TABLE IF NOT EXISTS memory_fts USING fts5(
  content, title, obs_id UNINDEXED, tokenize = 'porter unicode61');
CREATE TABLE IF NOT EXISTS memory_relations (
  id TEXT PRIMARY KEY, workspace_id TEXT NOT NULL, source_entity_id TEXT NOT NULL,
  target_entity_id TEXT NOT NULL, relation_type TEXT NOT NULL, weight REAL NOT NULL DEFAULT 1.0,
  created_at REAL NOT NULL);
CREATE INDEX IF NOT EXISTS ix_rel_src ON memory_relations(source_entity_id);
CREATE TABLE IF NOT EXISTS memory_meta (key TEXT PRIMARY KEY, value TEXT);
CREATE TABLE IF NOT EXISTS consent_revocations (
  workspace_id TEXT, virtual_user_id TEXT, category TEXT, revoked_at REAL,
  PRIMARY KEY (workspace_id, virtual_user_id, category));
CREATE TABLE IF NOT EXISTS memory_vector_log (
  seq INTEGER PRIMARY KEY AUTOINCREMENT, obs_id TEXT NOT NULL, workspace_id TEXT NOT NULL,
  op TEXT NOT NULL, at REAL NOT NULL);
CREATE TABLE IF NOT EXISTS memory_embedding_dim_change_consent (
  id INTEGER PRIMARY KEY CHECK (id = 1), target_dim INTEGER NOT NULL, recorded_at REAL);
"""

# the Postgres schema (migrations/*.up.sql equivalent); the embedding column is
# added by the dimension reconcile, not here, because its type carries the dim
_PG_SCHEMA = [
    "CREATE EXTENSION IF NOT EXISTS vector",
    "CREATE TABLE IF NOT EXISTS memory_entities (id TEXT PRIMARY KEY, workspace_id TEXT NOT "
    "NULL, kind TEXT NOT NULL DEFAULT 'fact', metadata TEXT NOT NULL DEFAULT '{}', created_at "
    "DOUBLE PRECISION NOT NULL, updated_at DOUBLE PRECISION NOT NULL, expires_at DOUBLE "
    "PRECISION, title TEXT, virtual_user_id TEXT, agent_id TEXT, source_type TEXT, "
    "trust_model TEXT, purpose TEXT, consent_category TEXT, about_kind TEXT, about_key TEXT, "
    "forgotten INTEGER NOT NULL DEFAULT 0)",
    "CREATE INDEX IF NOT EXISTS ix_ent_ws ON memory_entities(workspace_id, virtual_user_id, "
    "agent_id)",
    "CREATE UNIQUE INDEX IF NOT EXISTS ux_ent_about ON memory_entities(workspace_id, "
    "coalesce(virtual_user_id, ''), coalesce(agent_id, ''), about_kind, about_key) WHERE "
    "about_kind IS NOT NULL AND forgotten = 0",
    "CREATE TABLE IF NOT EXISTS memory_observations (id TEXT PRIMARY KEY, entity_id TEXT NOT "
    "NULL, content TEXT NOT NULL, confidence DOUBLE PRECISION NOT NULL DEFAULT 0.7, session_id "
    "TEXT, turn_range TEXT, observed_at DOUBLE PRECISION NOT NULL, accessed_at DOUBLE "
    "PRECISION, access_count INTEGER NOT NULL DEFAULT 0, summary TEXT, body_size_bytes "
    "INTEGER, superseded_by TEXT, valid_until DOUBLE PRECISION, embedding_model TEXT, "
    "search_vector tsvector GENERATED ALWAYS AS (to_tsvector('english', coalesce(content, "
    "''))) STORED)",
    "CREATE INDEX IF NOT EXISTS ix_obs_ent ON memory_observations(entity_id, observed_at)",
    "CREATE INDEX IF NOT EXISTS ix_obs_search ON memory_observations USING gin(search_vector)",
    "CREATE TABLE IF NOT EXISTS memory_relations (id TEXT PRIMARY KEY, workspace_id TEXT NOT "
    "NULL, source_entity_id TEXT NOT NULL, target_entity_id TEXT NOT NULL, relation_type TEXT "
    "NOT NULL, weight DOUBLE PRECISION NOT NULL DEFAULT 1.0, created_at DOUBLE PRECISION NOT "
    "NULL)",
    "CREATE INDEX IF NOT EXISTS ix_rel_src ON memory_relations(source_entity_id)",
    "CREATE TABLE IF NOT EXISTS memory_meta (key TEXT PRIMARY KEY, value TEXT)",
    "CREATE TABLE IF NOT EXISTS consent_revocations (workspace_id TEXT, virtual_user_id TEXT, "
    "category TEXT, revoked_at DOUBLE PRECISION, PRIMARY KEY (workspace_id, virtual_user_id, "
    "category))",
    "CREATE TABLE IF NOT EXISTS memory_vector_log (seq BIGSERIAL PRIMARY KEY, obs_id TEXT NOT "
    "NULL, workspace_id TEXT NOT NULL, op TEXT NOT NULL, at DOUBLE PRECISION NOT NULL)",
    f"CREATE TABLE IF NOT EXISTS {CONSENT_TABLE} (id INTEGER PRIMARY KEY CHECK (id = 1), "
    "target_dim INTEGER NOT NULL, recorded_at DOUBLE PRECISION)",
]

# conflict targets of the tables the store upserts into
_CONFLICT = {"memory_meta": ("key",), "consent_revocations": ("workspace_id", "virtual_user_id",
                                                             "category"),
             CONSENT_TABLE: ("id",)}
_PLACEHOLDER = re.compile(r"'(?:[^']|'')*'|\?")


class EmbeddingDimConsentRequired(RuntimeError):
    pass


class MemorySQLite:
    name = "sqlite"
    paramstyle = "qmark"
    emulated = False

    def q(self, sql: str) -> str:
        return sql

    def schema(self) -> list[str]:
        return [s.strip() for s in _SQLITE_SCHEMA.split(";") if s.strip()]

    def begin(self) -> str:
        return "BEGIN IMMEDIATE"

    def upsert(self, table: str, cols: list[str]) -> str:
        return (f"INSERT OR REPLACE INTO {table} ({', '.join(cols)}) VALUES "
                f"({', '.join('?' * len(cols))})")

    # ---- keyword search (FTS5 + porter; bm25: lower is better)
    uses_fts_table = True

    def fts_search(self, expr: str, limit: int) -> tuple[str, list]:
        return ("SELECT obs_id, bm25(memory_fts) FROM memory_fts WHERE memory_fts MATCH ? "
                "ORDER BY bm25(memory_fts) LIMIT ?", [expr, limit])

    # ---- embeddings
    def vec_param(self, blob: bytes | None, vec_text: str | None):
        return blob

    def vec_select(self, col: str = "o.embedding") -> str:
        return col

    def day_expr(self, col: str) -> str:
        return f"date({col}, 'unixepoch')"


class MemoryPostgres(MemorySQLite):
    """``paramstyle``: "dollar" ($1..$n, pgx/asyncpg) or "format" (%s, DB-API).
    ``emulate=True``: run the DML on SQLite (tests) -- schema, keyword search
    and vector I/O stay SQLite's there, every other statement is this dialect's."""

    name = "postgres"

    def __init__(self, paramstyle: str = "dollar", emulate: bool = False):
        self.paramstyle = paramstyle
        self.emulated = emulate

    def q(self, sql: str) -> str:
        n = [0]

        def sub(m):
            if m.group(0) != "?":
                return m.group(0)
            n[0] += 1
            return f"${n[0]}" if self.paramstyle == "dollar" else "%s"

        sql = _PLACEHOLDER.sub(sub, sql)
        return sql

    def schema(self) -> list[str]:
        return MemorySQLite.schema(self) if self.emulated else list(_PG_SCHEMA)

    def begin(self) -> str:
        return "BEGIN IMMEDIATE" if self.emulated else "BEGIN"

    def upsert(self, table: str, cols: list[str]) -> str:
        keys = _CONFLICT[table]
        rest = [c for c in cols if c not in keys]
        sets = ", ".join(f"{c} = excluded.{c}" for c in rest)
        return (f"INSERT INTO {table} ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))}) "
                f"ON CONFLICT ({', '.join(keys)}) DO " + (f"UPDATE SET {sets}" if rest
                                                           else "NOTHING"))

    @property
    def uses_fts_table(self) -> bool:  # type: ignore[override]
        return self.emulated

    def fts_search(self, expr: str, limit: int) -> tuple[str, list]:
        if self.emulated:
            return MemorySQLite.fts_search(self, expr, limit)
        # websearch syntax goes to Postgres verbatim; negate the rank so that, as
        # with bm25, lower is better for the callers
        return ("SELECT o.id, -ts_rank_cd(o.search_vector, q) FROM memory_observations o, "
                "websearch_to_tsquery('english', ?) q WHERE o.search_vector @@ q "
                "ORDER BY 2 LIMIT ?", [expr, limit])

    def vec_param(self, blob: bytes | None, vec_text: str | None):
        return blob if self.emulated else vec_text

    def vec_select(self, col: str = "o.embedding") -> str:
        return col if self.emulated else f"{col}::text"

    def day_expr(self, col: str) -> str:
        return (MemorySQLite.day_expr(self, col) if self.emulated else
                f"to_char(to_timestamp({col}), 'YYYY-MM-DD')")

    # ---- embedding dimension reconcile (embedding_schema.go:125)
    # the column's dimension from the catalog (the column may not exist yet:
    # _PG_SCHEMA never creates it) -- ``currentEmbeddingDim``, embedding_schema.go
    CURRENT_DIM_SQL = ("SELECT format_type(a.atttypid, a.atttypmod) FROM pg_attribute a "
                       "WHERE a.attrelid = 'memory_observations'::regclass AND "
                       "a.attname = 'embedding' AND NOT a.attisdropped")
    INDEX_NAME = "idx_memory_observations_embedding"
    INVALID_INDEX_SQL = ("SELECT NOT i.indisvalid FROM pg_index i JOIN pg_class c ON "
                         "c.oid = i.indexrelid WHERE c.relname = "
                         "'idx_memory_observations_embedding'")
    SCHEMA_LOCK, INDEX_LOCK = 1309, 1310

    @staticmethod
    def parse_dim(format_type: str | None) -> int | None:
        import re

        m = re.fullmatch(r"vector\((\d+)\)", (format_type or "").strip())
        return int(m.group(1)) if m else None

    @staticmethod
    def embedding_schema(dim: int, current_dim: int | None, has_data: bool,
                         consent_dim: int | None) -> list[str]:
        """TRANSACTIONAL statements that bring ``memory_observations.embedding`` to
        ``vector(dim)`` (``reconcileEmbeddingTx``): advisory xact lock, drop / add
        the column, settle the consent.  ``current_dim`` None = no column yet.
        Raises when the reshape would drop stored embeddings without consent for
        exactly ``dim``.  The HNSW index is built AFTER the commit, outside any
        transaction (:meth:`embedding_index_schema`)."""
        if dim <= 0:
            raise ValueError(f"invalid embedding dimension {dim}")
        if dim > MAX_INDEXABLE_DIM:
            raise ValueError(f"embedding dimension {dim} exceeds the maximum indexable "
                             f"dimension {MAX_INDEXABLE_DIM} (pgvector HNSW cap)")
        out = [f"SELECT pg_advisory_xact_lock({MemoryPostgres.SCHEMA_LOCK})"]
        if current_dim == dim:
            return out + [f"DELETE FROM {CONSENT_TABLE}"]  # stale consent cleared
        destructive = current_dim is not None and has_data
        if destructive and consent_dim != dim:
            raise EmbeddingDimConsentRequired(
                f"changing the embedding dimension to {dim} would discard existing embeddings "
                f"and requires one-shot consent (recorded target={consent_dim}); record it via "
                f"POST /admin/embedding-dimension-change {{\"target_dim\": {dim}}} or "
                f"INSERT INTO {CONSENT_TABLE} (id, target_dim, recorded_at) VALUES (1, {dim}, "
                f"now())")
        if current_dim is not None:
            out.append("ALTER TABLE memory_observations DROP COLUMN embedding")
        out.append(f"ALTER TABLE memory_observations ADD COLUMN embedding vector({dim})")
        out.append(f"DELETE FROM {CONSENT_TABLE}")  # consumed (or stale)
        return out

    @staticmethod
    def embedding_index_schema(invalid_leftover: bool) -> list[str]:
        """AUTOCOMMIT statements (``ensureEmbeddingIndexes``): Postgres refuses
        ``CREATE INDEX CONCURRENTLY`` inside a transaction block, so the build
        runs on an autocommit connection under a SESSION advisory lock, after
        dropping an invalid index a failed concurrent build left behind."""
        out = [f"SELECT pg_advisory_lock({MemoryPostgres.INDEX_LOCK})"]
        if invalid_leftover:
            out.append(f"DROP INDEX CONCURRENTLY IF EXISTS {MemoryPostgres.INDEX_NAME}")
        out.append(f"CREATE INDEX CONCURRENTLY IF NOT EXISTS {MemoryPostgres.INDEX_NAME} "
                   "ON memory_observations USING hnsw (embedding vector_cosine_ops) WITH "
                   "(m = 16, ef_construction = 64)")
        out.append(f"SELECT pg_advisory_unlock({MemoryPostgres.INDEX_LOCK})")
        return out


def vector_literal(vec) -> str:
    """pgvector text input: ``[v1,v2,...]``."""
    return "[" + ",".join(f"{float(x):.7g}" for x in vec) + "]"


def parse_vector_literal(s: str):
    import numpy as np

    return np.array([float(x) for x in s.strip("[]").split(",") if x], dtype=np.float32)


def connect_postgres(dsn: str):
    """A DB-API connection when a Postgres driver is importable (None otherwise)."""
    for mod in ("psycopg", "psycopg2", "pg8000.dbapi"):
        try:
            m = __import__(mod, fromlist=["connect"])
        except ImportError:
            continue
        return m.connect(dsn)
    return None
