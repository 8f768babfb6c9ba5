"""SQL dialects of the warm session tier: SQLite (default, in-process) and
Postgres with weekly range partitions.

Reference: ``internal/session/providers/postgres/provider_partition.go``
(``EnsurePartitionsAhead`` / ``CreatePartition`` aligned to ISO weeks,
``DropPartition`` of ``<table>_wYYYY_WW`` children, ``ListPartitions`` from
``pg_inherits``), ``provider_write.go`` (upserts), migrations'
``create_weekly_partitions(table, start, end)``.

No Postgres driver is importable in this image, so the Postgres dialect is
exercised two ways: its DML (``$n`` placeholders, ``INSERT .. ON CONFLICT ..
DO UPDATE``) runs unchanged on SQLite (which accepts both forms) under the same
WarmStore tests, and its DDL / partition management is checked as generated
SQL plus the ISO-week arithmetic.  With a DB-API driver present
(``psycopg``/``psycopg2``/``pg8000``), :func:`connect_postgres` opens a real
connection and the same WarmStore code runs on it (``paramstyle`` "format").
"""
from __future__ import annotations

import datetime as dt
import re

# (table, time column, columns) -- the warm schema, one definition for both dialects
TABLES: dict[str, tuple[str, list[tuple[str, str]]]] = {
    "sessions": ("created", [("id", "TEXT"), ("namespace", "TEXT"), ("agent", "TEXT"),
                             ("workspace", "TEXT"), ("status", "TEXT"), ("created", "REAL"),
                             ("updated", "REAL"), ("expires", "REAL"), ("user", "TEXT"),
                             ("doc", "TEXT")]),
    "messages": ("ts", [("id", "TEXT"), ("session_id", "TEXT"), ("seq", "INTEGER"),
                        ("ts", "REAL"), ("role", "TEXT"), ("content", "TEXT"),
                        ("doc", "TEXT")]),
    "tool_calls": ("created", [("id", "TEXT"), ("session_id", "TEXT"), ("created", "REAL"),
                               ("name", "TEXT"), ("status", "TEXT"), ("doc", "TEXT")]),
    "provider_calls": ("created", [("id", "TEXT"), ("session_id", "TEXT"),
                                   ("created", "REAL"), ("provider", "TEXT"),
                                   ("model", "TEXT"), ("input", "INTEGER"),
                                   ("output", "INTEGER"), ("cost", "REAL"), ("doc", "TEXT")]),
    "events": ("created", [("id", "TEXT"), ("session_id", "TEXT"), ("created", "REAL"),
                           ("type", "TEXT"), ("doc", "TEXT")]),
    "eval_results": ("created", [("id", "TEXT"), ("session_id", "TEXT"), ("created", "REAL"),
                                 ("eval_id", "TEXT"), ("passed", "INTEGER"), ("score", "REAL"),
                                 ("doc", "TEXT")]),
}
INDEXES = [("sessions_ns", "sessions", "namespace, agent, created"),
           ("messages_sid", "messages", "session_id, seq")]
PARTITIONED = ["sessions", "messages", "tool_calls", "provider_calls", "events",
               "eval_results"]


class SQLiteDialect:
    name = "sqlite"
    paramstyle = "qmark"

    def q(self, sql: str) -> str:
        return sql

    def cols(self, table: str) -> list[str]:
        # "user" is a reserved word (a function) in Postgres: always quoted
        return ['"user"' if c == "user" else c for c, _ in TABLES[table][1]]

    def upsert(self, table: str) -> str:
        cols = self.cols(table)
        return self.q(f"INSERT OR REPLACE INTO {table} ({', '.join(cols)}) VALUES "
                      f"({', '.join('?' * len(cols))})")

    def schema(self) -> list[str]:
        out = []
        for t, (_, cols) in TABLES.items():
            body = ", ".join(f"{c} {ty}" + (" PRIMARY KEY" if c == "id" else "")
                             for c, ty in cols)
            out.append(f"CREATE TABLE IF NOT EXISTS {t} ({body})")
        out += [f"CREATE INDEX IF NOT EXISTS {n} ON {t}({c})" for n, t, c in INDEXES]
        # the Postgres conflict target of a partitioned table is (id, time column)
        out += [f"CREATE UNIQUE INDEX IF NOT EXISTS {t}_id_time ON {t}(id, {TABLES[t][0]})"
                for t in PARTITIONED]
        out.append("CREATE TABLE IF NOT EXISTS provider_usage (id INTEGER PRIMARY KEY "
                   "AUTOINCREMENT, workspace TEXT, created REAL, doc TEXT)")
        return out


_PG_TYPES = {"TEXT": "TEXT", "REAL": "DOUBLE PRECISION", "INTEGER": "BIGINT"}


class PostgresDialect(SQLiteDialect):
    """``paramstyle``: "dollar" ($1..$n, the server-native form) or "format"
    (%s, what psycopg / pg8000 take)."""
    name = "postgres"

    def __init__(self, paramstyle: str = "dollar"):
        self.paramstyle = paramstyle

    def q(self, sql: str) -> str:
        if self.paramstyle == "format":
            return sql.replace("?", "%s")
        n = iter(range(1, 10_000))
        return re.sub(r"\?", lambda _: f"${next(n)}", sql)

    def upsert(self, table: str) -> str:
        cols = self.cols(table)
        tcol = TABLES[table][0]
        key = f"id, {tcol}" if table in PARTITIONED else "id"
        sets = ", ".join(f"{c} = EXCLUDED.{c}" for c in cols if c not in ("id", tcol))
        # (SQLite accepts this statement verbatim, which the dialect tests rely on)
        return self.q(f"INSERT INTO {table} ({', '.join(cols)}) VALUES "
                      f"({', '.join('?' * len(cols))}) ON CONFLICT ({key}) DO UPDATE SET {sets}")

    def schema(self) -> list[str]:
        out = []
        for t, (tcol, cols) in TABLES.items():
            body = ", ".join(f'"{c}" {_PG_TYPES[ty]}' if c == "user" else f"{c} {_PG_TYPES[ty]}"
                             for c, ty in cols)
            out.append(f"CREATE TABLE IF NOT EXISTS {t} ({body}, PRIMARY KEY (id, {tcol})) "
                       f"PARTITION BY RANGE ({tcol})")
        out += [f"CREATE INDEX IF NOT EXISTS {n} ON {t}({c})" for n, t, c in INDEXES]
        out.append("CREATE TABLE IF NOT EXISTS provider_usage (id BIGSERIAL PRIMARY KEY, "
                   "workspace TEXT, created DOUBLE PRECISION, doc TEXT)")
        out.append(CREATE_WEEKLY_PARTITIONS_FN)
        return out

    # ---------------------------------------------------------------- partitions
    def create_partition(self, table: str, week_start: dt.date) -> str:
        return f"SELECT create_weekly_partitions('{table}', DATE '{week_start.isoformat()}', " \
               f"DATE '{(week_start + dt.timedelta(days=7)).isoformat()}')"

    def drop_partitions(self, day: dt.date) -> list[str]:
        sfx = partition_suffix(day)
        return [f'DROP TABLE IF EXISTS "{t}_{sfx}"' for t in reversed(PARTITIONED)]

    def list_partitions(self) -> str:
        return ("SELECT c.relname, pg_get_expr(c.relpartbound, c.oid) FROM pg_class c "
                "JOIN pg_inherits i ON i.inhrelid = c.oid JOIN pg_class parent ON "
                "parent.oid = i.inhparent JOIN pg_namespace n ON n.oid = parent.relnamespace "
                "WHERE parent.relname = 'sessions' AND n.nspname = current_schema() "
                "AND c.relispartition ORDER BY c.relname")


# epoch-second bounds for a week [start, end), one child per partitioned table;
# returns how many children it created (0 = the week already existed)
CREATE_WEEKLY_PARTITIONS_FN = """
CREATE OR REPLACE FUNCTION create_weekly_partitions(parent TEXT, start_d DATE, end_d DATE)
RETURNS INTEGER LANGUAGE plpgsql AS $$
DECLARE
  child TEXT := parent || '_w' || to_char(start_d, 'IYYY') || '_' || to_char(start_d, 'IW');
BEGIN
  IF to_regclass(child) IS NOT NULL THEN RETURN 0; END IF;
  EXECUTE format('CREATE TABLE %I PARTITION OF %I FOR VALUES FROM (%s) TO (%s)', child, parent,
                 extract(epoch FROM start_d::timestamptz), extract(epoch FROM end_d::timestamptz));
  RETURN 1;
END $$"""


# ------------------------------------------------------------------ ISO weeks
def iso_week_start(day: dt.date) -> dt.date:
    """Monday of ``day``'s ISO week."""
    y, w, _ = day.isocalendar()
    return dt.date.fromisocalendar(y, w, 1)


def partition_suffix(day: dt.date) -> str:
    y, w, _ = day.isocalendar()
    return f"w{y:04d}_{w:02d}"


def _parse_bound(expr: str):
    m = re.search(r"FROM \('?([\d.]+)'?\) TO \('?([\d.]+)'?\)", expr)
    return (float(m.group(1)), float(m.group(2))) if m else None


class PartitionManager:
    """Weekly partition upkeep (``provider_partition.go``): keep the current
    week and ``weeks_ahead`` more created; drop whole weeks that ended before
    the retention horizon.  ``execute(sql) -> rows`` is the connection."""

    def __init__(self, execute, dialect: PostgresDialect | None = None):
        self.execute = execute
        self.d = dialect or PostgresDialect()

    def ensure_ahead(self, weeks_ahead: int = 2, now: dt.datetime | None = None) -> int:
        now = now or dt.datetime.now(dt.timezone.utc)
        created = 0
        for i in range(weeks_ahead + 1):
            week = iso_week_start((now + dt.timedelta(days=7 * i)).date())
            for t in PARTITIONED:
                rows = self.execute(self.d.create_partition(t, week))
                created += int(rows[0][0]) if rows else 0
        return created

    def list(self) -> list[dict]:
        out = []
        for name, expr in self.execute(self.d.list_partitions()):
            b = _parse_bound(expr)
            if b:
                out.append({"name": name, "start": b[0], "end": b[1]})
        return out

    def drop_older_than(self, horizon: dt.datetime) -> list[str]:
        """Drop every week whose end is at or before ``horizon``."""
        dropped = []
        cutoff = horizon.timestamp()
        for p in self.list():
            if p["end"] <= cutoff:
                day = dt.datetime.fromtimestamp(p["start"], dt.timezone.utc).date()
                for sql in self.d.drop_partitions(day):
                    self.execute(sql)
                dropped.append(partition_suffix(day))
        return dropped


def connect_postgres(dsn: str):
    """A DB-API connection from whichever Postgres driver is installed."""
    for mod in ("psycopg", "psycopg2", "pg8000.dbapi"):
        try:
            m = __import__(mod, fromlist=["connect"])
        except ImportError:
            continue
        return m.connect(dsn), PostgresDialect(paramstyle="format")
    raise RuntimeError("no Postgres driver (psycopg, psycopg2 or pg8000) is installed; the "
                       "warm tier runs on SQLite (--db PATH)")
