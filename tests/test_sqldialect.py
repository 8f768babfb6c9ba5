"""Warm-tier SQL dialects (``internal/session/providers/postgres``): the
Postgres dialect's DML runs verbatim on SQLite under the full WarmStore
behaviour, its DDL declares weekly range partitions, and the partition manager
creates/drops ISO weeks (``provider_partition.go`` + its unit tests)."""
import datetime as dt
import sqlite3

import pytest

from omnia_amd.session.model import Message, ProviderCall, Session, ToolCall
from omnia_amd.session.sqldialect import (PARTITIONED, PartitionManager, PostgresDialect,
                                          SQLiteDialect, connect_postgres, iso_week_start,
                                          partition_suffix)
from omnia_amd.session.store import TieredSessionService, WarmStore


@pytest.fixture(params=["sqlite", "postgres-dml"])
def warm(request):
    if request.param == "sqlite":
        return WarmStore()
    # Postgres statements ($n placeholders, ON CONFLICT upserts, quoted "user") on a
    # SQLite connection: same rows, same answers
    return WarmStore(dialect=PostgresDialect("dollar"),
                     conn=sqlite3.connect(":memory:", check_same_thread=False),
                     schema_dialect=SQLiteDialect())


def test_warm_store_behaviour_is_dialect_independent(warm):
    import asyncio

    svc = TieredSessionService(warm=warm)
    s = svc.create(Session(id="s1", agent_name="a", namespace="ns", virtual_user_id="u1"))
    for i in range(3):
        asyncio.run(svc.append_message("s1", Message(role="user", content=f"m{i} needle"
                                                     if i == 1 else f"m{i}")))
    svc.create(Session(id="s2", agent_name="b", namespace="ns", virtual_user_id="u2"))
    svc.record("tool_calls", "s1", ToolCall(name="t", status="success"))
    svc.record("provider_calls", "s1", ProviderCall(provider="omnia", model="m",
                                                    input_tokens=5, output_tokens=2))
    svc.update_status("s1", "completed")
    got = warm.get_session("s1")
    assert got.status == "completed" and got.message_count == 3 and got.tool_call_count == 1
    assert [m.content for m in warm.messages("s1")] == ["m0", "m1 needle", "m2"]
    assert [x.id for x in warm.list_sessions(user="u1")] == ["s1"]
    assert [x.id for x in warm.list_sessions(q="needle")] == ["s1"]
    assert {x.id for x in warm.list_sessions(namespace="ns")} == {"s1", "s2"}
    assert warm.aggregate_provider_calls()[0]["inputTokens"] == 5
    # upsert of an existing message id updates in place (no duplicate row)
    m = warm.messages("s1")[0]
    m.content = "edited"
    warm.add_message("s1", m)
    assert [x.content for x in warm.messages("s1")][0] == "edited"
    assert len(warm.messages("s1")) == 3
    assert warm.delete_session("s1") and warm.get_session("s1") is None


def test_postgres_statements():
    d = PostgresDialect("dollar")
    up = d.upsert("messages")
    assert up.startswith("INSERT INTO messages (id, session_id, seq, ts, role, content, doc) "
                         "VALUES ($1, $2, $3, $4, $5, $6, $7) ON CONFLICT (id, ts) DO UPDATE SET")
    assert "ts = EXCLUDED.ts" not in up and "content = EXCLUDED.content" in up
    assert '"user" = EXCLUDED."user"' in d.upsert("sessions")
    assert d.q("SELECT a FROM t WHERE x=? AND y=?") == "SELECT a FROM t WHERE x=$1 AND y=$2"
    assert PostgresDialect("format").q("x=? AND y=?") == "x=%s AND y=%s"
    ddl = d.schema()
    assert any(s.startswith("CREATE TABLE IF NOT EXISTS sessions (") and
               s.endswith("PRIMARY KEY (id, created)) PARTITION BY RANGE (created)") and
               '"user" TEXT' in s and "created DOUBLE PRECISION" in s for s in ddl)
    assert any("messages" in s and "PARTITION BY RANGE (ts)" in s for s in ddl)
    assert any("BIGSERIAL" in s for s in ddl)
    assert any("create_weekly_partitions" in s and "plpgsql" in s for s in ddl)


def test_iso_weeks_across_year_boundaries():
    assert iso_week_start(dt.date(2026, 10, 16)) == dt.date(2026, 10, 12)  # a Friday
    assert partition_suffix(dt.date(2026, 10, 12)) == "w2026_42"
    # 2027-01-01 is a Friday in ISO week 2026-W53
    assert iso_week_start(dt.date(2027, 1, 1)) == dt.date(2026, 12, 28)
    assert partition_suffix(dt.date(2027, 1, 1)) == "w2026_53"
    assert partition_suffix(dt.date(2027, 1, 4)) == "w2027_01"
    # 2024-12-30 (Monday) already belongs to 2025-W01
    assert partition_suffix(dt.date(2024, 12, 30)) == "w2025_01"


class FakePG:
    """Records statements; create_weekly_partitions returns 1 the first time
    a (table, week) is seen; the catalogue query lists created sessions weeks."""

    def __init__(self):
        self.sql, self.weeks = [], {}

    def __call__(self, sql):
        self.sql.append(sql)
        if sql.startswith("SELECT create_weekly_partitions"):
            table = sql.split("'")[1]
            start = sql.split("DATE '")[1][:10]
            key = (table, start)
            fresh = key not in self.weeks
            self.weeks[key] = True
            return [(1 if fresh else 0,)]
        if "FROM pg_class" in sql:
            out = []
            for (t, start) in sorted(self.weeks):
                if t != "sessions":
                    continue
                d0 = dt.datetime.fromisoformat(start).replace(tzinfo=dt.timezone.utc)
                d1 = d0 + dt.timedelta(days=7)
                out.append((f"sessions_{partition_suffix(d0.date())}",
                            f"FOR VALUES FROM ('{d0.timestamp():.0f}') TO "
                            f"('{d1.timestamp():.0f}')"))
            return out
        if sql.startswith("DROP TABLE"):
            name = sql.split('"')[1]
            t, sfx = name.rsplit("_w", 1)
            for k in list(self.weeks):
                if k[0] == t and partition_suffix(dt.date.fromisoformat(k[1])) == "w" + sfx:
                    del self.weeks[k]
            return []
        raise AssertionError(sql)


def test_partition_manager_ensures_ahead_and_drops_expired():
    pg = FakePG()
    pm = PartitionManager(pg)
    now = dt.datetime(2026, 12, 24, 15, tzinfo=dt.timezone.utc)  # Thursday of W52
    assert pm.ensure_ahead(2, now) == 3 * len(PARTITIONED)
    assert pm.ensure_ahead(2, now) == 0  # idempotent
    starts = sorted({k[1] for k in pg.weeks})
    assert starts == ["2026-12-21", "2026-12-28", "2027-01-04"]
    assert [p["name"] for p in pm.list()] == ["sessions_w2026_52", "sessions_w2026_53",
                                             "sessions_w2027_01"]
    # retention horizon inside W53: only W52 (ended 2026-12-28) is dropped, children first
    dropped = pm.drop_older_than(dt.datetime(2026, 12, 30, tzinfo=dt.timezone.utc))
    assert dropped == ["w2026_52"]
    drops = [s for s in pg.sql if s.startswith("DROP")]
    assert drops[0] == 'DROP TABLE IF EXISTS "eval_results_w2026_52"' and \
        drops[-1] == 'DROP TABLE IF EXISTS "sessions_w2026_52"'
    assert {k[1] for k in pg.weeks} == {"2026-12-28", "2027-01-04"}


def test_connect_postgres_says_what_is_missing():
    with pytest.raises(RuntimeError, match="no Postgres driver"):
        connect_postgres("postgresql://localhost/omnia")
