"""Session data plane: tier fallback matrix, session-api REST, event streams,
ring-buffer client, compaction (warm -> cold Parquet)."""
import asyncio
import time

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.session.api import MemoryPublisher, StreamPublisher, build_app
from omnia_amd.session.compaction import CompactionConfig, CompactionEngine
from omnia_amd.session.httpclient import RingBuffer, SessionHTTPClient
from omnia_amd.session.model import Message, Session
from omnia_amd.session.store import (ColdArchive, HotCache, MemoryBlobStore, TierError,
                                     TieredSessionService, WarmStore)
from omnia_amd.utils.resp import MiniRedis, RedisClient


def _svc(cold=True):
    return TieredSessionService(HotCache(), WarmStore(), ColdArchive(MemoryBlobStore())
                                if cold else None)


def test_tier_matrix_hit_miss_error():
    svc = _svc()
    s = svc.create(Session(id="a", agent_name="ag", namespace="ns"))
    asyncio.run(svc.append_message("a", Message(role="user", content="hello")))
    # hot hit
    assert svc.get("a")[1][0].content == "hello"
    # hot miss -> warm hit (and hot refill)
    svc.hot.invalidate("a")
    assert svc.get("a")[0].id == "a" and "a" in svc.hot.d
    # hot error -> warm answers
    svc.hot.fail = True
    assert svc.get("a")[0].id == "a"
    svc.hot.fail = False
    # all-miss -> definitive None
    assert svc.get("zzz") is None
    # warm error + cold miss -> NOT a definitive miss
    svc.warm.fail = True
    with pytest.raises(TierError):
        svc.get("zzz")
    svc.warm.fail = False
    # empty session (no messages) is a hit, not a miss
    svc.create(Session(id="empty", namespace="ns"))
    svc.hot.invalidate("empty")
    assert svc.get("empty") == (svc.warm.get_session("empty"), []) or svc.get("empty")[1] == []


def test_compaction_archives_to_cold_and_reads_back():
    svc = _svc()
    old = time.time() - 30 * 86400
    for i in range(5):
        s = Session(id=f"s{i}", namespace="ns", created_at=old, updated_at=old)
        svc.warm.put_session(s)
        for j in range(3):
            svc.warm.add_message(s.id, Message(role="user", content=f"m{i}-{j}",
                                               sequence_num=j))
    svc.create(Session(id="fresh", namespace="ns"))
    eng = CompactionEngine(svc.warm, svc.cold, svc.hot, CompactionConfig(
        warm_retention_s=7 * 86400, batch_size=2), sleep=lambda s: None)
    r = eng.run()
    assert r.archived == 5 and r.errors == 0
    assert svc.warm.get_session("s0") is None and svc.warm.get_session("fresh") is not None
    sess, msgs = svc.get("s3")  # served from cold parquet
    assert sess.id == "s3" and [m.content for m in msgs] == ["m3-0", "m3-1", "m3-2"]
    # cold expiry drops whole batches
    assert svc.cold.expire(time.time() + 1) == 5
    assert svc.get("s3") is None


def test_compaction_skips_unreadable_and_purges_without_cold():
    svc = _svc(cold=False)
    old = time.time() - 30 * 86400
    svc.warm.put_session(Session(id="x", namespace="ns", created_at=old, updated_at=old))
    r = CompactionEngine(svc.warm, None, svc.hot, CompactionConfig(),
                         sleep=lambda s: None).run()
    assert r.purged == 1 and svc.warm.get_session("x") is None


def test_session_api_rest_and_event_stream():
    async def go():
        red = await MiniRedis().start()
        svc = TieredSessionService(publisher=StreamPublisher(RedisClient(red.url)))
        app = build_app(svc)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        base = f"http://127.0.0.1:{port}/api/v1"
        out = {}
        async with aiohttp.ClientSession() as s:
            r = await s.post(f"{base}/sessions", json={"id": "sid1", "agentName": "ag",
                                                       "namespace": "ns"})
            out["create"] = r.status
            r = await s.post(f"{base}/sessions", json={"id": "sid1", "namespace": "ns"})
            out["create_again"] = r.status  # idempotent
            for role, c in (("user", "hello world"), ("assistant", "hi!")):
                await s.post(f"{base}/sessions/sid1/messages", json={
                    "role": role, "content": c, "inputTokens": 3, "outputTokens": 2})
            out["msgs"] = (await (await s.get(f"{base}/sessions/sid1/messages")).json())
            await s.post(f"{base}/sessions/sid1/tool-calls", json={"name": "t", "status":
                                                                    "success"})
            await s.post(f"{base}/sessions/sid1/provider-calls", json={
                "provider": "local", "model": "llama-3-8b", "inputTokens": 10,
                "outputTokens": 5, "costUsd": 0.01})
            out["agg"] = await (await s.get(f"{base}/provider-calls/aggregate")).json()
            await s.post(f"{base}/eval-results", json={"sessionId": "sid1", "evalId": "e1",
                                                       "passed": False})
            out["evsum"] = await (await s.get(f"{base}/sessions/sid1/eval-results/summary"))\
                .json()
            out["sess"] = await (await s.get(f"{base}/sessions/sid1")).json()
            out["search"] = await (await s.get(f"{base}/sessions?q=world")).json()
            r = await s.patch(f"{base}/sessions/sid1/status", json={"status": "completed"})
            out["status"] = (await r.json())["status"]
            out["404"] = (await s.get(f"{base}/sessions/nope")).status
            out["bulk"] = await (await s.delete(f"{base}/sessions?namespace=ns")).json()
        stream = red.streams.get(b"omnia:eval-events:ns", [])
        await runner.cleanup()
        await red.stop()
        return out, stream

    out, stream = asyncio.run(go())
    assert out["create"] == 201 and out["create_again"] == 201
    assert [m["role"] for m in out["msgs"]["messages"]] == ["user", "assistant"]
    assert out["agg"]["groups"][0]["costUsd"] == pytest.approx(0.01)
    assert out["evsum"]["total"] == 1 and out["evsum"]["passed"] == 0
    assert out["sess"]["messageCount"] == 2 and out["sess"]["toolCallCount"] == 1
    assert out["sess"]["totalInputTokens"] == 6
    assert len(out["search"]["sessions"]) == 1
    assert out["status"] == "completed" and out["404"] == 404
    assert out["bulk"]["deleted"] == 1
    import json as _json

    types = [_json.loads(dict(zip(f[::2], f[1::2]))[b"event"])["type"] for _, f in stream]
    # message.appended per message + session.completed on the status transition
    assert types == ["message.appended", "message.appended", "session.completed"], types


def test_ring_buffer_parks_and_flushes():
    async def go():
        c = SessionHTTPClient("http://127.0.0.1:9", buffer=2, timeout_s=0.5)  # nothing listens
        for i in range(3):
            ok = await c.append("s", "user", f"m{i}")
            assert ok is False
        n_parked, dropped = len(c.ring), c.ring.dropped
        await c.close()
        return n_parked, dropped

    assert asyncio.run(go()) == (2, 1)
    rb = RingBuffer(3)
    for i in range(5):
        rb.push(i)
    assert rb.drain() == [2, 3, 4] and rb.dropped == 2


def test_miniredis_streams_consumer_group():
    async def go():
        red = await MiniRedis().start()
        c = RedisClient(red.url)
        await c.set("k", "v", ex=100)
        v = await c.get("k")
        await c.xgroup_create("st", "g")
        await c.xadd("st", {"a": "1"})
        await c.xadd("st", {"a": "2"})
        got = await c.xreadgroup("g", "c1", {"st": ">"}, count=10)
        ids = [e[0] for e in got[0][1]]
        acked = await c.xack("st", "g", *ids)
        again = await c.xreadgroup("g", "c1", {"st": ">"}, count=10)
        c.close()
        await red.stop()
        return v, len(ids), acked, again

    v, n, acked, again = asyncio.run(go())
    assert v == b"v" and n == 2 and acked == 2 and again is None


# ------------------------------------------------------------------ service semantics
def _svc2():
    from omnia_amd.session.store import TieredSessionService, WarmStore

    events = []

    async def pub(ev):
        events.append(ev)

    return TieredSessionService(warm=WarmStore(), publisher=pub), events


def test_append_accounting_sequence_and_events():
    import asyncio

    from omnia_amd.session.model import Message, Session

    svc, events = _svc2()
    s0 = svc.create(Session(id="s1", agent_name="a", namespace="ns"))
    assert svc.create(Session(id="s1", agent_name="other")) is not None  # idempotent
    assert svc.get("s1")[0].agent_name == "a"
    for i in range(3):
        asyncio.run(svc.append_message("s1", Message(
            role="user" if i % 2 == 0 else "assistant", content=f"m{i}" * 100,
            input_tokens=10, output_tokens=5, cost_usd=0.01)))
    s, msgs = svc.get("s1")
    assert [m.sequence_num for m in msgs] == [0, 1, 2] and s.message_count == 3
    assert (s.total_input_tokens, s.total_output_tokens) == (30, 15)
    assert abs(s.estimated_cost_usd - 0.03) < 1e-9 and len(s.last_message_preview) == 120
    assert [e["type"] for e in events] == ["message.appended"] * 3
    assert events[0]["namespace"] == "ns" and events[1]["role"] == "assistant"
    # hot cache dropped: the warm tier answers with the same view
    svc.hot.invalidate("s1")
    s2, msgs2 = svc.get("s1")
    assert s2.message_count == 3 and [m.content for m in msgs2] == [m.content for m in msgs]
    with pytest.raises(KeyError):
        asyncio.run(svc.append_message("nope", Message(content="x")))
    assert s0.expires_at > 0  # default TTL applied on create


def test_status_ttl_decorate_delete_and_tool_calls():
    import time

    from omnia_amd.session.model import Session, ToolCall

    svc, _ = _svc2()
    svc.create(Session(id="s2", agent_name="a", namespace="ns"))
    svc.record("tool_calls", "s2", ToolCall(name="search", status="success"))
    svc.record("tool_calls", "s2", ToolCall(name="fetch", status="error"))
    s, _ = svc.get("s2")
    assert s.tool_call_count == 2
    assert [r["name"] for r in svc.warm.list_rows("tool_calls", "s2")] == ["search", "fetch"]
    t = time.time()
    s = svc.update_status("s2", "completed", ended_at=t)
    assert s.status == "completed" and s.ended_at == t
    s = svc.refresh_ttl("s2", 60)
    assert 55 < s.expires_at - time.time() <= 61
    s = svc.decorate("s2", tags=["vip"], state={"k": 1})
    assert "vip" in s.tags and s.state.get("k") == 1
    assert svc.delete("s2") and svc.get("s2") is None
    with pytest.raises(KeyError):
        svc.record("tool_calls", "s2", ToolCall(name="x"))


def test_list_sessions_filters_and_search():
    import asyncio

    from omnia_amd.session.model import Message, Session

    svc, _ = _svc2()
    base = 1_700_000_000.0
    for i in range(6):
        svc.create(Session(id=f"q{i}", agent_name="a" if i % 2 else "b",
                           namespace="ns1" if i < 4 else "ns2", created_at=base + i))
    asyncio.run(svc.append_message("q3", Message(content="the refund policy")))
    w = svc.warm
    assert {s.id for s in w.list_sessions(namespace="ns1")} == {"q0", "q1", "q2", "q3"}
    assert {s.id for s in w.list_sessions(namespace="ns1", agent="a")} == {"q1", "q3"}
    assert [s.id for s in w.list_sessions(after=base + 3.5)] == ["q5", "q4"]  # newest first
    assert [s.id for s in w.list_sessions(before=base + 1.5)] == ["q1", "q0"]
    assert [s.id for s in w.list_sessions(q="refund")] == ["q3"]
    page1 = [s.id for s in w.list_sessions(limit=2)]
    page2 = [s.id for s in w.list_sessions(limit=2, offset=2)]
    assert page1 == ["q5", "q4"] and page2 == ["q3", "q2"]


def test_admin_compaction_endpoint_and_remote_cli():
    """``POST /api/v1/admin/compaction`` runs one compaction on the replica's own
    tiers (the workspace compaction CronJob's target): policy retention by
    default, overridable per call; the CLI's ``--session-api`` mode drives it."""
    from omnia_amd.session import compaction as C

    async def go():
        svc = _svc()
        old = time.time() - 30 * 86400
        svc.warm.put_session(Session(id="old", namespace="ns", created_at=old, updated_at=old))
        svc.warm.add_message("old", Message(role="user", content="hi", sequence_num=0))
        svc.create(Session(id="new", namespace="ns"))
        app = build_app(svc, retention={"warm_retention_s": 7 * 86400})
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        url = f"http://127.0.0.1:{port}"
        out = {}
        async with aiohttp.ClientSession() as s:
            r = await s.post(f"{url}/api/v1/admin/compaction", json={"dryRun": True})
            out["dry"] = await r.json()
            r = await s.post(f"{url}/api/v1/admin/compaction")
            out["policy"] = await r.json()
            out["bad"] = (await s.post(f"{url}/api/v1/admin/compaction",
                                       json={"warmRetentionSeconds": -1})).status
        # the CronJob's CLI form, zero retention: the fresh session goes too
        out["cli"] = await asyncio.to_thread(
            C.main, ["--session-api", url, "--warm-retention", "0"])
        await runner.cleanup()
        return svc, out

    svc, out = asyncio.run(go())
    assert out["dry"]["archived"] == 1
    assert out["policy"]["archived"] == 1 and out["policy"]["coldArchive"] is True
    assert out["bad"] == 400
    assert out["cli"] == 0
    assert svc.warm.get_session("old") is None and svc.warm.get_session("new") is None
    sess, msgs = svc.get("old")  # read back from the cold archive
    assert sess.id == "old" and [m.content for m in msgs] == ["hi"]
    assert svc.get("new")[0].id == "new"
