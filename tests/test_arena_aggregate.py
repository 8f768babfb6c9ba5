"""Arena job results: aggregation by scenario / provider with error and
assertion roll-ups (``ee/pkg/arena/aggregator``), and played runs recorded
into session-api as ``source:arena`` sessions (``session_recording.go``)."""
import asyncio
import json

from aiohttp import web

from omnia_amd.ee.arena.aggregate import aggregate, to_job_result
from omnia_amd.ee.arena.queue import MemoryQueue, WorkItem
from omnia_amd.ee.arena.recording import ArenaSessionRecorder, session_uuid
from omnia_amd.session.api import build_app
from omnia_amd.session.httpclient import SessionHTTPClient
from omnia_amd.session.store import TieredSessionService


def _res(scen, prov, passed, cost=0.01, toks=10, err=None, iid="i", checks=()):
    r = {"scenario": scen, "provider": prov, "passed": passed, "cost": cost,
         "output_tokens": toks, "item_id": iid,
         "turns": [{"latency_ms": 100.0, "ttft_ms": 20.0,
                    "assertions": [{"id": n, "type": "contains", "passed": ok}
                                   for n, ok in checks]}]}
    if err is not None:
        r["error"] = err
    return r


def test_aggregate_groups_errors_assertions():
    results = [_res("s1", "p1", True, iid="a", checks=[("has-x", True)]),
               _res("s1", "p2", False, iid="b", checks=[("has-x", False)]),
               _res("s2", "p1", True, iid="c", checks=[("has-x", True), ("short", True)]),
               {"passed": False, "error": "timeout", "scenario": "s2", "provider": "p2",
                "item_id": "d"},
               {"passed": False, "error": "timeout", "scenario": "s2", "provider": "p2",
                "item_id": "e"},
               {"passed": False, "error": "", "scenario": "s1", "provider": "p1",
                "item_id": "f"}]
    a = aggregate(results)
    assert a["totalItems"] == 6 and a["passedItems"] == 2 and a["failedItems"] == 4
    assert abs(a["passRate"] - 100 * 2 / 6) < 1e-3
    assert a["totalTokens"] == 30 and abs(a["totalCost"] - 0.03) < 1e-9
    assert a["byScenario"]["s1"]["total"] == 3 and a["byScenario"]["s1"]["passed"] == 1
    assert a["byProvider"]["p2"]["failed"] == 3 and a["byProvider"]["p1"]["passRate"] > 66
    errs = {e["message"]: e for e in a["errors"]}
    assert errs["timeout"]["count"] == 2 and errs["timeout"]["workItemIds"] == ["d", "e"]
    assert errs["unknown error"]["count"] == 1
    asum = {x["name"]: x for x in a["assertions"]}
    assert asum["has-x"]["total"] == 3 and asum["has-x"]["failed"] == 1
    assert asum["short"]["passRate"] == 100.0
    jr = to_job_result(a)
    assert jr["summary"]["passRate"] == "33.3" and jr["summary"]["totalItems"] == "6"
    det = json.loads(jr["summary"]["details"])
    assert {s["name"] for s in det["scenarios"]} == {"s1", "s2"}
    assert {p["name"] for p in det["providers"]} == {"p1", "p2"}
    assert aggregate([])["totalItems"] == 0


def test_queue_failure_result_carries_item_identity():
    async def go():
        q = MemoryQueue()
        it = WorkItem(job_id="j", scenario_id="s", provider_id="p", max_attempts=1)
        await q.enqueue([it])
        [c] = await q.claim("j", "w")
        await q.fail(c, "boom")
        return (await q.results_of("j"))[0]

    r = asyncio.run(go())
    assert r == {"passed": False, "error": "boom", "scenario": "s", "provider": "p",
                 "item_id": r["item_id"], "attempt": 1}


def test_recorder_writes_arena_sessions_idempotently():
    async def go():
        svc = TieredSessionService()
        runner = web.AppRunner(build_app(svc))
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
        c = SessionHTTPClient(url)
        rec = ArenaSessionRecorder(c, "job1", "ns", "ws1")
        it = WorkItem(job_id="job1", scenario_id="greet", provider_id="local",
                      config={"trial": 2})
        res = {"passed": True, "turns": [
            {"user": "hi", "content": "hello!", "ttft_ms": 5.0, "latency_ms": 9.0,
             "usage": {"output_tokens": 3, "cost": 0.001}},
            {"user": "bye", "content": "ciao", "ttft_ms": 4.0, "latency_ms": 7.0}]}
        sid = await rec.record(it, res)
        again = await rec.record(it, res)  # a reclaimed item re-plays into the same id
        bad = WorkItem(job_id="job1", scenario_id="greet", provider_id="other")
        sid2 = await rec.record(bad, {"passed": False, "turns": [{"user": "x",
                                                                  "content": "y"}]})
        s, msgs = svc.get(sid)
        s2, _ = svc.get(sid2)
        await c.close()
        await runner.cleanup()
        return sid, again, it, s, msgs, s2

    sid, again, it, s, msgs, s2 = asyncio.run(go())
    assert sid == again == session_uuid(it.id, it.id)
    assert s.agent_name == "job1" and s.workspace_name == "ws1" and s.status == "completed"
    assert {"source:arena", "arena-job:job1", "scenario:greet", "provider:local",
            "trial:2"} <= set(s.tags)
    assert s.state["arena.provider.id"] == "local" and s.state["arena.trial.index"] == "2"
    assert s.virtual_user_id and s.virtual_user_id != it.id
    roles = [m.role for m in msgs]
    assert roles[:4] == ["user", "assistant", "user", "assistant"]
    assert msgs[1].output_tokens == 3
    assert s2.status == "error"  # the failed run is visible as such


def test_recorder_gives_up_without_session_api():
    class Down:
        calls = 0

        async def write(self, method, path, body=None):
            Down.calls += 1
            return False

    rec = ArenaSessionRecorder(Down(), "j", "ns", base_wait_s=0.0)
    it = WorkItem(job_id="j", scenario_id="s", provider_id="p")
    assert asyncio.run(rec.record(it, {"passed": True, "turns": []})) is None
    assert Down.calls == 3  # retried, then the run is played but not recorded


def test_sessions_with_failed_evals_become_scenarios():
    from omnia_amd.ee.arena.sources import SessionAPISource

    async def go():
        svc = TieredSessionService()
        runner = web.AppRunner(build_app(svc))
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
        c = SessionHTTPClient(url)
        ids = {}
        for sid, ok in (("sess-bad-0001", False), ("sess-good-001", True)):
            await c.request("POST", "/api/v1/sessions", {"id": sid, "agentName": "support",
                                                         "namespace": "ns"})
            for role, text in (("system", "be nice"), ("user", "where is my order"),
                               ("assistant", "it shipped"), ("user", "thanks"),
                               ("assistant", "bye")):
                m = await c.request("POST", f"/api/v1/sessions/{sid}/messages",
                                    {"role": role, "content": text})
                ids[(sid, text)] = m["id"]
            await c.request("POST", "/api/v1/eval-results", [
                {"sessionId": sid, "messageId": ids[(sid, "it shipped")], "evalId": "polite",
                 "evalType": "llm_judge", "passed": ok, "details": {"criteria": "tone"}},
                {"sessionId": sid, "evalId": "resolved", "evalType": "contains",
                 "passed": ok, "details": {"value": "shipped"}},
                {"sessionId": sid, "messageId": "not-in-transcript", "evalId": "ghost",
                 "passed": ok}])
        src = SessionAPISource(c)
        listed = await src.list(passed=False, limit=5)
        scen = await src.scenarios(passed=False, limit=5)
        all_ = await src.list(passed=None, limit=5)
        await c.close()
        await runner.cleanup()
        return listed, scen, all_

    listed, scen, all_ = asyncio.run(go())
    assert [x["id"] for x in listed] == ["sess-bad-0001"]  # de-duplicated per session
    assert {x["id"] for x in all_} == {"sess-bad-0001", "sess-good-001"}
    [s] = scen
    assert s["id"] == "session-sess-bad-000" and s["system"] == "be nice"
    assert [t["user"] for t in s["turns"]] == ["where is my order", "thanks"]
    assert s["turns"][0]["reference"] == "it shipped"
    a = s["turns"][0]["assertions"]
    assert [x["id"] for x in a] == ["polite"] and a[0]["params"] == {"criteria": "tone"}
    assert [x["id"] for x in s["conversation_assertions"]] == ["resolved"]
    assert s["metadata"]["failedEvals"] == ["ghost", "polite", "resolved"]
    assert s["turns"][1]["assertions"] == []  # the ghost result matched no message
