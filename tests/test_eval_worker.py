"""Eval worker to reference depth (``ee/pkg/evals``): PromptPack-loaded evals,
worker groups, judge-provider resolution from Provider CRs, the session
completion trigger (explicit + inactivity), on-demand evaluate requests, alert
webhooks, and at-least-once delivery (no ack on failure, XAUTOCLAIM reclaim,
dead-letter) -- against the in-repo RESP server and session-api."""
import asyncio
import json

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.ee.eval_worker import (CompletionTracker, EvalWorker, PackEvalLoader,
                                      ProviderResolver, SessionAPIClient, WebhookDispatcher,
                                      eval_groups, validate_webhook_url)
from omnia_amd.session.api import StreamPublisher, build_app
from omnia_amd.session.store import TieredSessionService
from omnia_amd.utils.resp import MiniRedis, RedisClient

PACK = {"id": "support", "version": "1.2.0", "evals": [
    {"id": "has-4", "type": "contains", "trigger": "every_turn",
     "params": {"value": "4", "groups": ["long-running"]}},
    {"id": "fast-only", "type": "contains", "trigger": "every_turn", "params": {"value": "x"}},
    {"id": "judge-turn", "type": "llm_judge", "trigger": "every_turn",
     "params": {"provider": "grader", "criteria": "correct"}},
    {"id": "session-judge", "type": "llm_judge", "trigger": "on_session_complete",
     "params": {"provider": "grader"}},
    {"id": "session-json", "type": "json_valid", "trigger": "on_session_complete",
     "params": {"groups": ["external"]}},
    {"id": "disabled", "type": "contains", "trigger": "every_turn", "enabled": False,
     "params": {"groups": ["long-running"]}},
]}


class _Judge:
    """Provider stand-in: always grades ``score`` out of 5."""

    def __init__(self, score):
        self.score = score
        self.calls = 0

    async def stream(self, msgs, tools, params, session_id=None, metadata=None):
        from omnia_amd.runtime.providers import ProviderEvent, Usage

        self.calls += 1
        yield ProviderEvent("text", text=f"SCORE: {self.score}\nreason")
        yield ProviderEvent("done", usage=Usage(input_tokens=3, output_tokens=4))


class _Kube:
    def __init__(self, objs):
        self.objs = objs

    def get(self, kind, name, ns="default"):
        o = self.objs.get((kind, ns, name))
        if o is None:
            raise KeyError((kind, ns, name))
        return o


def _kube(groups=None):
    ar = {"spec": {"providers": [{"name": "grader", "providerRef": {"name": "judge-prov"}}],
                   "evals": {"enabled": True, "sampling": {"defaultRate": 100,
                                                           "extendedRate": 100},
                             **({"worker": {"groups": groups}} if groups else {})}}}
    return _Kube({("AgentRuntime", "ns1", "agent-a"): ar,
                  ("Provider", "ns1", "judge-prov"): {"spec": {"type": "mock", "model": "m"}},
                  ("PromptPack", "ns1", "support"): {"spec": {"source": {
                      "configMapRef": {"name": "support-cm"}}}},
                  ("ConfigMap", "ns1", "support-cm"): {"data": {"pack.json": json.dumps(PACK)}}})


async def _session_api():
    redis = await MiniRedis().start()
    svc = TieredSessionService(publisher=StreamPublisher(RedisClient(redis.url)))
    runner = web.AppRunner(build_app(svc))
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
    return redis, svc, runner, url


async def _post(s, url, path, body, method="POST"):
    async with s.request(method, url + path, json=body) as r:
        return r.status, await r.json(content_type=None)


def test_eval_groups_defaults_are_disjoint():
    assert eval_groups({"type": "contains"}) == ["fast-running"]
    assert set(eval_groups({"type": "llm_judge"})) == {"long-running", "external"}
    assert eval_groups({"type": "contains", "params": {"groups": ["external"]}}) == ["external"]


def test_pack_loader_caches_per_version():
    loads = []

    async def source(ns, name, version):
        loads.append((ns, name, version))
        return dict(PACK, version=version or PACK["version"])

    async def go():
        L = PackEvalLoader(source)
        a = await L.load("ns1", "support", "1.2.0")
        assert {e["id"] for e in a["evals"]} >= {"has-4", "judge-turn"}
        assert "disabled" not in {e["id"] for e in a["evals"]}
        await L.load("ns1", "support", "1.2.0")
        assert len(loads) == 1  # cached
        await L.load("ns1", "support", "1.3.0")
        assert len(loads) == 2  # version moved: reload
        assert await L.load("ns1", "", "") is None

    asyncio.run(go())


def test_worker_end_to_end_triggers_groups_providers():
    """Real session-api publishing to Redis Streams; the worker loads the pack's
    evals through the kube source, filters by worker groups, resolves the judge
    from the Provider CR, and writes results back."""
    judge = _Judge(5)

    async def go():
        from omnia_amd.ee.eval_worker import KubePackSource

        redis, svc, runner, url = await _session_api()
        kube = _kube()
        sess = SessionAPIClient(url)
        w = EvalWorker(RedisClient(redis.url), sess, ["ns1"],
                       pack_loader=PackEvalLoader(KubePackSource(kube)),
                       resolver=ProviderResolver(kube, build=lambda spec: judge),
                       inactivity_timeout_s=60)
        await w.setup()
        try:
            async with aiohttp.ClientSession() as s:
                st, sj = await _post(s, url, "/api/v1/sessions", {
                    "agentName": "agent-a", "namespace": "ns1", "promptPackName": "support",
                    "promptPackVersion": "1.2.0"})
                sid = sj["id"]
                await _post(s, url, f"/api/v1/sessions/{sid}/messages",
                            {"role": "user", "content": "what is 2+2"})
                await _post(s, url, f"/api/v1/sessions/{sid}/messages",
                            {"role": "assistant", "content": "The answer is 4."})
                await w.poll_once()
                async with s.get(f"{url}/api/v1/sessions/{sid}/eval-results") as r:
                    rows = (await r.json())
                rows = rows.get("results", rows.get("items", rows)) if isinstance(rows, dict) \
                    else rows
                got = {r["evalId"] for r in rows}
                # worker groups default (long-running, external): the fast-running
                # deterministic eval stays inline in the runtime
                assert got == {"has-4", "judge-turn"}, got
                assert judge.calls == 1
                # completion: PATCH status -> session.completed -> session evals once
                st, _ = await _post(s, url, f"/api/v1/sessions/{sid}/status",
                                    {"status": "completed"}, method="PATCH")
                assert st == 200
                await w.poll_once()
                await _post(s, url, f"/api/v1/sessions/{sid}/status", {"status": "completed"},
                            method="PATCH")  # no transition: no second event
                await w.poll_once()
                async with s.get(f"{url}/api/v1/sessions/{sid}/eval-results") as r:
                    rows = await r.json()
                rows = rows.get("results", rows.get("items", rows)) if isinstance(rows, dict) \
                    else rows
                ids = [r["evalId"] for r in rows]
                assert ids.count("session-judge") == 1 and ids.count("session-json") == 1
                assert w.stats["session_completions"] == 1
                # on-demand evaluate: session + turn evals, source manual
                st, body = await _post(s, url, f"/api/v1/sessions/{sid}/evaluate", {})
                assert st == 202 and body["status"] == "queued"
                await w.poll_once()
                async with s.get(f"{url}/api/v1/sessions/{sid}/eval-results") as r:
                    rows = await r.json()
                rows = rows.get("results", rows.get("items", rows)) if isinstance(rows, dict) \
                    else rows
                manual = [r for r in rows if r.get("source") == "manual"]
                assert {r["evalId"] for r in manual} >= {"session-judge", "has-4"}
                st, _ = await _post(s, url, "/api/v1/sessions/nope/evaluate", {})
                assert st == 404
        finally:
            await sess.close()
            await runner.cleanup()
            await redis.stop()

    asyncio.run(go())


def test_worker_groups_from_agentruntime_include_fast_running():
    judge = _Judge(2)

    class Sess:
        posted = []

        async def get_messages(self, sid):
            return [{"id": "u", "role": "user", "content": "q"},
                    {"id": "a", "role": "assistant", "content": "x marks it"}]

        async def post_eval_results(self, results):
            self.posted.extend(results)

    async def go():
        async def src(ns, name, v):
            return PACK

        w = EvalWorker(None, Sess(), ["ns1"], pack_loader=PackEvalLoader(src),
                       resolver=ProviderResolver(_kube(groups=["fast-running"]),
                                                 build=lambda spec: judge))
        out = await w.handle({"type": "message.appended", "role": "assistant",
                              "sessionId": "s1", "messageId": "a", "agentName": "agent-a",
                              "namespace": "ns1", "promptPackName": "support",
                              "promptPackVersion": "1.2.0"})
        return out

    out = asyncio.run(go())
    assert {r["evalId"] for r in out} == {"fast-only"}
    assert out[0]["passed"] is True and judge.calls == 0


def test_completion_tracker_inactivity_once_and_eviction():
    t = [0.0]
    fired = []

    async def cb(sid):
        fired.append(sid)

    async def go():
        tr = CompletionTracker(10.0, cb, now=lambda: t[0])
        tr.record_activity("a")
        tr.record_activity("b")
        t[0] = 5.0
        tr.record_activity("b")
        t[0] = 11.0
        assert await tr.check_inactive() == ["a"]
        await tr.mark_completed("a")  # already completed: no second fire
        t[0] = 16.0
        assert await tr.check_inactive() == ["b"]
        tr.record_activity("a")  # completed sessions ignore late activity
        t[0] = 40.0
        await tr.check_inactive()
        assert tr.tracked == 0  # evicted after 2x timeout
        await tr.mark_completed("c")
        await tr.mark_completed("c")

    asyncio.run(go())
    assert fired == ["a", "b", "c"]


def test_explicit_completion_failure_propagates_and_retries():
    """session.completed whose evals fail raises (the stream entry stays
    pending) and does NOT mark the session done, so the redelivery runs them."""
    calls = []

    async def cb(sid):
        calls.append(sid)
        if len(calls) == 1:
            raise ConnectionError("session-api down")

    async def go():
        tr = CompletionTracker(10.0, cb, now=lambda: 0.0)
        with pytest.raises(ConnectionError):
            await tr.mark_completed("s")
        assert "s" not in tr.completed
        await tr.mark_completed("s")  # redelivery
        assert "s" in tr.completed
        await tr.mark_completed("s")  # exactly once after success

    asyncio.run(go())
    assert calls == ["s", "s"]


def test_webhook_dispatcher_window_consecutive_ratelimit_retry():
    calls = []
    fail = {"n": 2}

    async def post(url, body, headers):
        calls.append((url, json.loads(body), headers))
        if fail["n"] > 0:
            fail["n"] -= 1
            return 503
        return 200

    def res(passed, i):
        return {"evalId": "e1", "passed": passed, "sessionId": f"s{i}", "messageId": f"m{i}"}

    async def go():
        d = WebhookDispatcher([{"url": "https://hooks.example/a", "threshold": 0.8,
                                "windowSize": 4, "headers": {"X-Token": "t"}},
                               {"url": "ftp://bad/x", "threshold": 0.9}], post=post,
                              backoff_s=0.0)
        ok = [res(True, i) for i in range(6)]
        assert await d.check_and_fire("e1", "a", "ns", ok) == 0
        recent = ok + [res(False, 7), res(False, 8)]  # window of 4: pass rate 0.5
        assert await d.check_and_fire("e1", "a", "ns", recent) == 1
        assert len(calls) == 3  # two failed attempts, then success
        payload = calls[-1][1]
        assert payload["currentPassRate"] == 0.5 and payload["windowSize"] == 4
        assert {f["sessionId"] for f in payload["recentFailures"]} == {"s7", "s8"}
        assert calls[-1][2]["X-Token"] == "t"
        assert d.stats["invalid_url"] == 1
        # rate limited for a minute per (eval, url)
        assert await d.check_and_fire("e1", "a", "ns", recent) == 0
        assert d.stats["rate_limited"] >= 1
        d2 = WebhookDispatcher([{"url": "http://h/x", "threshold": 0.0,
                                 "consecutiveFails": 3}], post=post)
        streak = [res(True, 0), res(False, 1), res(False, 2)]
        assert await d2.check_and_fire("e1", "a", "ns", streak) == 0
        assert await d2.check_and_fire("e1", "a", "ns", streak + [res(False, 3)]) == 1

    asyncio.run(go())
    with pytest.raises(ValueError):
        validate_webhook_url("/relative")


def test_failed_event_stays_pending_then_reclaimed_or_dead_lettered():
    class Flaky:
        def __init__(self, fails):
            self.fails = fails
            self.posted = []

        async def get_messages(self, sid):
            return [{"id": "u", "role": "user", "content": "2+2"},
                    {"id": "a", "role": "assistant", "content": "4"}]

        async def post_eval_results(self, results):
            if self.fails > 0:
                self.fails -= 1
                raise RuntimeError("session-api 503")
            self.posted.extend(results)

    defs = [{"id": "has4", "type": "contains", "params": {"value": "4"}}]
    ev = {"type": "message.appended", "sessionId": "s", "namespace": "ns1",
          "agentName": "a", "messageId": "a", "role": "assistant"}

    async def go():
        red = await MiniRedis().start()
        try:
            rc = RedisClient(red.url)
            sess = Flaky(1)
            w = EvalWorker(rc, sess, ["ns1"], lambda a, n: defs, reclaim_min_idle_s=0.0,
                           reclaim_interval_s=0.0, max_deliveries=3)
            await w.setup()
            await rc.xadd("omnia:eval-events:ns1", {"event": json.dumps(ev)})
            await w.poll_once()  # first delivery fails, then reclaimed + retried
            assert w.stats["failed"] == 1 and w.stats["reclaimed"] == 1
            assert [r["evalId"] for r in sess.posted] == ["has4"]
            grp = red.groups[b"omnia:eval-events:ns1"][b"eval-workers"]
            assert not grp["pending"]  # acked only after the write succeeded
            # a poison event is dead-lettered after max_deliveries
            sess.fails = 99
            await rc.xadd("omnia:eval-events:ns1", {"event": json.dumps(ev)})
            for _ in range(4):
                await w.poll_once()
            assert w.stats["dead_lettered"] == 1 and not grp["pending"]
            # unparsable payloads are acked at once
            await rc.xadd("omnia:eval-events:ns1", {"event": "{not json"})
            await w.poll_once()
            assert not grp["pending"]
        finally:
            await red.stop()

    asyncio.run(go())


def test_session_client_reuses_one_http_session():
    async def go():
        redis, svc, runner, url = await _session_api()
        c = SessionAPIClient(url)
        try:
            s1 = await c._session()
            await c.get_messages("x") if False else None
            s2 = await c._session()
            assert s1 is s2
        finally:
            await c.close()
            await runner.cleanup()
            await redis.stop()

    asyncio.run(go())
