"""omnia doctor (``internal/doctor``): the runner's category concurrency and
sequential groups, every check family against live in-process services (facade
+ runtime with a tool, session-api with the runtime's event sink, memory-api
with its workers, privacy-api, the operator API server with a Workspace and an
AgentRuntime), the SSE server, and the ``omnia doctor`` CLI."""
import asyncio
import json
import time

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.doctor import build_runner, parser
from omnia_amd.doctor.checks import metrics_prefix
from omnia_amd.doctor.result import FAIL, PASS, SKIP, TestResult, failed, passed
from omnia_amd.doctor.runner import Check, Runner
from omnia_amd.doctor.server import build_app as doctor_app


def test_runner_concurrency_sequential_groups_and_failures():
    log = []

    def mk(name, cat, delay, result=None, exc=None):
        async def run():
            log.append(("start", name))
            await asyncio.sleep(delay)
            log.append(("end", name))
            if exc:
                raise exc
            return result or passed("ok")
        return Check(name, cat, run)

    r = Runner().register(mk("a1", "A", 0.05), mk("a2", "A", 0.0),
                          mk("b1", "B", 0.01, exc=RuntimeError("boom")),
                          mk("c1", "C", 0.0, result=TestResult(status=SKIP, detail="n/a")),
                          mk("d1", "D", 0.0))
    r.sequential_group("g", "C", "D")
    seen = []

    async def on(res):
        seen.append((res.name, res.status))

    run = asyncio.run(r.run(on_result=on))
    # A and B overlap (concurrent categories); inside A the checks are ordered
    assert log.index(("start", "b1")) < log.index(("end", "a1"))
    assert log.index(("end", "a1")) < log.index(("start", "a2"))
    # C and D share a sequential group: D starts after C ended
    assert log.index(("end", "c1")) < log.index(("start", "d1"))
    assert [c.name for c in run.categories] == ["A", "B", "C", "D"]
    b1 = run.categories[1].tests[0]
    assert b1.status == FAIL and "boom" in b1.error and b1.category == "B"
    assert run.status == FAIL and run.summary == {"total": 5, "passed": 3, "failed": 1,
                                                  "skipped": 1}
    assert ("a1", "running") in seen and ("a1", PASS) in seen
    assert json.loads(json.dumps(run.to_json()))["summary"]["failed"] == 1


def test_metrics_prefix_matches_reference_rule():
    assert metrics_prefix("SessionAPI") == "omnia_session_api_"
    assert metrics_prefix("APIFoo") == "omnia_api_foo_"
    assert metrics_prefix("Facade") == "omnia_facade_"


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


def _stack():
    """Context manager-ish coroutine pair: start every service, yield URLs."""
    from omnia_amd.api import crds
    from omnia_amd.ee.privacy import PrivacyStore
    from omnia_amd.ee.privacy import build_app as privacy_app
    from omnia_amd.facade.runtime_client import InProcessRuntimeClient
    from omnia_amd.facade.app import build_facade
    from omnia_amd.memory.api import build_app as memory_app
    from omnia_amd.memory.service import MemoryService
    from omnia_amd.memory.workers import CompactionWorker
    from omnia_amd.operator.apiserver import build_app as api_app
    from omnia_amd.operator.apistore import APIStore
    from omnia_amd.runtime.app import build_runtime
    from omnia_amd.runtime.config import RuntimeConfig
    from omnia_amd.session.api import build_app as session_app
    from omnia_amd.session.store import TieredSessionService

    async def up():
        runners = []
        r, s_url = await _serve(session_app(TieredSessionService()))
        runners.append(r)
        msvc = MemoryService()
        r, m_url = await _serve(memory_app(msvc))
        runners.append(r)
        r, p_url = await _serve(privacy_app(PrivacyStore()))
        runners.append(r)
        store = APIStore()
        for k in crds.KINDS.values():
            store.register_kind(k) if hasattr(store, "register_kind") else None
        store.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace",
                     "metadata": {"name": "ws-doc"},
                     "spec": {"displayName": "D", "namespace": {"name": "agents"}},
                     "status": {"phase": "Ready", "services": [
                         {"name": "default", "sessionURL": s_url, "memoryURL": m_url}]}})
        store.apply({"apiVersion": crds.API_VERSION, "kind": "AgentRuntime",
                     "metadata": {"name": "a", "namespace": "agents"},
                     "spec": {"promptPackRef": {"name": "p"}, "facades": [{"type": "websocket"}],
                              "memory": {"enabled": True}},
                     "status": {"phase": "Running"}})
        r, o_url = await _serve(api_app(store))
        runners.append(r)
        svc = await build_runtime(RuntimeConfig(provider={"type": "mock"},
                                                session_api_url=s_url))
        fac = build_facade({"OMNIA_SESSION_API_URL": s_url, "OMNIA_AGENT_NAME": "a",
                            "OMNIA_NAMESPACE": "agents"}, InProcessRuntimeClient(svc))
        port = await fac.start("127.0.0.1", 0)
        worker = asyncio.ensure_future(CompactionWorker(msvc, interval=3600).run())
        await asyncio.sleep(0.05)
        urls = {"facade": f"ws://127.0.0.1:{port}/ws", "session": s_url, "memory": m_url,
                "privacy": p_url, "operator": o_url,
                "facade_metrics": f"http://127.0.0.1:{port}/metrics"}

        async def down():
            worker.cancel()
            await fac.stop()
            for x in runners:
                await x.cleanup()

        return urls, down

    return up


def _args(u, *extra):
    return parser().parse_args([
        "--run-once", "--facade", u["facade"], "--namespace", "agents",
        "--operator-url", u["operator"], "--privacy-api-url", u["privacy"],
        "--memory-api-url", u["memory"],
        "--metrics", f"Agent={u['facade_metrics']}",
        "--metrics", f"SessionAPI={u['session']}", *extra])


def test_doctor_full_run_against_live_services():
    async def go():
        urls, down = await _stack()()
        try:
            return await build_runner(_args(urls)).run()
        finally:
            await down()

    run = asyncio.run(go())
    res = {t.name: t for t in run.results()}
    must_pass = ["SessionAPIHealthy", "MemoryAPIHealthy", "PrivacyAPIHealthy",
                 "OperatorAPIHealthy", "AgentRuntimesExist", "MemoryEnabled",
                 "WorkspacesConfigured", "WorkspaceResolved", "WebSocketConnect",
                 "SendMessageGetResponse", "SessionAPIDocsServed", "SessionCreated",
                 "SessionSearch", "MessagesRecorded", "MemoryAPIDocsServed", "MemorySave",
                 "MemoryRetrieve", "MemoryList", "MemoryExport", "MemoryUserOwnership",
                 "MemoryUserIsolation", "MemoryDelete", "ConsolidationWorkerRunning",
                 "MemoryOptOutRespected", "MemoryDeletionCascade", "Agent metrics",
                 "SessionAPI metrics"]
    bad = {n: res[n] for n in must_pass if res[n].status != PASS}
    assert not bad, bad
    # the session-api URL came from the Workspace status (not a flag)
    assert "ws-doc" in res["WorkspaceResolved"].detail
    assert res["RedisReachable"].status == SKIP
    assert res["GPUKernelsLoaded"].status in (SKIP, PASS)
    assert run.status == PASS, [t for t in run.results() if t.status == FAIL]


def test_doctor_detects_a_broken_service():
    async def go():
        urls, down = await _stack()()
        try:
            urls["memory"] = "http://127.0.0.1:9"  # nothing listens
            return await build_runner(_args(urls)).run()
        finally:
            await down()

    run = asyncio.run(go())
    res = {t.name: t for t in run.results()}
    assert res["MemoryAPIHealthy"].status == FAIL and res["MemorySave"].status == FAIL
    assert run.status == FAIL


def test_doctor_server_sse_trigger_and_latest():
    async def go():
        calls = []

        def build():
            calls.append(1)

            async def ok():
                return passed("fine")

            async def bad():
                return failed("nope")
            return Runner().register(Check("Ok", "X", ok), Check("Bad", "Y", bad))

        r, base = await _serve(doctor_app(build))
        try:
            async with aiohttp.ClientSession() as s:
                assert (await s.get(base + "/api/v1/results/latest")).status == 404
                assert (await s.get(base + "/api/v1/run")).status == 400
                resp = await s.get(base + "/api/v1/run?stream=true")
                assert resp.headers["Content-Type"].startswith("text/event-stream")
                text = await resp.text()
                trig = await (await s.post(base + "/api/v1/run")).json()
                latest = await (await s.get(base + "/api/v1/results/latest")).json()
                page = await (await s.get(base + "/")).text()
                hz = (await s.get(base + "/healthz")).status
            return text, trig, latest, page, hz, len(calls)
        finally:
            await r.cleanup()

    text, trig, latest, page, hz, n = asyncio.run(go())
    frames = [f for f in text.split("\n\n") if f.strip()]
    data = [json.loads(f.split("data: ", 1)[1]) for f in frames if f.startswith("data: ")]
    assert [(d["name"], d["status"]) for d in data if d["status"] != "running"] == \
        [("Ok", "pass"), ("Bad", "fail")] or {(d["name"], d["status"]) for d in data} >= \
        {("Ok", "pass"), ("Bad", "fail")}
    assert frames[-1].startswith("event: complete")
    done = json.loads(frames[-1].split("data: ", 1)[1])
    assert done["status"] == "fail" and done["summary"]["total"] == 2
    assert trig["runId"] == latest["id"] and hz == 200 and n == 2
    assert "EventSource" in page


def test_doctor_cli_run_once_exit_code(tmp_path):
    import subprocess
    import sys

    out = subprocess.run([sys.executable, "-m", "omnia_amd.cli", "doctor", "--run-once",
                          "--exit-code", "--memory-api-url", "http://127.0.0.1:9"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 1, out.stderr
    run = json.loads(out.stdout)
    names = {t["name"]: t["status"] for c in run["categories"] for t in c["tests"]}
    assert names["MemoryAPIHealthy"] == "fail" and names["CRDManifestsValid"] == "pass"
    assert names["WebSocketConnect"] == "skip"
