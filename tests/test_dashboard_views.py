"""Dashboard analysis views (verdict r5 L6 / C47 gap): costs, quality,
memories, memory analytics, privacy stats, topology, tools, skills and
settings -- against a real session-api, a fake operator REST API and fake
memory / privacy APIs, through the dashboard's HTTP routes."""
import asyncio

import aiohttp
from aiohttp import web

from omnia_amd.api import crds
from omnia_amd.operator import dashboard
from omnia_amd.operator.dashboard_views import skills_view, tools_view, topology
from omnia_amd.session.api import build_app as session_app
from omnia_amd.session.store import TieredSessionService

OBJS = {
    "workspaces": [{"metadata": {"name": "team-a"},
                    "spec": {"namespace": {"name": "ns-a"}}}],
    "agentruntimes": [{"metadata": {"namespace": "ns-a", "name": "support"},
                       "spec": {"promptPackRef": {"name": "pack"},
                                "providers": [{"name": "default",
                                               "providerRef": {"name": "llama"}}],
                                "toolRegistryRef": {"name": "tools"}},
                       "status": {"phase": "Running"}}],
    "promptpacks": [{"metadata": {"namespace": "ns-a", "name": "pack"},
                     "status": {"phase": "Active"}}],
    "providers": [{"metadata": {"namespace": "ns-a", "name": "llama"},
                   "spec": {"type": "local"}, "status": {"phase": "Ready"}}],
    "toolregistries": [{"metadata": {"namespace": "ns-a", "name": "tools"},
                        "spec": {"handlers": [{"name": "weather", "type": "http"}]},
                        "status": {"phase": "Ready", "discoveredTools": [
                            {"name": "get_weather", "handlerName": "weather",
                             "endpoint": "http://w", "status": "Available"}]}}],
    "skillsources": [{"metadata": {"namespace": "ns-a", "name": "kb-skills"},
                      "spec": {"source": {"type": "git"}},
                      "status": {"phase": "Ready", "skillCount": 3}}],
}


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


def _operator_api():
    app = web.Application()

    async def lst(request):
        return web.json_response({"items": OBJS.get(request.match_info["plural"], [])})

    app.router.add_get(f"/apis/{crds.GROUP}/{crds.VERSION}/{{plural}}", lst)
    return app


def _memory_api(seen):
    app = web.Application()

    async def h(request):
        seen.append((request.path, dict(request.query)))
        if request.path.endswith("/aggregate"):
            return web.json_response({"groups": [{"key": "hot", "count": 2}], "total": 2})
        if request.path.endswith("/projection"):
            return web.json_response({"tiers": {"hot": 2}})
        if request.path.endswith("/stats"):
            return web.json_response({"consolidated": 1})
        return web.json_response({"memories": [{"id": "m1", "category": "pref",
                                                "content": "likes tea", "confidence": 0.9}]})

    app.router.add_get("/api/v1/memories{tail:.*}", h)
    return app


def _privacy_api():
    app = web.Application()
    app.router.add_get("/api/v1/privacy/consent/stats",
                       lambda r: web.json_response({"granted": 5, "revoked": 1}))
    app.router.add_get("/api/v1/privacy/enforcement-stats",
                       lambda r: web.json_response({"redactions": 7}))
    return app


def test_views_end_to_end():
    async def go():
        seen = []
        runners = []
        out = {}
        try:
            r, api = await _serve(_operator_api())
            runners.append(r)
            r, sess = await _serve(session_app(TieredSessionService()))
            runners.append(r)
            r, mem = await _serve(_memory_api(seen))
            runners.append(r)
            r, priv = await _serve(_privacy_api())
            runners.append(r)
            async with aiohttp.ClientSession() as s:
                # one session in ns-a with two provider calls and eval results
                await s.post(f"{sess}/api/v1/sessions", json={"id": "s1", "agentName": "support",
                                                               "namespace": "ns-a"})
                for cost in (0.01, 0.02):
                    await s.post(f"{sess}/api/v1/sessions/s1/provider-calls",
                                 json={"provider": "local", "model": "llama-3-8b",
                                       "inputTokens": 100, "outputTokens": 20, "costUsd": cost})
                await s.post(f"{sess}/api/v1/eval-results", json={"results": [
                    {"sessionId": "s1", "evalId": "tools-called", "evalType": "tools_called",
                     "passed": True, "score": 1.0},
                    {"sessionId": "s1", "evalId": "tools-called", "evalType": "tools_called",
                     "passed": False, "score": 0.0}]})
            r, dash = await _serve(dashboard.build_app(api, sess, priv, memory_api=mem))
            runners.append(r)
            async with aiohttp.ClientSession() as s:
                for k, path in (("costs", "/api/workspaces/team-a/costs"),
                                ("quality", "/api/workspaces/team-a/eval-results/aggregate"),
                                ("mems", "/api/workspaces/team-a/memories"),
                                ("agg", "/api/workspaces/team-a/memory/aggregate?groupBy=tier"),
                                ("proj", "/api/workspaces/team-a/memory/projection"),
                                ("mstats", "/api/workspaces/team-a/memory/stats"),
                                ("consent", "/api/workspaces/team-a/privacy/consent/stats"),
                                ("enf", "/api/workspaces/team-a/privacy/enforcement-stats"),
                                ("topo", "/api/topology"), ("tools", "/api/tools"),
                                ("skills", "/api/skills"), ("settings", "/api/settings")):
                    async with s.get(dash + path) as resp:
                        out[k] = (resp.status, await resp.json())
                async with s.get(dash + "/") as resp:
                    out["page"] = await resp.text()
        finally:
            for r in runners:
                await r.cleanup()
        return out, seen

    out, seen = asyncio.run(go())
    st, costs = out["costs"]
    assert st == 200 and costs["namespace"] == "ns-a"  # workspace -> its namespace
    assert abs(costs["totalCostUsd"] - 0.03) < 1e-9 and costs["totalTokens"] == 240
    st, q = out["quality"]
    assert st == 200 and q["total"] == 2 and q["passed"] == 1 and q["passRate"] == 0.5
    assert out["mems"][1]["memories"][0]["id"] == "m1"
    assert out["agg"][1]["total"] == 2 and out["proj"][1]["tiers"]["hot"] == 2
    assert out["mstats"][1]["consolidated"] == 1
    # memory-api calls carry the workspace scope
    assert all(q.get("workspace") == "team-a" for _, q in seen)
    assert out["consent"][1]["granted"] == 5 and out["enf"][1]["redactions"] == 7
    topo = out["topo"][1]
    ids = {n["id"] for n in topo["nodes"]}
    assert {"AgentRuntime/ns-a/support", "PromptPack/ns-a/pack", "Provider/ns-a/llama",
            "ToolRegistry/ns-a/tools", "SkillSource/ns-a/kb-skills", "Workspace//team-a"} <= ids
    rels = {(e["from"].split("/")[0], e["to"].split("/")[0], e["rel"]) for e in topo["edges"]}
    assert ("AgentRuntime", "Provider", "default") in rels
    assert ("Workspace", "AgentRuntime", "contains") in rels
    assert out["tools"][1]["tools"][0]["tool"] == "get_weather"
    assert out["skills"][1]["sources"][0]["skills"] == 3
    assert out["settings"][1]["endpoints"]["memoryApi"]
    for sec in ("Costs", "Quality", "Memories", "Memory analytics", "Topology", "Tools",
                "Skills", "Settings"):
        assert f">{sec}<" in out["page"]


def test_unconfigured_backends_are_404_not_500():
    async def go():
        r, api = await _serve(_operator_api())
        r2, dash = await _serve(dashboard.build_app(api))
        try:
            async with aiohttp.ClientSession() as s:
                codes = []
                for p in ("/api/workspaces/x/costs", "/api/workspaces/x/memories",
                          "/api/workspaces/x/privacy/consent/stats"):
                    async with s.get(dash + p) as resp:
                        codes.append(resp.status)
                return codes
        finally:
            await r2.cleanup()
            await r.cleanup()

    assert asyncio.run(go()) == [404, 404, 404]


def test_pure_view_builders():
    t = topology({"agentruntimes": OBJS["agentruntimes"], "providers": [], "promptpacks": []})
    assert any(n["id"] == "Provider/ns-a/llama" for n in t["nodes"])  # referenced, not listed
    tv = tools_view([{"metadata": {"namespace": "n", "name": "r"},
                      "spec": {"handlers": [{"name": "h", "tool": {"name": "t"}}]},
                      "status": {"phase": "Pending"}}])
    assert tv == [{"namespace": "n", "registry": "r", "tool": "t", "handler": "h",
                   "endpoint": "", "status": "Pending", "description": ""}]
    assert skills_view([])[:1] == []
