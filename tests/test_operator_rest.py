"""Operator REST extras: ToolRegistry tool-test through the real executor,
DeployIntent translation (dry-run + apply, re-apply updates), workspace content
API with traversal guard."""
import asyncio
import json

import aiohttp
from aiohttp import web

from omnia_amd.operator.apiserver import build_app
from omnia_amd.operator.apistore import APIStore

PACK = {"id": "p", "name": "P", "version": "1.0.0",
        "prompts": {"default": {"id": "default", "name": "d", "version": "1.0.0",
                                "system_template": "hi"}}}


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


def test_tool_test_deploy_and_content(tmp_path, monkeypatch):
    monkeypatch.setenv("OMNIA_CONTENT_ROOT", str(tmp_path))

    async def backend(request):
        return web.json_response({"temp": 21, "city": request.query.get("city")})

    async def go():
        tools_app = web.Application()
        tools_app.router.add_get("/weather", backend)
        r_tools, turl = await _serve(tools_app)
        store = APIStore()
        store.create({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "ToolRegistry",
                      "metadata": {"name": "wx", "namespace": "default"},
                      "spec": {"handlers": [{"name": "weather", "type": "http", "tool": {
                          "name": "get_weather", "description": "w",
                          "inputSchema": {"type": "object", "properties": {
                              "city": {"type": "string"}}}},
                          "httpConfig": {"endpoint": turl + "/weather", "method": "GET",
                                         "queryParams": ["city"]}}]}})
        r_api, base = await _serve(build_app(store))
        out = {}
        try:
            async with aiohttp.ClientSession() as s:
                r = await s.post(f"{base}/api/v1/namespaces/default/toolregistries/wx/test",
                                 json={"tool": "get_weather", "arguments": {"city": "Oslo"}})
                out["tool"] = await r.json()
                r = await s.post(f"{base}/api/v1/namespaces/default/toolregistries/wx/test",
                                 json={"tool": "nope"})
                out["tool404"] = r.status
                intent = {"pack": {"name": "support", "content": PACK},
                          "agents": [{"name": "a1", "providers": [{"ref": "llm"}]},
                                     {"name": "a2", "providers": [{"ref": "llm"}],
                                      "facades": [{"type": "websocket"}, {"type": "a2a"}]}]}
                r = await s.post(f"{base}/api/v1/namespaces/default/deploy?dryRun=true",
                                 json=intent)
                out["dry"] = (r.status, await r.json())
                r = await s.post(f"{base}/api/v1/namespaces/default/deploy", json=intent)
                out["apply"] = (r.status, await r.json())
                r = await s.post(f"{base}/api/v1/namespaces/default/deploy", json=intent)
                out["reapply"] = await r.json()
                r = await s.post(f"{base}/api/v1/namespaces/default/deploy", json={"pack": {}})
                out["bad"] = r.status
                r = await s.put(f"{base}/api/v1/workspaces/w1/content/skills/a/SKILL.md",
                                data=b"# a")
                out["put"] = r.status
                r = await s.get(f"{base}/api/v1/workspaces/w1/content/skills/a")
                out["ls"] = await r.json()
                r = await s.get(f"{base}/api/v1/workspaces/w1/content/..%2F..%2Fetc%2Fpasswd")
                out["trav"] = r.status
        finally:
            await r_api.cleanup()
            await r_tools.cleanup()
        return out, store

    out, store = asyncio.run(go())
    assert out["tool"].get("ok"), out["tool"]
    assert out["tool"]["ok"] and out["tool"]["result"]["city"] == "Oslo"
    assert out["tool404"] == 404
    assert out["dry"][0] == 200 and all(x["action"] == "validated" for x in out["dry"][1]["applied"])
    assert out["apply"][0] == 201
    kinds = [(x["kind"], x["action"]) for x in out["apply"][1]["applied"]]
    assert kinds == [("ConfigMap", "created"), ("PromptPack", "created"),
                     ("AgentRuntime", "created"), ("AgentRuntime", "created")]
    assert all(x["action"] == "updated" for x in out["reapply"]["applied"])
    assert out["bad"] == 400 and out["put"] == 201
    assert out["ls"]["entries"][0]["name"] == "SKILL.md"
    assert out["trav"] in (403, 404)
    ar = store.get("AgentRuntime", "a2", "default")
    assert [f["type"] for f in ar["spec"]["facades"]] == ["websocket", "a2a"]
