"""Arena dev console (reference ``ee/cmd/arena-dev-console``).

Interactive WebSocket server for testing an agent definition while editing it:

* ``{"type": "config", "promptpack": {...pack.json...} | null, "system": str,
  "provider": {...Provider spec...}, "tools": {...ToolRegistry spec...},
  "defaults": {...}}`` -- (re)build the agent: HOT RELOAD, conversation
  history of the connection's sessions is kept across reloads (the context
  store outlives the agent);
* ``{"type": "message", "content": "...", "session_id": "..."}`` -- one turn
  through the same agent loop the runtime serves (PromptPack rendering, tool
  rounds, provider streaming): frames ``chunk`` / ``tool_call`` / ``done`` /
  ``error`` like the facade protocol;
* ``{"type": "providers"}`` -- list the Provider objects the operator knows
  (``--api``), so the dashboard can offer them.
Turns are optionally recorded to session-api (``--session-api``) with
``metadata.dev_session = true``.  The provider may be ``type: local`` -- the
in-node MI355X engine -- when the console runs inside a runtime pod.
"""
from __future__ import annotations

import argparse
import json
import uuid

from aiohttp import WSMsgType, web

from ..runtime.agent import Agent, AgentConfig, TurnIO
from ..runtime.context_store import MemoryContextStore
from ..runtime.promptpack import PromptPack
from ..runtime.providers import build_provider


class _WSIO(TurnIO):
    def __init__(self, sock, sid):
        self.sock, self.sid = sock, sid

    async def chunk(self, text: str) -> None:
        await self.sock.send_json({"type": "chunk", "session_id": self.sid, "content": text})


class DevConsole:
    def __init__(self, api: str = "", session_api: str = "", engine_factory=None):
        self.api = api.rstrip("/")
        self.session_api = session_api
        self.engine_factory = engine_factory
        self.store = MemoryContextStore()
        self.reloads = 0

    def build_agent(self, cfg: dict) -> Agent:
        pack = PromptPack(cfg["promptpack"]) if cfg.get("promptpack") else \
            PromptPack.minimal(cfg.get("system") or "You are a helpful assistant.")
        pspec = cfg.get("provider") or {"type": "mock"}
        engine = None
        if (pspec.get("type") or "").lower() in ("local", "omnia", "engine", "rocm"):
            if self.engine_factory is None:
                raise ValueError("local provider unavailable in this console")
            engine = self.engine_factory(cfg.get("engine") or {})
        provider = build_provider(pspec, engine=engine)
        executor = None
        if cfg.get("tools"):
            from ..tools.executor import OmniaExecutor

            executor = OmniaExecutor(cfg["tools"])
        return Agent(pack, provider, self.store, executor,
                     AgentConfig(defaults=cfg.get("defaults") or {}))

    async def providers(self) -> list[dict]:
        if not self.api:
            return []
        import aiohttp

        from ..api import crds

        async with aiohttp.ClientSession() as s:
            async with s.get(f"{self.api}/apis/{crds.GROUP}/{crds.VERSION}/providers",
                             timeout=aiohttp.ClientTimeout(total=10)) as r:
                body = await r.json(content_type=None)
        return [{"name": it["metadata"]["name"], "namespace": it["metadata"].get("namespace"),
                 "type": it["spec"].get("type"), "model": it["spec"].get("model")}
                for it in body.get("items", [])]

    async def record(self, sid: str, role: str, content: str) -> None:
        if not self.session_api:
            return
        import aiohttp

        async with aiohttp.ClientSession() as s:
            await s.post(f"{self.session_api}/api/v1/sessions",
                         json={"id": sid, "agent_name": "dev-console",
                               "state": {"dev_session": True}})
            await s.post(f"{self.session_api}/api/v1/sessions/{sid}/messages",
                         json={"role": role, "content": content,
                               "metadata": {"dev_session": "true"}})

    async def handle_ws(self, request):
        sock = web.WebSocketResponse(heartbeat=30)
        await sock.prepare(request)
        agent = None
        async for m in sock:
            if m.type != WSMsgType.TEXT:
                break
            try:
                msg = json.loads(m.data)
            except json.JSONDecodeError:
                await sock.send_json({"type": "error", "error": {"code": "INVALID_MESSAGE",
                                                                  "message": "bad json"}})
                continue
            t = msg.get("type")
            try:
                if t in ("config", "reload"):
                    agent = self.build_agent(msg)
                    if t == "reload":
                        self.reloads += 1
                    await sock.send_json({"type": "configured",
                                          "provider": agent.provider.type,
                                          "model": agent.provider.model})
                elif t == "providers":
                    await sock.send_json({"type": "providers", "items": await self.providers()})
                elif t == "message":
                    if agent is None:
                        agent = self.build_agent({})
                    sid = msg.get("session_id") or uuid.uuid4().hex
                    res = await agent.run_turn(sid, msg.get("content", ""), _WSIO(sock, sid),
                                               metadata={"dev_session": "true"})
                    await self.record(sid, "user", msg.get("content", ""))
                    await self.record(sid, "assistant", res.content)
                    await sock.send_json({"type": "done", "session_id": sid,
                                          "content": res.content,
                                          "tool_calls": res.tool_calls, "rounds": res.rounds,
                                          "usage": {"input_tokens": res.usage.input_tokens,
                                                    "output_tokens": res.usage.output_tokens}})
                else:
                    await sock.send_json({"type": "error", "error": {
                        "code": "INVALID_MESSAGE", "message": f"unknown type {t!r}"}})
            except Exception as e:  # noqa: BLE001 - reported to the developer
                await sock.send_json({"type": "error", "error": {"code": "DEV_CONSOLE_ERROR",
                                                                 "message": str(e)}})
        return sock


def build_app(console: DevConsole) -> web.Application:
    app = web.Application()

    async def healthz(_):
        return web.json_response({"status": "ok"})

    async def providers(_):
        return web.json_response({"items": await console.providers()})

    app.router.add_get("/ws", console.handle_ws)
    app.router.add_get("/api/providers", providers)
    app.router.add_get("/healthz", healthz)
    return app


def main(argv=None):
    ap = argparse.ArgumentParser("arena-dev-console")
    ap.add_argument("--port", type=int, default=8086)
    ap.add_argument("--api", default="")
    ap.add_argument("--session-api", default="")
    ap.add_argument("--engine", action="store_true", help="allow type: local providers")
    a = ap.parse_args(argv)
    factory = None
    if a.engine:
        from ..runtime.app import shared_engine

        factory = shared_engine
    web.run_app(build_app(DevConsole(a.api, a.session_api, factory)), port=a.port)


if __name__ == "__main__":
    main()
