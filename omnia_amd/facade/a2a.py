"""A2A (agent-to-agent) facade: JSON-RPC 2.0 + agent card, task store, and
outbound A2A clients exposed as tools for multi-agent chains.

Reference: ``internal/facade/a2a/server.go:56-104`` (PromptKit server/a2a),
``card_provider.go:29-105`` (``/.well-known/agent.json``),
``redis_task_store.go`` (tasks in memory or Redis), ``client_resolver.go:28-71``
(``spec.facades[].a2a.clients[].exposeAsTools``).

Methods: ``message/send`` (+ legacy ``tasks/send``), ``message/stream``
(SSE; legacy ``tasks/sendSubscribe``), ``tasks/get``, ``tasks/cancel``.
"""
from __future__ import annotations

import asyncio
import json
import time
import uuid

from aiohttp import web

from ..api.proto import runtime_v1 as pb
from ..observability import metrics as M

TERMINAL = {"completed", "failed", "canceled", "rejected"}


class MemoryTaskStore:
    def __init__(self):
        self.tasks: dict[str, dict] = {}

    async def put(self, task: dict):
        self.tasks[task["id"]] = json.loads(json.dumps(task))

    async def get(self, tid: str):
        t = self.tasks.get(tid)
        return json.loads(json.dumps(t)) if t else None


class RedisTaskStore:
    def __init__(self, client, ttl_s: int = 86400):
        self.r = client
        self.ttl_s = ttl_s

    async def put(self, task):
        await self.r.set(f"omnia:a2a:task:{task['id']}", json.dumps(task), ex=self.ttl_s)

    async def get(self, tid):
        v = await self.r.get(f"omnia:a2a:task:{tid}")
        return json.loads(v) if v else None


def agent_card(name: str, description: str, url: str, skills: list | None = None,
               streaming: bool = True) -> dict:
    return {"name": name, "description": description, "url": url, "version": "1.0.0",
            "protocolVersion": "0.3.0",
            "capabilities": {"streaming": streaming, "pushNotifications": False,
                             "stateTransitionHistory": True},
            "defaultInputModes": ["text/plain", "application/json"],
            "defaultOutputModes": ["text/plain"],
            "skills": skills or [{"id": "chat", "name": name, "description": description,
                                  "tags": ["chat"]}]}


def _text_of(message: dict) -> str:
    out = []
    for p in message.get("parts", []):
        if p.get("kind", p.get("type")) == "text":
            out.append(p.get("text", ""))
        elif p.get("kind") == "data":
            out.append(json.dumps(p.get("data")))
    return "\n".join(out)


class A2AServer:
    def __init__(self, runtime_client, name: str, description: str = "", base_url: str = "",
                 task_store=None, metadata: dict | None = None, skills: list | None = None):
        self.client = runtime_client
        self.skills = skills
        self.name = name
        self.description = description or f"Omnia agent {name}"
        self.base_url = base_url
        self.tasks = task_store or MemoryTaskStore()
        self.md = metadata or {}
        self.cancelled: set = set()

    async def card(self, request):
        url = self.base_url or f"http://{request.host}/a2a"
        return web.json_response(agent_card(self.name, self.description, url, self.skills))

    async def _run(self, message: dict, emit=None) -> dict:
        tid = message.get("taskId") or str(uuid.uuid4())
        ctx = message.get("contextId") or str(uuid.uuid4())
        task = {"id": tid, "contextId": ctx, "kind": "task",
                "status": {"state": "working", "timestamp": time.time()},
                "history": [message], "artifacts": []}
        await self.tasks.put(task)
        if emit:
            await emit({"kind": "status-update", "taskId": tid, "contextId": ctx,
                        "status": task["status"], "final": False})
        stream = await self.client.open({**self.md, "x-omnia-session-id": ctx,
                                         "x-omnia-origin": "a2a"})
        text = []
        try:
            await stream.send(pb.ClientMessage(session_id=ctx, content=_text_of(message)))
            while True:
                f = await stream.recv()
                if f is None:
                    task["status"] = {"state": "failed", "timestamp": time.time()}
                    break
                k = f.WhichOneof("message")
                if tid in self.cancelled:
                    task["status"] = {"state": "canceled", "timestamp": time.time()}
                    break
                if k == "chunk":
                    text.append(f.chunk.content)
                    if emit:
                        await emit({"kind": "artifact-update", "taskId": tid, "contextId": ctx,
                                    "artifact": {"artifactId": "response", "parts": [
                                        {"kind": "text", "text": f.chunk.content}]},
                                    "append": True})
                elif k == "done":
                    final = f.done.final_content or "".join(text)
                    task["artifacts"] = [{"artifactId": "response", "parts": [
                        {"kind": "text", "text": final}]}]
                    reply = {"role": "agent", "kind": "message", "messageId": str(uuid.uuid4()),
                             "parts": [{"kind": "text", "text": final}], "contextId": ctx,
                             "taskId": tid}
                    task["history"].append(reply)
                    task["status"] = {"state": "completed", "message": reply,
                                      "timestamp": time.time()}
                    task["metadata"] = {"usage": {"input_tokens": f.done.usage.input_tokens,
                                                  "output_tokens": f.done.usage.output_tokens}}
                    break
                elif k == "error":
                    task["status"] = {"state": "failed", "timestamp": time.time(),
                                      "message": {"role": "agent", "parts": [
                                          {"kind": "text", "text": f.error.message}]}}
                    break
                elif k == "tool_call":
                    task["status"] = {"state": "input-required", "timestamp": time.time()}
                    break
        finally:
            await stream.close()
        await self.tasks.put(task)
        if emit:
            await emit({"kind": "status-update", "taskId": tid, "contextId": ctx,
                        "status": task["status"], "final": True})
        return task

    async def rpc(self, request):
        try:
            req = await request.json()
        except Exception:  # noqa: BLE001
            return web.json_response({"jsonrpc": "2.0", "id": None,
                                      "error": {"code": -32700, "message": "parse error"}})
        rid, method, params = req.get("id"), req.get("method"), req.get("params") or {}

        def ok(result):
            M.A2A_REQUESTS.labels(method or "?", "ok").inc()
            return web.json_response({"jsonrpc": "2.0", "id": rid, "result": result})

        def err(code, msg):
            M.A2A_REQUESTS.labels(method or "?", "error").inc()
            return web.json_response({"jsonrpc": "2.0", "id": rid,
                                      "error": {"code": code, "message": msg}})

        if method in ("message/send", "tasks/send"):
            msg = params.get("message")
            if not msg:
                return err(-32602, "params.message required")
            return ok(await self._run(msg))
        if method in ("message/stream", "tasks/sendSubscribe"):
            msg = params.get("message")
            if not msg:
                return err(-32602, "params.message required")
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                               "Cache-Control": "no-cache"})
            await resp.prepare(request)

            async def emit(ev):
                data = {"jsonrpc": "2.0", "id": rid, "result": ev}
                await resp.write(f"data: {json.dumps(data)}\n\n".encode())

            await self._run(msg, emit)
            await resp.write_eof()
            M.A2A_REQUESTS.labels(method, "ok").inc()
            return resp
        if method == "tasks/get":
            t = await self.tasks.get(params.get("id", ""))
            return ok(t) if t else err(-32001, "task not found")
        if method == "tasks/cancel":
            t = await self.tasks.get(params.get("id", ""))
            if t is None:
                return err(-32001, "task not found")
            if t["status"]["state"] in TERMINAL:
                return err(-32002, "task is not cancelable")
            self.cancelled.add(t["id"])
            t["status"] = {"state": "canceled", "timestamp": time.time()}
            await self.tasks.put(t)
            return ok(t)
        return err(-32601, f"method {method} not found")


def pack_card_skills(path: str | None) -> list | None:
    """Card skills of a multi-agent PromptPack (one per ``agents.members``
    entry); None for plain packs or an unreadable pack."""
    if not path:
        return None
    from ..runtime.promptpack import PackError, PromptPack
    from ..runtime.workflow import card_skills

    try:
        pack = PromptPack.load(path)
    except (OSError, PackError):
        return None
    return card_skills(pack) or None


def mount_a2a(facade, runtime_client, path: str = "/a2a", **kw) -> A2AServer:
    import os

    kw.setdefault("skills", pack_card_skills(os.environ.get("OMNIA_PROMPTPACK_PATH")))
    srv = A2AServer(runtime_client, facade.cfg.agent, **kw)
    facade.app.router.add_get("/.well-known/agent.json", srv.card)
    facade.app.router.add_get("/.well-known/agent-card.json", srv.card)
    facade.app.router.add_post(path, srv.rpc)
    return srv


class A2AClient:
    """Outbound A2A client (``BuildA2AAgentOptions``) -- also usable as a tool."""

    def __init__(self, url: str, timeout_s: float = 120.0, headers: dict | None = None):
        self.url = url.rstrip("/")
        self.timeout_s = timeout_s
        self.headers = headers or {}

    async def card(self) -> dict:
        import aiohttp

        base = self.url.rsplit("/a2a", 1)[0]
        async with aiohttp.ClientSession() as s:
            async with s.get(base + "/.well-known/agent.json") as r:
                return await r.json()

    async def send(self, text: str, context_id: str | None = None) -> dict:
        import aiohttp

        body = {"jsonrpc": "2.0", "id": str(uuid.uuid4()), "method": "message/send",
                "params": {"message": {"role": "user", "kind": "message",
                                       "messageId": str(uuid.uuid4()),
                                       "parts": [{"kind": "text", "text": text}],
                                       **({"contextId": context_id} if context_id else {})}}}
        async with aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
            async with s.post(self.url, json=body, headers=self.headers) as r:
                d = await r.json()
        if "error" in d:
            raise RuntimeError(d["error"].get("message"))
        return d["result"]


def a2a_tool_handler(name: str, url: str, description: str = "",
                     headers: dict | None = None):
    """An InProcessHandler exposing a remote agent as a tool (multi-agent chains)."""
    from ..tools.executor import InProcessHandler

    client = A2AClient(url if url.rstrip("/").endswith("/a2a") else url.rstrip("/") + "/a2a",
                       headers=headers)

    async def call(args, ctx):
        task = await client.send(args.get("message") or args.get("input") or json.dumps(args),
                                 context_id=(ctx.session_id or None) and f"{ctx.session_id}-"
                                                                         f"{name}")
        st = task.get("status", {})
        parts = (st.get("message") or {}).get("parts") or (task.get("artifacts") or [{}])[0].get(
            "parts", [])
        return {"agent": name, "state": st.get("state"),
                "response": " ".join(p.get("text", "") for p in parts)}

    # bounded so the local engine's tool-call grammar always closes the string
    schema = {"type": "object", "properties": {"message": {"type": "string", "maxLength": 512,
                                                           "description": "what to ask"}},
              "required": ["message"]}
    return InProcessHandler(f"a2a-{name}", {f"ask_{name}": (
        description or f"Delegate a question to the {name} agent", schema, call)})
