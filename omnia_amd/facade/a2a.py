"""A2A (agent-to-agent) facade: JSON-RPC 2.0 + agent card, task store, and
outbound A2A clients exposed as tools for multi-agent chains.

Reference: ``internal/facade/a2a/server.go:56-104`` (PromptKit server/a2a),
``card_provider.go:29-105`` (``/.well-known/agent.json``),
``redis_task_store.go`` (tasks in memory or Redis), ``client_resolver.go:28-71``
(``spec.facades[].a2a.clients[].exposeAsTools``).

Methods: ``message/send`` (+ legacy ``tasks/send``), ``message/stream``
(SSE; legacy ``tasks/sendSubscribe``), ``tasks/get``, ``tasks/cancel``,
``tasks/resubscribe`` (SSE).  Task lifecycle and cross-replica cancel:
``redis_task_store.go:361-395`` (validated transitions, state changes published
on a pub/sub channel per task).
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
# isValidTransition (internal/facade/a2a/redis_task_store.go:379-395)
TRANSITIONS = {
    "submitted": {"working"},
    "working": {"completed", "failed", "canceled", "input-required", "auth-required",
                "rejected"},
    "input-required": {"working", "canceled"},
    "auth-required": {"working", "canceled"},
}


class InvalidTransition(Exception):
    pass


class TaskNotFound(Exception):
    pass


def _check(frm: str, to: str):
    if to not in TRANSITIONS.get(frm, ()):
        raise InvalidTransition(f"invalid task state transition {frm} -> {to}")


class _TaskStoreBase:
    """Lifecycle over a key/value + pub/sub backend: tasks are created
    ``submitted``; every state change is validated against :data:`TRANSITIONS`
    and published on the task's event channel, which is what makes a cancel on
    one facade replica reach the replica running the task, and what
    ``tasks/resubscribe`` streams."""

    async def create(self, tid: str, ctx: str, message: dict) -> dict:
        task = {"id": tid, "contextId": ctx, "kind": "task",
                "status": {"state": "submitted", "timestamp": time.time()},
                "history": [message], "artifacts": []}
        await self.put(task)
        return task

    async def set_state(self, task: dict, state: str, message: dict | None = None) -> dict:
        # validate against the STORED state (another replica may have canceled the
        # task); a task the store no longer holds (evicted once terminal) stays gone
        cur = await self.get(task["id"])
        if cur is None:
            raise TaskNotFound(task["id"])
        _check(cur["status"]["state"], state)
        task["status"] = {"state": state, "timestamp": time.time(),
                          **({"message": message} if message else {})}
        await self.put(task)
        await self.publish(task["id"], state)
        return task

    async def cancel(self, tid: str) -> dict:
        t = await self.get(tid)
        if t is None:
            raise TaskNotFound(tid)
        _check(t["status"]["state"], "canceled")
        t["status"] = {"state": "canceled", "timestamp": time.time()}
        await self.put(t)
        await self.publish(tid, "canceled")
        return t


class MemoryTaskStore(_TaskStoreBase):
    def __init__(self, max_tasks: int = 10000):
        self.tasks: dict[str, dict] = {}
        self.max_tasks = max_tasks
        self.subs: dict[str, set] = {}

    async def put(self, task: dict):
        self.tasks[task["id"]] = json.loads(json.dumps(task))
        if len(self.tasks) > self.max_tasks:  # evict the oldest terminal tasks
            for k in [k for k, t in self.tasks.items()
                      if t["status"]["state"] in TERMINAL][: len(self.tasks) - self.max_tasks]:
                self.tasks.pop(k, None)

    async def get(self, tid: str):
        t = self.tasks.get(tid)
        return json.loads(json.dumps(t)) if t else None

    async def publish(self, tid: str, state: str):
        for q in list(self.subs.get(tid, ())):
            q.put_nowait(state)

    async def subscribe(self, tid: str):
        q: asyncio.Queue = asyncio.Queue()
        self.subs.setdefault(tid, set()).add(q)
        store = self

        class _Sub:
            async def get(self, timeout=None):
                try:
                    return await asyncio.wait_for(q.get(), timeout)
                except asyncio.TimeoutError:
                    return None

            def close(self):
                store.subs.get(tid, set()).discard(q)
                if not store.subs.get(tid):
                    store.subs.pop(tid, None)

        return _Sub()


class RedisTaskStore(_TaskStoreBase):
    """Tasks as JSON under ``omnia:a2a:task:<id>`` (TTL) and state events on the
    pub/sub channel ``omnia:a2a:events:<id>`` (``redis_task_store.go``)."""

    def __init__(self, client, ttl_s: int = 86400):
        self.r = client
        self.ttl_s = ttl_s

    async def put(self, task):
        await self.r.set(f"omnia:a2a:task:{task['id']}", json.dumps(task), ex=self.ttl_s)

    async def get(self, tid):
        v = await self.r.get(f"omnia:a2a:task:{tid}")
        return json.loads(v) if v else None

    async def publish(self, tid: str, state: str):
        try:
            await self.r.publish(f"omnia:a2a:events:{tid}", state)
        except Exception:  # noqa: BLE001 - best effort, like the reference
            pass

    async def subscribe(self, tid: str):
        sub = await self.r.subscribe(f"omnia:a2a:events:{tid}")

        class _Sub:
            async def get(self, timeout=None):
                m = await sub.get(timeout)
                return m[1] if m else None

            def close(self):
                sub.close()

        return _Sub()


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
    for p in message.get("parts") or []:
        if p.get("kind", p.get("type")) == "text":
            out.append(p.get("text") or "")
        elif p.get("kind") == "data":
            out.append(json.dumps(p.get("data")))
    return "\n".join(out)


def _tool_results(message: dict, pending: list[dict]) -> dict[str, str]:
    """Client-tool results carried by a resume message: ``data`` parts
    ``{"toolCallId": id, "result": ...}`` (or ``{"call_id", "result"}``); a
    single pending call also accepts the message's text / data as its result."""
    out = {}
    for p in message.get("parts") or []:
        d = p.get("data") if p.get("kind") == "data" else None
        if isinstance(d, dict) and (d.get("toolCallId") or d.get("call_id")):
            cid = d.get("toolCallId") or d.get("call_id")
            out[cid] = json.dumps(d.get("result"))
    if not out and len(pending) == 1:
        txt = _text_of(message)
        try:
            json.loads(txt)
        except ValueError:
            txt = json.dumps(txt)
        out[pending[0]["id"]] = txt
    return out


class _Parked:
    """A runtime stream waiting for a client-tool result (task input-required)."""

    def __init__(self, stream, text: list, task: dict, timer):
        self.stream, self.text, self.task, self.timer = stream, text, task, timer


class A2AServer:
    """JSON-RPC task lifecycle (PromptKit ``server/a2a`` semantics):
    ``submitted -> working -> completed | failed | canceled | input-required``.
    A client-tool call leaves the task ``input-required`` with its runtime
    stream parked (``park_timeout_s``); a ``message/send`` on the same task with
    the tool result resumes it (``input-required -> working``) on that stream.
    ``tasks/cancel`` goes through the task store: the state change is published,
    and whichever replica runs the task aborts its stream mid-turn.
    ``tasks/resubscribe`` streams a task's remaining state events (SSE)."""

    def __init__(self, runtime_client, name: str, description: str = "", base_url: str = "",
                 task_store=None, metadata: dict | None = None, skills: list | None = None,
                 park_timeout_s: float = 300.0):
        self.client = runtime_client
        self.skills = skills
        self.name = name
        self.description = description or f"Omnia agent {name}"
        self.base_url = base_url
        self.tasks = task_store or MemoryTaskStore()
        self.md = metadata or {}
        self.park_timeout_s = park_timeout_s
        self.parked: dict[str, _Parked] = {}

    async def card(self, request):
        url = self.base_url or f"http://{request.host}/a2a"
        return web.json_response(agent_card(self.name, self.description, url, self.skills))

    async def _watch_cancel(self, tid: str, flag: asyncio.Event, stream):
        sub = await self.tasks.subscribe(tid)
        try:
            while True:
                st = await sub.get()
                if st is None:
                    return
                if st == "canceled":
                    flag.set()
                    await stream.close()  # unblocks a recv() waiting mid-turn
                    return
        finally:
            sub.close()

    async def _run(self, message: dict, emit=None) -> dict:
        tid = message.get("taskId") or ""
        existing = await self.tasks.get(tid) if tid else None
        if existing is not None:
            return await self._resume(existing, message, emit)
        tid = tid or str(uuid.uuid4())
        ctx = message.get("contextId") or str(uuid.uuid4())
        task = await self.tasks.create(tid, ctx, message)
        await self.tasks.set_state(task, "working")
        if emit:
            await emit({"kind": "status-update", "taskId": tid, "contextId": ctx,
                        "status": task["status"], "final": False})
        stream = await self.client.open({**self.md, "x-omnia-session-id": ctx,
                                         "x-omnia-origin": "a2a"})
        md = {str(k): str(v) for k, v in (message.get("metadata") or {}).items()}
        await stream.send(pb.ClientMessage(session_id=ctx, content=_text_of(message),
                                           metadata=md))
        return await self._pump(task, stream, [], emit)

    async def _resume(self, task: dict, message: dict, emit=None) -> dict:
        tid, ctx = task["id"], task["contextId"]
        if task["status"]["state"] != "input-required":
            raise InvalidTransition(f"task {tid} is {task['status']['state']}, not "
                                    "input-required")
        task["history"].append(message)
        pending = (task.get("metadata") or {}).get("pendingToolCalls") or []
        parked = self.parked.pop(tid, None)
        await self.tasks.set_state(task, "working")
        if emit:
            await emit({"kind": "status-update", "taskId": tid, "contextId": ctx,
                        "status": task["status"], "final": False})
        results = _tool_results(message, pending)
        if parked is not None:
            parked.timer.cancel()
            stream, text = parked.stream, parked.text
            for c in pending:
                r = results.get(c["id"])
                await stream.send(pb.ClientMessage(session_id=ctx, client_tool_result=(
                    pb.ClientToolResult(call_id=c["id"], result_json=r) if r is not None else
                    pb.ClientToolResult(call_id=c["id"], is_rejected=True,
                                        rejection_reason="no result supplied"))))
        else:
            # the stream was parked on another replica (or timed out): continue the
            # conversation on a fresh turn carrying the tool results as the message
            stream, text = await self.client.open({**self.md, "x-omnia-session-id": ctx,
                                                   "x-omnia-origin": "a2a"}), []
            await stream.send(pb.ClientMessage(session_id=ctx, content=json.dumps(
                {"tool_results": results}) if results else _text_of(message)))
        task.setdefault("metadata", {}).pop("pendingToolCalls", None)
        return await self._pump(task, stream, text, emit)

    async def _park_watch(self, tid: str):
        """A parked stream lives until the resume, a cancel published by ANY
        replica, or ``park_timeout_s`` (then the task is canceled)."""
        sub = await self.tasks.subscribe(tid)
        try:
            t0 = time.monotonic()
            while True:
                left = self.park_timeout_s - (time.monotonic() - t0)
                st = await sub.get(timeout=max(0.0, left)) if left > 0 else None
                if st in (None, "canceled"):
                    break
        finally:
            sub.close()
        p = self.parked.pop(tid, None)
        if p is None:
            return
        await p.stream.close()
        try:
            await self.tasks.cancel(tid)
        except (InvalidTransition, TaskNotFound):
            pass  # already canceled (or gone)

    async def _pump(self, task: dict, stream, text: list, emit=None) -> dict:
        tid, ctx = task["id"], task["contextId"]
        cancelled = asyncio.Event()
        watcher = asyncio.ensure_future(self._watch_cancel(tid, cancelled, stream))
        park = False
        final_state = None
        raced = False

        async def settle(state, msg=None) -> bool:
            """The final transition; another replica may have canceled the task
            before its cancel notice reached us (or the task is gone): then the
            stored state wins and is what the client gets."""
            nonlocal raced
            try:
                await self.tasks.set_state(task, state, msg)
                return True
            except (InvalidTransition, TaskNotFound):
                raced = True
                return False

        try:
            while True:
                try:
                    f = await stream.recv()
                except (asyncio.CancelledError, Exception):
                    # a cancel closes the stream under a pending recv (gRPC raises)
                    if not cancelled.is_set():
                        raise
                    f = None
                if cancelled.is_set():
                    final_state = "canceled"
                    break
                if f is None:
                    await settle("failed")
                    break
                k = f.WhichOneof("message")
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
                    task.setdefault("metadata", {})["usage"] = {
                        "input_tokens": f.done.usage.input_tokens,
                        "output_tokens": f.done.usage.output_tokens}
                    await settle("completed", reply)
                    break
                elif k == "error":
                    await settle("failed", {"role": "agent", "parts": [
                        {"kind": "text", "text": f.error.message}]})
                    break
                elif k == "tool_call":
                    tc = f.tool_call
                    calls = [{"id": tc.id, "name": tc.name, "arguments": tc.arguments_json}]
                    task.setdefault("metadata", {})["pendingToolCalls"] = calls
                    msg = {"role": "agent", "kind": "message", "messageId": str(uuid.uuid4()),
                           "contextId": ctx, "taskId": tid,
                           "parts": [{"kind": "data", "data": {"toolCalls": calls}}]}
                    park = await settle("input-required", msg)
                    break
        except (ConnectionError, OSError):
            final_state = "canceled" if cancelled.is_set() else None
            if final_state is None:
                await settle("failed")
        finally:
            watcher.cancel()
            if park and not cancelled.is_set():
                self.parked[tid] = _Parked(stream, text, task, asyncio.ensure_future(
                    self._park_watch(tid)))
            else:
                await stream.close()
        if final_state == "canceled" or raced:
            task = await self.tasks.get(tid) or task
        if emit:
            await emit({"kind": "status-update", "taskId": tid, "contextId": ctx,
                        "status": task["status"],
                        "final": task["status"]["state"] in TERMINAL or park})
        return task

    async def resubscribe(self, tid: str, emit) -> dict | None:
        """``tasks/resubscribe``: the task's current status, then every state
        change published for it until a terminal / input-required state."""
        sub = await self.tasks.subscribe(tid)
        try:
            t = await self.tasks.get(tid)
            if t is None:
                return None
            done = lambda s: s in TERMINAL or s == "input-required"  # noqa: E731
            await emit({"kind": "status-update", "taskId": tid, "contextId": t["contextId"],
                        "status": t["status"], "final": done(t["status"]["state"])})
            while not done(t["status"]["state"]):
                st = await sub.get(timeout=self.park_timeout_s)
                if st is None:
                    break
                t = await self.tasks.get(tid) or t
                if t["status"]["state"] == "completed" and t.get("artifacts"):
                    await emit({"kind": "artifact-update", "taskId": tid,
                                "contextId": t["contextId"], "artifact": t["artifacts"][0],
                                "append": False})
                await emit({"kind": "status-update", "taskId": tid, "contextId": t["contextId"],
                            "status": t["status"], "final": done(t["status"]["state"])})
            return t
        finally:
            sub.close()

    async def rpc(self, request):
        try:
            req = await request.json()
        except Exception:  # noqa: BLE001
            return web.json_response({"jsonrpc": "2.0", "id": None,
                                      "error": {"code": -32700, "message": "parse error"}})
        if not isinstance(req, dict):
            return web.json_response({"jsonrpc": "2.0", "id": None,
                                      "error": {"code": -32600, "message": "invalid request"}})
        rid, method, params = req.get("id"), req.get("method"), req.get("params") or {}
        if not isinstance(method, str):
            method = None

        def ok(result):
            M.A2A_REQUESTS.labels(method or "?", "ok").inc()
            return web.json_response({"jsonrpc": "2.0", "id": rid, "result": result})

        def err(code, msg):
            M.A2A_REQUESTS.labels(method or "?", "error").inc()
            return web.json_response({"jsonrpc": "2.0", "id": rid,
                                      "error": {"code": code, "message": msg}})

        async def sse(run):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                               "Cache-Control": "no-cache"})
            await resp.prepare(request)

            async def emit(ev):
                data = {"jsonrpc": "2.0", "id": rid, "result": ev}
                await resp.write(f"data: {json.dumps(data)}\n\n".encode())

            await run(emit)
            await resp.write_eof()
            M.A2A_REQUESTS.labels(method, "ok").inc()
            return resp

        # JSON-RPC invalid params: wrongly typed params / message / ids answer -32602
        # instead of failing inside the handler
        if not isinstance(params, dict):
            return err(-32602, "params must be an object")
        if not isinstance(params.get("id", ""), str):
            return err(-32602, "params.id must be a string")
        m0 = params.get("message")
        if m0 is not None and (not isinstance(m0, dict) or not all(
                isinstance(m0.get(k) or "", str) for k in ("taskId", "contextId", "messageId",
                                                          "role")) or
                not isinstance(m0.get("metadata") or {}, dict) or
                not isinstance(m0.get("parts") or [], list) or
                not all(isinstance(p, dict) and all(isinstance(p.get(k) or "", str)
                                                    for k in ("text", "kind", "type"))
                        for p in m0.get("parts") or [])):
            return err(-32602, "params.message must be an A2A message object")
        if method in ("message/send", "tasks/send"):
            msg = params.get("message")
            if not msg:
                return err(-32602, "params.message required")
            try:
                return ok(await self._run(msg))
            except InvalidTransition as e:
                return err(-32002, str(e))
            except TaskNotFound as e:
                return err(-32001, f"task {e} not found")
        if method in ("message/stream", "tasks/sendSubscribe"):
            msg = params.get("message")
            if not msg:
                return err(-32602, "params.message required")
            t = await self.tasks.get(msg.get("taskId") or "") if msg.get("taskId") else None
            if t is not None and t["status"]["state"] != "input-required":
                return err(-32002, f"task {t['id']} is {t['status']['state']}, not "
                                   "input-required")
            return await sse(lambda emit: self._run(msg, emit))
        if method == "tasks/resubscribe":
            tid = params.get("id", "")
            if await self.tasks.get(tid) is None:
                return err(-32001, "task not found")
            return await sse(lambda emit: self.resubscribe(tid, emit))
        if method == "tasks/get":
            t = await self.tasks.get(params.get("id", ""))
            return ok(t) if t else err(-32001, "task not found")
        if method == "tasks/cancel":
            tid = params.get("id", "")
            try:
                t = await self.tasks.cancel(tid)
            except TaskNotFound:
                return err(-32001, "task not found")
            except InvalidTransition:
                return err(-32002, "task is not cancelable")
            p = self.parked.pop(tid, None)
            if p is not None:  # parked here: release its runtime stream now
                p.timer.cancel()
                await p.stream.close()
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
                     headers: dict | None = None, timeout=None):
    """An InProcessHandler exposing a remote agent as a tool (multi-agent chains).
    ``timeout`` (seconds or a duration string; default the executor's 30 s)
    bounds one delegated turn."""
    from ..tools.executor import InProcessHandler, _dur

    # one parse, both bounds: the HTTP session (A2AClient) and the tool call
    # (InProcessHandler) -- a spec timeout above the client's 120 s default must
    # not be cut off by aiohttp
    secs = _dur(timeout, None)
    client = A2AClient(url if url.rstrip("/").endswith("/a2a") else url.rstrip("/") + "/a2a",
                       headers=headers, **({"timeout_s": secs} if secs else {}))

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
        description or f"Delegate a question to the {name} agent", schema, call)},
        timeout=secs if secs else timeout)
