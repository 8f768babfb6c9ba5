"""``omnia.runtime.v1`` RuntimeService: Converse / Invoke / Health / HasConversation.

Transport-agnostic core (:class:`RuntimeService`, driven through a small
``Stream`` interface so tests, the bench and the in-process facade can call it
without sockets) plus the grpc.aio adapter (:func:`serve_grpc`) and the
health/metrics HTTP listener (:9001 ``/healthz`` ``/readyz`` ``/metrics``).

Protocol rules enforced (``pkg/runtime/conformance/checks.go:44-230``,
``internal/runtime/server.go:715-777``):
  * the first ServerMessage of every text Converse stream is RuntimeHello with
    the same capability set Health reports;
  * each turn ends with Done{usage}; errors become an Error frame with a
    generic message (provider details are never leaked) and the stream stays up;
  * only implemented capabilities are advertised (``invoke``, ``client_tools``,
    ``consent_grants``); Invoke is served, DuplexStart is answered on-protocol
    with an Error frame because ``duplex_audio`` is NOT advertised.
"""
from __future__ import annotations

import asyncio
import os
import json
import logging
import time
import uuid

from ..utils.arrivals import mark
from ..api.proto import runtime_v1 as pb
from ..observability import metrics as M
from ..observability import tracing
from ..tools.executor import CallContext
from .agent import Agent, TurnIO
from .providers import ProviderError
from .chat import ToolCallReq
from .context_store import StoreUnavailable

log = logging.getLogger("omnia.runtime.server")

CAPABILITIES = [pb.CAP_INVOKE, pb.CAP_CLIENT_TOOLS, pb.CAP_CONSENT_GRANTS]
GENERIC_ERROR = "an internal error occurred while processing the message"


def identity_from_metadata(md: dict, session_id: str = "") -> CallContext:
    """Flat x-omnia-* metadata (``pkg/policy/context.go:80-147``)."""
    claims = {k[len("x-omnia-claim-"):]: v for k, v in md.items()
              if k.startswith("x-omnia-claim-")}
    headers = {k: v for k, v in md.items() if k.startswith("x-omnia-")}
    return CallContext(session_id=session_id or md.get("x-omnia-session-id", ""),
                       agent=md.get("x-omnia-agent-name", ""),
                       namespace=md.get("x-omnia-namespace", ""),
                       workspace=md.get("x-omnia-workspace", ""),
                       user_id=md.get("x-omnia-user-id", ""), origin=md.get("x-omnia-origin", ""),
                       claims=claims, headers=headers)


class Stream:
    """Minimal bidi stream interface."""

    async def recv(self):  # -> pb.ClientMessage | None
        raise NotImplementedError

    async def send(self, msg) -> None:
        raise NotImplementedError

    def metadata(self) -> dict:
        return {}


class QueueStream(Stream):
    """In-process stream over asyncio queues (tests, bench, in-pod facade)."""

    def __init__(self, md: dict | None = None):
        self.inbox: asyncio.Queue = asyncio.Queue()
        self.outbox: asyncio.Queue = asyncio.Queue()
        self._md = md or {}

    async def recv(self):
        return await self.inbox.get()

    async def send(self, msg):
        await self.outbox.put(msg)

    def metadata(self):
        return self._md

    def close(self):
        self.inbox.put_nowait(None)


class _GrpcTurnIO(TurnIO):
    """Turn output onto the Converse stream.

    ``interval_s`` > 0 coalesces text deltas: the first delta of a turn goes out
    at once (TTFT is unaffected), later deltas are sent at most once per
    interval as one Chunk with their concatenated text (a timer flushes a
    partial buffer, so no text waits longer than the interval).  Every other
    frame (tool calls, Done, Error) first flushes the buffer, so frame order is
    the order of the deltas.  ``interval_s`` = 0 sends one Chunk per delta
    (the reference's behaviour, ``internal/runtime/server.go:742-760``)."""

    def __init__(self, stream: Stream, pending_msgs: list, interval_s: float = 0.0):
        self.stream = stream
        self.pending = pending_msgs
        self.nchunks = 0
        self.interval = interval_s
        self.buf: list[str] = []
        self.last = -1e9
        self.timer = None
        self.lock = asyncio.Lock()

    async def chunk(self, text: str) -> None:
        if self.interval <= 0:
            self.nchunks += 1
            await self.stream.send(pb.ServerMessage(chunk=pb.Chunk(content=text)))
            return
        self.buf.append(text)
        wait = self.interval - (time.monotonic() - self.last)
        if wait <= 0:
            await self.flush()
        elif self.timer is None:
            self.timer = asyncio.get_running_loop().call_later(wait, self._on_timer)

    def _on_timer(self):
        self.timer = None
        if self.buf:
            asyncio.ensure_future(self.flush())

    async def flush(self) -> None:
        async with self.lock:
            if self.timer is not None:
                self.timer.cancel()
                self.timer = None
            if not self.buf:
                return
            text = "".join(self.buf)
            self.buf.clear()
            self.last = time.monotonic()
            self.nchunks += 1
            await self.stream.send(pb.ServerMessage(chunk=pb.Chunk(content=text)))

    async def client_tool_calls(self, calls: list[ToolCallReq], meta: dict) -> dict:
        await self.flush()
        for c in calls:
            m = meta.get(c.id, {})
            await self.stream.send(pb.ServerMessage(tool_call=pb.ToolCall(
                id=c.id, name=c.name, arguments_json=c.arguments_json,
                execution=pb.TOOL_EXECUTION_CLIENT,
                consent_message=m.get("consentMessage", ""),
                categories=m.get("categories", []))))
        want = {c.id for c in calls}
        got: dict[str, dict] = {}
        while want - set(got):
            msg = await self.stream.recv()
            if msg is None:
                raise ConnectionError("stream closed while waiting for client tool results")
            if msg.HasField("client_tool_result"):
                r = msg.client_tool_result
                got[r.call_id] = {"result_json": r.result_json, "is_rejected": r.is_rejected,
                                  "rejection_reason": r.rejection_reason}
            else:
                self.pending.append(msg)  # a new user message racing the tool result
        return got


class RuntimeService:
    def __init__(self, agent: Agent, capabilities: list[str] | None = None,
                 invoke_agent: Agent | None = None, duplex=None, stream_interval_s: float = 0.0):
        self.agent = agent
        # text-delta coalescing window of Converse streams (OMNIA_STREAM_INTERVAL_MS)
        self.stream_interval_s = stream_interval_s
        self.invoke_agent = invoke_agent or agent
        self.capabilities = list(capabilities or CAPABILITIES)
        self.duplex = duplex  # DuplexConfig when STT + TTS providers are configured
        if duplex is not None:
            for c in (pb.CAP_DUPLEX_AUDIO, pb.CAP_INTERRUPTION):
                if c not in self.capabilities:
                    self.capabilities.append(c)
        self.ready = True
        self.active_streams = 0

    # ------------------------------------------------------------ Health
    async def health(self, req=None) -> pb.HealthResponse:
        ok = self.ready
        try:
            ok = ok and await self.agent.provider.health()
        except Exception:  # noqa: BLE001
            ok = False
        return pb.HealthResponse(healthy=ok, status="ok" if ok else "degraded",
                                 contract_version=pb.CONTRACT_VERSION,
                                 capabilities=self.capabilities)

    # ------------------------------------------------------------ HasConversation
    async def has_conversation(self, req) -> pb.HasConversationResponse:
        if not req.session_id:
            return pb.HasConversationResponse(state=pb.RESUME_STATE_NOT_FOUND)
        try:
            st = await self.agent.store.load(req.session_id)
        except StoreUnavailable as e:
            return pb.HasConversationResponse(state=pb.RESUME_STATE_UNAVAILABLE, detail=str(e))
        except Exception as e:  # noqa: BLE001
            return pb.HasConversationResponse(state=pb.RESUME_STATE_UNAVAILABLE, detail=str(e))
        if st is None:
            return pb.HasConversationResponse(state=pb.RESUME_STATE_NOT_FOUND)
        return pb.HasConversationResponse(state=pb.RESUME_STATE_RESUMABLE)

    # ------------------------------------------------------------ Invoke
    async def invoke(self, req, md: dict | None = None) -> pb.InvocationResponse:
        t0 = time.perf_counter()
        inv = req.invocation_id or uuid.uuid4().hex
        ctx = identity_from_metadata(dict(md or {}), inv)

        class _Collect(TurnIO):
            async def chunk(self, text):
                pass

        res = await self.invoke_agent.run_turn(inv, req.input_json, _Collect(),
                                               metadata=dict(req.metadata), ctx=ctx,
                                               persist=False)
        return pb.InvocationResponse(output_json=res.content,
                                     usage=pb.Usage(input_tokens=res.usage.input_tokens,
                                                    output_tokens=res.usage.output_tokens,
                                                    cost_usd=res.cost),
                                     duration_ms=int((time.perf_counter() - t0) * 1000),
                                     invocation_id=inv)

    # ------------------------------------------------------------ Converse
    async def converse(self, stream: Stream) -> None:
        self.active_streams += 1
        hello_sent = False
        pending: list = []
        md = dict(stream.metadata() or {})
        sids: set = set()
        try:
            while True:
                msg = pending.pop(0) if pending else await stream.recv()
                if msg is None:
                    return
                if msg.HasField("duplex_start"):
                    if self.duplex is None:
                        await stream.send(pb.ServerMessage(error=pb.Error(
                            code="DUPLEX_UNSUPPORTED",
                            message="this runtime does not advertise duplex_audio")))
                        return
                    from .duplex import DuplexSession

                    sid = msg.session_id or md.get("x-omnia-session-id") or uuid.uuid4().hex
                    await DuplexSession(self.agent, self.duplex, stream, sid,
                                        identity_from_metadata(md, sid)).run(msg)
                    return
                if not hello_sent:
                    await stream.send(pb.ServerMessage(runtime_hello=pb.RuntimeHello(
                        capabilities=self.capabilities)))
                    hello_sent = True
                if msg.HasField("client_tool_result") and not msg.content and not msg.parts:
                    continue  # stray result outside a turn
                sids.add(await self._turn(stream, msg, md, pending))
        finally:
            self.active_streams -= 1
            # the conversation stream closed: its session-trigger inline evals
            ev = getattr(self.agent, "evaluator", None)
            if ev is not None and hasattr(ev, "on_session_complete"):
                for sid in sids - {None}:
                    asyncio.get_running_loop().create_task(ev.on_session_complete(sid))

    async def _turn(self, stream: Stream, msg, md: dict, pending: list):
        mark("runtime_turn")
        sid = msg.session_id or md.get("x-omnia-session-id") or uuid.uuid4().hex
        content = msg.content
        parts = []
        for p in msg.parts:
            if p.type == "text":
                content = (content + "\n" + p.text) if content else p.text
            else:
                parts.append({"type": p.type, "mime_type": p.media.mime_type,
                              "url": p.media.url, "storage_ref": p.media.storage_ref})
        if not content and not parts:
            await stream.send(pb.ServerMessage(error=pb.Error(code="INVALID_MESSAGE",
                                                              message="empty message")))
            return None
        ctx = identity_from_metadata(md, sid)
        metadata = dict(msg.metadata)
        if msg.consent_grants:
            metadata["consent_grants"] = ",".join(msg.consent_grants)
        io = _GrpcTurnIO(stream, pending, self.stream_interval_s)
        tp = tracing.parse_traceparent(md.get("traceparent"))
        span = tracing.start_span("omnia.runtime.message", {"session.id": sid},
                                  trace_id=tracing.session_trace_id(sid), link=tp)
        try:
            res = await self.agent.run_turn(sid, content, io, parts=parts, metadata=metadata,
                                            ctx=ctx)
            await io.flush()
        except ProviderError as e:  # coded provider failure (e.g. ENGINE_FAULT)
            await io.flush()
            log.error("turn failed for session %s: %s (%s)", sid, e, e.code)
            tracing.end_span(span, error=True)
            await stream.send(pb.ServerMessage(error=pb.Error(code=e.code,
                                                              message=GENERIC_ERROR)))
            return sid
        except Exception:  # noqa: BLE001 - never leak provider details
            await io.flush()
            log.exception("turn failed for session %s", sid)
            tracing.end_span(span, error=True)
            await stream.send(pb.ServerMessage(error=pb.Error(code="INTERNAL_ERROR",
                                                              message=GENERIC_ERROR)))
            return sid
        tracing.end_span(span)
        mark("runtime_done")
        await stream.send(pb.ServerMessage(done=pb.Done(
            final_content=res.content,
            usage=pb.Usage(input_tokens=res.usage.input_tokens,
                           output_tokens=res.usage.output_tokens, cost_usd=res.cost,
                           cached_tokens=res.usage.cached_tokens))))
        return sid


# ===================================================================== gRPC
class _GrpcStream(Stream):
    def __init__(self, context):
        self.ctx = context
        self._md = {k: v for k, v in (context.invocation_metadata() or [])}

    async def recv(self):
        import grpc

        m = await self.ctx.read()
        if m is grpc.aio.EOF:
            return None
        return m

    async def send(self, msg):
        await self.ctx.write(msg)

    def metadata(self):
        return self._md


def grpc_handler(svc: RuntimeService):
    import grpc

    async def invoke(req, context):
        md = {k: v for k, v in (context.invocation_metadata() or [])}
        if pb.CAP_INVOKE not in svc.capabilities:
            await context.abort(grpc.StatusCode.UNIMPLEMENTED, "invoke not supported")
        try:
            return await svc.invoke(req, md)
        except Exception:  # noqa: BLE001
            log.exception("invoke failed")
            await context.abort(grpc.StatusCode.INTERNAL, GENERIC_ERROR)

    async def health(req, context):
        return await svc.health(req)

    async def has_conversation(req, context):
        return await svc.has_conversation(req)

    adapter = _ConverseAdapter(svc)

    async def converse_gen(request_iterator, context):
        async for m in adapter._run(request_iterator, context):
            yield m

    async def converse_direct(_request_iterator, context):
        # frames go straight through context.read() / context.write(): no output
        # queue + async-generator hop per streamed chunk (one token frame per
        # request per decode step -- ~27K frames/s at 256 concurrent turns)
        await svc.converse(_GrpcStream(context))

    conv = converse_gen if os.environ.get("OMNIA_GRPC_QUEUE_ADAPTER") == "1" else \
        converse_direct
    handlers = {
        "Converse": grpc.stream_stream_rpc_method_handler(
            conv, request_deserializer=pb.ClientMessage.FromString,
            response_serializer=pb.ServerMessage.SerializeToString),
        "Invoke": grpc.unary_unary_rpc_method_handler(
            invoke, request_deserializer=pb.InvocationRequest.FromString,
            response_serializer=pb.InvocationResponse.SerializeToString),
        "Health": grpc.unary_unary_rpc_method_handler(
            health, request_deserializer=pb.HealthRequest.FromString,
            response_serializer=pb.HealthResponse.SerializeToString),
        "HasConversation": grpc.unary_unary_rpc_method_handler(
            has_conversation, request_deserializer=pb.HasConversationRequest.FromString,
            response_serializer=pb.HasConversationResponse.SerializeToString),
    }
    return grpc.method_handlers_generic_handler(pb.SERVICE, handlers)


class _ConverseAdapter:
    """Stream-stream behaviour using the request iterator + an output queue, so
    reads and writes can interleave freely (client tool round-trips)."""

    def __init__(self, svc: RuntimeService):
        self.svc = svc

    def __call__(self, request_iterator, context):
        return self._run(request_iterator, context)

    async def _run(self, request_iterator, context):
        out: asyncio.Queue = asyncio.Queue()
        md = {k: v for k, v in (context.invocation_metadata() or [])}

        class S(Stream):
            def __init__(self):
                self.it = request_iterator.__aiter__()

            async def recv(self):
                try:
                    return await self.it.__anext__()
                except StopAsyncIteration:
                    return None

            async def send(self, msg):
                await out.put(msg)

            def metadata(self):
                return md

        async def drive():
            try:
                await self.svc.converse(S())
            finally:
                await out.put(None)

        task = asyncio.ensure_future(drive())
        try:
            while True:
                m = await out.get()
                if m is None:
                    break
                yield m
        finally:
            if not task.done():
                task.cancel()


async def serve_grpc(svc: RuntimeService, port: int = 9000, host: str = "0.0.0.0"):
    import grpc

    server = grpc.aio.server(options=[("grpc.max_receive_message_length", 32 * 2**20),
                                      ("grpc.max_send_message_length", 32 * 2**20)])
    server.add_generic_rpc_handlers((grpc_handler(svc),))
    bound = server.add_insecure_port(f"{host}:{port}")
    await server.start()
    return server, bound


def _engine_stats(agent, reset: bool = False):
    """Stats (or a reset) of the agent's in-node engine: the engine-core client
    (``engine/core_proc.py``) or the in-process engine; None without one."""
    eng = getattr(getattr(agent, "provider", None), "engine", None)
    if eng is None:
        return None
    if hasattr(eng, "call") and hasattr(eng, "stats"):  # engine-core child process
        return eng.call("reset_timing") if reset else eng.stats()
    inner = getattr(eng, "engine", None)
    if inner is None or not hasattr(inner, "busy_seconds"):
        return None
    if reset:
        inner.busy_seconds(reset=True)
        return True
    return {"timing": dict(inner.timing), "counters": dict(inner.counters),
            "gpu_busy_s": inner.busy_seconds()}


async def serve_health(svc: RuntimeService, port: int = 9001, host: str = "0.0.0.0"):
    from aiohttp import web

    async def healthz(_):
        return web.json_response({"status": "ok"})

    async def readyz(_):
        h = await svc.health()
        return web.json_response({"ready": h.healthy}, status=200 if h.healthy else 503)

    async def metrics(_):
        return web.Response(body=M.exposition(), content_type="text/plain")

    app = web.Application()
    app.router.add_get("/healthz", healthz)
    app.router.add_get("/readyz", readyz)
    app.router.add_get("/metrics", metrics)
    if os.environ.get("OMNIA_DEBUG_ENGINE_STATS") == "1":
        # benchmark / diagnostics only (off by default): the local engine's
        # counters and hipEvent-measured device busy time, and their reset
        async def engine_stats(request):
            reset = request.method == "POST"
            out = await asyncio.get_running_loop().run_in_executor(
                None, _engine_stats, svc.agent, reset)
            if out is None:
                return web.json_response({"error": "no local engine"}, status=404)
            return web.json_response(out if isinstance(out, dict) else {"ok": bool(out)})

        app.router.add_get("/debug/engine-stats", engine_stats)
        app.router.add_post("/debug/engine-stats", engine_stats)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]
