"""WebSocket / REST facade server (``internal/facade/server.go``, ``cmd/agent``).

Endpoints on the facade port (8080):
  GET  /ws  (also /)          WebSocket agent protocol (protocol.py)
  POST /functions/{name}      function mode: input schema -> Invoke -> output schema
  GET  /healthz /readyz /metrics
  A2A (a2a.py) and MCP (mcp.py) routers are mounted when enabled.

Connection semantics (``server_config.go:78-101``, ``connection.go``,
``message.go``, ``session.go``): 500 connections max, 16 MiB max message,
30 s ping / 60 s pong, 50 msg/s (burst 100) text and 2 MiB/s (burst 16 MiB)
media budgets, ONE in-flight message per connection (extra -> RATE_LIMITED,
connection stays up), ``connected`` frame sent immediately on upgrade, a
client-supplied foreign session id triggers the HasConversation resume probe
(NOT_FOUND -> SESSION_EXPIRED, UNAVAILABLE -> INTERNAL_ERROR), the trace id is
derived from the session UUID, and SIGTERM drains: no new upgrades, live
sessions get ``drain_timeout`` to finish.

Realtime blip-resume (:mod:`.realtime`): a connection that drops without a
``hangup`` while a duplex audio call is up parks the call for
``grace_window_s``; ``?resume=<session>`` from the same owner takes it back
(``connected.resumed = true``) and replays what the runtime said meanwhile.
Draining still admits such resume upgrades and waits for live + parked calls.
"""
from __future__ import annotations

import asyncio
import os
import json
import logging
import time
import uuid
from dataclasses import dataclass, field

from aiohttp import WSMsgType, web

from ..utils.arrivals import mark
from ..api.proto import runtime_v1 as pb
from ..observability import metrics as M
from ..observability import tracing
from ..utils import jsonschema
from ..utils.ratelimit import TokenBucket
from . import protocol as P
from ..observability import logging as logctx
from .auth import AuthChain, AuthError
from .handlers import PendingTools, RuntimeHandler, Writer
from .realtime import NoopRouteStore, RealtimeRegistry

log = logging.getLogger("omnia.facade")


@dataclass
class FacadeConfig:
    agent: str = "agent"
    namespace: str = "default"
    port: int = 8080
    max_connections: int = 500
    max_message_bytes: int = 16 * 2**20
    ping_interval_s: float = 30.0
    pong_timeout_s: float = 60.0
    msg_rate: float = 50.0
    msg_burst: float = 100.0
    media_rate: float = 2 * 2**20
    media_burst: float = 16 * 2**20
    max_inflight: int = 1
    max_audio_sessions: int = 8
    binary_frames: bool = True
    media_enabled: bool = False
    drain_timeout_s: float = 30.0
    grace_window_s: float = 15.0  # OMNIA_GRACE_WINDOW_SECONDS
    pod_addr: str = ""  # POD_IP:port, the route hint of parked calls
    functions: dict = field(default_factory=dict)  # name -> {"input_schema", "output_schema"}
    allowed_origins: list = field(default_factory=list)  # [] = any


class _WSWriter(Writer):
    def __init__(self, ws, labels):
        self.ws = ws
        self.labels = labels
        self.lock = asyncio.Lock()
        self.sent = M.child(M.MESSAGES_SENT, *labels)

    async def write(self, msg: dict) -> None:
        async with self.lock:
            if not self.ws.closed:
                await self.ws.send_str(json.dumps(msg, separators=(",", ":")))
                self.sent.inc()

    async def write_chunk(self, session_id: str, session_json: str, content: str,
                          role: str = "") -> None:
        # hot path (one frame per streamed token): pre-serialized, no dict
        async with self.lock:
            if not self.ws.closed:
                await self.ws.send_str(P.chunk_text(session_json, content, role))
                self.sent.inc()

    async def write_bytes(self, data: bytes) -> None:
        async with self.lock:
            if not self.ws.closed:
                await self.ws.send_bytes(data)
                M.child(M.MESSAGES_SENT, *self.labels).inc()


class FacadeServer:
    def __init__(self, cfg: FacadeConfig, handler=None, runtime_client=None,
                 auth: AuthChain | None = None, recorder=None, media_store=None,
                 routes=None):
        self.cfg = cfg
        self.client = runtime_client
        self.handler = handler or (RuntimeHandler(runtime_client) if runtime_client else None)
        self.auth = auth or AuthChain()
        self.recorder = recorder
        self.media = media_store
        self.connections = 0
        self.draining = False
        self.sessions: set = set()
        self.audio_sessions = 0
        self._caps: tuple[float, list] | None = None
        self.labels = (cfg.agent, cfg.namespace)
        self._conn_done = asyncio.Event()
        self._bg: set = set()
        self.routes = routes or NoopRouteStore()
        self.parked = RealtimeRegistry(self.routes, cfg.pod_addr, cfg.grace_window_s,
                                       self._park_expired)
        self.app = web.Application(client_max_size=cfg.max_message_bytes,
                                   middlewares=[self._auth_mw])
        r = self.app.router
        r.add_get("/ws", self.ws_handler)
        r.add_get("/", self.ws_handler)
        r.add_post("/functions/{name}", self.function_handler)
        r.add_get("/healthz", self.healthz)
        r.add_get("/readyz", self.readyz)
        r.add_get("/metrics", self.metrics)
        self.runner = None

    async def duplex_available(self) -> bool:
        """True when the runtime advertises ``duplex_audio`` (cached 30 s)."""
        if self.client is None:
            return False
        now = time.monotonic()
        if self._caps is None or now - self._caps[0] > 30.0:
            try:
                h = await self.client.health(timeout=2.0)
                self._caps = (now, list(h.capabilities))
            except Exception:  # noqa: BLE001
                self._caps = (now, [])
        return pb.CAP_DUPLEX_AUDIO in self._caps[1]

    async def _park_expired(self, session_id: str, persisted: bool):
        # parking skipped completion (the call might resume); expiry is where it
        # definitively did not -- complete only a session that was recorded
        if persisted and self.recorder is not None:
            try:
                await self.recorder.close_session(session_id)
            except Exception as e:  # noqa: BLE001
                log.warning("completing expired parked session %s failed: %s", session_id, e)

    @staticmethod
    def _owner(ident) -> str:
        return getattr(ident, "end_user", "") or getattr(ident, "subject", "") or ""

    # ---------------------------------------------------------------- health
    async def healthz(self, request):
        return web.json_response({"status": "ok"})

    async def readyz(self, request):
        if self.draining:
            return web.json_response({"ready": False, "reason": "draining"}, status=503)
        if self.client is not None:
            try:
                h = await self.client.health(timeout=2.0)
                if not h.healthy:
                    return web.json_response({"ready": False, "reason": "runtime"}, status=503)
            except Exception:  # noqa: BLE001
                return web.json_response({"ready": False, "reason": "runtime"}, status=503)
        return web.json_response({"ready": True})

    async def metrics(self, request):
        return web.Response(body=M.exposition(), content_type="text/plain")

    # ---------------------------------------------------------------- auth
    async def _authenticate(self, request):
        peer = request.remote or ""
        args = (request.headers, dict(request.query), peer)
        if self.auth.blocking:  # a JWKS fetch may run: keep it off the event loop
            return await asyncio.get_running_loop().run_in_executor(
                None, self.auth.authenticate, *args)
        return self.auth.authenticate(*args)

    # routes that authenticate themselves, and the public probes / agent card
    _SELF_AUTH = ("/ws", "/", "/healthz", "/readyz", "/metrics",
                  "/.well-known/agent.json", "/.well-known/agent-card.json")

    @web.middleware
    async def _auth_mw(self, request, handler):
        """The same chain in front of every other route (A2A JSON-RPC, MCP,
        media), so the management-plane twin serves them only to mgmt tokens."""
        path = request.path
        if path in self._SELF_AUTH or path.startswith("/functions/"):
            return await handler(request)
        try:
            request["omnia_identity"] = await self._authenticate(request)
        except AuthError as e:
            return web.json_response({"error": "unauthorized", "message": str(e)}, status=401)
        return await handler(request)

    def _metadata(self, ident, session_id: str, request) -> dict:
        md = {"x-omnia-agent-name": self.cfg.agent, "x-omnia-namespace": self.cfg.namespace,
              "x-omnia-session-id": session_id,
              "x-omnia-request-id": request.headers.get("X-Request-Id", uuid.uuid4().hex)}
        md.update(ident.to_metadata())
        tp = request.headers.get("traceparent")
        if tp:
            md["traceparent"] = tp
        return md

    # ---------------------------------------------------------------- websocket
    async def ws_handler(self, request):
        resume = request.query.get("resume")
        if self.draining and not resume:  # draining still admits realtime reattach
            return web.Response(status=503, text="draining")
        if self.connections >= self.cfg.max_connections:
            return web.Response(status=503, text="too many connections")
        origin = request.headers.get("Origin")
        if self.cfg.allowed_origins and origin and origin not in self.cfg.allowed_origins:
            return web.Response(status=403, text="origin not allowed")
        try:
            ident = await self._authenticate(request)
        except AuthError as e:
            return web.Response(status=401, text=str(e))
        ws = web.WebSocketResponse(heartbeat=self.cfg.ping_interval_s,
                                   max_msg_size=self.cfg.max_message_bytes)
        await ws.prepare(request)
        self.connections += 1
        M.child(M.CONNECTIONS_ACTIVE, *self.labels).inc()
        M.child(M.CONNECTIONS_TOTAL, *self.labels).inc()
        binary = request.query.get("binary", "false").lower() == "true" and self.cfg.binary_frames
        owner = self._owner(ident)
        parked = await self.parked.take(resume, owner) if resume else None
        session_id = resume or str(uuid.uuid4())
        writer = _WSWriter(ws, self.labels)
        await writer.write(P.connected(session_id, binary, self.cfg.max_message_bytes,
                                       resumed=bool(resume)))
        conn = _Connection(self, ws, writer, ident, request, session_id)
        if parked is not None:  # blip-resume: the live call continues on this socket
            conn.audio = parked
            conn.session_ensured = parked.persisted
            await parked.attach(conn)
        try:
            await conn.read_loop()
        finally:
            self.connections -= 1
            M.child(M.CONNECTIONS_ACTIVE, *self.labels).dec()
            for t in list(conn.tasks):
                t.cancel()
            if self.connections == 0:
                self._conn_done.set()
            audio, conn.audio = conn.audio, None
            if audio is not None:
                # aiohttp cancels the handler when the peer drops: release the
                # call in a task of its own so parking completes regardless
                if not (conn.hung_up or audio.finished):
                    audio.detach(persisted=conn.session_ensured)
                t = asyncio.get_running_loop().create_task(
                    self._release_audio(conn, audio, owner))
                self._bg.add(t)
                t.add_done_callback(self._bg.discard)
                await asyncio.shield(t)
        return ws

    async def _release_audio(self, conn, audio, owner: str):
        if conn.hung_up or audio.finished:
            await audio.close()
        else:  # dropped mid-call: park it for a reconnect
            await self.parked.park(conn.session_id, owner, audio, conn.session_ensured)

    # ---------------------------------------------------------------- function mode
    async def function_handler(self, request):
        """POST /functions/{name} (``internal/facade/functions_handler.go:159-300``)."""
        name = request.match_info.get("name", "")
        if not name:
            return web.json_response({"error": "missing_function_name"}, status=400)
        try:
            ident = await self._authenticate(request)
        except AuthError as e:
            return web.json_response({"error": "unauthorized", "message": str(e)}, status=401)
        try:
            raw = await request.read()
            body = json.loads(raw or b"{}")
        except Exception:  # noqa: BLE001
            return web.json_response({"error": "read_body_failed"}, status=400)
        spec = self.cfg.functions.get(name) or self.cfg.functions.get("*") or {}
        if spec.get("input_schema"):
            errs = jsonschema.Validator(spec["input_schema"]).errors(body)
            if errs:
                M.FUNCTION_REQUESTS.labels(name, "input_invalid").inc()
                return web.json_response({"error": "input_invalid",
                                          "details": [str(e) for e in errs[:10]]}, status=400)
        inv = str(uuid.uuid4())
        md = self._metadata(ident, inv, request)
        if self.recorder is not None:
            await self.recorder.ensure_session(inv, self.cfg.agent, self.cfg.namespace,
                                               {"mode": "function", "function": name})
            await self.recorder.record(inv, "user", json.dumps(body))
        try:
            resp = await self.client.invoke(pb.InvocationRequest(
                input_json=json.dumps(body), invocation_id=inv,
                metadata={"function": name}), metadata=md, timeout=120)
        except Exception as e:  # noqa: BLE001
            log.warning("invoke failed: %s", e)
            M.FUNCTION_REQUESTS.labels(name, "runtime_error").inc()
            return web.json_response({"error": "runtime_error"}, status=502)
        raw_out = resp.output_json
        try:
            out = json.loads(raw_out)
        except json.JSONDecodeError:
            out = None
            if spec.get("output_schema") is not None:
                M.FUNCTION_REQUESTS.labels(name, "output_invalid").inc()
                return web.json_response({"error": "output_invalid", "raw": raw_out,
                                          "details": ["output is not JSON"]}, status=502)
        if spec.get("output_schema") is not None:
            errs = jsonschema.Validator(spec["output_schema"]).errors(out)
            if errs:
                M.FUNCTION_REQUESTS.labels(name, "output_invalid").inc()
                return web.json_response({"error": "output_invalid", "raw": raw_out,
                                          "details": [str(e) for e in errs[:10]]}, status=502)
        if self.recorder is not None:
            await self.recorder.record(inv, "assistant", raw_out, usage={
                "input_tokens": resp.usage.input_tokens,
                "output_tokens": resp.usage.output_tokens, "cost_usd": resp.usage.cost_usd})
            await self.recorder.close_session(inv)
        M.FUNCTION_REQUESTS.labels(name, "ok").inc()
        return web.json_response(out if out is not None else {"output": raw_out},
                                 headers={"X-Omnia-Invocation-Id": inv,
                                          "X-Omnia-Duration-Ms": str(resp.duration_ms)})

    # ---------------------------------------------------------------- lifecycle
    async def start(self, host: str = "0.0.0.0", port: int | None = None,
                    extra_ports=()) -> int:
        # per-connection access logging is opt-in (OMNIA_ACCESS_LOG=1): a formatted
        # log record per closed session sits on the event loop exactly when a burst
        # of turns completes
        access = {} if os.environ.get("OMNIA_ACCESS_LOG") == "1" else {"access_log": None}
        self.runner = web.AppRunner(self.app, **access)
        await self.runner.setup()
        # listen backlog sized for connection bursts: aiohttp's default of 128
        # drops the SYNs of a burst of new sessions beyond it, and the kernel's
        # 1 s SYN retransmit then delays their first turn (a 256-session wave
        # otherwise loses ~1 s per wave); the kernel caps it at somaxconn
        site = web.TCPSite(self.runner, host, self.cfg.port if port is None else port,
                           backlog=max(1024, 2 * self.cfg.max_connections))
        await site.start()
        for p in extra_ports:  # A2A / MCP ports serve the same app (dual-protocol pods)
            await web.TCPSite(self.runner, host, p, backlog=1024).start()
        return site._server.sockets[0].getsockname()[1]

    async def drain(self) -> int:
        """SIGTERM: stop new upgrades (resume reattach still admitted), give live
        connections and realtime calls -- active or parked -- drain_timeout
        (drain.go:40-104).  Returns the realtime calls still live at the end."""
        self.draining = True
        M.DRAINING.set(1)
        M.REALTIME_DRAINING.set(1)
        t0 = time.monotonic()
        initial = self.audio_sessions
        deadline = t0 + self.cfg.drain_timeout_s
        reason = "all_drained"
        while self.connections or self.audio_sessions or len(self.parked):
            if time.monotonic() >= deadline:
                reason = "deadline"
                break
            await asyncio.sleep(0.05)
        remaining = self.audio_sessions
        M.REALTIME_DRAIN_DURATION.labels(reason).observe(time.monotonic() - t0)
        M.REALTIME_DRAINED.inc(max(0, initial - remaining))
        M.REALTIME_FORCE_ENDED.inc(remaining)
        M.REALTIME_DRAINING.set(0)
        return remaining

    async def stop(self):
        await self.parked.close_all()
        if self.runner is not None:
            await self.runner.cleanup()


class _Connection:
    def __init__(self, srv: FacadeServer, ws, writer, ident, request, session_id):
        self.srv = srv
        self.ws = ws
        self.writer = writer
        self.ident = ident
        self.request = request
        self.session_id = session_id
        self.inflight = 0
        self.pending = PendingTools()
        self.text_bucket = TokenBucket(srv.cfg.msg_rate, srv.cfg.msg_burst)
        self.media_bucket = TokenBucket(srv.cfg.media_rate, srv.cfg.media_burst)
        self.tasks: set = set()
        self.session_ensured = False
        self.audio = None  # _AudioSession while a duplex call is up
        self.hung_up = False

    async def on_audio(self, fr: dict):
        if self.audio is None:
            if self.srv.audio_sessions >= self.srv.cfg.max_audio_sessions:
                M.RATE_LIMITED.labels("audio").inc()
                await self.writer.write(P.error(self.session_id, P.E_RATE_LIMITED,
                                                "audio session limit reached"))
                return
            self.audio = _AudioSession(self)
            try:
                await self.audio.start(fr.get("meta") or {})
            except Exception as e:  # noqa: BLE001
                self.audio = None
                await self.writer.write(P.error(self.session_id, P.E_INVALID_MESSAGE,
                                                f"audio session start failed: {e}"))
                return
        await self.audio.frame(fr)
        if fr["flags"] & P.FLAG_LAST and not (fr["flags"] & P.FLAG_CHUNKED):
            await self.audio.wait_closed()
            self.audio = None

    async def read_loop(self):
        labels = self.srv.labels
        async for m in self.ws:
            if m.type == WSMsgType.TEXT:
                M.child(M.MESSAGES_RECEIVED, *labels).inc()
                if not self.text_bucket.allow():
                    M.RATE_LIMITED.labels("text").inc()
                    await self.writer.write(P.error(self.session_id, P.E_RATE_LIMITED,
                                                    "message rate limit exceeded"))
                    continue
                try:
                    msg = P.parse_client(m.data)
                except (ValueError, json.JSONDecodeError) as e:
                    await self.writer.write(P.error(self.session_id, P.E_INVALID_MESSAGE,
                                                    f"invalid message: {e}"))
                    continue
                if await self.on_message(msg) == "hangup":
                    self.hung_up = True
                    await self.ws.close()
                    break
            elif m.type == WSMsgType.BINARY:
                if not self.media_bucket.allow(len(m.data)):
                    M.RATE_LIMITED.labels("media").inc()
                    await self.writer.write(P.error(self.session_id, P.E_RATE_LIMITED,
                                                    "media rate limit exceeded"))
                    continue
                await self.on_binary(m.data)
            elif m.type in (WSMsgType.ERROR, WSMsgType.CLOSE):
                break
        for t in list(self.tasks):
            await asyncio.gather(t, return_exceptions=True)

    async def on_binary(self, data: bytes):
        try:
            peek = P.decode_frame(data)
        except ValueError as e:
            await self.writer.write(P.error(self.session_id, P.E_INVALID_MESSAGE, str(e)))
            return
        # media-chunk frames are a duplex audio call when the runtime speaks it
        # (reference: BinaryMessageTypeMediaChunk -> audio session); uploads stay uploads
        if peek["type"] == P.TYPE_MEDIA_CHUNK and (self.audio is not None or
                                                  await self.srv.duplex_available()):
            await self.on_audio(peek)
            return
        if not self.srv.cfg.media_enabled or self.srv.media is None:
            await self.writer.write(P.error(self.session_id, P.E_MEDIA_NOT_ENABLED,
                                            "media uploads are not enabled"))
            return
        try:
            fr = P.decode_frame(data)
        except ValueError as e:
            await self.writer.write(P.error(self.session_id, P.E_INVALID_MESSAGE, str(e)))
            return
        try:
            ref = await self.srv.media.put_frame(self.session_id, fr)
        except Exception as e:  # noqa: BLE001
            await self.writer.write(P.error(self.session_id, P.E_UPLOAD_FAILED, str(e)))
            return
        if ref:
            await self.writer.write(P.server_msg(P.UPLOAD_COMPLETE, self.session_id,
                                                 upload_complete=ref))

    async def on_message(self, msg: dict):
        t = msg["type"]
        if t == P.MESSAGE:
            mark("facade_msg")
        if t == P.HANGUP:
            return "hangup"
        if t == P.TOOL_RESULT:
            tr = msg.get("tool_result") or {}
            self.pending.result(tr.get("call_id", ""), tr)
            return None
        if t == P.TOOL_CALL_ACK:
            self.pending.ack((msg.get("tool_call_ack") or {}).get("call_id", ""), True)
            return None
        if t == P.TOOL_CALL_NACK:
            n = msg.get("tool_call_nack") or {}
            self.pending.ack(n.get("call_id", ""), False, n.get("reason", ""))
            return None
        if t == P.UPLOAD_REQUEST:
            if not self.srv.cfg.media_enabled or self.srv.media is None:
                await self.writer.write(P.error(self.session_id, P.E_MEDIA_NOT_ENABLED,
                                                "media uploads are not enabled"))
                return None
            info = await self.srv.media.upload_url(self.session_id, msg.get("upload_request")
                                                   or {})
            await self.writer.write(P.server_msg(P.UPLOAD_READY, self.session_id,
                                                 upload_ready=info))
            return None
        # message
        if self.inflight >= self.srv.cfg.max_inflight:
            M.RATE_LIMITED.labels("inflight").inc()
            await self.writer.write(P.error(self.session_id, P.E_RATE_LIMITED,
                                            "a message is already in flight"))
            return None
        if not msg.get("content") and not msg.get("parts"):
            await self.writer.write(P.error(self.session_id, P.E_INVALID_MESSAGE,
                                            "message content is empty"))
            return None
        self.inflight += 1
        task = asyncio.get_running_loop().create_task(self.process(msg))
        self.tasks.add(task)
        task.add_done_callback(self.tasks.discard)
        return None

    async def ensure_session(self, sid: str) -> bool:
        """Resume probe for a client-chosen foreign session id (session.go:263-372)."""
        srv = self.srv
        if sid != self.session_id and srv.client is not None:
            try:
                r = await srv.client.has_conversation(sid)
            except Exception:  # noqa: BLE001
                r = pb.HasConversationResponse(state=pb.RESUME_STATE_UNAVAILABLE)
            if r.state == pb.RESUME_STATE_NOT_FOUND:
                await self.writer.write(P.error(sid, P.E_SESSION_EXPIRED,
                                                "session has expired or does not exist"))
                return False
            if r.state != pb.RESUME_STATE_RESUMABLE:
                await self.writer.write(P.error(sid, P.E_INTERNAL,
                                                "session store temporarily unavailable"))
                return False
            self.session_id = sid
        if not self.session_ensured and srv.recorder is not None:
            try:
                from ..operator.authz import pseudonymize_id

                # recorded sessions carry the pseudonym, never the raw user id
                # (pkg/identity: facade ingestion and dashboard queries agree)
                await srv.recorder.ensure_session(self.session_id, srv.cfg.agent,
                                                  srv.cfg.namespace,
                                                  {"user": pseudonymize_id(
                                                      self.ident.end_user or
                                                      self.ident.subject or "")})
            except Exception as e:  # noqa: BLE001
                log.warning("session ensure failed: %s", e)
        self.session_ensured = True
        return True

    async def process(self, msg: dict):
        srv = self.srv
        labels = srv.labels
        t0 = time.perf_counter()
        logctx.bind(session_id=self.session_id, agent=srv.cfg.agent,
                    namespace=srv.cfg.namespace)
        M.child(M.REQUESTS_INFLIGHT, *labels).inc()
        status = "ok"
        sid = msg.get("session_id") or self.session_id
        span = tracing.start_span("omnia.facade.message", {"session.id": sid},
                                  trace_id=tracing.session_trace_id(sid),
                                  link=tracing.parse_traceparent(
                                      self.request.headers.get("traceparent")))
        try:
            if not await self.ensure_session(sid):
                status = "session_error"
                return
            sid = self.session_id
            if srv.recorder is not None:
                srv.recorder.submit(sid, "user", msg.get("content", ""))
            md = srv._metadata(self.ident, sid, self.request)
            md["traceparent"] = span.traceparent
            if srv.handler is None:
                await self.writer.write(P.error(sid, P.E_AGENT_UNAVAILABLE, "no agent handler"))
                status = "error"
                return
            try:
                res = await srv.handler.handle(sid, msg, self.writer, self.pending, md)
            except Exception as e:  # noqa: BLE001
                log.exception("turn failed")
                await self.writer.write(P.error(sid, P.E_AGENT_UNAVAILABLE,
                                                "agent unavailable"))
                status = "error"
                return
            if res.get("error"):
                status = "error"
            elif srv.recorder is not None:
                srv.recorder.submit(sid, "assistant", res.get("content", ""),
                                    usage=res.get("usage"))
        finally:
            self.inflight -= 1
            M.child(M.REQUESTS_INFLIGHT, *labels).dec()
            M.child(M.REQUESTS_TOTAL, *labels, status).inc()
            M.child(M.REQUEST_DURATION, *labels).observe(time.perf_counter() - t0)
            tracing.end_span(span, error=status != "ok")


class _AudioSession:
    """One duplex call over the runtime's Converse stream (reference
    ``internal/facade/audio_session.go``): DuplexStart from the first frame's
    metadata, every inbound media-chunk frame -> AudioInputChunk, and the
    runtime's frames relayed back (audio as binary media-chunk frames)."""

    MAX_BUFFERED = 4096  # frames held for a reconnect while parked

    def __init__(self, conn: "_Connection"):
        self.c = conn
        self.srv = conn.srv
        self.session_id = conn.session_id
        self.stream = None
        self.relay = None
        self.media_seq = 0
        self.persisted = False
        self.finished = False
        self.buffer: list = []  # (is_bytes, payload) produced while parked

    # ---------------------------------------------------------------- park / resume
    def detach(self, persisted: bool = False):
        self.c = None
        self.persisted = persisted

    async def attach(self, conn: "_Connection"):
        self.c = conn
        pending, self.buffer = self.buffer, []
        for is_bytes, payload in pending:
            await (conn.writer.write_bytes(payload) if is_bytes else conn.writer.write(payload))

    async def _out(self, msg):
        c = self.c
        if c is None or c.ws.closed:
            if len(self.buffer) < self.MAX_BUFFERED:
                self.buffer.append((isinstance(msg, bytes), msg))
            return
        await (c.writer.write_bytes(msg) if isinstance(msg, bytes) else c.writer.write(msg))

    async def close(self):
        # the relay's exit releases the call's slot and closes the stream
        if self.relay is not None and not self.relay.done():
            self.relay.cancel()
            await asyncio.gather(self.relay, return_exceptions=True)
        elif self.stream is not None:
            try:
                await self.stream.close()
            except Exception:  # noqa: BLE001
                pass

    async def start(self, meta: dict):
        c = self.c
        md = {"x-omnia-session-id": c.session_id, "x-omnia-agent-name": c.srv.cfg.agent}
        self.stream = await c.srv.client.open(md)
        await self.stream.send(pb.ClientMessage(session_id=c.session_id, duplex_start=pb.DuplexStart(
            codec=meta.get("codec") or "pcm", sample_rate=int(meta.get("sample_rate") or 16000),
            channels=int(meta.get("channels") or 1),
            system_instruction=meta.get("system_instruction", ""))))
        c.srv.audio_sessions += 1
        self.relay = asyncio.get_running_loop().create_task(self._relay())

    async def frame(self, fr: dict):
        await self.stream.send(pb.ClientMessage(audio_input=pb.AudioInputChunk(
            data=fr["payload"], sequence=fr["seq"],
            is_last=bool(fr["flags"] & P.FLAG_LAST) and not (fr["flags"] & P.FLAG_CHUNKED))))

    async def _relay(self):
        sid, out = self.session_id, self._out
        try:
            while True:
                resp = await self.stream.recv()
                if resp is None:
                    return
                kind = resp.WhichOneof("message")
                if kind == "runtime_hello":
                    m = resp.runtime_hello.media
                    await out(P.server_msg(P.SESSION_CONFIG, sid, media={
                        "codec": m.codec, "sample_rate": m.sample_rate, "channels": m.channels},
                        capabilities=list(resp.runtime_hello.capabilities)))
                elif kind == "chunk":
                    await out(P.chunk(sid, resp.chunk.content, resp.chunk.role))
                elif kind == "media_chunk":
                    mc = resp.media_chunk
                    fl = P.FLAG_LAST if mc.is_last else 0
                    await out(P.encode_frame(
                        P.TYPE_MEDIA_CHUNK, bytes(mc.data),
                        {"session_id": sid, "mime_type": mc.mime_type}, mc.sequence,
                        mc.media_id.encode()[:12], fl))
                elif kind == "interruption":
                    await out(P.server_msg(P.INTERRUPT, sid))
                elif kind == "done":
                    d = resp.done
                    await out(P.done(sid, d.final_content, None, {
                        "input_tokens": d.usage.input_tokens,
                        "output_tokens": d.usage.output_tokens,
                        "cached_tokens": d.usage.cached_tokens}))
                elif kind == "error":
                    await out(P.error(sid, resp.error.code or P.E_INTERNAL,
                                      resp.error.message))
                    return
        finally:
            self.finished = True
            self.srv.audio_sessions -= 1
            try:
                await self.stream.close()
            except Exception:  # noqa: BLE001
                pass
            if self.c is None and sid in self.srv.parked.parked:
                # the runtime ended the call while it was parked: nothing to resume
                asyncio.get_running_loop().create_task(self.srv.parked.expire(sid))

    async def wait_closed(self, timeout: float = 120.0):
        if self.relay is not None:
            try:
                await asyncio.wait_for(self.relay, timeout)
            except asyncio.TimeoutError:
                self.relay.cancel()
