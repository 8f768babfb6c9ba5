"""OTLP trace ingest for the session-api: OpenTelemetry GenAI spans become
session records.

Reference: ``internal/session/otlp/receiver.go:27-49`` (gRPC TraceService),
``handler.go:31-136`` (OTLP/HTTP ``POST /v1/traces``: protobuf or JSON, gzip,
4 MiB cap, response in the request's encoding), ``transformer.go:70-497`` and
``attributes.go:31-291`` (attribute keys, session-id resolution, message
extraction strategies).

Per span (spans of a scope are taken in start-time order):

* the session id is ``gen_ai.conversation.id`` / ``session.id`` /
  ``langfuse.session.id`` on the span, else ``session.id`` /
  ``langfuse.session.id`` on the resource -- never the trace id (a trace id
  would mint ghost sessions for services that have none); no id -> skipped;
* the session is created on first sight: agent = ``service.name``, namespace =
  ``service.namespace``, workspace / PromptPack from ``omnia.*`` attributes
  (span first, then resource), state = provider / model / pack, and a
  pseudonymous virtual user derived from the session id;
* ``tool.*`` spans -> a system message ``{type: tool.call.completed, tool_name,
  tool_args, status, duration_ms}``; ``workflow.transition`` /
  ``workflow.completed`` spans -> ``workflow.transitioned`` /
  ``workflow.completed`` system messages;
* anything else -> conversation messages, from (1) ``gen_ai.input.messages`` /
  ``gen_ai.output.messages`` (kvlists with ``role`` + ``content`` or text
  ``parts``), else (2) the ``gen_ai.client.inference.operation.details`` span
  event, else (3) legacy OpenLLMetry ``gen_ai.prompt.{i}.*`` /
  ``gen_ai.completion.{i}.*``; each carries ``gen_ai.model`` metadata, and the
  span's token usage (current or deprecated keys) is booked on its first
  output message so session totals follow.

A failing span is logged and the rest of the export still lands (partial
success, as the reference does).
"""
from __future__ import annotations

import gzip
import io
import logging
import re
import uuid
import zlib

from google.protobuf import json_format

from ..api.proto import otlp_trace_v1 as ot
from .model import ROLE_ASSISTANT, ROLE_SYSTEM, ROLE_USER, Message, Session

log = logging.getLogger("omnia.session.otlp")

MAX_BODY = 4 * 2**20
CT_PROTOBUF = "application/x-protobuf"
CT_JSON = "application/json"

# attribute keys (attributes.go:31-105)
CONVERSATION_ID = "gen_ai.conversation.id"
SESSION_ID = "session.id"
LANGFUSE_SESSION_ID = "langfuse.session.id"
REQUEST_MODEL, RESPONSE_MODEL = "gen_ai.request.model", "gen_ai.response.model"
PROVIDER_NAME, SYSTEM = "gen_ai.provider.name", "gen_ai.system"
INPUT_MESSAGES, OUTPUT_MESSAGES = "gen_ai.input.messages", "gen_ai.output.messages"
USAGE_INPUT, USAGE_OUTPUT = "gen_ai.usage.input_tokens", "gen_ai.usage.output_tokens"
USAGE_PROMPT, USAGE_COMPLETION = "gen_ai.usage.prompt_tokens", "gen_ai.usage.completion_tokens"
PROMPT_PREFIX, COMPLETION_PREFIX = "gen_ai.prompt.", "gen_ai.completion."
SERVICE_NAME, SERVICE_NAMESPACE = "service.name", "service.namespace"
WORKSPACE = "omnia.workspace.name"
PACK_NAME, PACK_VERSION = "omnia.promptpack.name", "omnia.promptpack.version"
COHORT, VARIANT = "omnia.cohort.id", "omnia.variant"
INFERENCE_EVENT = "gen_ai.client.inference.operation.details"

_ROLES = {"user": ROLE_USER, "assistant": ROLE_ASSISTANT, "system": ROLE_SYSTEM}
_INDEXED = re.compile(r"^(\d+)\.(role|content)$")


# ------------------------------------------------------------------ attribute access
def get_str(attrs, *keys) -> str:
    for key in keys:
        for kv in attrs:
            if kv.key == key and kv.value.WhichOneof("value") == "string_value" \
                    and kv.value.string_value:
                return kv.value.string_value
    return ""


def get_int(attrs, *keys) -> int:
    for key in keys:
        for kv in attrs:
            if kv.key == key:
                k = kv.value.WhichOneof("value")
                v = kv.value.int_value if k == "int_value" else \
                    int(kv.value.double_value) if k == "double_value" else \
                    int(kv.value.string_value) if k == "string_value" and \
                    kv.value.string_value.isdigit() else 0
                if v:
                    return v
    return 0


def get_array(attrs, key) -> list:
    for kv in attrs:
        if kv.key == key and kv.value.WhichOneof("value") == "array_value":
            return list(kv.value.array_value.values)
    return []


def session_id_of(span_attrs, resource_attrs) -> str:
    return get_str(span_attrs, CONVERSATION_ID, SESSION_ID, LANGFUSE_SESSION_ID) or \
        get_str(resource_attrs, SESSION_ID, LANGFUSE_SESSION_ID)


# ------------------------------------------------------------------ message extraction
def _content_of_parts(v) -> str:
    if v.WhichOneof("value") != "array_value":
        return ""
    for part in v.array_value.values:
        if part.WhichOneof("value") != "kvlist_value":
            continue
        kvs = part.kvlist_value.values
        if get_str(kvs, "type") in ("text", ""):
            c = get_str(kvs, "content")
            if c:
                return c
    return ""


def _message_of(v, default_role: str, ts: float) -> Message | None:
    if v.WhichOneof("value") != "kvlist_value":
        return None
    role, content = "", ""
    for kv in v.kvlist_value.values:
        if kv.key == "role":
            role = kv.value.string_value
        elif kv.key == "content":
            content = kv.value.string_value
        elif kv.key == "parts" and not content:
            content = _content_of_parts(kv.value)
    if not content:
        return None
    role = _ROLES.get(role, default_role)
    if not role:
        return None
    return Message(id=str(uuid.uuid4()), role=role, content=content, timestamp=ts)


def structured_messages(attrs, ts: float) -> list[Message]:
    out = [m for v in get_array(attrs, INPUT_MESSAGES) if (m := _message_of(v, "", ts))]
    out += [m for v in get_array(attrs, OUTPUT_MESSAGES)
            if (m := _message_of(v, ROLE_ASSISTANT, ts))]
    return out


def legacy_messages(attrs, ts: float) -> list[Message]:
    out = []
    for prefix in (PROMPT_PREFIX, COMPLETION_PREFIX):
        roles, contents = {}, {}
        for kv in attrs:
            if not kv.key.startswith(prefix):
                continue
            m = _INDEXED.match(kv.key[len(prefix):])
            if m:
                (roles if m.group(2) == "role" else contents)[int(m.group(1))] = \
                    kv.value.string_value
        for i in sorted(set(roles) | set(contents)):
            if contents.get(i):
                out.append(Message(id=str(uuid.uuid4()),
                                   role=_ROLES.get(roles.get(i, ""), ROLE_ASSISTANT),
                                   content=contents[i], timestamp=ts))
    return out


def resolve_messages(span, ts: float) -> list[Message]:
    attrs = span.attributes
    msgs = structured_messages(attrs, ts)
    if not msgs:
        for ev in span.events:
            if ev.name == INFERENCE_EVENT:
                msgs = structured_messages(ev.attributes, ts)
                break
    if not msgs:
        msgs = legacy_messages(attrs, ts)
    model = get_str(attrs, RESPONSE_MODEL, REQUEST_MODEL)
    for m in msgs:
        if model:
            m.metadata["gen_ai.model"] = model
    return msgs


# ------------------------------------------------------------------ transformer
class Transformer:
    """``svc``: the tiered session service (create / get / append_message)."""

    def __init__(self, svc):
        self.svc = svc
        self.stats = {"spans": 0, "skipped": 0, "failed": 0, "sessions_created": 0}

    async def process_export(self, req) -> tuple[int, str]:
        processed, first_err = 0, ""
        for rs in req.resource_spans:
            res_attrs = list(rs.resource.attributes)
            ctx = {"agent": get_str(res_attrs, SERVICE_NAME),
                   "namespace": get_str(res_attrs, SERVICE_NAMESPACE),
                   "workspace": get_str(res_attrs, WORKSPACE),
                   "pack": get_str(res_attrs, PACK_NAME),
                   "pack_version": get_str(res_attrs, PACK_VERSION), "attrs": res_attrs}
            for ss in rs.scope_spans:
                for span in sorted(ss.spans, key=lambda s: s.start_time_unix_nano):
                    try:
                        if await self.process_span(ctx, span):
                            processed += 1
                    except Exception as e:  # noqa: BLE001 - partial success
                        self.stats["failed"] += 1
                        log.error("otlp span %s failed: %s", span.span_id.hex(), e)
                        first_err = first_err or str(e)
        return processed, first_err

    def _ensure(self, sid: str, ctx: dict, attrs) -> None:
        v = self.svc.get(sid, with_messages=False)
        if v is not None:
            return
        from ..operator.authz import pseudonymize_id

        state = {}
        prov = get_str(attrs, PROVIDER_NAME, SYSTEM)
        model = get_str(attrs, RESPONSE_MODEL, REQUEST_MODEL)
        pack = get_str(attrs, PACK_NAME) or ctx["pack"]
        ver = get_str(attrs, PACK_VERSION) or ctx["pack_version"]
        if prov:
            state["gen_ai.provider"] = prov
        if model:
            state["gen_ai.model"] = model
        if get_str(attrs, PACK_NAME):
            state[PACK_NAME] = pack
        if get_str(attrs, PACK_VERSION):
            state[PACK_VERSION] = ver
        self.svc.create(Session(id=sid, agent_name=ctx["agent"], namespace=ctx["namespace"],
                                workspace_name=ctx["workspace"], prompt_pack_name=pack,
                                prompt_pack_version=ver, state=state,
                                cohort_id=get_str(attrs, COHORT),
                                variant=get_str(attrs, VARIANT),
                                virtual_user_id=pseudonymize_id(sid)))
        self.stats["sessions_created"] += 1

    async def process_span(self, ctx: dict, span) -> bool:
        attrs = list(span.attributes)
        sid = session_id_of(attrs, ctx["attrs"])
        if not sid:
            self.stats["skipped"] += 1
            return False
        self._ensure(sid, ctx, attrs)
        ts = span.start_time_unix_nano / 1e9 if span.start_time_unix_nano else None
        name = span.name
        if name.startswith("tool."):
            msgs = [Message(role=ROLE_SYSTEM, tool_call_id=get_str(attrs, "tool.call_id"),
                            metadata={"type": "tool.call.completed",
                                      "tool_name": get_str(attrs, "tool.name"),
                                      "tool_args": get_str(attrs, "tool.args"),
                                      "status": get_str(attrs, "tool.status"),
                                      "duration_ms": str(get_int(attrs, "tool.duration_ms"))})]
        elif name == "workflow.transition":
            msgs = [Message(role=ROLE_SYSTEM, metadata={
                "type": "workflow.transitioned",
                "from_state": get_str(attrs, "workflow.from_state"),
                "to_state": get_str(attrs, "workflow.to_state"),
                "event": get_str(attrs, "workflow.event"),
                "prompt_task": get_str(attrs, "workflow.prompt_task")})]
        elif name == "workflow.completed":
            msgs = [Message(role=ROLE_SYSTEM, metadata={
                "type": "workflow.completed",
                "final_state": get_str(attrs, "workflow.final_state"),
                "transition_count": str(get_int(attrs, "workflow.transition_count"))})]
        else:
            msgs = resolve_messages(span, ts or 0.0)
            out = next((m for m in msgs if m.role == ROLE_ASSISTANT), None)
            if out is not None:
                out.input_tokens = get_int(attrs, USAGE_INPUT, USAGE_PROMPT)
                out.output_tokens = get_int(attrs, USAGE_OUTPUT, USAGE_COMPLETION)
        for m in msgs:
            if ts:
                m.timestamp = ts
            await self.svc.append_message(sid, m)
        self.stats["spans"] += 1
        return True


# ------------------------------------------------------------------ transports
def build_otlp_app(transformer: "Transformer", tokens: dict | None = None):
    """The OTLP/HTTP listener (reference: its own ``:4318`` server sharing the
    session-api's bearer-token review, ``cmd/session-api/main.go:346-360``)."""
    from aiohttp import web

    @web.middleware
    async def guard(request, handler):
        if tokens is not None:
            h = request.headers.get("Authorization", "")
            if tokens.get(h[7:] if h.lower().startswith("bearer ") else "") is None:
                return web.json_response({"error": "unauthorized"}, status=401)
        return await handler(request)

    app = web.Application(middlewares=[guard], client_max_size=MAX_BODY + 1024)
    mount_otlp_http(app, transformer)
    return app


def mount_otlp_http(app, transformer: Transformer):
    """``POST /v1/traces`` (handler.go:55-101)."""
    from aiohttp import web

    async def traces(request):
        ct = (request.headers.get("Content-Type") or "").split(";")[0].strip()
        if ct not in (CT_PROTOBUF, CT_JSON):
            return web.Response(status=415, text="unsupported content type; expected "
                                                 "application/x-protobuf or application/json")
        try:
            # aiohttp inflates a gzip Content-Encoding itself; a body that still
            # carries the gzip magic (a proxy that strips the header) is inflated here
            body = await request.read()  # bounded by the app's client_max_size
        except web.HTTPRequestEntityTooLarge:
            return web.Response(status=413, text="request body too large")
        except Exception:  # noqa: BLE001 - the server's own inflate failed
            return web.Response(status=400, text="invalid gzip encoding")
        if body[:2] == b"\x1f\x8b":
            try:
                body = gzip.GzipFile(fileobj=io.BytesIO(body)).read(MAX_BODY + 1)
            except (OSError, EOFError, zlib.error):
                return web.Response(status=400, text="invalid gzip encoding")
        if len(body) > MAX_BODY:
            return web.Response(status=413, text="request body too large")
        try:
            if ct == CT_JSON:
                req = json_format.Parse(body.decode() or "{}", ot.ExportTraceServiceRequest(),
                                        ignore_unknown_fields=True)
            else:
                req = ot.ExportTraceServiceRequest.FromString(body)
        except Exception:  # noqa: BLE001
            return web.Response(status=400, text="invalid payload")
        processed, err = await transformer.process_export(req)
        if err:
            log.error("otlp partial export failure (%d processed): %s", processed, err)
        resp = ot.ExportTraceServiceResponse()
        if ct == CT_JSON:
            return web.Response(text=json_format.MessageToJson(resp), content_type=CT_JSON)
        return web.Response(body=resp.SerializeToString(), content_type=CT_PROTOBUF)

    app.router.add_post("/v1/traces", traces)


def grpc_trace_handler(transformer: Transformer):
    """``opentelemetry.proto.collector.trace.v1.TraceService/Export`` (receiver.go)."""
    import grpc

    async def export(req, context):
        processed, err = await transformer.process_export(req)
        if err:
            log.error("otlp partial export failure (%d processed): %s", processed, err)
        return ot.ExportTraceServiceResponse()

    return grpc.method_handlers_generic_handler(ot.SERVICE, {
        "Export": grpc.unary_unary_rpc_method_handler(
            export, request_deserializer=ot.ExportTraceServiceRequest.FromString,
            response_serializer=ot.ExportTraceServiceResponse.SerializeToString)})


def token_interceptor(tokens: dict):
    """gRPC twin of the HTTP guard: ``authorization: Bearer <token>`` metadata
    must name a token of the session-api's token map (reference
    ``otlpGRPCServerOptions``), else UNAUTHENTICATED before the handler runs."""
    import grpc

    async def deny(_req, context):
        await context.abort(grpc.StatusCode.UNAUTHENTICATED, "unauthorized")

    denied = grpc.unary_unary_rpc_method_handler(deny)

    class _Guard(grpc.aio.ServerInterceptor):
        async def intercept_service(self, continuation, details):
            md = {k.lower(): v for k, v in (details.invocation_metadata or ())}
            h = md.get("authorization", "")
            tok = h[7:] if isinstance(h, str) and h.lower().startswith("bearer ") else ""
            if tokens.get(tok) is None:
                return denied
            return await continuation(details)

    return _Guard()


async def serve_otlp_grpc(transformer: Transformer, port: int = 4317, host: str = "0.0.0.0",
                          tokens: dict | None = None):
    """``tokens``: the session-api bearer-token map; when set every export must
    carry one (same review as the HTTP listener)."""
    import grpc

    server = grpc.aio.server(options=[("grpc.max_receive_message_length", MAX_BODY)],
                             interceptors=[token_interceptor(tokens)] if tokens is not None
                             else None)
    server.add_generic_rpc_handlers((grpc_trace_handler(transformer),))
    bound = server.add_insecure_port(f"{host}:{port}")
    await server.start()
    return server, bound
