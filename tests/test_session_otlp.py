"""Session-api OTLP ingest (``internal/session/otlp/*_test.go`` behaviours):
GenAI spans over OTLP/HTTP (protobuf, JSON, gzip) and OTLP/gRPC become
sessions and messages; session-id resolution never falls back to the trace id;
tool and workflow spans become typed system messages."""
import asyncio
import gzip
import json

import pytest
from aiohttp.test_utils import TestClient, TestServer
from google.protobuf import json_format

from omnia_amd.api.proto import otlp_trace_v1 as ot
from omnia_amd.session.otlp import Transformer, build_otlp_app, serve_otlp_grpc
from omnia_amd.session.store import TieredSessionService


def _kv(attrs, key, value):
    kv = attrs.add()
    kv.key = key
    if isinstance(value, bool):
        kv.value.bool_value = value
    elif isinstance(value, int):
        kv.value.int_value = value
    elif isinstance(value, list):
        for item in value:
            v = kv.value.array_value.values.add()
            for k2, v2 in item.items():
                e = v.kvlist_value.values.add()
                e.key = k2
                if isinstance(v2, list):  # parts
                    for part in v2:
                        pv = e.value.array_value.values.add()
                        for k3, v3 in part.items():
                            pe = pv.kvlist_value.values.add()
                            pe.key = k3
                            pe.value.string_value = v3
                else:
                    e.value.string_value = v2
    else:
        kv.value.string_value = value


def _request(spans, resource=None):
    req = ot.ExportTraceServiceRequest()
    rs = req.resource_spans.add()
    for k, v in (resource or {"service.name": "support-agent",
                              "service.namespace": "prod",
                              "omnia.workspace.name": "ws1",
                              "omnia.promptpack.name": "support-pack",
                              "omnia.promptpack.version": "1.2.0"}).items():
        _kv(rs.resource.attributes, k, v)
    ss = rs.scope_spans.add()
    for name, start, attrs, events in spans:
        sp = ss.spans.add()
        sp.name = name
        sp.start_time_unix_nano = start
        sp.trace_id = bytes(range(16))
        sp.span_id = bytes(range(8))
        for k, v in attrs.items():
            _kv(sp.attributes, k, v)
        for ename, eattrs in events:
            ev = sp.events.add()
            ev.name = ename
            for k, v in eattrs.items():
                _kv(ev.attributes, k, v)
    return req


T0 = 1_760_000_000_000_000_000

CHAT = ("chat llama", T0 + 10, {
    "gen_ai.conversation.id": "conv-1", "gen_ai.provider.name": "omnia",
    "gen_ai.request.model": "llama-3-8b", "gen_ai.response.model": "llama-3-8b-instruct",
    "gen_ai.usage.input_tokens": 42, "gen_ai.usage.output_tokens": 7,
    "gen_ai.input.messages": [{"role": "system", "content": "be brief"},
                              {"role": "user", "parts": [{"type": "text",
                                                          "content": "hello?"}]}],
    "gen_ai.output.messages": [{"content": "hi there"}]}, [])
TOOL = ("tool.get_weather", T0 + 20, {
    "session.id": "conv-1", "tool.name": "get_weather", "tool.call_id": "c1",
    "tool.args": '{"city":"Paris"}', "tool.status": "success", "tool.duration_ms": 12}, [])
WF = ("workflow.transition", T0 + 30, {
    "session.id": "conv-1", "workflow.from_state": "triage", "workflow.to_state": "billing",
    "workflow.event": "billing_issue", "workflow.prompt_task": "billing"}, [])
WFC = ("workflow.completed", T0 + 40, {
    "session.id": "conv-1", "workflow.final_state": "closing",
    "workflow.transition_count": 2}, [])
NOSESSION = ("chat", T0 + 50, {"gen_ai.output.messages": [{"content": "orphan"}]}, [])


def _check_conv1(svc):
    sess, msgs = svc.get("conv-1")
    assert sess.agent_name == "support-agent" and sess.namespace == "prod"
    assert sess.workspace_name == "ws1" and sess.prompt_pack_name == "support-pack"
    assert sess.state == {"gen_ai.provider": "omnia", "gen_ai.model": "llama-3-8b-instruct"}
    assert sess.virtual_user_id
    roles = [m.role for m in msgs]
    assert roles == ["system", "user", "assistant", "system", "system", "system"]
    assert msgs[1].content == "hello?" and msgs[2].content == "hi there"
    assert msgs[2].metadata["gen_ai.model"] == "llama-3-8b-instruct"
    assert sess.total_input_tokens == 42 and sess.total_output_tokens == 7
    assert msgs[3].metadata == {"type": "tool.call.completed", "tool_name": "get_weather",
                                "tool_args": '{"city":"Paris"}', "status": "success",
                                "duration_ms": "12"}
    assert msgs[3].tool_call_id == "c1"
    assert msgs[4].metadata["type"] == "workflow.transitioned" and \
        msgs[4].metadata["to_state"] == "billing"
    assert msgs[5].metadata == {"type": "workflow.completed", "final_state": "closing",
                                "transition_count": "2"}
    assert abs(msgs[2].timestamp - (T0 + 10) / 1e9) < 1e-6


@pytest.mark.parametrize("encoding", ["protobuf", "json", "protobuf+gzip"])
def test_otlp_http_ingest(encoding):
    svc = TieredSessionService()
    # out of order on the wire: ingest sorts a scope's spans by start time
    req = _request([WFC, TOOL, CHAT, WF, NOSESSION])

    async def run():
        c = TestClient(TestServer(build_otlp_app(Transformer(svc))))
        await c.start_server()
        try:
            if encoding == "json":
                body = json_format.MessageToJson(req).encode()
                headers = {"Content-Type": "application/json"}
            else:
                body = req.SerializeToString()
                headers = {"Content-Type": "application/x-protobuf"}
                if encoding.endswith("gzip"):
                    body = gzip.compress(body)
                    headers["Content-Encoding"] = "gzip"
            r = await c.post("/v1/traces", data=body, headers=headers)
            return r.status, r.headers["Content-Type"], await r.read()
        finally:
            await c.close()

    status, ct, body = asyncio.run(run())
    assert status == 200
    if encoding == "json":
        assert ct.startswith("application/json") and json.loads(body) == {}
    else:
        assert ct == "application/x-protobuf"
        ot.ExportTraceServiceResponse.FromString(body)
    _check_conv1(svc)
    # the orphan span (no session attribute) never became a session
    assert len(svc.warm.list_sessions()) == 1


def test_otlp_http_rejections():
    svc = TieredSessionService()

    async def run():
        c = TestClient(TestServer(build_otlp_app(Transformer(svc), tokens={"t": "sa"})))
        await c.start_server()
        try:
            auth = {"Authorization": "Bearer t"}
            out = [(await c.post("/v1/traces", data=b"{}",
                                 headers={"Content-Type": "application/json"})).status]
            out.append((await c.post("/v1/traces", data=b"x", headers={
                **auth, "Content-Type": "text/plain"})).status)
            out.append((await c.post("/v1/traces", data=b"\xff\x01garbage", headers={
                **auth, "Content-Type": "application/x-protobuf"})).status)
            # gzip magic but a corrupt stream (aiohttp itself resets the connection
            # when a declared Content-Encoding fails to inflate)
            out.append((await c.post("/v1/traces", data=b"\x1f\x8bcorrupt", headers={
                **auth, "Content-Type": "application/x-protobuf"})).status)
            out.append((await c.post("/v1/traces", data=b"\x00" * (4 * 2**20 + 10), headers={
                **auth, "Content-Type": "application/x-protobuf"})).status)
            return out
        finally:
            await c.close()

    assert asyncio.run(run()) == [401, 415, 400, 400, 413]


def test_otlp_grpc_export():
    import grpc

    svc = TieredSessionService()

    async def run():
        tr = Transformer(svc)
        server, port = await serve_otlp_grpc(tr, 0, "127.0.0.1")
        try:
            async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
                export = ch.unary_unary(ot.METHOD_EXPORT,
                                        request_serializer=ot.ExportTraceServiceRequest
                                        .SerializeToString,
                                        response_deserializer=ot.ExportTraceServiceResponse
                                        .FromString)
                await export(_request([CHAT, TOOL, WF, WFC]))
            return tr.stats
        finally:
            await server.stop(0)

    stats = asyncio.run(run())
    assert stats["spans"] == 4 and stats["sessions_created"] == 1
    _check_conv1(svc)


def test_otlp_grpc_requires_a_session_api_token():
    import grpc

    svc = TieredSessionService()

    async def run():
        tr = Transformer(svc)
        server, port = await serve_otlp_grpc(tr, 0, "127.0.0.1", tokens={"sekrit": "sa:x"})
        codes = []
        try:
            async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
                export = ch.unary_unary(ot.METHOD_EXPORT,
                                        request_serializer=ot.ExportTraceServiceRequest
                                        .SerializeToString,
                                        response_deserializer=ot.ExportTraceServiceResponse
                                        .FromString)
                for md in (None, (("authorization", "Bearer wrong"),)):
                    try:
                        await export(_request([CHAT]), metadata=md)
                        codes.append("OK")
                    except grpc.aio.AioRpcError as e:
                        codes.append(e.code().name)
                await export(_request([CHAT, TOOL, WF, WFC]),
                             metadata=(("authorization", "Bearer sekrit"),))
            return codes, tr.stats
        finally:
            await server.stop(0)

    codes, stats = asyncio.run(run())
    assert codes == ["UNAUTHENTICATED", "UNAUTHENTICATED"]
    assert stats["spans"] == 4  # only the authorised export was ingested
    _check_conv1(svc)


def test_event_and_legacy_strategies_and_resource_session_id():
    svc = TieredSessionService()
    ev_span = ("chat", T0 + 1, {"gen_ai.request.model": "m1"}, [
        ("gen_ai.client.inference.operation.details", {
            "gen_ai.input.messages": [{"role": "user", "content": "from event"}],
            "gen_ai.output.messages": [{"role": "assistant", "content": "event reply"}]})])
    legacy = ("openllmetry.chat", T0 + 2, {
        "gen_ai.prompt.1.role": "user", "gen_ai.prompt.1.content": "second",
        "gen_ai.prompt.0.role": "system", "gen_ai.prompt.0.content": "first",
        "gen_ai.completion.0.content": "legacy reply",
        "gen_ai.usage.prompt_tokens": 5, "gen_ai.usage.completion_tokens": 3}, [])
    req = _request([ev_span, legacy], resource={"service.name": "a", "session.id": "res-sid"})
    tr = Transformer(svc)
    asyncio.run(tr.process_export(req))
    sess, msgs = svc.get("res-sid")
    assert [(m.role, m.content) for m in msgs] == [
        ("user", "from event"), ("assistant", "event reply"), ("system", "first"),
        ("user", "second"), ("assistant", "legacy reply")]
    assert msgs[1].metadata["gen_ai.model"] == "m1"
    assert sess.total_input_tokens == 5 and sess.total_output_tokens == 3


def test_failed_span_does_not_drop_the_rest():
    svc = TieredSessionService()
    calls = {"n": 0}
    orig = svc.append_message

    async def flaky(sid, m):
        calls["n"] += 1
        if calls["n"] == 1:
            raise RuntimeError("warm store hiccup")
        return await orig(sid, m)

    svc.append_message = flaky
    tr = Transformer(svc)
    processed, err = asyncio.run(tr.process_export(_request([TOOL, WF])))
    assert processed == 1 and "hiccup" in err and tr.stats["failed"] == 1
    assert [m.metadata["type"] for m in svc.get("conv-1")[1]] == ["workflow.transitioned"]
