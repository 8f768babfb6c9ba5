"""Tracing (reference ``internal/tracing/tracing.go``): the span
tree of one runtime turn with a server-side tool, the session-derived trace id,
the caller's traceparent as a link (not a parent), ParentBased sampling, and the
OTLP/HTTP JSON export body."""
import asyncio
import json
import uuid

from aiohttp import web

from omnia_amd.api.proto import runtime_v1 as pb
from omnia_amd.observability import tracing
from tests.test_runtime import _turn, make_service

CALLER = "00-" + "ab" * 16 + "-" + "cd" * 8 + "-01"


def _run_traced_turn(ratio=1.0):
    mem = tracing.MemoryExporter()
    tracing.configure(exporter=mem, ratio=ratio)
    sid = str(uuid.uuid4())
    try:
        svc, _, calls = make_service()
        frames = asyncio.run(_turn(svc, [pb.ClientMessage(
            session_id=sid, content="weather?", metadata={"mock_scenario": "weather"})],
            md={"traceparent": CALLER}))
    finally:
        tracing.configure(exporter=None, endpoint="")
    assert frames[-1].WhichOneof("message") == "done" and calls
    return sid, mem.spans


def test_turn_span_tree_and_genai_attributes():
    sid, spans = _run_traced_turn()
    by = {}
    for s in spans:
        by.setdefault(s.name, []).append(s)
    root = by["omnia.runtime.message"][0]
    turn = by["omnia.runtime.conversation.turn"][0]
    chats = by["genai.chat"]
    tool = by["omnia.tool.call"][0]
    # one trace per session: the trace id IS the session UUID (lossless)
    assert {s.trace_id for s in spans} == {uuid.UUID(sid).hex}
    # the caller's traceparent is a link of the root, never its parent
    assert root.parent_id is None
    assert root.links == [{"trace_id": "ab" * 16, "span_id": "cd" * 8, "sampled": True}]
    assert turn.parent_id == root.span_id
    assert len(chats) == 2 and all(c.parent_id == turn.span_id for c in chats)  # tool round
    assert tool.parent_id == turn.span_id and tool.attributes["tool.name"] == "get_weather"
    assert chats[0].attributes["gen_ai.system"] and "gen_ai.request.model" in chats[0].attributes
    assert turn.attributes["gen_ai.usage.output_tokens"] > 0
    assert all(s.status == "OK" and s.end_ns >= s.start_ns for s in spans)


def test_parent_based_sampling_keeps_a_trace_whole():
    _, spans = _run_traced_turn(ratio=0.0)  # root unsampled -> nothing exported
    assert spans == []


def test_traceparent_parsing_rejects_garbage():
    assert tracing.parse_traceparent(CALLER)["sampled"] is True
    for bad in (None, "", "00-xyz", "00-" + "a" * 31 + "-" + "b" * 16 + "-01"):
        assert tracing.parse_traceparent(bad) is None
    # non-UUID session ids still map to a stable 128-bit trace id
    assert tracing.session_trace_id("not-a-uuid") == tracing.session_trace_id("not-a-uuid")
    assert len(tracing.session_trace_id("not-a-uuid")) == 32


def test_otlp_http_json_export_body():
    got = []

    async def go():
        async def h(request):
            got.append(await request.json())
            return web.json_response({})

        app = web.Application()
        app.router.add_post("/v1/traces", h)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        try:
            exp = tracing.OTLPHTTPExporter(f"http://127.0.0.1:{port}", "omnia-runtime",
                                           interval_s=3600)
            tracing.configure(exporter=exp)
            sp = tracing.start_span("omnia.runtime.message", {"session.id": "s", "n": 3,
                                                              "ok": True, "x": 0.5})
            tracing.end_span(sp)
            tracing.record_span("omnia.engine.decode_step", 1, 2, {"omnia.engine.batch_size": 8})
            await asyncio.get_running_loop().run_in_executor(None, exp.flush)
        finally:
            tracing.configure(exporter=None, endpoint="")
            await runner.cleanup()

    asyncio.run(go())
    rs = got[0]["resourceSpans"][0]
    assert rs["resource"]["attributes"][0] == {"key": "service.name",
                                               "value": {"stringValue": "omnia-runtime"}}
    spans = rs["scopeSpans"][0]["spans"]
    assert [s["name"] for s in spans] == ["omnia.runtime.message", "omnia.engine.decode_step"]
    attrs = {a["key"]: a["value"] for a in spans[0]["attributes"]}
    assert attrs["n"] == {"intValue": "3"} and attrs["ok"] == {"boolValue": True}
    assert attrs["x"] == {"doubleValue": 0.5}
    assert spans[1]["startTimeUnixNano"] == "1" and spans[1]["status"] == {"code": 1}
    json.dumps(got)  # plain JSON end to end
