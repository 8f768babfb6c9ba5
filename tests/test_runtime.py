"""omnia.runtime.v1 server: conformance gate (cf. internal/runtime/conformance_test.go),
agent loop with server/client tools, resume states, function-mode invoke."""
import asyncio
import json

import pytest

from omnia_amd.api.proto import runtime_v1 as pb
from omnia_amd.runtime import conformance
from omnia_amd.runtime.agent import Agent, AgentConfig
from omnia_amd.runtime.config import RuntimeConfig
from omnia_amd.runtime.context_store import MemoryContextStore
from omnia_amd.runtime.promptpack import PromptPack
from omnia_amd.runtime.providers import MockProvider
from omnia_amd.runtime.server import QueueStream, RuntimeService, serve_grpc
from omnia_amd.tools.executor import InProcessHandler, OmniaExecutor

PACK = {
    "id": "t", "name": "t", "version": "1.0.0",
    "template_engine": {"version": "v1", "syntax": "{{variable}}", "features": ["fragments"]},
    "fragments": {"tone": "Be {{style}}."},
    "tools": {"get_weather": {"name": "get_weather", "description": "weather",
                              "parameters": {"type": "object",
                                             "properties": {"city": {"type": "string"}}}},
              "get_location": {"name": "get_location", "description": "gps"}},
    "prompts": {"default": {"id": "default", "name": "d", "version": "1.0.0",
                            "system_template": "You are {{name}}. {{tone}}",
                            "variables": [{"name": "name", "type": "string", "required": False,
                                           "default": "Omnia"},
                                          {"name": "style", "type": "string", "required": False,
                                           "default": "brief"}],
                            "tools": ["get_weather", "get_location"],
                            "tool_policy": {"max_rounds": 3}}},
}

SCEN = {
    "default_response": "hello there friend",
    "scenarios": {
        "weather": {"turns": [
            {"tool_calls": [{"id": "c1", "name": "get_weather", "arguments": {"city": "Paris"}}]},
            {"response": "It is sunny in Paris."}]},
        "client": {"turns": [
            {"tool_calls": [{"id": "c9", "name": "get_location", "arguments": {}}]},
            {"response": "You are at home."}]},
        "loop": {"turns": [{"tool_calls": [{"name": "get_weather", "arguments": {}}]}]},
    },
}


def _run_sync(coro):
    try:
        asyncio.get_running_loop()
    except RuntimeError:
        return asyncio.run(coro)
    import concurrent.futures

    with concurrent.futures.ThreadPoolExecutor(1) as ex:
        return ex.submit(asyncio.run, coro).result()


def make_service(store=None):
    pack = PromptPack(PACK)
    calls = []

    async def weather(args, ctx):
        calls.append(args)
        return {"temp_c": 21, "city": args.get("city")}

    ex = OmniaExecutor({"handlers": [{"name": "client-tools", "type": "client",
                                      "tool": {"name": "get_location", "description": "gps"},
                                      "clientConfig": {"consentMessage": "share location?",
                                                       "categories": ["location"]}}]})
    ex.add_handler(InProcessHandler("builtin", {"get_weather": (
        "weather", {"type": "object"}, weather)}))
    _run_sync(ex.discover())
    prov = MockProvider(scenarios=SCEN)
    agent = Agent(pack, prov, store or MemoryContextStore(), ex, AgentConfig())
    return RuntimeService(agent), prov, calls


async def _turn(svc, msgs, md=None, replies=None):
    st = QueueStream(md)
    task = asyncio.create_task(svc.converse(st))
    frames = []
    for m in msgs:
        await st.inbox.put(m)
    while True:
        f = await asyncio.wait_for(st.outbox.get(), 5)
        frames.append(f)
        k = f.WhichOneof("message")
        if k == "tool_call" and replies:
            await st.inbox.put(replies(f.tool_call))
        if k in ("done", "error"):
            break
    st.close()
    await asyncio.wait_for(task, 5)
    return frames


def test_conformance_over_grpc():
    svc, _, _ = make_service()

    async def go():
        server, port = await serve_grpc(svc, 0, "127.0.0.1")
        try:
            res = await conformance.run(f"127.0.0.1:{port}", timeout=10)
        finally:
            await server.stop(0)
        return res

    res = asyncio.run(go())
    names = {r.name: r for r in res}
    assert set(names) == {"health/contract", "hello-first", "text-turn-shape",
                          "graceful-malformed-input", "invoke-honesty", "duplex-honesty"}
    failed = [str(r) for r in res if not r.passed]
    assert not failed, failed


def test_hello_then_chunks_then_done_with_usage():
    svc, prov, _ = make_service()
    frames = asyncio.run(_turn(svc, [pb.ClientMessage(session_id="s1", content="hi")]))
    kinds = [f.WhichOneof("message") for f in frames]
    assert kinds[0] == "runtime_hello" and kinds[-1] == "done"
    text = "".join(f.chunk.content for f in frames if f.WhichOneof("message") == "chunk")
    assert text == "hello there friend"
    assert frames[-1].done.usage.output_tokens > 0
    # system prompt rendered with fragment + defaults
    sys_msg = prov.calls[0]["messages"][0]
    assert sys_msg["content"] == "You are Omnia. Be brief."


def test_server_tool_loop_is_internal():
    svc, prov, calls = make_service()
    frames = asyncio.run(_turn(svc, [pb.ClientMessage(
        session_id="s2", content="weather?", metadata={"mock_scenario": "weather"})]))
    kinds = [f.WhichOneof("message") for f in frames]
    assert "tool_call" not in kinds  # server-side tools never reach the facade
    assert calls == [{"city": "Paris"}]
    assert frames[-1].done.final_content == "It is sunny in Paris."
    # the tool result was fed back to the model
    assert prov.calls[1]["messages"][-1]["role"] == "tool"


def test_client_tool_round_trip():
    svc, prov, _ = make_service()

    def reply(tc):
        assert tc.execution == pb.TOOL_EXECUTION_CLIENT
        assert tc.consent_message == "share location?"
        return pb.ClientMessage(session_id="s3", client_tool_result=pb.ClientToolResult(
            call_id=tc.id, result_json='{"lat": 1}'))

    frames = asyncio.run(_turn(svc, [pb.ClientMessage(
        session_id="s3", content="where am i", metadata={"mock_scenario": "client"})],
        replies=reply))
    kinds = [f.WhichOneof("message") for f in frames]
    assert "tool_call" in kinds and kinds[-1] == "done"
    assert frames[-1].done.final_content == "You are at home."
    assert json.loads(prov.calls[1]["messages"][-1]["content"]) == {"lat": 1}


def test_max_rounds_bounds_tool_loop():
    svc, prov, calls = make_service()
    frames = asyncio.run(_turn(svc, [pb.ClientMessage(
        session_id="s4", content="x", metadata={"mock_scenario": "loop"})]))
    assert frames[-1].WhichOneof("message") == "done"
    assert len(calls) == 3  # max_rounds=3 tool rounds, then the turn ends


def test_has_conversation_three_states():
    store = MemoryContextStore()
    svc, _, _ = make_service(store)

    async def go():
        r0 = await svc.has_conversation(pb.HasConversationRequest(session_id="nope"))
        await _turn(svc, [pb.ClientMessage(session_id="s5", content="hi")])
        r1 = await svc.has_conversation(pb.HasConversationRequest(session_id="s5"))
        store.fail = True
        r2 = await svc.has_conversation(pb.HasConversationRequest(session_id="s5"))
        return r0, r1, r2

    r0, r1, r2 = asyncio.run(go())
    assert r0.state == pb.RESUME_STATE_NOT_FOUND
    assert r1.state == pb.RESUME_STATE_RESUMABLE
    assert r2.state == pb.RESUME_STATE_UNAVAILABLE and r2.detail


def test_multi_turn_history_persisted():
    svc, prov, _ = make_service()

    async def go():
        await _turn(svc, [pb.ClientMessage(session_id="s6", content="first")])
        await _turn(svc, [pb.ClientMessage(session_id="s6", content="second")])

    asyncio.run(go())
    roles = [m["role"] for m in prov.calls[1]["messages"]]
    assert roles == ["system", "user", "assistant", "user"]


def test_provider_error_is_generic():
    svc, prov, _ = make_service()

    async def boom(*a, **k):
        raise RuntimeError("secret api key sk-123 leaked")
        yield  # noqa

    prov.stream = boom
    frames = asyncio.run(_turn(svc, [pb.ClientMessage(session_id="s7", content="hi")]))
    err = frames[-1].error
    assert err.code == "INTERNAL_ERROR" and "sk-123" not in err.message


def test_invoke_function_mode():
    svc, _, _ = make_service()
    resp = asyncio.run(svc.invoke(pb.InvocationRequest(input_json='{"message":"x"}',
                                                       invocation_id="inv1")))
    assert resp.invocation_id == "inv1" and resp.output_json == "hello there friend"


def test_runtime_config_env_roundtrip():
    c = RuntimeConfig(agent_name="a", namespace="ns", context_type="redis",
                      context_url="redis://x:6379/0", provider={"type": "local"},
                      engine={"model": "llama-3-8b", "tp": 1})
    c2 = RuntimeConfig.from_env(c.to_env())
    assert c2.agent_name == "a" and c2.context_url == "redis://x:6379/0"
    assert c2.provider["type"] == "local" and c2.engine["model"] == "llama-3-8b"


def test_local_engine_provider_end_to_end_cpu():
    from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine
    from omnia_amd.runtime.providers import LocalEngineProvider

    eng = AsyncLLMEngine(LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=64,
                                                block_size=16, max_batch=4,
                                                max_model_len=2048)))
    try:
        prov = LocalEngineProvider(eng)
        pack = PromptPack.minimal("sys")
        agent = Agent(pack, prov, MemoryContextStore(), None,
                      AgentConfig(defaults={"maxTokens": 5, "temperature": 0}))
        svc = RuntimeService(agent)
        f1 = asyncio.run(_turn(svc, [pb.ClientMessage(session_id="e1", content="hi")]))
        assert f1[-1].WhichOneof("message") == "done"
        assert f1[-1].done.usage.output_tokens == 5
        f2 = asyncio.run(_turn(svc, [pb.ClientMessage(session_id="e1", content="again")]))
        assert f2[-1].done.usage.input_tokens > f1[-1].done.usage.input_tokens
        # second turn hit the resident session KV prefix
        assert eng.engine.blocks.stats["prefix_hit_tokens"] > 0
    finally:
        eng.shutdown()


def test_stream_interval_coalesces_chunks():
    """OMNIA_STREAM_INTERVAL_MS: the first delta goes out at once, later deltas are
    merged per window, the text is complete and ends before Done."""
    words = " ".join(f"w{i}" for i in range(30))

    async def run(interval):
        prov = MockProvider(scenarios={"default_response": words}, delay_s=0.004)
        agent = Agent(PromptPack.minimal("sys"), prov, MemoryContextStore(), None, AgentConfig())
        svc = RuntimeService(agent, stream_interval_s=interval)
        st = QueueStream({"x-omnia-session-id": "s"})
        task = asyncio.ensure_future(svc.converse(st))
        await st.inbox.put(pb.ClientMessage(session_id="s", content="hi"))
        chunks = []
        while True:
            f = await st.outbox.get()
            k = f.WhichOneof("message")
            if k == "chunk":
                chunks.append(f.chunk.content)
            elif k == "done":
                break
        st.close()
        await task
        return chunks

    per_delta = _run_sync(run(0.0))
    merged = _run_sync(run(0.03))
    assert len(per_delta) == 30 and "".join(per_delta) == words
    assert "".join(merged) == words and merged[0] == "w0"
    assert 2 <= len(merged) < 15


# ------------------------------------------------------------------ context window
class _WordTok:
    def encode(self, s):
        return s.split()


def _agent_with(truncation, window, summary="the user asked about weather"):
    from omnia_amd.runtime.agent import Agent, AgentConfig

    class _Summ(MockProvider):
        async def complete(self, msgs, params=None, **kw):
            return summary, None, None

    a = Agent(PromptPack(PACK), _Summ(scenarios=SCEN), MemoryContextStore(), None,
              AgentConfig(context_window=window, truncation=truncation), tokenizer=_WordTok())
    return a


def _msgs():
    from omnia_amd.runtime.chat import Message

    return [Message("system", "sys prompt"), Message("user", "one two three"),
            Message("assistant", "call tool"), Message("tool", "tool result here"),
            Message("user", "four five"), Message("assistant", "six")]


def test_sliding_window_keeps_system_and_tool_pairs():
    a = _agent_with("sliding", 0)
    assert len(_run_sync(a._truncate(_msgs(), 0))) == len(_msgs())  # 0 = unlimited
    full = _msgs()
    assert [m.content for m in _run_sync(a._truncate(full, 10_000))] == [m.content for m in full]
    out = _run_sync(a._truncate(_msgs(), 19))
    roles = [m.role for m in out]
    assert roles[0] == "system" and out[0].content == "sys prompt"
    # the assistant tool call and its tool result went together; never a lone tool row
    assert "tool" not in roles and roles[1:] == ["user", "assistant"]
    assert sum(a._count(m) for m in out) <= 19


def test_summarize_strategy_replaces_old_turns_with_a_summary():
    a = _agent_with("summarize", 30)
    out = _run_sync(a._truncate(_msgs(), 30))
    assert out[0].content == "sys prompt"
    assert out[1].role == "system" and "the user asked about weather" in out[1].content
    assert out[-1].content == "six" and sum(a._count(m) for m in out) <= 30
    assert all(m.role != "tool" for m in out[:3])  # no orphaned tool result
    # custom falls back to sliding
    c = _agent_with("custom", 19)
    assert [m.role for m in _run_sync(c._truncate(_msgs(), 19))][0] == "system"
