"""BASELINE config 3 on the real engine: AgentRuntime + ToolRegistry with HTTP,
gRPC and MCP tool adapters, a multi-round tool-call loop driven by the in-node
engine, a Redis context store (the in-repo RESP server), and resume after a
runtime restart.

The local engine cannot be asked nicely to call a tool (random-init weights):
``tool_choice: required`` is enforced by the tool-call grammar (engine/guided.py),
so every forced round emits a valid call of an offered tool with
schema-valid arguments, which the executor routes to the adapter that owns the
tool.  The CPU variant runs tiny-llama; the GPU variant Llama-3-8B."""
import asyncio
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tool_fakes import GRPCToolFake, HTTPToolFake, MCPToolFake  # noqa: E402

from omnia_amd.api.proto import runtime_v1 as pb  # noqa: E402
from omnia_amd.utils.jsonschema import validate  # noqa: E402

WEATHER = {"name": "get_weather", "description": "Current weather for a city",
           "parameters": {"type": "object", "properties": {
               "city": {"type": "string", "maxLength": 12}, "unit": {"enum": ["C", "F"]}},
               "required": ["city", "unit"]}}
CLOCK = {"name": "get_time", "description": "Time in a zone",
         "parameters": {"type": "object", "properties": {"tz": {"enum": ["UTC", "PST", "CET"]}},
                        "required": ["tz"]}}
KB = {"name": "lookup", "description": "Search the knowledge base",
      "parameters": {"type": "object", "properties": {"q": {"type": "string", "maxLength": 16}},
                     "required": ["q"]}}


async def _turn(client, sid, content):
    st = await client.open({"x-omnia-session-id": sid})
    await st.send(pb.ClientMessage(session_id=sid, content=content))
    frames = []
    while True:
        m = await asyncio.wait_for(st.recv(), 600)
        if m is None:
            break
        k = m.WhichOneof("message")
        frames.append((k, m))
        if k in ("done", "error"):
            break
    await st.close()
    return frames


def _run(device: str, model: str, tmp_path, max_rounds=3):
    from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine
    from omnia_amd.facade.runtime_client import GrpcRuntimeClient
    from omnia_amd.runtime.app import build_runtime
    from omnia_amd.runtime.config import RuntimeConfig
    from omnia_amd.runtime.server import serve_grpc
    from omnia_amd.utils.resp import MiniRedis

    pack = {"id": "cfg3", "name": "cfg3", "version": "1.0.0",
            "template_engine": {"version": "v1", "syntax": "{{variable}}"},
            "prompts": {"default": {
                "id": "default", "name": "d", "version": "1.0.0",
                "system_template": "You are a helpful operations agent.",
                "tools": ["get_weather", "get_time", "lookup"],
                "tool_policy": {"tool_choice": "required", "max_rounds": max_rounds},
                "parameters": {"temperature": 0.9, "max_tokens": 160}}}}
    (tmp_path / "pack.json").write_text(json.dumps(pack))

    async def go():
        redis = await _start(MiniRedis())
        http = await HTTPToolFake().start()
        grpcf = await GRPCToolFake([CLOCK]).start()
        mcp = await MCPToolFake([KB]).start()
        tools = {"handlers": [
            {"name": "weather", "type": "http", "endpoint": f"http://127.0.0.1:{http.port}/",
             "tool": {"name": "get_weather", "description": WEATHER["description"],
                      "inputSchema": WEATHER["parameters"]}},
            {"name": "clock", "type": "grpc", "endpoint": f"127.0.0.1:{grpcf.port}"},
            {"name": "kb", "type": "mcp",
             "mcpConfig": {"endpoint": f"http://127.0.0.1:{mcp.port}/mcp"}}]}
        (tmp_path / "tools.json").write_text(json.dumps(tools))
        cfg = RuntimeConfig(provider={"type": "local"}, context_type="redis",
                            context_url=redis.url, promptpack_path=str(tmp_path / "pack.json"),
                            tools_config_path=str(tmp_path / "tools.json"))
        ecfg = EngineConfig(model=model, device=device, max_batch=8, max_model_len=4096,
                            num_blocks=1024, block_size=32, seed=11)

        async def start_runtime():
            eng = AsyncLLMEngine(LLMEngine(ecfg))
            svc = await build_runtime(cfg, engine=eng)
            server, port = await serve_grpc(svc, 0, "127.0.0.1")
            client = GrpcRuntimeClient(f"127.0.0.1:{port}")
            assert await client.wait_ready()
            return eng, svc, server, client

        eng, svc, server, client = await start_runtime()
        try:
            f1 = await _turn(client, "s-cfg3", "What is the weather and time, and look up X?")
            state1 = json.loads(await svc.agent.store.client.get("omnia:ctx:s-cfg3"))
        finally:
            await client.close()
            await server.stop(0)
            eng.shutdown()
        # ---- runtime restart: a fresh engine and runtime over the same Redis
        eng2, svc2, server2, client2 = await start_runtime()
        try:
            hc = await client2.has_conversation("s-cfg3")
            f2 = await _turn(client2, "s-cfg3", "And tomorrow?")
            state2 = json.loads(await svc2.agent.store.client.get("omnia:ctx:s-cfg3"))
        finally:
            await client2.close()
            await server2.stop(0)
            eng2.shutdown()
            for x in (http, grpcf, mcp):
                await x.stop()
            await redis.stop()
        return f1, f2, hc, state1, state2, http.calls, grpcf.calls, mcp.calls

    return asyncio.run(go())


async def _start(r):
    await r.start()
    return r


def _check(res, max_rounds=3):
    f1, f2, hc, state1, state2, http_calls, grpc_calls, mcp_calls = res
    kinds = [k for k, _ in f1]
    assert kinds[-1] == "done", kinds
    # every forced round called a tool through its adapter: max_rounds calls per turn
    msgs = state1["messages"]
    calls = [tc for m in msgs if m["role"] == "assistant" for tc in m.get("tool_calls") or []]
    results = [m for m in msgs if m["role"] == "tool"]
    assert len(calls) == max_rounds and len(results) == max_rounds
    schemas = {t["name"]: t["parameters"] for t in (WEATHER, CLOCK, KB)}
    for c in calls:
        args = c["arguments"] if isinstance(c["arguments"], dict) else json.loads(c["arguments"])
        validate(args, schemas[c["name"]])
    served = len(http_calls) + len(grpc_calls) + len(mcp_calls)
    assert served == 2 * max_rounds  # both turns, every call reached a fake
    by_name = {"get_weather": len(http_calls), "get_time": len(grpc_calls),
               "lookup": len(mcp_calls)}
    made = [c["name"] for m in state1["messages"] + state2["messages"][len(msgs):]
            if m["role"] == "assistant" for c in m.get("tool_calls") or []]
    for n, k in by_name.items():
        assert made.count(n) == k  # routed to the adapter owning that tool
    for m in results:
        assert json.loads(m["content"])  # tool results fed back to the model
    # resume after restart: the transcript came back from Redis
    assert hc.state == pb.RESUME_STATE_RESUMABLE
    assert [k for k, _ in f2][-1] == "done"
    assert state2["turn"] == 2 and len(state2["messages"]) > len(msgs)
    assert state2["messages"][:len(msgs)] == msgs


def test_config3_tool_loop_cpu(tmp_path):
    _check(_run("cpu", "tiny-llama", tmp_path))


@pytest.mark.gpu
def test_config3_tool_loop_llama3_8b_gpu(tmp_path):
    _check(_run("cuda", "llama-3-8b", tmp_path))
