"""OpenAI-compatible engine server: chat (stream / non-stream, tools,
response_format), completions, embeddings, driven through the in-tree
OpenAICompatProvider client and raw HTTP (CPU tiny-llama)."""
import asyncio
import json
import socket

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine
from omnia_amd.engine.openai_server import build_app
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.memory.embedding import HashEmbedder
from omnia_amd.runtime.chat import Message
from omnia_amd.runtime.providers import OpenAICompatProvider


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _serve(eng, embedder=None):
    app = build_app(eng, "tiny-llama", embedder)
    runner = web.AppRunner(app)
    await runner.setup()
    port = _port()
    site = web.TCPSite(runner, "127.0.0.1", port)
    await site.start()
    return runner, f"http://127.0.0.1:{port}"


@pytest.fixture(scope="module")
def eng():
    e = AsyncLLMEngine(LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=256,
                                              block_size=32, max_batch=8, max_model_len=1024)))
    yield e
    e.shutdown()


def test_chat_stream_and_nonstream_agree(eng):
    async def main():
        runner, url = await _serve(eng, HashEmbedder(64))
        try:
            prov = OpenAICompatProvider(url, model="tiny-llama")
            msgs = [Message("system", "be brief"), Message("user", "hello there")]
            p = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
            text, usage = [], None
            async for ev in prov.stream(msgs, [], p, session_id="oa1"):
                if ev.type == "text":
                    text.append(ev.text)
                elif ev.type == "done":
                    usage = ev.usage
            async with aiohttp.ClientSession() as s:
                body = {"model": "tiny-llama", "temperature": 0, "max_tokens": 12,
                        "ignore_eos": True, "messages": [m.to_dict() for m in msgs]}
                async with s.post(url + "/v1/chat/completions", json=body) as r:
                    assert r.status == 200
                    full = await r.json()
                async with s.get(url + "/v1/models") as r:
                    models = await r.json()
                async with s.post(url + "/v1/completions",
                                  json={"prompt": "abc", "max_tokens": 5, "temperature": 0,
                                        "ignore_eos": True}) as r:
                    comp = await r.json()
                async with s.post(url + "/v1/embeddings", json={"input": ["a b", "c"]}) as r:
                    emb = await r.json()
                async with s.post(url + "/v1/chat/completions", json={"messages": "x"}) as r:
                    bad = r.status
            return "".join(text), usage, full, models, comp, emb, bad
        finally:
            await runner.cleanup()

    text, usage, full, models, comp, emb, bad = asyncio.run(main())
    assert full["choices"][0]["message"]["content"] == text
    assert usage.output_tokens == 12 == full["usage"]["completion_tokens"]
    assert models["data"][0]["id"] == "tiny-llama"
    assert comp["usage"]["completion_tokens"] == 5
    assert len(emb["data"]) == 2 and len(emb["data"][0]["embedding"]) == 64
    assert bad == 400


def test_chat_response_format_json_schema(eng):
    schema = {"type": "object", "properties": {"ok": {"type": "boolean"}}, "required": ["ok"]}

    async def main():
        runner, url = await _serve(eng)
        try:
            async with aiohttp.ClientSession() as s:
                body = {"messages": [{"role": "user", "content": "answer"}], "temperature": 0.7,
                        "seed": 3, "max_tokens": 64,
                        "response_format": {"type": "json_schema",
                                            "json_schema": {"name": "r", "schema": schema}}}
                async with s.post(url + "/v1/chat/completions", json=body) as r:
                    return await r.json()
        finally:
            await runner.cleanup()

    out = asyncio.run(main())
    obj = json.loads(out["choices"][0]["message"]["content"])
    assert isinstance(obj["ok"], bool) and set(obj) == {"ok"}
    assert out["choices"][0]["finish_reason"] == "stop"
