"""LLM providers behind the agent loop.

The reference builds a PromptKit ``providers.Provider`` from the Provider CRD
(``internal/runtime/provider.go:95-151``; types ``pkg/provider/types.go:28-110``)
and every call leaves the pod.  Here the default is **local**: the in-node
MI355X engine (:class:`LocalEngineProvider`).  Remote OpenAI-compatible
endpoints (``openai`` / ``vllm`` / ``ollama`` types) and Anthropic's Messages
API (``claude``) remain available, the other vendor types and the bedrock /
vertex / azure platforms are in :mod:`.vendors`, and ``mock`` reproduces the
reference's scenario-driven mock provider for tests
(``internal/runtime/scenario.go``).
"""
from __future__ import annotations

import asyncio
import dataclasses
import json
import time
import uuid
from dataclasses import dataclass, field
from typing import AsyncIterator

import yaml

from ..engine.sampling_params import SamplingParams
from .chat import Message, ToolCallReq, parse_tool_calls, render_llama3, shared_prefix_len


@dataclass
class Usage:
    input_tokens: int = 0
    output_tokens: int = 0
    cached_tokens: int = 0

    def __iadd__(self, o: "Usage"):
        self.input_tokens += o.input_tokens
        self.output_tokens += o.output_tokens
        self.cached_tokens += o.cached_tokens
        return self


@dataclass
class ProviderEvent:
    type: str  # text | tool_calls | done | error
    text: str = ""
    tool_calls: list = field(default_factory=list)
    usage: Usage | None = None
    finish_reason: str = ""
    ttft: float | None = None
    code: str = ""  # error events: machine code surfaced in the runtime Error frame


class ProviderError(RuntimeError):
    """A provider failure with a client-visible code (``ENGINE_FAULT``,
    ``PROVIDER_ERROR``...).  The message stays generic on the wire."""

    def __init__(self, message: str = "provider error", code: str = "PROVIDER_ERROR"):
        super().__init__(message)
        self.code = code


@dataclass
class Pricing:
    input_per_1k: float = 0.0
    output_per_1k: float = 0.0
    cached_per_1k: float = 0.0

    def cost(self, u: Usage) -> float:
        fresh_in = max(0, u.input_tokens - u.cached_tokens)
        return (fresh_in * self.input_per_1k + u.cached_tokens * self.cached_per_1k
                + u.output_tokens * self.output_per_1k) / 1000.0


class Provider:
    type = "base"

    def __init__(self, name: str = "", model: str = "", pricing: Pricing | None = None,
                 defaults: dict | None = None):
        self.name = name or self.type
        self.model = model
        self.pricing = pricing or Pricing()
        self.defaults = defaults or {}

    async def stream(self, messages: list[Message], tools: list[dict],
                     params: SamplingParams, session_id: str | None = None,
                     metadata: dict | None = None) -> AsyncIterator[ProviderEvent]:
        raise NotImplementedError
        yield  # pragma: no cover

    async def complete(self, messages, tools=None, params=None, session_id=None,
                       metadata=None) -> tuple[str, list, Usage]:
        text, calls, usage = [], [], Usage()
        async for ev in self.stream(messages, tools or [], params or SamplingParams(),
                                    session_id, metadata):
            if ev.type == "text":
                text.append(ev.text)
            elif ev.type == "tool_calls":
                calls.extend(ev.tool_calls)
            elif ev.type == "done" and ev.usage:
                usage = ev.usage
        return "".join(text), calls, usage

    async def embed(self, texts: list[str]) -> list[list[float]]:
        raise NotImplementedError(f"{self.type} provider has no embedding role")

    async def health(self) -> bool:
        return True

    def close(self):
        pass


# ===================================================================== local
class LocalEngineProvider(Provider):
    """In-node MI355X engine: Llama-3 chat template -> AsyncLLMEngine stream.

    The session id keys the engine's resident KV prefix, so turn n of a session
    prefills only the tokens added since turn n-1."""

    type = "local"

    def __init__(self, engine, name="local", model="", pricing=None, defaults=None,
                 embedder=None):
        super().__init__(name, model or engine.engine.model_cfg.name, pricing, defaults)
        self.engine = engine
        self.embedder = embedder

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        tok = self.engine.tokenizer
        prompt_text = render_llama3(messages, tools or None)
        prompt_ids = tok.encode(prompt_text, add_bos=False)
        params = params or SamplingParams()
        if params.share_limit is None:
            # publish only the PromptPack prefix for cross-session KV sharing, in
            # the caller's workspace scope (engine/kv_manager.py "Isolation")
            md = metadata or {}
            params = dataclasses.replace(
                params, share_limit=shared_prefix_len(
                    messages, tools, lambda t: tok.encode(t, add_bos=False), prompt_ids),
                cache_salt=params.cache_salt or md.get("workspace") or md.get("namespace"))
        tool_names = {t["name"] for t in tools or []}
        buf: list[str] = []
        holding = None  # decide after the first non-space text whether this is a tool call
        usage = Usage(input_tokens=len(prompt_ids))
        t0 = time.perf_counter()
        ttft = None
        async for ev in self.engine.generate(prompt_ids, params, session_id=session_id):
            if ev.text:
                if ttft is None:
                    ttft = time.perf_counter() - t0
                if tool_names and holding is None:
                    buf.append(ev.text)
                    joined = "".join(buf).lstrip()
                    if joined:
                        holding = joined.startswith("{") or joined.startswith("<|python_tag|>") \
                            or joined.startswith("[")
                        if not holding:
                            yield ProviderEvent("text", text="".join(buf))
                            buf = []
                elif holding:
                    buf.append(ev.text)
                else:
                    yield ProviderEvent("text", text=ev.text)
            if ev.finished:
                usage.output_tokens = ev.output_tokens
                usage.cached_tokens = ev.cached_tokens
                text = "".join(buf)
                if holding and text:
                    rest, calls = parse_tool_calls(text, tool_names)
                    if calls:
                        if rest:
                            yield ProviderEvent("text", text=rest)
                        yield ProviderEvent("tool_calls", tool_calls=calls)
                    else:
                        yield ProviderEvent("text", text=text)
                elif text:
                    yield ProviderEvent("text", text=text)
                if ev.finish_reason == "error":
                    yield ProviderEvent("error", text="engine fault", code="ENGINE_FAULT")
                yield ProviderEvent("done", usage=usage, finish_reason=ev.finish_reason or "",
                                    ttft=ev.ttft if ev.ttft is not None else ttft)
                return

    async def embed(self, texts):
        if self.embedder is None:
            raise NotImplementedError("no embedding model configured")
        return await self.embedder.embed(texts)

    async def health(self) -> bool:
        h = getattr(self.engine, "health", None)
        if not callable(h):
            return True
        # an engine-core health call is a blocking round trip: keep it off the loop
        return bool(await asyncio.get_running_loop().run_in_executor(None, h))


# ===================================================================== mock
class MockProvider(Provider):
    """Scenario-driven mock (reference: PromptKit mock provider + scenario.go).

    Scenario file (YAML/JSON)::

        default_response: "Hello from the mock"
        scenarios:
          weather:
            turns:
              - tool_calls: [{name: get_weather, arguments: {city: Paris}}]
              - response: "It is sunny in Paris."
    The scenario is picked from metadata ``mock_scenario`` (then content_type,
    then "default"); the turn index advances per (session, scenario)."""

    type = "mock"

    def __init__(self, name="mock", model="mock-model", scenarios: dict | None = None,
                 path: str | None = None, chunk_words: int = 1, delay_s: float = 0.0, **kw):
        super().__init__(name, model, **kw)
        data = scenarios or {}
        if path:
            with open(path) as f:
                data = yaml.safe_load(f) or {}
        self.default_response = data.get("default_response", "This is a mock response.")
        self.scenarios = data.get("scenarios", {})
        self.turns: dict[tuple, int] = {}
        self.chunk_words = chunk_words
        self.delay_s = delay_s
        self.calls: list[dict] = []

    @staticmethod
    def pick_scenario(metadata: dict | None, content: str = "") -> str:
        md = metadata or {}
        if md.get("mock_scenario"):
            return md["mock_scenario"]
        ct = md.get("content_type", "")
        if ct.startswith("image/"):
            return "image-analysis"
        if ct.startswith("audio/"):
            return "audio-analysis"
        if ct in ("application/pdf", "text/plain") or ct.startswith("application/vnd"):
            return "document-qa"
        return "default"

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        last_user = next((m.content for m in reversed(messages) if m.role == "user"), "")
        scen = self.pick_scenario(metadata, last_user)
        self.calls.append({"scenario": scen, "messages": [m.to_dict() for m in messages],
                           "tools": [t["name"] for t in tools or []]})
        key = (session_id or "", scen)
        turn_idx = self.turns.get(key, 0)
        self.turns[key] = turn_idx + 1
        spec = self.scenarios.get(scen)
        text, calls = self.default_response, []
        if spec is not None:
            turns = spec.get("turns", [])
            if turns:
                t = turns[min(turn_idx, len(turns) - 1)]
                text = t.get("response", "")
                calls = [ToolCallReq(id=c.get("id") or "call_" + uuid.uuid4().hex[:12],
                                     name=c["name"], arguments=c.get("arguments", {}))
                         for c in t.get("tool_calls", [])]
            elif "response" in spec:
                text = spec["response"]
        in_tok = sum(len(m.content.split()) for m in messages)
        words = text.split(" ") if text else []
        for i in range(0, len(words), self.chunk_words):
            if self.delay_s:
                await asyncio.sleep(self.delay_s)
            piece = " ".join(words[i:i + self.chunk_words])
            yield ProviderEvent("text", text=(piece if i == 0 else " " + piece))
        if calls:
            yield ProviderEvent("tool_calls", tool_calls=calls)
        yield ProviderEvent("done", usage=Usage(in_tok, max(1, len(words))),
                            finish_reason="tool_calls" if calls else "stop")

    async def embed(self, texts):
        import hashlib

        out = []
        for t in texts:
            h = hashlib.sha256(t.encode()).digest()
            v = [((b / 255.0) - 0.5) for b in h[:32]]
            n = sum(x * x for x in v) ** 0.5 or 1.0
            out.append([x / n for x in v])
        return out


# ===================================================================== openai-compatible
class OpenAICompatProvider(Provider):
    """``/v1/chat/completions`` SSE client (openai, vllm, ollama, and our own
    engine's OpenAI shim)."""

    type = "openai"

    def __init__(self, base_url: str, api_key: str | None = None, name="openai", model="",
                 headers: dict | None = None, timeout_s: float = 120.0, **kw):
        super().__init__(name, model, **kw)
        self.base_url = base_url.rstrip("/")
        self.api_key = api_key
        self.headers = headers or {}
        self.timeout_s = timeout_s

    def _url(self, path):
        b = self.base_url
        return b + path if b.endswith("/v1") else b + "/v1" + path

    def _hdrs(self):
        h = {"Content-Type": "application/json", **self.headers}
        if self.api_key:
            h["Authorization"] = f"Bearer {self.api_key}"
        return h

    @staticmethod
    def to_openai(messages: list[Message]) -> list[dict]:
        out = []
        for m in messages:
            d = {"role": m.role, "content": m.content}
            if m.role == "assistant" and m.tool_calls:
                d["tool_calls"] = [{"id": t.id, "type": "function",
                                    "function": {"name": t.name,
                                                 "arguments": t.arguments_json}}
                                   for t in m.tool_calls]
            if m.role == "tool":
                d["tool_call_id"] = m.tool_call_id
            out.append(d)
        return out

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        import aiohttp

        body = {"model": self.model, "messages": self.to_openai(messages), "stream": True,
                "temperature": params.temperature, "top_p": params.top_p,
                "max_tokens": params.max_tokens,
                "stream_options": {"include_usage": True}}
        if params.frequency_penalty:
            body["frequency_penalty"] = params.frequency_penalty
        if params.presence_penalty:
            body["presence_penalty"] = params.presence_penalty
        if params.stop:
            body["stop"] = params.stop
        if params.seed is not None:
            body["seed"] = params.seed
        if session_id:
            body["user"] = session_id
        if tools:
            body["tools"] = [{"type": "function", "function": t} for t in tools]
        elif params.json_schema is not None:
            body["response_format"] = {"type": "json_schema", "json_schema": {
                "name": "response", "schema": params.json_schema, "strict": True}}
        elif params.json_object:
            body["response_format"] = {"type": "json_object"}
        usage = Usage()
        calls: dict[int, dict] = {}
        finish = ""
        timeout = aiohttp.ClientTimeout(total=self.timeout_s)
        async with aiohttp.ClientSession(timeout=timeout) as sess:
            async with sess.post(self._url("/chat/completions"), json=body,
                                 headers=self._hdrs()) as resp:
                if resp.status >= 400:
                    raise RuntimeError(f"provider HTTP {resp.status}")
                async for raw in resp.content:
                    line = raw.decode().strip()
                    if not line.startswith("data:"):
                        continue
                    data = line[5:].strip()
                    if data == "[DONE]":
                        break
                    obj = json.loads(data)
                    if obj.get("usage"):
                        u = obj["usage"]
                        usage = Usage(u.get("prompt_tokens", 0), u.get("completion_tokens", 0),
                                      (u.get("prompt_tokens_details") or {}).get("cached_tokens",
                                                                                 0))
                    for ch in obj.get("choices", []):
                        delta = ch.get("delta", {})
                        if delta.get("content"):
                            yield ProviderEvent("text", text=delta["content"])
                        for tc in delta.get("tool_calls", []) or []:
                            slot = calls.setdefault(tc.get("index", 0),
                                                    {"id": "", "name": "", "args": ""})
                            slot["id"] = tc.get("id") or slot["id"]
                            fn = tc.get("function", {})
                            slot["name"] += fn.get("name", "") or ""
                            slot["args"] += fn.get("arguments", "") or ""
                        if ch.get("finish_reason"):
                            finish = ch["finish_reason"]
        if calls:
            out = []
            for c in calls.values():
                try:
                    args = json.loads(c["args"] or "{}")
                except json.JSONDecodeError:
                    args = {"input": c["args"]}
                out.append(ToolCallReq(id=c["id"] or "call_" + uuid.uuid4().hex[:12],
                                       name=c["name"], arguments=args))
            yield ProviderEvent("tool_calls", tool_calls=out)
        yield ProviderEvent("done", usage=usage, finish_reason=finish)

    async def embed(self, texts):
        import aiohttp

        async with aiohttp.ClientSession() as sess:
            async with sess.post(self._url("/embeddings"), headers=self._hdrs(),
                                 json={"model": self.model, "input": texts}) as resp:
                if resp.status >= 400:
                    raise RuntimeError(f"embedding HTTP {resp.status}")
                obj = await resp.json()
        return [d["embedding"] for d in obj["data"]]


class AnthropicProvider(Provider):
    """Anthropic Messages API (``type: claude``) streaming client."""

    type = "claude"

    def __init__(self, api_key: str | None, base_url="https://api.anthropic.com", name="claude",
                 model="", timeout_s=120.0, **kw):
        super().__init__(name, model, **kw)
        self.api_key = api_key
        self.base_url = base_url.rstrip("/")
        self.timeout_s = timeout_s

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        import aiohttp

        system = "\n".join(m.content for m in messages if m.role == "system")
        msgs = []
        for m in messages:
            if m.role == "system":
                continue
            if m.role == "tool":
                msgs.append({"role": "user", "content": [{"type": "tool_result",
                                                          "tool_use_id": m.tool_call_id,
                                                          "content": m.content}]})
            elif m.role == "assistant" and m.tool_calls:
                content = ([{"type": "text", "text": m.content}] if m.content else []) + [
                    {"type": "tool_use", "id": t.id, "name": t.name, "input": t.arguments}
                    for t in m.tool_calls]
                msgs.append({"role": "assistant", "content": content})
            else:
                msgs.append({"role": m.role, "content": m.content})
        body = {"model": self.model, "system": system, "messages": msgs, "stream": True,
                "max_tokens": params.max_tokens, "temperature": params.temperature}
        if tools:
            body["tools"] = [{"name": t["name"], "description": t.get("description", ""),
                              "input_schema": t.get("parameters", {"type": "object"})}
                             for t in tools]
        hdrs = {"x-api-key": self.api_key or "", "anthropic-version": "2023-06-01",
                "content-type": "application/json"}
        usage = Usage()
        calls, cur = [], None
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
            async with s.post(self.base_url + "/v1/messages", json=body, headers=hdrs) as resp:
                if resp.status >= 400:
                    raise RuntimeError(f"provider HTTP {resp.status}")
                async for raw in resp.content:
                    line = raw.decode().strip()
                    if not line.startswith("data:"):
                        continue
                    ev = json.loads(line[5:])
                    t = ev.get("type")
                    if t == "message_start":
                        u = ev["message"].get("usage", {})
                        usage.input_tokens = u.get("input_tokens", 0)
                    elif t == "content_block_start" and ev["content_block"]["type"] == "tool_use":
                        cb = ev["content_block"]
                        cur = {"id": cb["id"], "name": cb["name"], "json": ""}
                    elif t == "content_block_delta":
                        d = ev["delta"]
                        if d.get("type") == "text_delta":
                            yield ProviderEvent("text", text=d["text"])
                        elif d.get("type") == "input_json_delta" and cur is not None:
                            cur["json"] += d.get("partial_json", "")
                    elif t == "content_block_stop" and cur is not None:
                        calls.append(ToolCallReq(cur["id"], cur["name"],
                                                 json.loads(cur["json"] or "{}")))
                        cur = None
                    elif t == "message_delta":
                        usage.output_tokens = ev.get("usage", {}).get("output_tokens", 0)
        if calls:
            yield ProviderEvent("tool_calls", tool_calls=calls)
        yield ProviderEvent("done", usage=usage)


def build_provider(spec: dict, engine=None, secrets: dict | None = None) -> Provider:
    """Provider from a Provider CRD ``spec`` (``api/v1alpha1/provider_types.go:273-413``)."""
    t = (spec.get("type") or "mock").lower()
    model = spec.get("model", "")
    pr = spec.get("pricing") or {}
    pricing = Pricing(float(pr.get("inputCostPer1K", 0) or 0),
                      float(pr.get("outputCostPer1K", 0) or 0),
                      float(pr.get("cachedCostPer1K", 0) or 0))
    defaults = spec.get("defaults") or {}
    key = spec.get("apiKey")  # resolved from a devroot Secret (OMNIA_CONFIG_DIR)
    cred = spec.get("credential") or {}
    if secrets and key is None:
        key = secrets.get(cred.get("secretRef", {}).get("key", "api-key")) or \
            next(iter(secrets.values()), None)
    if t in ("local", "omnia", "rocm", "engine"):
        if engine is None:
            raise ValueError("local provider needs an engine")
        return LocalEngineProvider(engine, name=spec.get("name", "local"), model=model,
                                   pricing=pricing, defaults=defaults)
    if t == "mock":
        return MockProvider(name="mock", model=model or "mock-model",
                            path=(spec.get("mock") or {}).get("path"),
                            scenarios=(spec.get("mock") or {}).get("scenarios"),
                            pricing=pricing, defaults=defaults)
    from .vendors import build_vendor_provider

    vendor = build_vendor_provider(spec, key, secrets,
                                   {"pricing": pricing, "defaults": defaults})
    if vendor is not None:
        return vendor
    if t in ("openai", "vllm", "ollama", "openrouter", "azure"):
        base = spec.get("baseURL") or {"openai": "https://api.openai.com/v1",
                                       "ollama": "http://127.0.0.1:11434",
                                       "openrouter": "https://openrouter.ai/api/v1"}.get(t, "")
        return OpenAICompatProvider(base, api_key=key, name=t, model=model,
                                    headers=spec.get("headers"), pricing=pricing,
                                    defaults=defaults)
    if t in ("claude", "anthropic"):
        return AnthropicProvider(key, base_url=spec.get("baseURL") or "https://api.anthropic.com",
                                 model=model, pricing=pricing, defaults=defaults)
    raise ValueError(f"unsupported provider type {t!r}")
