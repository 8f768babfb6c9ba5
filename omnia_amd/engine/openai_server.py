"""OpenAI-compatible HTTP front for the in-node engine.

The reference reaches its LLMs through PromptKit providers of type openai /
vllm / ollama (``api/v1alpha1/provider_types.go``); serving the MI355X engine
behind the same wire lets any of those Provider specs -- and external clients --
point at it unchanged (``OpenAICompatProvider`` in ``runtime/providers.py`` is
the in-tree client).

Routes
  GET  /v1/models                      the served model
  POST /v1/chat/completions            Llama-3 chat template, SSE streaming,
                                       tools -> ``tool_calls``, response_format
                                       (json_object / json_schema -> K13 guided
                                       decoding), seed, stop, n=1
  POST /v1/completions                 raw prompt (text or token ids)
  POST /v1/embeddings                  when an embedding model is attached
  GET  /health, /metrics

Session affinity: ``x-omnia-session-id`` (or the body's ``user``) keys the
engine's resident KV prefix, so a multi-turn client re-prefills only the new
turn.  Works over :class:`AsyncLLMEngine` or the engine-core process client.

``python -m omnia_amd.engine.openai_server --model llama-3-8b --port 8000``
"""
from __future__ import annotations

import argparse
import json
import logging
import time
import uuid

from aiohttp import web

from ..observability import metrics as M
from ..runtime.chat import (Message, ToolCallReq, parse_tool_calls, render_llama3,
                            shared_prefix_len)
from .sampling_params import SamplingParams

log = logging.getLogger("omnia.engine.openai")

ENGINE = web.AppKey("engine", object)
EMBEDDER = web.AppKey("embedder", object)
MODEL = web.AppKey("model", str)


def _err(status: int, msg: str, typ: str = "invalid_request_error"):
    return web.json_response({"error": {"message": msg, "type": typ}}, status=status)


def _str_field(obj: dict, key: str, default: str = "") -> str:
    v = obj.get(key)
    if v is None:
        return default
    if not isinstance(v, str):
        raise TypeError(f"{key} must be a string")
    return v


def _content(raw) -> str:
    """OpenAI message content: a string, null, or an array of content parts (the
    text parts are kept; other part types carry no text)."""
    if raw is None:
        return ""
    if isinstance(raw, str):
        return raw
    if isinstance(raw, list):
        out = []
        for p in raw:
            if not isinstance(p, dict):
                raise TypeError("content parts must be objects")
            t = p.get("text")
            if t is None:
                continue
            if not isinstance(t, str):
                raise TypeError("content part text must be a string")
            out.append(t)
        return "".join(out)
    raise TypeError("content must be a string, an array of parts or null")


def _messages(raw: list) -> list[Message]:
    """Validated chat messages: a wrongly typed field raises TypeError (-> 400)."""
    out = []
    for m in raw:
        content = _content(m.get("content"))
        calls = []
        tcs = m.get("tool_calls")
        if tcs is not None and not isinstance(tcs, list):
            raise TypeError("tool_calls must be an array")
        for tc in tcs or []:
            if not isinstance(tc, dict):
                raise TypeError("tool_calls entries must be objects")
            fn = tc.get("function") or {}
            if not isinstance(fn, dict):
                raise TypeError("tool_calls[].function must be an object")
            args = fn.get("arguments", "{}")
            try:
                args = json.loads(args) if isinstance(args, str) else dict(args)
            except (json.JSONDecodeError, TypeError, ValueError):
                args = {"input": args}
            if not isinstance(args, dict):
                args = {"input": args}
            calls.append(ToolCallReq(id=_str_field(tc, "id"), name=_str_field(fn, "name"),
                                     arguments=args))
        out.append(Message(role=_str_field(m, "role", "user"), content=content, tool_calls=calls,
                           tool_call_id=_str_field(m, "tool_call_id"),
                           name=_str_field(m, "name")))
    return out


def _params(body: dict) -> SamplingParams:
    d = {k: body[k] for k in ("temperature", "top_p", "top_k", "max_tokens", "seed", "stop",
                              "frequency_penalty", "presence_penalty", "repetition_penalty",
                              "min_tokens", "ignore_eos", "response_format")
         if body.get(k) is not None}
    if "max_completion_tokens" in body and "max_tokens" not in d:
        d["max_tokens"] = body["max_completion_tokens"]
    return SamplingParams.from_dict(d)


def _usage(fin) -> dict:
    return {"prompt_tokens": fin.prompt_tokens, "completion_tokens": fin.output_tokens,
            "total_tokens": fin.prompt_tokens + fin.output_tokens,
            "prompt_tokens_details": {"cached_tokens": fin.cached_tokens}}


def _session(request, body) -> str | None:
    return request.headers.get("x-omnia-session-id") or body.get("user") or None


def build_app(engine, model_name: str, embedder=None) -> web.Application:
    app = web.Application(client_max_size=32 << 20)
    app[ENGINE] = engine
    app[MODEL] = model_name
    app[EMBEDDER] = embedder

    async def models(_):
        return web.json_response({"object": "list", "data": [
            {"id": model_name, "object": "model", "created": 0, "owned_by": "omnia-amd"}]})

    async def health(_):
        err = getattr(engine, "error", None)
        return web.json_response({"status": "error" if err else "ok"}, status=500 if err else 200)

    async def metrics(_):
        return web.Response(body=M.exposition(), content_type="text/plain")

    async def chat(request):
        try:
            body = await request.json()
            if not isinstance(body, dict):
                raise TypeError("the request body must be a JSON object")
            if not isinstance(body.get("messages"), list) or not all(
                    isinstance(m, dict) for m in body["messages"]):
                raise TypeError("messages must be an array of objects")
            msgs = _messages(body["messages"])
            params = _params(body)
            n = body.get("n", 1)
            tools = body.get("tools") or []
            if not isinstance(tools, list) or not all(isinstance(t, dict) for t in tools):
                raise TypeError("tools must be an array of objects")
            tools = [t.get("function", t) for t in tools if body.get("tool_choice") != "none"]
            if not all(isinstance(t, dict) and isinstance(t.get("name", ""), str)
                       for t in tools):
                raise TypeError("tool functions must be objects with a string name")
            tool_names = {t["name"] for t in tools if "name" in t}
            if not isinstance(body.get("stream_options") or {}, dict):
                raise TypeError("stream_options must be an object")
            if not isinstance(body.get("user") or "", str):
                raise TypeError("user must be a string")
            if isinstance(n, bool) or not isinstance(n, int):
                raise TypeError("n must be an integer")
        except (KeyError, TypeError, ValueError, AttributeError) as e:
            return _err(400, f"bad request: {e}")
        if n != 1:
            return _err(400, "only n=1 is supported")
        if tools and params.guided:
            return _err(400, "response_format cannot be combined with tools")
        enc = engine.tokenizer.encode
        prompt = enc(render_llama3(msgs, tools or None), add_bos=False)
        # cross-session KV sharing: only the system prompt + tool schemas are
        # published, within the request's ``cache_salt`` scope (kv_manager.py)
        salt = body.get("cache_salt")
        if salt is not None and not isinstance(salt, str):
            return _err(400, "bad request: cache_salt must be a string")
        params.cache_salt = salt or None
        params.share_limit = shared_prefix_len(msgs, tools, lambda t: enc(t, add_bos=False),
                                               prompt)
        rid = "chatcmpl-" + uuid.uuid4().hex[:24]
        created = int(time.time())
        sid = _session(request, body)
        gen = engine.generate(prompt, params, session_id=sid)
        if body.get("stream"):
            return await _chat_stream(request, gen, rid, created, tool_names,
                                      bool((body.get("stream_options") or {}).get(
                                          "include_usage")))
        text, fin = [], None
        try:
            async for ev in gen:
                if ev.finished:
                    fin = ev
                    break
                text.append(ev.text)
        except RuntimeError as e:
            return _err(400, str(e))
        content = "".join(text)
        msg = {"role": "assistant", "content": content}
        finish = fin.finish_reason if fin else "stop"
        if tool_names:
            rest, calls = parse_tool_calls(content, tool_names)
            if calls:
                msg = {"role": "assistant", "content": rest or None, "tool_calls": [
                    {"id": c.id, "type": "function",
                     "function": {"name": c.name, "arguments": c.arguments_json}}
                    for c in calls]}
                finish = "tool_calls"
        return web.json_response({
            "id": rid, "object": "chat.completion", "created": created, "model": model_name,
            "choices": [{"index": 0, "message": msg, "finish_reason": finish}],
            "usage": _usage(fin) if fin else None})

    async def _chat_stream(request, gen, rid, created, tool_names, include_usage):
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                           "Cache-Control": "no-cache"})
        await resp.prepare(request)

        def frame(delta, finish=None, usage=None):
            d = {"id": rid, "object": "chat.completion.chunk", "created": created,
                 "model": model_name,
                 "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}
            if usage is not None:
                d["usage"] = usage
            return b"data: " + json.dumps(d).encode() + b"\n\n"

        await resp.write(frame({"role": "assistant", "content": ""}))
        held: list[str] = []  # tool-call candidates are held until complete
        holding = None
        fin = None
        try:
            async for ev in gen:
                if ev.finished:
                    fin = ev
                    break
                if not ev.text:
                    continue
                if tool_names and holding is None:
                    held.append(ev.text)
                    lead = "".join(held).lstrip()
                    if lead:
                        holding = lead.startswith("{") or lead.startswith("<|python_tag|>")
                        if not holding:
                            await resp.write(frame({"content": "".join(held)}))
                            held = []
                elif holding:
                    held.append(ev.text)
                else:
                    await resp.write(frame({"content": ev.text}))
        except RuntimeError as e:
            await resp.write(b"data: " + json.dumps({"error": {"message": str(e)}}).encode()
                             + b"\n\n")
            await resp.write(b"data: [DONE]\n\n")
            return resp
        finish = fin.finish_reason if fin else "stop"
        if held:
            text = "".join(held)
            rest, calls = parse_tool_calls(text, tool_names)
            if calls:
                await resp.write(frame({"tool_calls": [
                    {"index": i, "id": c.id, "type": "function",
                     "function": {"name": c.name, "arguments": c.arguments_json}}
                    for i, c in enumerate(calls)]}))
                finish = "tool_calls"
            else:
                await resp.write(frame({"content": text}))
        await resp.write(frame({}, finish))
        if include_usage and fin is not None:
            d = {"id": rid, "object": "chat.completion.chunk", "created": created,
                 "model": model_name, "choices": [], "usage": _usage(fin)}
            await resp.write(b"data: " + json.dumps(d).encode() + b"\n\n")
        await resp.write(b"data: [DONE]\n\n")
        return resp

    async def completions(request):
        try:
            body = await request.json()
            if not isinstance(body, dict):
                raise TypeError("the request body must be a JSON object")
            params = _params(body)
            p = body["prompt"]
            if not isinstance(body.get("user") or "", str):
                raise TypeError("user must be a string")
            if not isinstance(body.get("cache_salt") or "", str):
                raise TypeError("cache_salt must be a string")
            # a raw prompt has no system-prompt boundary: it publishes KV pages
            # for cross-session sharing only inside an explicit cache_salt scope
            params.cache_salt = body.get("cache_salt") or None
            params.share_limit = None if params.cache_salt else 0
        except (KeyError, TypeError, ValueError, AttributeError) as e:
            return _err(400, f"bad request: {e}")
        vocab = getattr(engine.tokenizer, "vocab_size", None) or 1 << 31
        if isinstance(p, list) and p and all(isinstance(t, int) and not isinstance(t, bool)
                                             and 0 <= t < vocab for t in p):
            ids = p
        elif isinstance(p, str):
            ids = engine.tokenizer.encode(p, add_bos=True)
        else:
            return _err(400, "prompt must be a string or a list of token ids")
        rid = "cmpl-" + uuid.uuid4().hex[:24]
        created = int(time.time())
        gen = engine.generate(ids, params, session_id=_session(request, body))
        if body.get("stream"):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
            await resp.prepare(request)
            async for ev in gen:
                d = {"id": rid, "object": "text_completion", "created": created,
                     "model": model_name,
                     "choices": [{"index": 0, "text": ev.text or "",
                                  "finish_reason": ev.finish_reason if ev.finished else None}]}
                await resp.write(b"data: " + json.dumps(d).encode() + b"\n\n")
                if ev.finished:
                    break
            await resp.write(b"data: [DONE]\n\n")
            return resp
        text, fin = [], None
        try:
            async for ev in gen:
                if ev.finished:
                    fin = ev
                    break
                text.append(ev.text)
        except RuntimeError as e:
            return _err(400, str(e))
        return web.json_response({
            "id": rid, "object": "text_completion", "created": created, "model": model_name,
            "choices": [{"index": 0, "text": "".join(text),
                         "finish_reason": fin.finish_reason if fin else "stop"}],
            "usage": _usage(fin) if fin else None})

    async def embeddings(request):
        emb = app[EMBEDDER]
        if emb is None:
            return _err(404, "no embedding model is attached to this server")
        try:
            body = await request.json()
            inp = body["input"]
        except (KeyError, TypeError, ValueError, json.JSONDecodeError) as e:
            return _err(400, f"bad request: {e}")
        texts = [inp] if isinstance(inp, str) else inp
        if not isinstance(texts, list) or not texts or not all(isinstance(t, str) for t in texts):
            return _err(400, "input must be a string or a non-empty array of strings")
        vecs = await emb.embed(texts)
        return web.json_response({"object": "list", "model": body.get("model", "embed"), "data": [
            {"object": "embedding", "index": i, "embedding": [float(x) for x in v]}
            for i, v in enumerate(vecs)],
            "usage": {"prompt_tokens": 0, "total_tokens": 0}})

    app.router.add_get("/v1/models", models)
    app.router.add_post("/v1/chat/completions", chat)
    app.router.add_post("/v1/completions", completions)
    app.router.add_post("/v1/embeddings", embeddings)
    app.router.add_get("/health", health)
    app.router.add_get("/metrics", metrics)
    return app


def main(argv=None):
    from .engine import AsyncLLMEngine, EngineConfig

    ap = argparse.ArgumentParser(description="OpenAI-compatible server for the omnia engine")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--inproc", action="store_true", help="engine thread instead of process")
    ap.add_argument("--embed-model", default=None, help="attach an embedding model (K17)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    cfg = EngineConfig.from_env(model=a.model, device=a.device, max_batch=a.max_batch,
                                checkpoint=a.checkpoint)
    if a.inproc or a.device != "cuda":
        eng = AsyncLLMEngine.from_config(cfg)
    else:
        from .core_proc import EngineCoreClient

        eng = EngineCoreClient(cfg)
    embedder = None
    if a.embed_model:
        from ..memory.embedding import build_embedder

        embedder = build_embedder({"type": "local", "model": a.embed_model, "device": a.device})
    web.run_app(build_app(eng, a.model, embedder), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
