"""Vendor providers and hyperscaler platforms against local
fakes of each API: Gemini (direct + Vertex, SSE stream with a function call),
Bedrock Converse (SigV4 with the double-encoded model segment), Azure OpenAI
(deployment URL + api-key), Voyage / HuggingFace embeddings, Imagen, and the
Cartesia / ElevenLabs TTS byte endpoints.  The fakes assert auth headers and
request shapes; no vendor SDK is involved."""
import asyncio
import base64
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.runtime import vendors as V
from omnia_amd.runtime.chat import Message, ToolCallReq
from omnia_amd.runtime.duplex import build_audio_provider
from omnia_amd.runtime.providers import build_provider

CALLS = []


class _H(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):
        pass

    def _send(self, raw: bytes, ctype="application/json"):
        self.send_response(200)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(raw)))
        self.end_headers()
        self.wfile.write(raw)

    def do_POST(self):
        raw = self.rfile.read(int(self.headers.get("Content-Length", 0)))
        body = json.loads(raw or b"{}")
        CALLS.append((self.path, {k.lower(): v for k, v in self.headers.items()}, body))
        p = self.path
        if ":streamGenerateContent" in p:
            assert p.endswith("?alt=sse")
            evs = [{"candidates": [{"content": {"role": "model", "parts": [{"text": "Hel"}]}}]},
                   {"candidates": [{"content": {"parts": [{"text": "lo"}, {"functionCall": {
                       "name": "get_weather", "args": {"city": "Oslo"}}}]},
                       "finishReason": "STOP"}],
                    "usageMetadata": {"promptTokenCount": 7, "candidatesTokenCount": 3}}]
            return self._send("".join(f"data: {json.dumps(e)}\r\n\r\n" for e in evs).encode(),
                              "text/event-stream")
        if p.endswith(":batchEmbedContents"):
            return self._send(json.dumps({"embeddings": [
                {"values": [float(len(r["content"]["parts"][0]["text"])), 1.0]}
                for r in body["requests"]]}).encode())
        if p.endswith(":predict"):
            if "instances" in body and "prompt" in body["instances"][0]:
                n = body["parameters"]["sampleCount"]
                return self._send(json.dumps({"predictions": [
                    {"bytesBase64Encoded": base64.b64encode(b"\x89PNG%d" % i).decode()}
                    for i in range(n)]}).encode())
            return self._send(json.dumps({"predictions": [
                {"embeddings": {"values": [0.5, 0.5]}} for _ in body["instances"]]}).encode())
        if p.endswith("/converse"):
            return self._send(json.dumps({
                "output": {"message": {"role": "assistant", "content": [
                    {"text": "bedrock says hi"},
                    {"toolUse": {"toolUseId": "tu1", "name": "lookup", "input": {"q": 1}}}]}},
                "usage": {"inputTokens": 11, "outputTokens": 4}, "stopReason": "tool_use"}
            ).encode())
        if "/openai/deployments/" in p:
            evs = [{"choices": [{"delta": {"content": "azure ok"}}]},
                   {"choices": [{"delta": {}, "finish_reason": "stop"}],
                    "usage": {"prompt_tokens": 5, "completion_tokens": 2}}]
            out = "".join(f"data: {json.dumps(e)}\n\n" for e in evs) + "data: [DONE]\n\n"
            return self._send(out.encode(), "text/event-stream")
        if p == "/v1/embeddings":
            return self._send(json.dumps({"data": [
                {"index": i, "embedding": [float(i), 2.0]} for i in range(len(body["input"]))
            ][::-1]}).encode())
        if p.endswith("/pipeline/feature-extraction"):
            return self._send(json.dumps([[[1.0, 3.0], [3.0, 5.0]] for _ in body["inputs"]]
                                         ).encode())
        if p == "/tts/bytes" or p.startswith("/v1/text-to-speech/"):
            return self._send(b"\x01\x00" * 8, "application/octet-stream")
        self.send_response(404)
        self.send_header("Content-Length", "0")
        self.end_headers()


@pytest.fixture(scope="module")
def base():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


def _collect(prov, msgs, tools=None):
    async def go():
        return [e async for e in prov.stream(msgs, tools or [], SamplingParams(max_tokens=16))]
    return asyncio.run(go())


MSGS = [Message("system", "be brief"), Message("user", "weather in Oslo?"),
        Message("assistant", "", tool_calls=[ToolCallReq("c1", "get_weather", {"city": "Oslo"})]),
        Message("tool", '{"temp": 3}', tool_call_id="c1", name="get_weather")]
TOOLS = [{"name": "get_weather", "description": "w", "parameters": {"type": "object"}}]


def test_gemini_direct_stream_tools_and_embed(base):
    CALLS.clear()
    p = build_provider({"type": "gemini", "model": "gemini-2.0-flash", "baseURL": base},
                       secrets={"api-key": "GKEY"})
    assert isinstance(p, V.GeminiProvider)
    evs = _collect(p, MSGS, TOOLS)
    assert "".join(e.text for e in evs if e.type == "text") == "Hello"
    tc = [e for e in evs if e.type == "tool_calls"][0].tool_calls[0]
    assert (tc.name, tc.arguments) == ("get_weather", {"city": "Oslo"})
    done = evs[-1]
    assert done.type == "done" and done.usage.input_tokens == 7 and done.usage.output_tokens == 3
    path, hdrs, body = CALLS[-1]
    assert path.startswith("/v1beta/models/gemini-2.0-flash:streamGenerateContent")
    assert hdrs["x-goog-api-key"] == "GKEY"
    assert body["systemInstruction"]["parts"][0]["text"] == "be brief"
    roles = [c["role"] for c in body["contents"]]
    assert roles == ["user", "model", "user"]
    assert body["contents"][1]["parts"][0]["functionCall"]["name"] == "get_weather"
    assert body["contents"][2]["parts"][0]["functionResponse"]["response"] == {"temp": 3}
    assert body["tools"][0]["functionDeclarations"][0]["name"] == "get_weather"
    vecs = asyncio.run(p.embed(["ab", "abcd"]))
    assert vecs == [[2.0, 1.0], [4.0, 1.0]]


def test_gemini_on_vertex_uses_bearer_and_project_path(base):
    CALLS.clear()
    p = build_provider({"type": "gemini", "model": "gemini-1.5-pro",
                        "platform": {"type": "vertex", "project": "proj", "region": "europe-west4",
                                     "endpoint": base},
                        "auth": {"type": "workloadIdentity"}},
                       secrets={"access-token": "ya29.tok"})
    evs = _collect(p, [Message("user", "hi")])
    assert evs[-1].type == "done"
    path, hdrs, _ = CALLS[-1]
    assert path.startswith("/v1/projects/proj/locations/europe-west4/publishers/google/models/"
                           "gemini-1.5-pro:streamGenerateContent")
    assert hdrs["authorization"] == "Bearer ya29.tok"
    assert asyncio.run(p.embed(["x"])) == [[0.5, 0.5]]


def test_bedrock_converse_sigv4(base):
    CALLS.clear()
    p = build_provider({"type": "claude", "model": "anthropic.claude-3-5-sonnet-20240620-v1:0",
                        "platform": {"type": "bedrock", "region": "us-west-2", "endpoint": base},
                        "auth": {"type": "accessKey"}},
                       secrets={"aws-access-key-id": "AKID", "aws-secret-access-key": "SECRET"})
    assert isinstance(p, V.BedrockConverseProvider)
    evs = _collect(p, MSGS, TOOLS)
    assert evs[0].text == "bedrock says hi"
    assert evs[1].tool_calls[0].name == "lookup"
    assert evs[-1].usage.input_tokens == 11 and evs[-1].finish_reason == "tool_use"
    path, hdrs, body = CALLS[-1]
    assert path == "/model/anthropic.claude-3-5-sonnet-20240620-v1%3A0/converse"
    auth = hdrs["authorization"]
    assert auth.startswith("AWS4-HMAC-SHA256 Credential=AKID/")
    assert "/us-west-2/bedrock/aws4_request" in auth
    assert "x-amz-date" in hdrs
    assert body["system"] == [{"text": "be brief"}]
    assert body["messages"][1]["content"][0]["toolUse"]["name"] == "get_weather"
    assert body["messages"][2]["content"][0]["toolResult"]["toolUseId"] == "c1"
    assert body["toolConfig"]["tools"][0]["toolSpec"]["name"] == "get_weather"


def test_bedrock_signature_is_deterministic():
    import datetime as dt

    p = V.BedrockConverseProvider("m:1", "us-east-1", "AK", "SK")
    now = dt.datetime(2024, 1, 1, tzinfo=dt.timezone.utc)
    u1, h1 = p.signed_request(b"{}", now=now)
    u2, h2 = p.signed_request(b"{}", now=now)
    assert u1 == u2 and h1 == h2 and u1.endswith("/model/m%3A1/converse")
    _, h3 = p.signed_request(b"{ }", now=now)
    assert h3["Authorization"] != h1["Authorization"]


def test_azure_openai_deployment_url_and_key(base):
    CALLS.clear()
    p = build_provider({"type": "openai", "model": "gpt4o-deploy",
                        "platform": {"type": "azure", "endpoint": base},
                        "auth": {"type": "servicePrincipal"}}, secrets={"api-key": "AZKEY"})
    assert isinstance(p, V.AzureOpenAIProvider)
    evs = _collect(p, [Message("user", "hi")])
    assert evs[0].text == "azure ok" and evs[-1].usage.output_tokens == 2
    path, hdrs, _ = CALLS[-1]
    assert path == "/openai/deployments/gpt4o-deploy/chat/completions?api-version=2024-10-21"
    assert hdrs["api-key"] == "AZKEY" and "authorization" not in hdrs


def test_platform_matrix_rejections():
    with pytest.raises(ValueError):
        build_provider({"type": "openai", "model": "m",
                        "platform": {"type": "vertex", "project": "p"}})
    with pytest.raises(ValueError):
        build_provider({"type": "gemini", "model": "m", "platform": {"type": "bedrock"}})
    with pytest.raises(ValueError):
        build_provider({"type": "gemini", "model": "m",
                        "platform": {"type": "azure", "endpoint": "http://x"}})


def test_voyage_and_huggingface_embeddings(base):
    v = build_provider({"type": "voyageai", "model": "voyage-3", "baseURL": base + "/v1"},
                       secrets={"api-key": "VK"})
    assert asyncio.run(v.embed(["a", "b"])) == [[0.0, 2.0], [1.0, 2.0]]  # sorted by index
    assert CALLS[-1][1]["authorization"] == "Bearer VK"
    hf = V.HuggingFaceProvider("sentence-transformers/x", "HFK", feature_url=base + "/models")
    assert asyncio.run(hf.embed(["q"])) == [[2.0, 4.0]]  # token vectors mean-pooled
    assert CALLS[-1][0] == "/models/sentence-transformers/x/pipeline/feature-extraction"


def test_imagen_generate(base):
    p = build_provider({"type": "imagen", "model": "imagen-3.0-generate-002", "baseURL": base},
                       secrets={"api-key": "IK"})
    imgs = asyncio.run(p.generate("a cat", n=2))
    assert imgs == [b"\x89PNG0", b"\x89PNG1"]
    assert CALLS[-1][0] == "/v1beta/models/imagen-3.0-generate-002:predict"


def test_tts_vendors(base):
    c = build_audio_provider({"type": "cartesia", "baseURL": base, "apiKey": "CK",
                              "audio": {"voice": "v1"}}, "tts")
    pcm = asyncio.run(c.synthesize("hello", 16000))
    assert pcm == b"\x01\x00" * 8
    path, hdrs, body = CALLS[-1]
    assert path == "/tts/bytes" and hdrs["x-api-key"] == "CK"
    assert body["output_format"] == {"container": "raw", "encoding": "pcm_s16le",
                                     "sample_rate": 16000}
    e = build_audio_provider({"type": "elevenlabs", "baseURL": base, "apiKey": "EK"}, "tts")
    asyncio.run(e.synthesize("hello", 24000))
    path, hdrs, body = CALLS[-1]
    assert path.endswith("?output_format=pcm_24000") and hdrs["xi-api-key"] == "EK"
