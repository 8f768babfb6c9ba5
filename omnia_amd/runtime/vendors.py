"""Remote vendor providers and hyperscaler platforms.

The reference resolves every Provider CRD type (``pkg/provider/types.go:28-110``)
and hosting platform (``api/v1alpha1/provider_types.go:188-315``: bedrock /
vertex / azure with their auth types) to a PromptKit provider that leaves the
pod.  Here the in-node engine is the default, and these clients keep the other
types working for users who point an AgentRuntime at a hosted model:

* :class:`GeminiProvider` -- ``gemini`` direct (API key) or on Vertex AI
  (``streamGenerateContent?alt=sse``, bearer token), chat + tools + embeddings.
* :class:`BedrockConverseProvider` -- ``claude`` on AWS Bedrock via the Converse
  API, SigV4-signed (access key or workload-identity credentials).
* :class:`AzureOpenAIProvider` -- ``openai`` on Azure AI Foundry (deployment
  URL, ``api-key`` or Entra bearer token).
* :class:`VoyageEmbeddings` (``voyageai``, embedding role),
  :class:`HuggingFaceProvider` (``huggingface``, OpenAI-compatible router +
  feature-extraction embeddings), :class:`ImagenProvider` (``imagen``, image
  role), :class:`CartesiaTTS` / :class:`ElevenLabsTTS` (tts role, PCM out for
  the duplex pipeline).

No vendor SDKs: plain aiohttp, so every client is exercised against local fakes
in ``tests/test_vendors.py``.
"""
from __future__ import annotations

import base64
import json
import os
import urllib.parse
import uuid

from .chat import Message, ToolCallReq
from .providers import OpenAICompatProvider, Provider, ProviderEvent, Usage


async def _post_json(url: str, body: dict, headers: dict, timeout_s: float = 120.0):
    import aiohttp

    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout_s)) as s:
        async with s.post(url, data=json.dumps(body).encode(),
                          headers={"Content-Type": "application/json", **headers}) as r:
            if r.status >= 400:
                raise RuntimeError(f"provider HTTP {r.status}")
            return await r.json(content_type=None)


async def _post_bytes(url: str, body: dict, headers: dict, timeout_s: float = 60.0) -> bytes:
    import aiohttp

    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout_s)) as s:
        async with s.post(url, json=body, headers=headers) as r:
            if r.status >= 400:
                raise RuntimeError(f"provider HTTP {r.status}")
            return await r.read()


# ------------------------------------------------------------------ credentials
class TokenSource:
    """Bearer token for Vertex / Azure workload identity: a static token, or
    one fetched from a metadata endpoint (GCE ``computeMetadata`` or Azure IMDS
    style JSON with ``access_token`` + ``expires_in``) and cached until expiry."""

    def __init__(self, token: str = "", url: str = "", headers: dict | None = None):
        self.static, self.url, self.headers = token, url, headers or {}
        self._tok, self._exp = "", 0.0

    async def token(self) -> str:
        import time

        if self.static:
            return self.static
        if self._tok and time.time() < self._exp - 60:
            return self._tok
        import aiohttp

        async with aiohttp.ClientSession() as s:
            async with s.get(self.url, headers=self.headers,
                             timeout=aiohttp.ClientTimeout(total=10)) as r:
                r.raise_for_status()
                d = await r.json(content_type=None)
        self._tok = d["access_token"]
        self._exp = time.time() + float(d.get("expires_in", 300))
        return self._tok


GCE_TOKEN_URL = ("http://metadata.google.internal/computeMetadata/v1/instance/"
                 "service-accounts/default/token")


# ------------------------------------------------------------------ gemini
class GeminiProvider(Provider):
    type = "gemini"

    def __init__(self, model: str, api_key: str | None = None, base_url: str = "",
                 vertex: dict | None = None, token: TokenSource | None = None,
                 timeout_s: float = 120.0, **kw):
        super().__init__(kw.pop("name", "gemini"), model, **kw)
        self.key, self.vertex, self.tok, self.timeout_s = api_key, vertex, token, timeout_s
        if vertex:
            region = vertex.get("region") or "us-central1"
            self.base = (base_url or f"https://{region}-aiplatform.googleapis.com").rstrip("/") + \
                f"/v1/projects/{vertex['project']}/locations/{region}/publishers/google/models"
        else:
            self.base = (base_url or "https://generativelanguage.googleapis.com").rstrip("/") + \
                "/v1beta/models"

    async def _auth(self) -> tuple[dict, str]:
        if self.vertex:
            return {"Authorization": f"Bearer {await self.tok.token()}"}, ""
        return {"x-goog-api-key": self.key or ""}, ""

    @staticmethod
    def to_contents(messages: list[Message]) -> tuple[dict | None, list[dict]]:
        system = "\n".join(m.content for m in messages if m.role == "system")
        contents = []
        for m in messages:
            if m.role == "system":
                continue
            if m.role == "tool":
                try:
                    resp = json.loads(m.content)
                except (json.JSONDecodeError, TypeError):
                    resp = {"result": m.content}
                if not isinstance(resp, dict):
                    resp = {"result": resp}
                contents.append({"role": "user", "parts": [{"functionResponse": {
                    "name": m.name or m.tool_call_id, "response": resp}}]})
            elif m.role == "assistant":
                parts = [{"text": m.content}] if m.content else []
                parts += [{"functionCall": {"name": t.name, "args": t.arguments}}
                          for t in (m.tool_calls or [])]
                contents.append({"role": "model", "parts": parts})
            else:
                contents.append({"role": "user", "parts": [{"text": m.content}]})
        sys_inst = {"parts": [{"text": system}]} if system else None
        return sys_inst, contents

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        import aiohttp

        sys_inst, contents = self.to_contents(messages)
        gen = {"temperature": params.temperature, "topP": params.top_p,
               "maxOutputTokens": params.max_tokens}
        if params.top_k and params.top_k > 0:
            gen["topK"] = params.top_k
        if params.stop:
            gen["stopSequences"] = list(params.stop)
        if params.json_schema is not None and not tools:
            gen["responseMimeType"] = "application/json"
            gen["responseSchema"] = params.json_schema
        body = {"contents": contents, "generationConfig": gen}
        if sys_inst:
            body["systemInstruction"] = sys_inst
        if tools:
            body["tools"] = [{"functionDeclarations": [
                {"name": t["name"], "description": t.get("description", ""),
                 "parameters": t.get("parameters", {"type": "object"})} for t in tools]}]
        hdrs, _ = await self._auth()
        url = f"{self.base}/{self.model}:streamGenerateContent?alt=sse"
        usage, calls, finish = Usage(), [], ""
        async with aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
            async with s.post(url, json=body, headers=hdrs) as r:
                if r.status >= 400:
                    raise RuntimeError(f"provider HTTP {r.status}")
                async for raw in r.content:
                    line = raw.decode().strip()
                    if not line.startswith("data:"):
                        continue
                    obj = json.loads(line[5:])
                    um = obj.get("usageMetadata")
                    if um:
                        usage = Usage(um.get("promptTokenCount", 0),
                                      um.get("candidatesTokenCount", 0),
                                      um.get("cachedContentTokenCount", 0))
                    for cand in obj.get("candidates", []):
                        for part in (cand.get("content") or {}).get("parts", []):
                            if part.get("text"):
                                yield ProviderEvent("text", text=part["text"])
                            if part.get("functionCall"):
                                fc = part["functionCall"]
                                calls.append(ToolCallReq("call_" + uuid.uuid4().hex[:12],
                                                         fc["name"], fc.get("args") or {}))
                        finish = cand.get("finishReason", finish)
        if calls:
            yield ProviderEvent("tool_calls", tool_calls=calls)
        yield ProviderEvent("done", usage=usage, finish_reason=finish.lower())

    async def embed(self, texts):
        hdrs, _ = await self._auth()
        if self.vertex:
            out = await _post_json(f"{self.base}/{self.model}:predict",
                                   {"instances": [{"content": t} for t in texts]}, hdrs)
            return [p["embeddings"]["values"] for p in out["predictions"]]
        out = await _post_json(
            f"{self.base}/{self.model}:batchEmbedContents",
            {"requests": [{"model": f"models/{self.model}",
                           "content": {"parts": [{"text": t}]}} for t in texts]}, hdrs)
        return [e["values"] for e in out["embeddings"]]


# ------------------------------------------------------------------ bedrock
class BedrockConverseProvider(Provider):
    """Anthropic (or any Converse-capable) model on AWS Bedrock.  The Converse
    API returns one JSON document; it is replayed as a single text event."""

    type = "claude"

    def __init__(self, model: str, region: str, access_key: str, secret_key: str,
                 session_token: str = "", endpoint: str = "", timeout_s: float = 120.0, **kw):
        super().__init__(kw.pop("name", "bedrock"), model, **kw)
        self.region = region
        self.creds = (access_key, secret_key, session_token)
        self.endpoint = (endpoint or f"https://bedrock-runtime.{region}.amazonaws.com").rstrip("/")
        self.timeout_s = timeout_s

    @staticmethod
    def to_converse(messages: list[Message]) -> tuple[list, list]:
        system = [{"text": m.content} for m in messages if m.role == "system" and m.content]
        msgs = []
        for m in messages:
            if m.role == "system":
                continue
            if m.role == "tool":
                msgs.append({"role": "user", "content": [{"toolResult": {
                    "toolUseId": m.tool_call_id, "content": [{"text": m.content}]}}]})
            elif m.role == "assistant":
                content = [{"text": m.content}] if m.content else []
                content += [{"toolUse": {"toolUseId": t.id, "name": t.name,
                                         "input": t.arguments}} for t in (m.tool_calls or [])]
                msgs.append({"role": "assistant", "content": content})
            else:
                msgs.append({"role": "user", "content": [{"text": m.content}]})
        return system, msgs

    def signed_request(self, body: bytes, now=None) -> tuple[str, dict]:
        from ..ee.encryption import sigv4_headers

        seg = urllib.parse.quote(self.model, safe="")
        url = f"{self.endpoint}/model/{seg}/converse"
        # SigV4 canonical URI for non-S3 services: each segment encoded twice
        sign_url = f"{self.endpoint}/model/{urllib.parse.quote(seg, safe='')}/converse"
        ak, sk, st = self.creds
        hdrs = sigv4_headers("POST", sign_url, body, self.region, "bedrock", ak, sk, st,
                             extra={"content-type": "application/json"}, now=now)
        return url, hdrs

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        import aiohttp
        import yarl

        system, msgs = self.to_converse(messages)
        body = {"messages": msgs,
                "inferenceConfig": {"maxTokens": params.max_tokens,
                                    "temperature": params.temperature, "topP": params.top_p}}
        if system:
            body["system"] = system
        if params.stop:
            body["inferenceConfig"]["stopSequences"] = list(params.stop)
        if tools:
            body["toolConfig"] = {"tools": [{"toolSpec": {
                "name": t["name"], "description": t.get("description", ""),
                "inputSchema": {"json": t.get("parameters", {"type": "object"})}}}
                for t in tools]}
        raw = json.dumps(body).encode()
        url, hdrs = self.signed_request(raw)
        async with aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
            # send the path exactly as signed (':' of model ids stays %3A)
            async with s.post(yarl.URL(url, encoded=True), data=raw, headers=hdrs) as r:
                if r.status >= 400:
                    raise RuntimeError(f"provider HTTP {r.status}")
                out = await r.json(content_type=None)
        calls = []
        for c in ((out.get("output") or {}).get("message") or {}).get("content", []):
            if "text" in c:
                yield ProviderEvent("text", text=c["text"])
            if "toolUse" in c:
                tu = c["toolUse"]
                calls.append(ToolCallReq(tu["toolUseId"], tu["name"], tu.get("input") or {}))
        if calls:
            yield ProviderEvent("tool_calls", tool_calls=calls)
        u = out.get("usage") or {}
        yield ProviderEvent("done", usage=Usage(u.get("inputTokens", 0), u.get("outputTokens", 0),
                                                u.get("cacheReadInputTokens", 0)),
                            finish_reason=out.get("stopReason", ""))


# ------------------------------------------------------------------ azure openai
class AzureOpenAIProvider(OpenAICompatProvider):
    type = "openai"

    def __init__(self, endpoint: str, deployment: str, api_key: str | None = None,
                 token: TokenSource | None = None, api_version: str = "2024-10-21", **kw):
        super().__init__(endpoint, api_key=None, name=kw.pop("name", "azure"),
                         model=deployment, **kw)
        self.azure_key, self.tok, self.api_version = api_key, token, api_version
        self._bearer = ""

    def _url(self, path):
        return (f"{self.base_url}/openai/deployments/{self.model}{path}"
                f"?api-version={self.api_version}")

    def _hdrs(self):
        h = {"Content-Type": "application/json", **self.headers}
        if self.azure_key:
            h["api-key"] = self.azure_key
        elif self._bearer:
            h["Authorization"] = f"Bearer {self._bearer}"
        return h

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        if not self.azure_key and self.tok is not None:
            self._bearer = await self.tok.token()
        async for ev in super().stream(messages, tools, params, session_id, metadata):
            yield ev


# ------------------------------------------------------------------ embeddings / inference
class VoyageEmbeddings(Provider):
    type = "voyageai"

    def __init__(self, model: str, api_key: str | None, base_url: str = "", **kw):
        super().__init__(kw.pop("name", "voyageai"), model or "voyage-3", **kw)
        self.key = api_key
        self.base = (base_url or "https://api.voyageai.com/v1").rstrip("/")

    async def stream(self, *a, **k):
        raise RuntimeError("voyageai is an embedding-role provider")
        yield  # pragma: no cover

    async def embed(self, texts):
        out = await _post_json(f"{self.base}/embeddings", {"input": texts, "model": self.model},
                               {"Authorization": f"Bearer {self.key or ''}"})
        return [d["embedding"] for d in sorted(out["data"], key=lambda d: d.get("index", 0))]


class HuggingFaceProvider(OpenAICompatProvider):
    """HF Inference: chat through the OpenAI-compatible router, embeddings through
    the feature-extraction pipeline."""

    type = "huggingface"

    def __init__(self, model: str, api_key: str | None, base_url: str = "",
                 feature_url: str = "", **kw):
        super().__init__(base_url or "https://router.huggingface.co/v1", api_key=api_key,
                         name=kw.pop("name", "huggingface"), model=model, **kw)
        self.feature_base = (feature_url or
                             "https://router.huggingface.co/hf-inference/models").rstrip("/")

    async def embed(self, texts):
        out = await _post_json(f"{self.feature_base}/{self.model}/pipeline/feature-extraction",
                               {"inputs": texts}, {"Authorization": f"Bearer {self.api_key}"})
        return [v if not (v and isinstance(v[0], list)) else
                [sum(c) / len(v) for c in zip(*v)] for v in out]  # token vectors -> mean


class ImagenProvider(Provider):
    """Image role: ``generate(prompt, n)`` -> PNG bytes (Gemini API or Vertex)."""

    type = "imagen"

    def __init__(self, model: str, api_key: str | None = None, vertex: dict | None = None,
                 token: TokenSource | None = None, base_url: str = "", **kw):
        super().__init__(kw.pop("name", "imagen"), model or "imagen-3.0-generate-002", **kw)
        self._g = GeminiProvider(self.model, api_key=api_key, vertex=vertex, token=token,
                                 base_url=base_url)

    async def stream(self, *a, **k):
        raise RuntimeError("imagen is an image-role provider")
        yield  # pragma: no cover

    async def generate(self, prompt: str, n: int = 1, aspect_ratio: str = "1:1") -> list[bytes]:
        hdrs, _ = await self._g._auth()
        out = await _post_json(f"{self._g.base}/{self.model}:predict",
                               {"instances": [{"prompt": prompt}],
                                "parameters": {"sampleCount": n, "aspectRatio": aspect_ratio}},
                               hdrs)
        return [base64.b64decode(p["bytesBase64Encoded"]) for p in out.get("predictions", [])]


# ------------------------------------------------------------------ tts
class CartesiaTTS:
    type = "cartesia"

    def __init__(self, api_key: str | None, model: str = "", voice: str = "",
                 base_url: str = "", version: str = "2024-11-13"):
        self.key, self.model, self.voice, self.version = api_key, model or "sonic-2", voice, version
        self.base = (base_url or "https://api.cartesia.ai").rstrip("/")

    async def transcribe(self, pcm: bytes, sample_rate: int) -> str:
        raise RuntimeError("cartesia is a tts-role provider")

    async def synthesize(self, text: str, sample_rate: int) -> bytes:
        return await _post_bytes(
            f"{self.base}/tts/bytes",
            {"model_id": self.model, "transcript": text, "voice": {"mode": "id", "id": self.voice},
             "output_format": {"container": "raw", "encoding": "pcm_s16le",
                               "sample_rate": sample_rate}},
            {"X-API-Key": self.key or "", "Cartesia-Version": self.version})


class ElevenLabsTTS:
    type = "elevenlabs"

    def __init__(self, api_key: str | None, model: str = "", voice: str = "",
                 base_url: str = ""):
        self.key, self.model = api_key, model or "eleven_multilingual_v2"
        self.voice = voice or "21m00Tcm4TlvDq8ikWAM"
        self.base = (base_url or "https://api.elevenlabs.io").rstrip("/")

    async def transcribe(self, pcm: bytes, sample_rate: int) -> str:
        raise RuntimeError("elevenlabs is a tts-role provider")

    async def synthesize(self, text: str, sample_rate: int) -> bytes:
        return await _post_bytes(
            f"{self.base}/v1/text-to-speech/{self.voice}?output_format=pcm_{sample_rate}",
            {"text": text, "model_id": self.model}, {"xi-api-key": self.key or ""})


# ------------------------------------------------------------------ factory
def _secret(secrets: dict | None, *names: str) -> str:
    for n in names:
        if secrets and secrets.get(n):
            return secrets[n]
        if os.environ.get(n.upper().replace("-", "_")):
            return os.environ[n.upper().replace("-", "_")]
    return ""


def build_vendor_provider(spec: dict, key: str | None, secrets: dict | None, common: dict):
    """Vendor / platform provider for a Provider ``spec``, or None when the type
    is not a vendor type handled here."""
    t = (spec.get("type") or "").lower()
    model = spec.get("model", "")
    base = spec.get("baseURL") or ""
    plat = spec.get("platform") or {}
    ptype = (plat.get("type") or "").lower()
    auth = spec.get("auth") or {}
    if ptype == "bedrock":
        if t != "claude":
            raise ValueError(f"{t} on bedrock is not supported")
        return BedrockConverseProvider(
            model, plat.get("region") or "us-east-1",
            _secret(secrets, "aws-access-key-id", "AWS_ACCESS_KEY_ID"),
            _secret(secrets, "aws-secret-access-key", "AWS_SECRET_ACCESS_KEY"),
            _secret(secrets, "aws-session-token", "AWS_SESSION_TOKEN"),
            endpoint=plat.get("endpoint", ""), **common)
    if ptype in ("vertex", "azure"):
        tok = TokenSource(_secret(secrets, "access-token", "token"),
                          url=GCE_TOKEN_URL if ptype == "vertex" else
                          auth.get("tokenURL", ""),
                          headers={"Metadata-Flavor": "Google"} if ptype == "vertex" else {})
        if ptype == "vertex":
            if t == "openai":
                raise ValueError("openai on vertex is not supported")
            vx = {"project": plat.get("project", ""), "region": plat.get("region", "")}
            return GeminiProvider(model, vertex=vx, token=tok, base_url=plat.get("endpoint", ""),
                                  **common)
        if t == "gemini":
            raise ValueError("gemini on azure is not supported")
        return AzureOpenAIProvider(plat["endpoint"], model, api_key=key or None, token=tok,
                                   **common)
    if t == "gemini":
        return GeminiProvider(model, api_key=key, base_url=base, **common)
    if t == "voyageai":
        return VoyageEmbeddings(model, key, base_url=base, **common)
    if t == "huggingface":
        return HuggingFaceProvider(model, key, base_url=base, **common)
    if t == "imagen":
        return ImagenProvider(model, api_key=key, base_url=base, **common)
    return None


def build_tts_provider(spec: dict, api_key: str | None = None):
    t = (spec.get("type") or "").lower()
    audio = spec.get("audio") or {}
    if t == "cartesia":
        return CartesiaTTS(api_key, spec.get("model", ""), audio.get("voice", ""),
                           spec.get("baseURL", ""))
    if t == "elevenlabs":
        return ElevenLabsTTS(api_key, spec.get("model", ""), audio.get("voice", ""),
                             spec.get("baseURL", ""))
    return None
