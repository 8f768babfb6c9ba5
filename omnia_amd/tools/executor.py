"""OmniaExecutor: server-side tool dispatch for the agent loop.

Reference: ``internal/runtime/tools/omnia_executor.go:56-552`` (dispatch by
handler type ``:403-434``, policy-broker decision before every call, fail
closed ``:436-473``), ``http_client.go`` (URL templates, query/header params,
static query/body, JMESPath body/response mapping, redaction, bearer/basic
auth), ``omnia_executor_mcp.go`` (MCP streamable-http / sse / stdio),
``omnia_executor_grpc.go`` (``omnia.tools.v1.ToolService/Execute``),
``openapi_adapter.go`` (operations -> tools) and client tools, which are NOT
executed here but surfaced to the facade (``runtime.proto:119-127``).

Tools config file format = the operator-generated ``handlers[]``
(``internal/runtime/tools/config.go:118-145``) mounted at /etc/omnia/tools.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
import re
import time
import uuid
from dataclasses import dataclass, field
from pathlib import Path

import yaml

from ..utils import failpoints
from ..observability import metrics as M
from ..utils import jmespath
from .resilience import (CircuitBreaker, CircuitOpen, PermanentError, RetryPolicy,
                         TransientError, call_with_retry)

log = logging.getLogger("omnia.tools")

DEFAULT_TIMEOUT_S = 30.0


class PolicyDenied(Exception):
    pass


@dataclass
class ToolDef:
    name: str
    description: str = ""
    input_schema: dict = field(default_factory=lambda: {"type": "object"})
    handler: str = ""
    handler_type: str = "http"
    remote_name: str = ""  # name at the backend (MCP/gRPC/OpenAPI operation)
    meta: dict = field(default_factory=dict)

    @property
    def is_client(self) -> bool:
        return self.handler_type == "client"

    def spec(self) -> dict:
        return {"name": self.name, "description": self.description,
                "parameters": self.input_schema or {"type": "object"}}


@dataclass
class CallContext:
    session_id: str = ""
    agent: str = ""
    namespace: str = ""
    workspace: str = ""
    user_id: str = ""
    origin: str = ""
    claims: dict = field(default_factory=dict)
    headers: dict = field(default_factory=dict)  # x-omnia-* propagation


def load_tools_config(path: str | Path) -> dict:
    p = Path(path)
    if p.is_dir():
        for cand in ("tools.yaml", "tools.json", "config.yaml"):
            if (p / cand).exists():
                p = p / cand
                break
        else:
            return {"handlers": []}
    if not p.exists():
        return {"handlers": []}
    text = p.read_text()
    return (json.loads(text) if p.suffix == ".json" else yaml.safe_load(text)) or {"handlers": []}


def _dur(v, default):
    if v in (None, "", 0):
        return default
    if isinstance(v, (int, float)):
        return float(v)
    from ..runtime.context_store import parse_ttl

    s = str(v)
    if s.endswith("ms"):
        return float(s[:-2]) / 1000.0
    return float(parse_ttl(s))


def redact(obj, fields: list[str]):
    if not fields:
        return obj
    if isinstance(obj, dict):
        return {k: ("[REDACTED]" if k in fields else redact(v, fields)) for k, v in obj.items()}
    if isinstance(obj, list):
        return [redact(x, fields) for x in obj]
    return obj


# ===================================================================== handlers
class Handler:
    type = "base"

    def __init__(self, entry: dict, secrets_dir: str | None = None):
        self.entry = entry
        self.name = entry["name"]
        self.endpoint = entry.get("endpoint", "")
        self.timeout = _dur(entry.get("timeout"), DEFAULT_TIMEOUT_S)
        self.secrets_dir = secrets_dir

    async def discover(self) -> list[ToolDef]:
        t = self.entry.get("tool")
        if not t:
            return []
        return [ToolDef(name=t["name"], description=t.get("description", ""),
                        input_schema=t.get("inputSchema") or {"type": "object"},
                        handler=self.name, handler_type=self.type, remote_name=t["name"],
                        meta={"outputSchema": t.get("outputSchema")})]

    async def call(self, tool: ToolDef, args: dict, ctx: CallContext) -> str:
        raise NotImplementedError

    async def close(self):
        pass

    token_acquirer = None  # workloadIdentity (tools/workload_identity.py); None: the pod's

    async def _wif_headers(self, cfg: dict) -> dict:
        """The workloadIdentity auth header, resolved per call (tokens are cached
        per audience by the acquirer); {} when the handler uses other auth.
        Unsupported clouds / no identity fail the call loudly."""
        from .workload_identity import (WorkloadIdentityError, default_acquirer,
                                        resolve_header, wif_config)

        wif = wif_config(self.entry, cfg)
        if wif is None:
            return {}
        try:
            name, val = await resolve_header(self.token_acquirer or default_acquirer(), wif)
        except WorkloadIdentityError as e:
            raise PermanentError(str(e)) from None
        return {name: val}

    def _secret(self, key: str | None) -> str | None:
        if not key:
            return None
        if self.secrets_dir:
            p = Path(self.secrets_dir) / self.name / key
            if p.exists():
                return p.read_text().strip()
            p = Path(self.secrets_dir) / key
            if p.exists():
                return p.read_text().strip()
        return os.environ.get(key)


class HTTPHandler(Handler):
    type = "http"

    def __init__(self, entry, secrets_dir=None):
        super().__init__(entry, secrets_dir)
        self.cfg = entry.get("httpConfig") or {}
        self.retry = RetryPolicy.from_cfg(self.cfg.get("retryPolicy"))

    def _auth_headers(self) -> dict:
        c = self.cfg
        auth = self.entry.get("auth") or {}
        atype = (auth.get("type") or c.get("authType") or "").lower()
        token = c.get("authToken") or self._secret(auth.get("tokenKey") or c.get("authTokenKey"))
        if not token and c.get("authTokenPath") and Path(c["authTokenPath"]).exists():
            token = Path(c["authTokenPath"]).read_text().strip()
        if atype == "bearer" and token:
            return {c.get("authHeader") or "Authorization": f"Bearer {token}"}
        if atype == "basic" and token:
            if ":" in token:
                token = base64.b64encode(token.encode()).decode()
            return {"Authorization": f"Basic {token}"}
        if atype == "header" and token:
            return {c.get("authHeader") or "X-API-Key": token}
        return {}

    def build_request(self, args: dict, ctx: CallContext) -> tuple[str, str, dict, dict, object]:
        c = self.cfg
        args = dict(args or {})
        method = (c.get("method") or "POST").upper()
        url = c.get("endpoint") or self.endpoint
        tmpl = c.get("urlTemplate")
        if tmpl:
            def rep(m):
                k = m.group(1)
                return str(args.pop(k, m.group(0)))

            url = re.sub(r"\{([A-Za-z_][\w]*)\}", rep, tmpl if "://" in tmpl else url + tmpl)
        headers = {"Content-Type": c.get("contentType") or "application/json",
                   **(c.get("headers") or {}), **self._auth_headers(), **ctx.headers}
        for arg, hdr in (c.get("headerParams") or {}).items():
            if arg in args:
                headers[hdr] = str(args.pop(arg))
        query = dict(c.get("staticQuery") or {})
        for q in c.get("queryParams") or []:
            if q in args:
                query[q] = args.pop(q)
        body: object = args
        if c.get("staticBody"):
            body = {**c["staticBody"], **args}
        if c.get("bodyMapping"):
            body = jmespath.search(c["bodyMapping"], body)
        if method in ("GET", "DELETE", "HEAD"):
            for k, v in (body or {}).items() if isinstance(body, dict) else []:
                query.setdefault(k, v)
            body = None
        return method, url, headers, query, body

    async def call(self, tool, args, ctx):
        import aiohttp

        method, url, headers, query, body = self.build_request(args, ctx)
        headers.update(await self._wif_headers(self.cfg))
        timeout = aiohttp.ClientTimeout(total=self.timeout)

        async def once():
            async with aiohttp.ClientSession(timeout=timeout) as s:
                async with s.request(method, url, params={k: str(v) for k, v in query.items()},
                                     json=body if body is not None else None,
                                     headers=headers) as r:
                    text = await r.text()
                    if r.status in self.retry.retryable_status or r.status >= 500:
                        ra = r.headers.get("Retry-After")
                        raise TransientError(f"HTTP {r.status}",
                                             float(ra) if ra and ra.isdigit() else None)
                    if r.status >= 400:
                        raise PermanentError(f"HTTP {r.status}: {text[:200]}")
                    return text

        text = await call_with_retry(once, self.retry)
        try:
            data = json.loads(text) if text else None
        except json.JSONDecodeError:
            return json.dumps({"result": text})
        if self.cfg.get("responseMapping"):
            data = jmespath.search(self.cfg["responseMapping"], data)
        data = redact(data, self.cfg.get("redact") or [])
        return json.dumps(data)


class GRPCHandler(Handler):
    """``omnia.tools.v1.ToolService`` client (``api/proto/tools/v1/tools.proto``)."""

    type = "grpc"

    def __init__(self, entry, secrets_dir=None):
        super().__init__(entry, secrets_dir)
        self.cfg = entry.get("grpcConfig") or {}
        self.target = (self.cfg.get("endpoint") or self.endpoint).replace("grpc://", "")
        self.retry = RetryPolicy.from_cfg(self.cfg.get("retryPolicy"))
        self._ch = None

    def _channel(self):
        import grpc

        if self._ch is None:
            if self.cfg.get("tls"):
                self._ch = grpc.aio.secure_channel(self.target, grpc.ssl_channel_credentials())
            else:
                self._ch = grpc.aio.insecure_channel(self.target)
        return self._ch

    async def discover(self):
        base = await super().discover()
        if base:
            return base
        from ..api.proto import tools_v1 as T

        try:
            rpc = self._channel().unary_unary(T.METHOD_LIST_TOOLS,
                                              request_serializer=T.ListToolsRequest.SerializeToString,
                                              response_deserializer=T.ListToolsResponse.FromString)
            resp = await rpc(T.ListToolsRequest(), timeout=self.timeout)
        except Exception as e:  # noqa: BLE001
            log.warning("grpc tool discovery failed for %s: %s", self.name, e)
            return []
        return [ToolDef(name=t.name, description=t.description,
                        input_schema=json.loads(t.input_schema or '{"type":"object"}'),
                        handler=self.name, handler_type=self.type, remote_name=t.name)
                for t in resp.tools]

    async def call(self, tool, args, ctx):
        import grpc

        from ..api.proto import tools_v1 as T

        rpc = self._channel().unary_unary(T.METHOD_EXECUTE,
                                          request_serializer=T.ToolRequest.SerializeToString,
                                          response_deserializer=T.ToolResponse.FromString)
        req = T.ToolRequest(tool_name=tool.remote_name or tool.name, arguments_json=json.dumps(args),
                            metadata={k: str(v) for k, v in ctx.headers.items()})
        # credentials ride the call metadata (authorization / the configured header)
        md = [(k.lower(), v) for k, v in (await self._wif_headers(self.cfg)).items()]
        tok = self.cfg.get("authToken") or self._secret(self.cfg.get("authTokenKey"))
        if not md and tok and (self.cfg.get("authType") or "").lower() == "bearer":
            md = [("authorization", "Bearer " + tok)]

        async def once():
            try:
                return await rpc(req, timeout=self.timeout, metadata=md or None)
            except grpc.aio.AioRpcError as e:
                if e.code() in (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED,
                                grpc.StatusCode.RESOURCE_EXHAUSTED):
                    raise TransientError(str(e.code())) from e
                raise PermanentError(f"{e.code()}: {e.details()}") from e

        resp = await call_with_retry(once, self.retry)
        if resp.is_error:
            raise PermanentError(resp.error_message or "tool error")
        return resp.result_json or "null"

    async def close(self):
        if self._ch is not None:
            await self._ch.close()


class MCPHandler(Handler):
    """MCP client: streamable-http (JSON or SSE responses), sse, stdio."""

    type = "mcp"

    def __init__(self, entry, secrets_dir=None):
        super().__init__(entry, secrets_dir)
        self.cfg = entry.get("mcpConfig") or {}
        self.transport = self.cfg.get("transport", "streamable-http")
        self.url = self.cfg.get("endpoint") or self.endpoint
        self.session_id = None
        self._id = 0
        self._proc = None
        self._lock = asyncio.Lock()
        self._init = False
        self.tool_filter = self.cfg.get("toolFilter") or {}

    def _next_id(self):
        self._id += 1
        return self._id

    async def _rpc_http(self, method, params):
        import aiohttp

        body = {"jsonrpc": "2.0", "id": self._next_id(), "method": method, "params": params}
        hdrs = {"Content-Type": "application/json",
                "Accept": "application/json, text/event-stream",
                **(self.cfg.get("headers") or {}), **(await self._wif_headers(self.cfg))}
        if self.session_id:
            hdrs["Mcp-Session-Id"] = self.session_id
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout)) as s:
            async with s.post(self.url, json=body, headers=hdrs) as r:
                if r.status >= 500:
                    raise TransientError(f"MCP HTTP {r.status}")
                if r.status >= 400:
                    raise PermanentError(f"MCP HTTP {r.status}")
                self.session_id = r.headers.get("Mcp-Session-Id", self.session_id)
                ctype = r.headers.get("Content-Type", "")
                if "text/event-stream" in ctype:
                    async for raw in r.content:
                        line = raw.decode().strip()
                        if line.startswith("data:"):
                            msg = json.loads(line[5:])
                            if msg.get("id") == body["id"]:
                                return self._result(msg)
                    raise PermanentError("MCP stream ended without a response")
                if r.status == 202:
                    return None
                return self._result(await r.json())

    async def _rpc_stdio(self, method, params):
        if self._proc is None:
            cmd = self.cfg.get("command")
            args = self.cfg.get("args") or []
            env = {**os.environ, **(self.cfg.get("env") or {})}
            self._proc = await asyncio.create_subprocess_exec(
                cmd, *args, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
                env=env)
        rid = self._next_id()
        msg = {"jsonrpc": "2.0", "id": rid, "method": method, "params": params}
        self._proc.stdin.write((json.dumps(msg) + "\n").encode())
        await self._proc.stdin.drain()
        while True:
            line = await asyncio.wait_for(self._proc.stdout.readline(), self.timeout)
            if not line:
                raise TransientError("MCP stdio server exited")
            resp = json.loads(line)
            if resp.get("id") == rid:
                return self._result(resp)

    @staticmethod
    def _result(msg):
        if "error" in msg:
            raise PermanentError(f"MCP error {msg['error'].get('code')}: "
                                 f"{msg['error'].get('message')}")
        return msg.get("result")

    async def _rpc(self, method, params):
        async with self._lock:
            if self.transport == "stdio":
                return await self._rpc_stdio(method, params)
            return await self._rpc_http(method, params)

    async def _ensure_init(self):
        if self._init:
            return
        await self._rpc("initialize", {"protocolVersion": "2025-03-26", "capabilities": {},
                                       "clientInfo": {"name": "omnia-runtime", "version": "1.0"}})
        try:
            await self._rpc("notifications/initialized", {})
        except PermanentError:
            pass
        self._init = True

    async def discover(self):
        try:
            await self._ensure_init()
            res = await self._rpc("tools/list", {})
        except Exception as e:  # noqa: BLE001
            log.warning("MCP discovery failed for %s: %s", self.name, e)
            return []
        allow = set(self.tool_filter.get("allowlist") or [])
        block = set(self.tool_filter.get("blocklist") or [])
        out = []
        for t in (res or {}).get("tools", []):
            if (allow and t["name"] not in allow) or t["name"] in block:
                continue
            out.append(ToolDef(name=t["name"], description=t.get("description", ""),
                               input_schema=t.get("inputSchema") or {"type": "object"},
                               handler=self.name, handler_type=self.type, remote_name=t["name"]))
        return out

    async def call(self, tool, args, ctx):
        await self._ensure_init()
        res = await self._rpc("tools/call", {"name": tool.remote_name or tool.name,
                                             "arguments": args})
        res = res or {}
        if res.get("isError"):
            txt = " ".join(c.get("text", "") for c in res.get("content", []))
            raise PermanentError(txt or "MCP tool error")
        if "structuredContent" in res:
            return json.dumps(res["structuredContent"])
        texts = [c.get("text", "") for c in res.get("content", []) if c.get("type") == "text"]
        if len(texts) == 1:
            try:
                json.loads(texts[0])
                return texts[0]
            except json.JSONDecodeError:
                return json.dumps({"result": texts[0]})
        return json.dumps({"content": res.get("content", [])})

    async def close(self):
        if self._proc is not None:
            self._proc.kill()
            await self._proc.wait()


class OpenAPIHandler(HTTPHandler):
    """OpenAPI spec -> one tool per operation (``openapi_adapter.go``)."""

    type = "openapi"

    def __init__(self, entry, secrets_dir=None):
        entry = dict(entry)
        entry.setdefault("httpConfig", {})
        super().__init__(entry, secrets_dir)
        self.ocfg = entry.get("openAPIConfig") or {}
        for k in ("authType", "authToken", "authTokenPath", "authHeader", "authCloud",
                  "authAudience"):  # the spec's auth applies to every operation call
            if k in self.ocfg and k not in self.cfg:
                self.cfg[k] = self.ocfg[k]
        self.ops: dict[str, dict] = {}

    async def _load_spec(self) -> dict:
        src = self.ocfg.get("specURL") or self.ocfg.get("specPath") or self.endpoint
        if self.ocfg.get("spec"):
            return self.ocfg["spec"]
        if src and Path(src).exists():
            t = Path(src).read_text()
            return json.loads(t) if src.endswith(".json") else yaml.safe_load(t)
        import aiohttp

        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout)) as s:
            async with s.get(src) as r:
                t = await r.text()
        try:
            return json.loads(t)
        except json.JSONDecodeError:
            return yaml.safe_load(t)

    async def discover(self):
        try:
            spec = await self._load_spec()
        except Exception as e:  # noqa: BLE001
            log.warning("openapi spec load failed for %s: %s", self.name, e)
            return []
        base = self.ocfg.get("baseURL") or (spec.get("servers") or [{}])[0].get("url", "")
        allow = set(self.ocfg.get("operationFilter") or [])
        out = []
        for path, item in (spec.get("paths") or {}).items():
            for method, op in item.items():
                if method.lower() not in ("get", "post", "put", "patch", "delete"):
                    continue
                oid = op.get("operationId") or f"{method}_{path}".replace("/", "_").strip("_")
                if allow and oid not in allow:
                    continue
                props, req, qp = {}, [], []
                for p in op.get("parameters", []) + item.get("parameters", []):
                    if "$ref" in p:
                        continue
                    props[p["name"]] = p.get("schema", {"type": "string"})
                    if p.get("required"):
                        req.append(p["name"])
                    if p.get("in") == "query":
                        qp.append(p["name"])
                body = (op.get("requestBody") or {}).get("content", {}).get("application/json")
                if body and body.get("schema", {}).get("properties"):
                    props.update(body["schema"]["properties"])
                    req += body["schema"].get("required", [])
                self.ops[oid] = {"method": method.upper(), "url": base.rstrip("/") + path,
                                 "query": qp}
                out.append(ToolDef(name=oid, description=op.get("summary") or
                                   op.get("description", ""),
                                   input_schema={"type": "object", "properties": props,
                                                 "required": req},
                                   handler=self.name, handler_type=self.type, remote_name=oid))
        return out

    async def call(self, tool, args, ctx):
        op = self.ops[tool.remote_name]
        self.cfg = {**self.cfg, "method": op["method"], "urlTemplate": op["url"],
                    "queryParams": op["query"]}
        return await super().call(tool, args, ctx)


class ClientHandler(Handler):
    type = "client"

    async def call(self, tool, args, ctx):
        raise RuntimeError("client tools are fulfilled by the facade, not the runtime")


class InProcessHandler(Handler):
    """Python callables registered as tools (tests, built-in memory tools, A2A bridges)."""

    type = "inprocess"

    def __init__(self, name: str, fns: dict, timeout=None):
        super().__init__({"name": name, "timeout": timeout})
        self.fns = fns  # tool name -> (description, schema, async fn(args, ctx))

    async def discover(self):
        return [ToolDef(name=n, description=d, input_schema=s, handler=self.name,
                        handler_type=self.type, remote_name=n)
                for n, (d, s, _) in self.fns.items()]

    async def call(self, tool, args, ctx):
        fn = self.fns[tool.remote_name][2]
        res = await fn(args, ctx)
        return res if isinstance(res, str) else json.dumps(res)


HANDLERS = {"http": HTTPHandler, "grpc": GRPCHandler, "mcp": MCPHandler,
            "openapi": OpenAPIHandler, "client": ClientHandler}


# ===================================================================== policy broker
class PolicyBrokerClient:
    """POST {url}/v1/decision before every tool call; fail-closed by default
    (``internal/runtime/tools/policy_broker_client.go:71-215``)."""

    def __init__(self, url: str, fail_open: bool = False, timeout_s: float = 2.0):
        self.url = url.rstrip("/")
        self.fail_open = fail_open
        self.timeout_s = timeout_s

    async def decide(self, tool: ToolDef, args: dict, ctx: CallContext) -> dict:
        import aiohttp

        body = {"headers": {"x-omnia-tool-name": tool.name, "x-omnia-tool-registry": tool.handler,
                            **ctx.headers},
                "body": args,
                "identity": {"origin": ctx.origin, "subject": ctx.user_id,
                             "endUser": ctx.user_id, "workspace": ctx.workspace,
                             "agent": ctx.agent, "claims": ctx.claims}}
        t0 = time.perf_counter()
        try:
            async with aiohttp.ClientSession(
                    timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
                async with s.post(self.url + "/v1/decision", json=body) as r:
                    if r.status != 200:
                        raise RuntimeError(f"broker HTTP {r.status}")
                    d = await r.json()
        except Exception as e:  # noqa: BLE001
            M.TOOLPOLICY_DECISIONS.labels("error").inc()
            if self.fail_open:
                return {"allow": True, "injectedHeaders": {}}
            return {"allow": False, "deniedBy": "broker-unavailable",
                    "message": "policy broker unavailable (fail-closed)"}
        finally:
            M.TOOLPOLICY_LATENCY.observe(time.perf_counter() - t0)
        M.TOOLPOLICY_DECISIONS.labels("allow" if d.get("allow") else "deny").inc()
        return d


# ===================================================================== AgentPolicy
class ToolAccess:
    """In-node enforcement of the AgentPolicies selecting this agent
    (compiled by ``operator/policies.compile_tool_access``; the mesh form is the
    Istio AuthorizationPolicies keyed on ``X-Omnia-Tool-Name: registry/tool``).

    Enforcing policies: a denylist match denies; when any allowlist applies, a
    tool must match one of them.  Permissive policies evaluate the same way but
    only record the decision (audit).  Tools outside the agent's ToolRegistry
    (skills, memory tools, workflow tools) are not registry tools and are not
    subject to tool-access rules, as in the reference."""

    def __init__(self, policies: list[dict] | None, registry: str = ""):
        self.policies = list(policies or [])
        self.registry = registry
        self.audit: list[dict] = []

    @staticmethod
    def _decide(policies, key: str):
        allow_lists = [p for p in policies if p["mode"] == "allowlist"]
        for p in policies:
            if p["mode"] == "denylist" and any(key in {f"{r['registry']}/{t}" for t in r["tools"]}
                                               for r in p["rules"]):
                return False, p["policy"]
        if allow_lists and not any(key in {f"{r['registry']}/{t}" for t in r["tools"]}
                                   for p in allow_lists for r in p["rules"]):
            return False, allow_lists[0]["policy"]
        return True, ""

    def check(self, tool: str) -> tuple[bool, str]:
        if not self.policies or not self.registry:
            return True, ""
        key = f"{self.registry}/{tool}"
        ok, by = self._decide([p for p in self.policies if p.get("enforce", True)], key)
        if not ok:
            M.TOOLPOLICY_DECISIONS.labels("deny").inc()
            return False, by
        would, pby = self._decide([p for p in self.policies if not p.get("enforce", True)], key)
        if not would:  # permissive: audit only
            self.audit.append({"tool": key, "policy": pby, "decision": "would-deny"})
            log.info("AgentPolicy %s (permissive) would deny tool %s", pby, key)
        return True, ""


# ===================================================================== executor
class OmniaExecutor:
    def __init__(self, config: dict | None = None, secrets_dir: str | None = None,
                 policy: PolicyBrokerClient | None = None, breaker_threshold: int = 5,
                 breaker_open_s: float = 30.0):
        self.handlers: dict[str, Handler] = {}
        self.tools: dict[str, ToolDef] = {}
        self.breakers: dict[str, CircuitBreaker] = {}
        self.policy = policy
        self.secrets_dir = secrets_dir
        self.breaker_threshold = breaker_threshold
        self.breaker_open_s = breaker_open_s
        for e in (config or {}).get("handlers", []):
            cls = HANDLERS.get(e.get("type", "http"))
            if cls is None:
                log.warning("unknown handler type %s", e.get("type"))
                continue
            self.handlers[e["name"]] = cls(e, secrets_dir)
        self._client_cfg = {e["name"]: e.get("clientConfig") or {}
                            for e in (config or {}).get("handlers", []) if e.get("type") == "client"}
        self.registry_handlers = {e["name"] for e in (config or {}).get("handlers", [])}
        self.access = ToolAccess((config or {}).get("toolAccess"),
                                 (config or {}).get("registry", ""))

    def add_handler(self, h: Handler):
        self.handlers[h.name] = h

    async def discover(self) -> dict[str, ToolDef]:
        for h in self.handlers.values():
            for t in await h.discover():
                if h.type == "client":
                    t.meta.update(self._client_cfg.get(h.name, {}))
                self.tools[t.name] = t
        return self.tools

    def specs(self, names: list[str] | None = None) -> dict[str, dict]:
        return {n: t.spec() for n, t in self.tools.items() if names is None or n in names}

    def is_client_tool(self, name: str) -> bool:
        t = self.tools.get(name)
        return t is not None and t.is_client

    def breaker(self, name: str) -> CircuitBreaker:
        b = self.breakers.get(name)
        if b is None:
            b = self.breakers[name] = CircuitBreaker(self.breaker_threshold, self.breaker_open_s)
        return b

    async def execute(self, name: str, args: dict, ctx: CallContext | None = None) -> tuple[str, bool]:
        """Run a server-side tool.  Returns (result_json, is_error)."""
        ctx = ctx or CallContext()
        tool = self.tools.get(name)
        if tool is None:
            return json.dumps({"error": f"unknown tool {name}"}), True
        h = self.handlers[tool.handler]
        t0 = time.perf_counter()
        status = "ok"
        try:
            if tool.handler in self.registry_handlers:
                ok, by = self.access.check(name)
                if not ok:
                    raise PolicyDenied(f"tool {self.access.registry}/{name} denied by "
                                       f"AgentPolicy {by}")
            if self.policy is not None:
                d = await self.policy.decide(tool, args, ctx)
                if not d.get("allow"):
                    raise PolicyDenied(d.get("message") or f"denied by {d.get('deniedBy')}")
                if d.get("injectedHeaders"):
                    ctx = CallContext(**{**ctx.__dict__,
                                         "headers": {**ctx.headers, **d["injectedHeaders"]}})
            br = self.breaker(name)
            if not br.allow():
                raise CircuitOpen(f"circuit open for tool {name}")
            try:
                failpoints.hit("tool.call")
                res = await asyncio.wait_for(h.call(tool, args, ctx), h.timeout + 1)
            except Exception:
                br.record(False)
                raise
            br.record(True)
            return res, False
        except PolicyDenied as e:
            status = "denied"
            return json.dumps({"error": "policy_denied", "message": str(e)}), True
        except CircuitOpen as e:
            status = "circuit_open"
            return json.dumps({"error": "circuit_open", "message": str(e)}), True
        except asyncio.TimeoutError:
            status = "timeout"
            return json.dumps({"error": "timeout"}), True
        except Exception as e:  # noqa: BLE001
            status = "error"
            return json.dumps({"error": type(e).__name__, "message": str(e)[:500]}), True
        finally:
            M.TOOL_CALLS.labels(name, status).inc()
            M.TOOL_DURATION.labels(name).observe(time.perf_counter() - t0)

    async def close(self):
        for h in self.handlers.values():
            await h.close()
