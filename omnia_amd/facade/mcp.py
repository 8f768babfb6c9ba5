"""MCP server facade: function-mode agents exposed as MCP tools over
Streamable HTTP (``internal/facade/mcp/server.go:62-109``,
``tool_adapter.go:55-133``).  ``tools/list`` advertises the function with its
input schema; ``tools/call`` runs the same invoker as ``POST /functions/{name}``
(input schema -> Invoke -> output schema) and returns text + structuredContent.
"""
from __future__ import annotations

import json
import uuid

from aiohttp import web

from ..api.proto import runtime_v1 as pb
from ..observability import metrics as M
from ..utils import jsonschema

PROTOCOL_VERSION = "2025-03-26"


class MCPServer:
    def __init__(self, runtime_client, name: str, functions: dict, description: str = ""):
        self.client = runtime_client
        self.name = name
        self.functions = functions or {}
        self.description = description or f"Omnia function {name}"
        self.sessions: set = set()

    def _tools(self):
        spec = self.functions.get("*") or self.functions.get(self.name) or {}
        t = {"name": self.name, "description": self.description,
             "inputSchema": spec.get("input_schema") or {"type": "object"}}
        if spec.get("output_schema"):
            t["outputSchema"] = spec["output_schema"]
        return [t]

    async def handle(self, request):
        try:
            req = await request.json()
        except Exception:  # noqa: BLE001
            return web.json_response({"jsonrpc": "2.0", "id": None,
                                      "error": {"code": -32700, "message": "parse error"}})
        if not isinstance(req, dict):
            return web.json_response({"jsonrpc": "2.0", "id": None,
                                      "error": {"code": -32600, "message": "invalid request"}})
        method, rid, params = req.get("method"), req.get("id"), req.get("params") or {}
        if rid is None:  # notification
            return web.Response(status=202)
        if not isinstance(method, str):
            method = None

        def ok(result, headers=None):
            M.MCP_REQUESTS.labels(method or "?", "ok").inc()
            return web.json_response({"jsonrpc": "2.0", "id": rid, "result": result},
                                     headers=headers)

        def err(code, msg):
            M.MCP_REQUESTS.labels(method or "?", "error").inc()
            return web.json_response({"jsonrpc": "2.0", "id": rid,
                                      "error": {"code": code, "message": msg}})

        if method == "initialize":
            sid = uuid.uuid4().hex
            self.sessions.add(sid)
            return ok({"protocolVersion": PROTOCOL_VERSION,
                       "capabilities": {"tools": {"listChanged": False}},
                       "serverInfo": {"name": f"omnia-{self.name}", "version": "1.0.0"}},
                      headers={"Mcp-Session-Id": sid})
        if method == "ping":
            return ok({})
        if method == "tools/list":
            return ok({"tools": self._tools()})
        if method == "tools/call":
            if not isinstance(params, dict) or not isinstance(params.get("arguments") or {},
                                                              dict):
                return err(-32602, "params must be an object with object arguments")
            if params.get("name") != self.name:
                return err(-32602, f"unknown tool {params.get('name')}")
            args = params.get("arguments") or {}
            spec = self.functions.get("*") or self.functions.get(self.name) or {}
            if spec.get("input_schema"):
                errs = jsonschema.Validator(spec["input_schema"]).errors(args)
                if errs:
                    return ok({"isError": True, "content": [
                        {"type": "text", "text": "input_invalid: " + "; ".join(
                            str(e) for e in errs[:5])}]})
            try:
                resp = await self.client.invoke(pb.InvocationRequest(
                    input_json=json.dumps(args), invocation_id=str(uuid.uuid4())),
                    metadata={"x-omnia-origin": "mcp"}, timeout=120)
            except Exception:  # noqa: BLE001
                return ok({"isError": True, "content": [{"type": "text",
                                                         "text": "runtime_error"}]})
            out = resp.output_json
            result = {"content": [{"type": "text", "text": out}], "isError": False}
            try:
                parsed = json.loads(out)
                if spec.get("output_schema") is not None:
                    errs = jsonschema.Validator(spec["output_schema"]).errors(parsed)
                    if errs:
                        return ok({"isError": True, "content": [
                            {"type": "text", "text": "output_invalid: " + out}]})
                if isinstance(parsed, dict):
                    result["structuredContent"] = parsed
            except json.JSONDecodeError:
                if spec.get("output_schema") is not None:
                    return ok({"isError": True, "content": [
                        {"type": "text", "text": "output_invalid: " + out}]})
            return ok(result)
        return err(-32601, f"method {method} not found")


def mount_mcp(facade, runtime_client, path: str = "/mcp") -> MCPServer:
    srv = MCPServer(runtime_client, facade.cfg.agent, facade.cfg.functions)
    facade.app.router.add_post(path, srv.handle)
    return srv
