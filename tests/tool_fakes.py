"""In-process fakes of the three remote tool transports the runtime's executor
speaks: a plain HTTP tool endpoint, an ``omnia.tools.v1.ToolService`` gRPC
server and an MCP streamable-http server (JSON-RPC).  Each records the calls it
served so tests can assert which adapter a tool call travelled through."""
from __future__ import annotations

import json

from aiohttp import web


class HTTPToolFake:
    """POST / with the arguments JSON -> {"weather": ...}."""

    def __init__(self):
        self.calls = []
        self.headers = []
        self.runner = None
        self.port = None

    async def start(self):
        async def handle(request):
            args = await request.json()
            self.calls.append(args)
            self.headers.append(dict(request.headers))
            return web.json_response({"weather": "sunny", "echo": args})

        app = web.Application()
        app.router.add_post("/", handle)
        self.runner = web.AppRunner(app)
        await self.runner.setup()
        site = web.TCPSite(self.runner, "127.0.0.1", 0)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        await self.runner.cleanup()


class GRPCToolFake:
    """omnia.tools.v1.ToolService: ListTools + Execute."""

    def __init__(self, tools: list[dict]):
        self.tools = tools
        self.calls = []
        self.metadata = []
        self.server = None
        self.port = None

    async def start(self):
        import grpc

        from omnia_amd.api.proto import tools_v1 as T

        async def list_tools(req, ctx):
            return T.ListToolsResponse(tools=[T.ToolInfo(name=t["name"],
                                                         description=t.get("description", ""),
                                                         input_schema=json.dumps(t["parameters"]))
                                              for t in self.tools])

        async def execute(req, ctx):
            self.calls.append((req.tool_name, json.loads(req.arguments_json or "{}")))
            self.metadata.append(dict(ctx.invocation_metadata() or ()))
            return T.ToolResponse(result_json=json.dumps({"time": "12:00", "tool": req.tool_name}))

        svc = T.SERVICE
        handlers = {
            T.METHOD_LIST_TOOLS.rsplit("/", 1)[-1]: grpc.unary_unary_rpc_method_handler(
                list_tools, request_deserializer=T.ListToolsRequest.FromString,
                response_serializer=T.ListToolsResponse.SerializeToString),
            T.METHOD_EXECUTE.rsplit("/", 1)[-1]: grpc.unary_unary_rpc_method_handler(
                execute, request_deserializer=T.ToolRequest.FromString,
                response_serializer=T.ToolResponse.SerializeToString),
        }
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(svc,
                                                                                  handlers),))
        self.port = self.server.add_insecure_port("127.0.0.1:0")
        await self.server.start()
        return self

    async def stop(self):
        await self.server.stop(0)


class MCPToolFake:
    """MCP streamable-http: initialize, tools/list, tools/call (JSON responses)."""

    def __init__(self, tools: list[dict]):
        self.tools = tools
        self.calls = []
        self.headers = []
        self.runner = None
        self.port = None

    async def start(self):
        async def handle(request):
            body = await request.json()
            self.headers.append(dict(request.headers))
            m = body.get("method")
            rid = body.get("id")
            if m == "initialize":
                res = {"protocolVersion": "2025-03-26", "capabilities": {"tools": {}},
                       "serverInfo": {"name": "fake-mcp", "version": "1"}}
            elif m == "tools/list":
                res = {"tools": [{"name": t["name"], "description": t.get("description", ""),
                                  "inputSchema": t["parameters"]} for t in self.tools]}
            elif m == "tools/call":
                p = body.get("params") or {}
                self.calls.append((p.get("name"), p.get("arguments")))
                res = {"content": [{"type": "text",
                                    "text": json.dumps({"found": True, "q": p.get("arguments")})}]}
            elif rid is None:  # notification
                return web.Response(status=202)
            else:
                return web.json_response({"jsonrpc": "2.0", "id": rid,
                                          "error": {"code": -32601, "message": "no method"}})
            return web.json_response({"jsonrpc": "2.0", "id": rid, "result": res},
                                     headers={"Mcp-Session-Id": "s1"})

        app = web.Application()
        app.router.add_post("/mcp", handle)
        self.runner = web.AppRunner(app)
        await self.runner.setup()
        site = web.TCPSite(self.runner, "127.0.0.1", 0)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        await self.runner.cleanup()
