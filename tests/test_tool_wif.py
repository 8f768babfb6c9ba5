"""``workloadIdentity`` tool auth (verdict r5 item 7; reference
``internal/runtime/tools/auth.go:26-50``, ``azure_token.go``): the projected
federated token is exchanged at a (fake) Entra ID token endpoint, the bearer
token reaches the tool over HTTP headers, gRPC metadata and MCP headers, tokens
are cached per audience until 5 minutes before expiry, and unsupported clouds /
missing identity fail the call loudly."""
import asyncio

import pytest
from aiohttp import web

from omnia_amd.tools.executor import OmniaExecutor
from omnia_amd.tools.workload_identity import (AzureTokenAcquirer, WorkloadIdentityError,
                                               resolve_header)
from tool_fakes import GRPCToolFake, HTTPToolFake, MCPToolFake


class _TokenEndpoint:
    """Entra ID v2 token endpoint stand-in: checks the client-assertion grant."""

    def __init__(self, tenant="tid", client="cid"):
        self.tenant, self.client = tenant, client
        self.forms = []
        self.runner = None
        self.url = ""

    async def start(self):
        async def token(request):
            form = dict(await request.post())
            self.forms.append(form)
            if request.match_info["tenant"] != self.tenant or form.get("client_id") != self.client:
                return web.json_response({"error": "invalid_client"}, status=401)
            if form.get("client_assertion_type") != \
                    "urn:ietf:params:oauth:client-assertion-type:jwt-bearer":
                return web.json_response({"error": "invalid_request"}, status=400)
            n = len(self.forms)
            return web.json_response({"access_token": f"tok{n}:{form['scope']}:"
                                                      f"{form['client_assertion']}",
                                      "expires_in": 3600, "token_type": "Bearer"})

        app = web.Application()
        app.router.add_post("/{tenant}/oauth2/v2.0/token", token)
        self.runner = web.AppRunner(app)
        await self.runner.setup()
        site = web.TCPSite(self.runner, "127.0.0.1", 0)
        await site.start()
        self.url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}/"
        return self

    async def stop(self):
        await self.runner.cleanup()


def _env(tmp_path, url, token="fed-1"):
    f = tmp_path / "azure-identity-token"
    f.write_text(token)
    return {"AZURE_TENANT_ID": "tid", "AZURE_CLIENT_ID": "cid",
            "AZURE_FEDERATED_TOKEN_FILE": str(f), "AZURE_AUTHORITY_HOST": url}, f


def test_exchange_cache_and_rotation(tmp_path):
    async def go():
        ep = await _TokenEndpoint().start()
        t = [1000.0]
        env, f = _env(tmp_path, ep.url)
        acq = AzureTokenAcquirer(env, now=lambda: t[0])
        try:
            a = await acq.token("api://tools")
            b = await acq.token("api://tools")  # cached
            c = await acq.token("https://other")  # per audience
            t[0] += 3600 - 299  # inside the 5-minute refresh margin
            f.write_text("fed-2")  # the kubelet rotated the projected token
            d = await acq.token("api://tools")
            return a, b, c, d, ep.forms
        finally:
            await ep.stop()

    a, b, c, d, forms = asyncio.run(go())
    assert a == b == "tok1:api://tools/.default:fed-1"
    assert c.startswith("tok2:https://other/.default")
    assert d == "tok3:api://tools/.default:fed-2"
    assert len(forms) == 3 and forms[0]["grant_type"] == "client_credentials"


def test_fail_loud():
    async def go():
        with pytest.raises(WorkloadIdentityError, match="not supported"):
            await resolve_header(AzureTokenAcquirer({}), {"cloud": "gcp", "audience": "x"})
        with pytest.raises(WorkloadIdentityError, match="no token acquirer"):
            await resolve_header(None, {"cloud": "azure", "audience": "x"})
        with pytest.raises(WorkloadIdentityError, match="AZURE_TENANT_ID"):
            await AzureTokenAcquirer({}).token("api://x")
    asyncio.run(go())


def test_token_endpoint_rejection_is_an_error(tmp_path):
    async def go():
        ep = await _TokenEndpoint(client="someone-else").start()
        env, _ = _env(tmp_path, ep.url)
        try:
            with pytest.raises(WorkloadIdentityError, match="HTTP 401"):
                await AzureTokenAcquirer(env).token("api://x")
        finally:
            await ep.stop()
    asyncio.run(go())


def _wif(aud, header=None):
    return {"type": "workloadIdentity",
            "workloadIdentity": {"cloud": "azure", "audience": aud,
                                 **({"header": header} if header else {})}}


def test_token_reaches_http_grpc_and_mcp_tools(tmp_path):
    async def go():
        ep = await _TokenEndpoint().start()
        http = await HTTPToolFake().start()
        grpc_ = await GRPCToolFake([{"name": "clock", "parameters": {"type": "object"}}]).start()
        mcp = await MCPToolFake([{"name": "kb", "parameters": {"type": "object"}}]).start()
        env, _ = _env(tmp_path, ep.url)
        acq = AzureTokenAcquirer(env)
        cfg = {"handlers": [
            {"name": "weather", "type": "http", "auth": _wif("api://weather"),
             "httpConfig": {"endpoint": f"http://127.0.0.1:{http.port}/"},
             "tool": {"name": "weather", "description": "w", "inputSchema": {"type": "object"}}},
            {"name": "clocksvc", "type": "grpc", "auth": _wif("api://clock", "x-api-token"),
             "grpcConfig": {"endpoint": f"127.0.0.1:{grpc_.port}"}},
            {"name": "kbsvc", "type": "mcp",
             "mcpConfig": {"transport": "streamable-http",
                           "endpoint": f"http://127.0.0.1:{mcp.port}/mcp",
                           "authType": "workloadIdentity", "authCloud": "azure",
                           "authAudience": "api://kb"}},
        ]}
        ex = OmniaExecutor(cfg)
        for h in ex.handlers.values():
            h.token_acquirer = acq
        try:
            await ex.discover()
            r1 = await ex.execute("weather", {"city": "Oslo"})
            r2 = await ex.execute("clock", {})
            r3 = await ex.execute("kb", {"q": "x"})
            return (r1, r2, r3, http.headers, grpc_.metadata, mcp.headers, ep.forms)
        finally:
            for x in (http, grpc_, mcp, ep):
                await x.stop()

    r1, r2, r3, hh, gm, mh, forms = asyncio.run(go())
    assert not r1[1] and not r2[1] and not r3[1], (r1, r2, r3)
    assert hh[-1]["Authorization"].startswith("Bearer tok") and "api://weather" in \
        hh[-1]["Authorization"]
    assert gm[-1]["x-api-token"].startswith("Bearer tok") and "api://clock" in gm[-1]["x-api-token"]
    assert mh[-1]["Authorization"].startswith("Bearer tok") and "api://kb" in mh[-1]["Authorization"]
    # one exchange per audience, however many MCP round trips
    assert sorted(f["scope"] for f in forms) == ["api://clock/.default", "api://kb/.default",
                                                 "api://weather/.default"]


def test_unsupported_cloud_fails_the_call():
    async def go():
        http = await HTTPToolFake().start()
        ex = OmniaExecutor({"handlers": [
            {"name": "w", "type": "http",
             "auth": {"type": "workloadIdentity",
                      "workloadIdentity": {"cloud": "aws", "audience": "x"}},
             "httpConfig": {"endpoint": f"http://127.0.0.1:{http.port}/"},
             "tool": {"name": "w", "description": "w", "inputSchema": {"type": "object"}}}]})
        try:
            await ex.discover()
            return await ex.execute("w", {}), http.calls
        finally:
            await http.stop()

    (res, err), calls = asyncio.run(go())
    assert err and "not supported" in res and calls == []  # never sent unauthenticated


def test_operator_rejects_wif_on_stdio_and_client_handlers():
    from omnia_amd.operator.controllers import ToolRegistryReconciler

    v = ToolRegistryReconciler.validate_handler
    assert v({"name": "a", "type": "mcp", "auth": _wif("x"),
              "mcpConfig": {"transport": "stdio", "command": "srv"}})
    assert v({"name": "b", "type": "client", "auth": _wif("x"),
              "tool": {"name": "b", "description": "", "inputSchema": {}}})
    assert v({"name": "c", "type": "http", "auth": _wif("x"),
              "httpConfig": {"endpoint": "http://x"},
              "tool": {"name": "c", "description": "", "inputSchema": {}}}) is None
