"""Management-plane twin listeners (``cmd/agent/websocket.go:148-153``,
``cmd/agent/mgmt_plane.go:46-71``, ``pkg/facade/auth/mgmt_plane.go``).

The facade serves its routes a second time on the internal port behind a chain
holding ONLY the mgmt-plane validator: RS256 JWTs minted by the dashboard,
verified against its JWKS (fetched over HTTP from ``OMNIA_MGMT_PLANE_JWKS_URL``),
origin ``management-plane``, agent / workspace claims matched.  The public chain
never accepts those tokens; the twin never accepts client credentials or
anonymous callers."""
import asyncio
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import aiohttp
import pytest

from omnia_amd.facade.app import build_facade, start_facade, stop_facade
from omnia_amd.facade.auth import (AuthError, JWKSResolver, MgmtPlaneValidator, jwk_from_private,
                                   mint_mgmt_token)
from omnia_amd.facade.runtime_client import InProcessRuntimeClient
from omnia_amd.utils.rsa import generate_private_key

from test_runtime import make_service


@pytest.fixture(scope="module")
def keys():
    return {"k1": generate_private_key(1024), "k2": generate_private_key(1024),
            "rogue": generate_private_key(1024)}


class _JWKS:
    """Threaded HTTP JWKS endpoint (the dashboard's /api/auth/jwks) whose key set
    can be rotated; counts fetches."""

    def __init__(self, jwks):
        self.jwks = jwks
        self.fetches = 0
        outer = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                outer.fetches += 1
                body = json.dumps(outer.jwks).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}/api/auth/jwks"
        self.t = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.t.start()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


def _env(jwks_url):
    return {"OMNIA_AGENT_NAME": "agent-a", "OMNIA_NAMESPACE": "ns", "OMNIA_WORKSPACE_NAME": "ws1",
            "OMNIA_AUTH_SHARED_TOKEN": "client-secret", "OMNIA_FACADE_PORT": "0",
            "OMNIA_INTERNAL_FACADE_PORT": "1", "OMNIA_MGMT_PLANE_JWKS_URL": jwks_url,
            "OMNIA_FACADE_TYPES": "websocket,a2a"}


async def _ws_status(url, token=None, query=""):
    hdrs = {"Authorization": f"Bearer {token}"} if token else {}
    async with aiohttp.ClientSession() as s:
        try:
            async with s.ws_connect(url + query, headers=hdrs) as ws:
                hello = await ws.receive_json(timeout=5)
                return 101, hello
        except aiohttp.WSServerHandshakeError as e:
            return e.status, None


def test_dashboard_token_only_on_twin(keys, monkeypatch):
    jw = _JWKS({"keys": [jwk_from_private(keys["k1"], "k1")]})

    async def go():
        svc, _, _ = make_service()
        env = _env(jw.url)
        fac = build_facade(env, InProcessRuntimeClient(svc))
        assert fac.internal is not None
        # bind ephemeral ports instead of 8080/18080
        pub = await fac.start("127.0.0.1", 0)
        mgmt = await fac.internal.start("127.0.0.1", 0)
        pub_ws, mgmt_ws = f"ws://127.0.0.1:{pub}/ws", f"ws://127.0.0.1:{mgmt}/ws"
        tok = mint_mgmt_token(keys["k1"], "k1", "alice@dashboard", agent="agent-a",
                              workspace="ws1")
        try:
            st, hello = await _ws_status(mgmt_ws, tok)
            assert st == 101 and hello["type"] == "connected"
            # the public chain does not know mgmt tokens (no HS256 / mgmt validator there)
            st, _ = await _ws_status(pub_ws, tok)
            assert st == 401
            # a client credential works on the public port, never on the twin
            st, _ = await _ws_status(pub_ws, "client-secret")
            assert st == 101
            st, _ = await _ws_status(mgmt_ws, "client-secret")
            assert st == 401
            st, _ = await _ws_status(mgmt_ws, None, "?token=client-secret")
            assert st == 401
            st, _ = await _ws_status(mgmt_ws)  # anonymous
            assert st == 401
            # wrong agent / workspace / origin / signer / expiry
            for bad in (mint_mgmt_token(keys["k1"], "k1", "x", agent="agent-b"),
                        mint_mgmt_token(keys["k1"], "k1", "x", workspace="ws2"),
                        mint_mgmt_token(keys["k1"], "k1", "x", origin="data-plane"),
                        mint_mgmt_token(keys["rogue"], "k1", "x"),
                        mint_mgmt_token(keys["k1"], "k1", "x", ttl_s=-120),
                        mint_mgmt_token(keys["k1"], "k1", "x", audience="other")):
                st, _ = await _ws_status(mgmt_ws, bad)
                assert st == 401
            # A2A JSON-RPC on the twin needs the mgmt token too; the card stays public
            body = {"jsonrpc": "2.0", "id": 1, "method": "tasks/get", "params": {"id": "nope"}}
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{mgmt}/a2a", json=body) as r:
                    assert r.status == 401
                async with s.post(f"http://127.0.0.1:{mgmt}/a2a", json=body,
                                  headers={"Authorization": f"Bearer {tok}"}) as r:
                    assert r.status == 200
                async with s.get(f"http://127.0.0.1:{mgmt}/.well-known/agent.json") as r:
                    assert r.status == 200
            # key rotation: an unknown kid triggers one JWKS re-fetch
            jw.jwks = {"keys": [jwk_from_private(keys["k1"], "k1"),
                                jwk_from_private(keys["k2"], "k2")]}
            await asyncio.sleep(2.1)  # past the resolver's min refresh interval
            tok2 = mint_mgmt_token(keys["k2"], "k2", "bob", agent="agent-a")
            st, _ = await _ws_status(mgmt_ws, tok2)
            assert st == 101
        finally:
            await stop_facade(fac)

    try:
        asyncio.run(go())
    finally:
        jw.close()
    assert jw.fetches >= 2


def test_twin_without_jwks_rejects_everyone(keys):
    async def go():
        svc, _, _ = make_service()
        env = {"OMNIA_AGENT_NAME": "a", "OMNIA_INTERNAL_FACADE_PORT": "18080"}
        fac = build_facade(env, InProcessRuntimeClient(svc))
        mgmt = await fac.internal.start("127.0.0.1", 0)
        pub = await fac.start("127.0.0.1", 0)
        try:
            st, _ = await _ws_status(f"ws://127.0.0.1:{mgmt}/ws")
            assert st == 401
            st, _ = await _ws_status(f"ws://127.0.0.1:{pub}/ws")  # dev default: anonymous
            assert st == 101
        finally:
            await stop_facade(fac)

    asyncio.run(go())


def test_no_twin_unless_allocated():
    svc, _, _ = make_service()
    fac = build_facade({"OMNIA_AGENT_NAME": "a"}, InProcessRuntimeClient(svc))
    assert fac.internal is None


def test_validator_unit(keys):
    jwks = {"keys": [jwk_from_private(keys["k1"], "k1")]}
    v = MgmtPlaneValidator(JWKSResolver(jwks=jwks), expected_agent="a")
    tok = mint_mgmt_token(keys["k1"], "k1", "sub-1", agent="a", workspace="w")
    ident = v.validate({"Authorization": f"Bearer {tok}"}, {}, "")
    assert ident.origin == "management-plane" and ident.subject == "sub-1"
    assert ident.workspace == "w" and ident.agent == "a"
    md = ident.to_metadata()
    assert md["x-omnia-origin"] == "management-plane"
    assert v.validate({}, {}, "") is None  # no credential: next validator
    with pytest.raises(AuthError):  # HS256 is not a mgmt-plane algorithm
        from omnia_amd.facade.auth import jwt_encode_hs256

        v.validate({"Authorization": "Bearer " + jwt_encode_hs256(
            {"origin": "management-plane", "exp": 2**40}, b"k", kid="k1")}, {}, "")


def test_builder_allocates_twin_ports():
    from omnia_amd.operator import builders as B

    ar = {"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "AgentRuntime",
          "metadata": {"name": "a", "namespace": "ns", "uid": "u"},
          "spec": {"facades": [{"type": "websocket"}, {"type": "a2a"},
                               {"type": "mcp", "managementPlane": False}]}}
    env = B.facade_env(ar, mgmt_jwks_url="http://dash:3000/api/auth/jwks")
    assert env["OMNIA_INTERNAL_FACADE_PORT"] == "18080"
    assert env["OMNIA_INTERNAL_A2A_PORT"] == "19999"
    assert "OMNIA_INTERNAL_MCP_PORT" not in env
    assert env["OMNIA_MGMT_PLANE_JWKS_URL"].endswith("/api/auth/jwks")
    assert B.management_endpoints(ar) == {"ws": 18080, "a2a": 19999}
    names = {p["name"] for p in B.service(ar)["spec"]["ports"]}
    assert {"facade-mgmt", "a2a-mgmt"} <= names and "mcp-mgmt" not in names
    ar["spec"]["facades"][0]["managementPlane"] = False
    assert "OMNIA_INTERNAL_FACADE_PORT" not in B.facade_env(ar, mgmt_jwks_url="")


def test_dashboard_console_proxies_to_twin(keys):
    """Browser -> dashboard WS proxy -> agent twin with a dashboard-minted token;
    the facade verifies it against the dashboard's own JWKS endpoint."""
    from aiohttp import web

    from omnia_amd.operator.dashboard import build_app

    async def go():
        twin = {}

        async def resolver(ns, name):
            return twin.get((ns, name)), "ws1"

        dash = build_app("http://127.0.0.1:1", mgmt_key=keys["k1"], mgmt_kid="dash-1",
                         twin_resolver=resolver, open_console=True)
        runner = web.AppRunner(dash)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        dport = site._server.sockets[0].getsockname()[1]
        svc, _, _ = make_service()
        env = _env(f"http://127.0.0.1:{dport}/api/auth/jwks")
        fac = build_facade(env, InProcessRuntimeClient(svc))
        pub = await fac.start("127.0.0.1", 0)
        mgmt = await fac.internal.start("127.0.0.1", 0)
        twin[("ns", "agent-a")] = f"ws://127.0.0.1:{mgmt}/ws"
        try:
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://127.0.0.1:{dport}/api/auth/jwks") as r:
                    assert (await r.json())["keys"][0]["kid"] == "dash-1"
                async with s.ws_connect(f"http://127.0.0.1:{dport}/api/agents/ns/agent-a/ws") as ws:
                    hello = await ws.receive_json(timeout=10)
                    assert hello["type"] == "connected"
                    await ws.send_json({"type": "message", "content": "hi"})
                    while True:
                        m = await ws.receive_json(timeout=10)
                        if m["type"] in ("done", "error"):
                            break
                    assert m["type"] == "done"
                # an agent without a management endpoint
                async with s.get(f"http://127.0.0.1:{dport}/api/agents/ns/other/ws") as r:
                    assert r.status == 404
            # the dashboard's token is useless on the public listener
            tok = mint_mgmt_token(keys["k1"], "dash-1", "x", agent="agent-a")
            st, _ = await _ws_status(f"ws://127.0.0.1:{pub}/ws", tok)
            assert st == 401
        finally:
            await stop_facade(fac)
            await runner.cleanup()

    asyncio.run(go())


def test_dashboard_kid_is_key_thumbprint_and_facade_refetches_rotated_key(keys):
    """A dashboard restarted with a new ephemeral key publishes a new kid (RFC 7638
    thumbprint), and a facade that cached the old key under a reused kid
    re-fetches once on a signature failure instead of 401-ing until restart."""
    from omnia_amd.facade.auth import (JWKSResolver, MgmtPlaneValidator, jwk_from_private,
                                       jwk_thumbprint, mint_mgmt_token)

    assert jwk_thumbprint(keys["k1"]) != jwk_thumbprint(keys["k2"])
    assert jwk_thumbprint(keys["k1"]) == jwk_thumbprint(keys["k1"])
    served = {"keys": [jwk_from_private(keys["k1"], "same")]}
    calls = []

    def fetch():
        calls.append(1)
        return served

    res = JWKSResolver(url="http://dash/jwks", fetch=fetch, min_refresh_s=0.0)
    v = MgmtPlaneValidator(res)
    tok1 = mint_mgmt_token(keys["k1"], "same", "u")
    assert v.validate({"Authorization": f"Bearer {tok1}"}, {}, None).subject == "u"
    # rotation under the same kid: the cached key fails, one re-fetch fixes it
    served["keys"] = [jwk_from_private(keys["k2"], "same")]
    tok2 = mint_mgmt_token(keys["k2"], "same", "u2")
    assert v.validate({"Authorization": f"Bearer {tok2}"}, {}, None).subject == "u2"
    assert len(calls) == 2
    # a forged token still fails after the re-fetch
    bad = tok2.rsplit(".", 1)[0] + "." + tok1.rsplit(".", 1)[1]
    with pytest.raises(AuthError):
        v.validate({"Authorization": f"Bearer {bad}"}, {}, None)


def test_dashboard_console_refuses_cross_origin_and_unauthenticated(keys):
    """The console mints mgmt tokens only for same-origin callers that are
    authenticated (OIDC ticket) or explicitly opted in (--open-console)."""
    from aiohttp import web

    from omnia_amd.facade.auth import jwk_from_private
    from omnia_amd.operator.dashboard import build_app

    async def resolver(ns, name):
        return None, ""  # no twin: an accepted request answers 404 after the checks

    async def go():
        idp = {"keys": [jwk_from_private(keys["k2"], "idp")]}
        apps = {"closed": build_app("http://127.0.0.1:1", mgmt_key=keys["k1"],
                                    twin_resolver=resolver),
                "open": build_app("http://127.0.0.1:1", mgmt_key=keys["k1"],
                                  twin_resolver=resolver, open_console=True),
                "oidc": build_app("http://127.0.0.1:1", mgmt_key=keys["k1"],
                                  twin_resolver=resolver, oidc={"jwks": idp})}
        runners, ports = [], {}
        for k, a in apps.items():
            r = web.AppRunner(a)
            await r.setup()
            site = web.TCPSite(r, "127.0.0.1", 0)
            await site.start()
            runners.append(r)
            ports[k] = site._server.sockets[0].getsockname()[1]
        try:
            async with aiohttp.ClientSession() as s:
                u = "http://127.0.0.1:{}/api/agents/ns/a/ws"
                async with s.get(u.format(ports["closed"])) as r:
                    assert r.status == 403
                async with s.get(u.format(ports["open"]),
                                 headers={"Origin": "https://evil.example"}) as r:
                    assert r.status == 403
                async with s.get(u.format(ports["open"]),
                                 headers={"Origin": f"http://127.0.0.1:{ports['open']}"}) as r:
                    assert r.status == 404  # passed the guards, no twin
                async with s.get(u.format(ports["oidc"])) as r:
                    assert r.status == 401  # no bearer, no ticket
                async with s.get(u.format(ports["oidc"]) + "?ticket=forged") as r:
                    assert r.status == 401
                idtok = _idp_token(keys["k2"], "idp")
                async with s.post(u.format(ports["oidc"]) + "-ticket",
                                  headers={"Authorization": f"Bearer {idtok}"}) as r:
                    assert r.status == 200
                    t = (await r.json())["ticket"]
                # a ticket is bound to its agent and is single-use
                async with s.get("http://127.0.0.1:{}/api/agents/ns/b/ws?ticket={}".format(
                        ports["oidc"], t)) as r:
                    assert r.status == 401
                async with s.post(u.format(ports["oidc"]) + "-ticket",
                                  headers={"Authorization": f"Bearer {idtok}"}) as r:
                    t = (await r.json())["ticket"]
                async with s.get(u.format(ports["oidc"]) + f"?ticket={t}") as r:
                    assert r.status == 404  # authenticated; no twin
                async with s.get(u.format(ports["oidc"]) + f"?ticket={t}") as r:
                    assert r.status == 401  # used up
        finally:
            for r in runners:
                await r.cleanup()

    asyncio.run(go())


def _idp_token(key, kid):
    import json as _json
    import time as _time

    from omnia_amd.facade.auth import _b64url_enc
    from omnia_amd.utils.rsa import sign_pkcs1_sha256

    hdr = _b64url_enc(_json.dumps({"alg": "RS256", "kid": kid}).encode())
    body = _b64url_enc(_json.dumps({"sub": "alice", "exp": int(_time.time()) + 60}).encode())
    sig = sign_pkcs1_sha256(key, f"{hdr}.{body}".encode())
    return f"{hdr}.{body}.{_b64url_enc(sig)}"
