"""examples/custom-facade: a third-party facade that authenticates its own
protocol, emits the x-omnia-* identity contract as gRPC metadata, speaks
RuntimeService/Converse directly (to a capturing fake runtime and to the stock
runtime), and serves a fail-closed RS256 management-plane twin."""
import asyncio
import base64
import json
import os
import sys
import time

import aiohttp
from aiohttp import web

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "custom-facade"))
import facade as cf  # noqa: E402

from omnia_amd.api.proto import runtime_v1 as pb  # noqa: E402


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _rs256(key, claims: dict, kid: str = "k1") -> str:
    from omnia_amd.utils.rsa import sign_pkcs1_sha256

    h = _b64(json.dumps({"alg": "RS256", "typ": "JWT", "kid": kid}).encode())
    p = _b64(json.dumps(claims).encode())
    return f"{h}.{p}.{_b64(sign_pkcs1_sha256(key, f'{h}.{p}'.encode()))}"


def _jwk(key, kid="k1"):
    n = key.n.to_bytes((key.n.bit_length() + 7) // 8, "big")
    e = key.e.to_bytes((key.e.bit_length() + 7) // 8, "big")
    return {"kty": "RSA", "kid": kid, "alg": "RS256", "n": _b64(n), "e": _b64(e)}


async def _fake_runtime(seen: list):
    import grpc

    async def converse(it, context):
        seen.append(dict(context.invocation_metadata()))
        yield pb.ServerMessage(runtime_hello=pb.RuntimeHello(capabilities=[]))
        async for m in it:
            yield pb.ServerMessage(chunk=pb.Chunk(content="echo: "))
            yield pb.ServerMessage(done=pb.Done(final_content="echo: " + m.content))

    h = grpc.method_handlers_generic_handler(pb.SERVICE, {
        "Converse": grpc.stream_stream_rpc_method_handler(
            converse, request_deserializer=pb.ClientMessage.FromString,
            response_serializer=pb.ServerMessage.SerializeToString)})
    server = grpc.aio.server()
    server.add_generic_rpc_handlers((h,))
    port = server.add_insecure_port("127.0.0.1:0")
    await server.start()
    return server, port


def test_custom_facade_identity_contract_and_health():
    async def go():
        seen = []
        server, rport = await _fake_runtime(seen)
        rc = cf.RuntimeClient(f"127.0.0.1:{rport}", "agent-x")
        r1, dport = await cf.start(cf.data_plane_app(cf.Authenticator(cf.DEMO_TOKENS), rc),
                                   0, "127.0.0.1")
        r2, hport = await cf.start(cf.health_app(), 0, "127.0.0.1")
        try:
            async with aiohttp.ClientSession() as s:
                ok = await s.post(f"http://127.0.0.1:{dport}/chat",
                                  headers={"Authorization": "Bearer demo-token"},
                                  json={"session_id": "s1", "message": "hi"})
                okb = await ok.json()
                bad = await s.post(f"http://127.0.0.1:{dport}/chat",
                                   headers={"Authorization": "Bearer nope"},
                                   json={"message": "hi"})
                empty = await s.post(f"http://127.0.0.1:{dport}/chat",
                                     headers={"Authorization": "Bearer demo-token"}, json={})
                hz = (await s.get(f"http://127.0.0.1:{hport}/healthz")).status
                rz = (await s.get(f"http://127.0.0.1:{hport}/readyz")).status
            return ok.status, okb, bad.status, empty.status, hz, rz, seen
        finally:
            await rc.close()
            await r1.cleanup()
            await r2.cleanup()
            await server.stop(0)

    st, body, bad, empty, hz, rz, seen = asyncio.run(go())
    assert st == 200 and body == {"reply": "echo: hi", "session_id": "s1"}
    assert bad == 401 and empty == 400 and hz == rz == 200
    md = seen[0]
    assert md["x-omnia-user-id"] == "user-42" and md["x-omnia-user-roles"] == "admin,editor"
    assert md["x-omnia-workspace"] == "acme" and md["x-omnia-origin"] == "shared-token"
    assert md["x-omnia-agent-name"] == "agent-x" and md["x-omnia-session-id"] == "s1"
    assert (md["x-omnia-claim-tier"], md["x-omnia-claim-team"],
            md["x-omnia-claim-region"]) == ("gold", "finance", "emea")
    assert not any(k.lower() == "authorization" for k in md)  # never the bearer


def test_custom_facade_mgmt_twin_fails_closed():
    from omnia_amd.facade.auth import jwt_encode_hs256
    from omnia_amd.utils.rsa import generate_private_key

    key, other = generate_private_key(1024), generate_private_key(1024)

    async def go():
        seen = []
        server, rport = await _fake_runtime(seen)
        jw = web.Application()
        jw.router.add_get("/jwks", lambda _: web.json_response({"keys": [_jwk(key)]}))
        rj, jport = await cf.start(jw, 0, "127.0.0.1")
        rc = cf.RuntimeClient(f"127.0.0.1:{rport}", "agent-x")
        v = cf.MgmtVerifier(f"http://127.0.0.1:{jport}/jwks")
        rm, mport = await cf.start(cf.data_plane_app(cf.Authenticator({}), rc, [v.middleware()]),
                                   0, "127.0.0.1")
        now = int(time.time())
        good = _rs256(key, {"sub": "dash-admin", "role": "admin", "workspace": "acme",
                            "exp": now + 300})
        cases = {"good": good,
                 "expired": _rs256(key, {"sub": "x", "exp": now - 10}),
                 "no_exp": _rs256(key, {"sub": "x"}),
                 "unknown_signer": _rs256(other, {"sub": "x", "exp": now + 300}),
                 "malformed": "not.a.jwt",
                 "hs256": jwt_encode_hs256({"sub": "x", "exp": now + 300}, b"k"),
                 "missing": None}
        out = {}
        try:
            async with aiohttp.ClientSession() as s:
                for name, tok in cases.items():
                    h = {"Authorization": f"Bearer {tok}"} if tok else {}
                    r = await s.post(f"http://127.0.0.1:{mport}/chat", headers=h,
                                     json={"message": "ping"})
                    out[name] = r.status
            return out, seen
        finally:
            await rc.close()
            for r in (rm, rj):
                await r.cleanup()
            await server.stop(0)

    out, seen = asyncio.run(go())
    assert out["good"] == 200, out
    assert all(v == 401 for k, v in out.items() if k != "good"), out
    assert len(seen) == 1 and seen[0]["x-omnia-origin"] == "management-plane"
    assert seen[0]["x-omnia-user-id"] == "dash-admin"


def test_custom_facade_against_stock_runtime():
    from omnia_amd.runtime.app import build_runtime
    from omnia_amd.runtime.config import RuntimeConfig
    from omnia_amd.runtime.server import serve_grpc

    async def go():
        svc = await build_runtime(RuntimeConfig(provider={"type": "mock"}))
        server, rport = await serve_grpc(svc, 0, "127.0.0.1")
        rc = cf.RuntimeClient(f"127.0.0.1:{rport}", "stock")
        try:
            return await rc.turn(cf.DEMO_TOKENS["demo-token"], "s-stock", "hello")
        finally:
            await rc.close()
            await server.stop(0)

    assert asyncio.run(go())
