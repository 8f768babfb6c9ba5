"""A minimal "bring your own" facade (``spec.facades[].type: custom``): the
smallest working third-party facade image, re-derived from the reference
example (``examples/custom-facade/main.go``).  It

1. authenticates its own protocol -- a static bearer-token table maps a token to
   a :class:`Principal` (swap in a real credential check);
2. emits the platform's flat identity contract -- ``x-omnia-user-id``,
   ``x-omnia-user-roles``, ``x-omnia-origin``, ``x-omnia-workspace``,
   ``x-omnia-agent-name`` and one ``x-omnia-claim-<name>`` per claim -- as gRPC
   metadata, so the runtime and the policy broker see the caller;
3. speaks the runtime contract directly: ``RuntimeService/Converse`` against
   ``OMNIA_RUNTIME_ADDRESS``, reading frames until ``done`` / ``error``;
4. serves ``/healthz`` + ``/readyz`` on the operator-probed health port 8081;
5. optionally serves the management-plane twin on 18080 when
   ``OMNIA_MGMT_PLANE_JWKS_URL`` is set: RS256 JWTs verified against the JWKS,
   failing closed on a missing / malformed / expired / unknown-signer token.

Ports: data plane 8080 (``POST /chat`` ``{"session_id", "message"}`` ->
``{"reply"}``), health 8081, mgmt twin 18080 -- ``OMNIA_FACADE_PORT``,
``OMNIA_HEALTH_PORT`` and ``OMNIA_MGMT_PORT`` override them for local runs.

It imports only the public contract pieces (``omnia_amd.api.proto.runtime_v1``
and the JWT verifier); none of the stock facade's server, session or auth chain.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import sys
import time
import uuid
from dataclasses import dataclass, field

from aiohttp import web

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from omnia_amd.api.proto import runtime_v1 as pb  # noqa: E402
from omnia_amd.facade.auth import AuthError, jwt_decode  # noqa: E402

log = logging.getLogger("custom-facade")


@dataclass
class Principal:
    user_id: str
    roles: list = field(default_factory=list)
    workspace: str = ""
    origin: str = "shared-token"
    claims: dict = field(default_factory=dict)

    def outbound_metadata(self, agent: str) -> list[tuple[str, str]]:
        md = [("x-omnia-user-id", self.user_id), ("x-omnia-origin", self.origin)]
        if self.roles:
            md.append(("x-omnia-user-roles", ",".join(self.roles)))
        if self.workspace:
            md.append(("x-omnia-workspace", self.workspace))
        if agent:
            md.append(("x-omnia-agent-name", agent))
        md += [(f"x-omnia-claim-{k.lower()}", str(v)) for k, v in sorted(self.claims.items())]
        return md


DEMO_TOKENS = {"demo-token": Principal("user-42", ["admin", "editor"], "acme", "shared-token",
                                       {"tier": "gold", "team": "finance", "region": "emea"})}


class Authenticator:
    def __init__(self, tokens: dict[str, Principal]):
        self.tokens = tokens

    def authenticate(self, request) -> Principal | None:
        h = request.headers.get("Authorization", "")
        return self.tokens.get(h[7:]) if h.lower().startswith("bearer ") else None


class RuntimeClient:
    """One Converse turn per call over ``RuntimeService``."""

    def __init__(self, address: str, agent: str = ""):
        import grpc

        self.grpc = grpc
        self.agent = agent
        self.channel = grpc.aio.insecure_channel(address)
        self.converse = self.channel.stream_stream(
            pb.METHOD_CONVERSE, request_serializer=pb.ClientMessage.SerializeToString,
            response_deserializer=pb.ServerMessage.FromString)

    async def turn(self, principal: Principal, session_id: str, message: str,
                   timeout: float = 120.0) -> str:
        md = principal.outbound_metadata(self.agent) + [("x-omnia-session-id", session_id)]
        call = self.converse(metadata=md, timeout=timeout)
        await call.write(pb.ClientMessage(session_id=session_id, content=message))
        text = []
        try:
            while True:
                f = await call.read()
                if f is self.grpc.aio.EOF:
                    raise RuntimeError("runtime closed the stream before done")
                kind = f.WhichOneof("message")
                if kind == "chunk":
                    text.append(f.chunk.content)
                elif kind == "done":
                    return f.done.final_content or "".join(text)
                elif kind == "error":
                    raise RuntimeError(f"{f.error.code}: {f.error.message}")
        finally:
            await call.done_writing()
            call.cancel()

    async def close(self):
        await self.channel.close()


class MgmtVerifier:
    """RS256 against a JWKS URL; every failure is a 401 (fail closed)."""

    def __init__(self, jwks_url: str, ttl_s: float = 300.0):
        self.url, self.ttl_s = jwks_url, ttl_s
        self.jwks, self.fetched = None, 0.0

    async def _keys(self, refresh: bool = False):
        import aiohttp

        if refresh or self.jwks is None or time.time() - self.fetched > self.ttl_s:
            async with aiohttp.ClientSession() as s:
                async with s.get(self.url) as r:
                    self.jwks = await r.json()
            self.fetched = time.time()
        return self.jwks

    async def verify(self, request) -> dict:
        h = request.headers.get("Authorization", "")
        if not h.lower().startswith("bearer "):
            raise AuthError("missing bearer token")
        tok = h[7:]
        if tok.count(".") != 2 or json.loads(_b64(tok.split(".")[0])).get("alg") != "RS256":
            raise AuthError("malformed or non-RS256 token")
        try:
            claims = jwt_decode(tok, jwks=await self._keys(), leeway=0)
        except AuthError:  # unknown signer: the JWKS may have rotated -- refetch once
            claims = jwt_decode(tok, jwks=await self._keys(refresh=True), leeway=0)
        if "exp" not in claims:
            raise AuthError("token without exp")
        return claims

    def middleware(self):
        @web.middleware
        async def mw(request, handler):
            try:
                request["mgmt_claims"] = await self.verify(request)
            except (AuthError, ValueError, KeyError) as e:
                return web.json_response({"error": f"unauthorized: {e}"}, status=401)
            return await handler(request)
        return mw


def _b64(s: str) -> bytes:
    import base64

    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def data_plane_app(auth: Authenticator, runtime: RuntimeClient, middlewares=()) -> web.Application:
    async def chat(request):
        p = auth.authenticate(request)
        if p is None and "mgmt_claims" in request:  # the mgmt twin's verified caller
            c = request["mgmt_claims"]
            p = Principal(str(c.get("sub", "")), [str(c.get("role", ""))] if c.get("role")
                          else [], str(c.get("workspace", "")), "management-plane")
        if p is None:
            return web.json_response({"error": "unauthorized"}, status=401)
        try:
            body = await request.json()
        except ValueError:
            return web.json_response({"error": "invalid JSON"}, status=400)
        if not body.get("message"):
            return web.json_response({"error": "message is required"}, status=400)
        sid = body.get("session_id") or str(uuid.uuid4())
        try:
            reply = await runtime.turn(p, sid, body["message"])
        except Exception as e:  # noqa: BLE001
            log.warning("turn failed: %s", e)
            return web.json_response({"error": "runtime error"}, status=502)
        return web.json_response({"reply": reply, "session_id": sid})

    app = web.Application(middlewares=list(middlewares))
    app.router.add_post("/chat", chat)
    return app


def health_app() -> web.Application:
    app = web.Application()
    ok = lambda _: web.Response(text="ok")  # noqa: E731
    app.router.add_get("/healthz", ok)
    app.router.add_get("/readyz", ok)
    return app


async def start(app: web.Application, port: int, host: str = "0.0.0.0"):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


async def main():
    logging.basicConfig(level=logging.INFO)
    env = os.environ
    rc = RuntimeClient(env.get("OMNIA_RUNTIME_ADDRESS", "localhost:9000"),
                       env.get("OMNIA_AGENT_NAME", ""))
    auth = Authenticator(DEMO_TOKENS)
    await start(health_app(), int(env.get("OMNIA_HEALTH_PORT", "8081")))
    await start(data_plane_app(auth, rc), int(env.get("OMNIA_FACADE_PORT", "8080")))
    if env.get("OMNIA_MGMT_PLANE_JWKS_URL"):
        v = MgmtVerifier(env["OMNIA_MGMT_PLANE_JWKS_URL"])
        await start(data_plane_app(auth, rc, [v.middleware()]),
                    int(env.get("OMNIA_MGMT_PORT", "18080")))
        log.info("management-plane twin enabled (jwks=%s)", env["OMNIA_MGMT_PLANE_JWKS_URL"])
    await asyncio.Event().wait()


if __name__ == "__main__":
    asyncio.run(main())
