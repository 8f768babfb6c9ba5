"""Facade process assembly from env (``cmd/agent/main.go:55-155``).

``build_facade(env, runtime_client)`` is shared by the standalone binary
(``python -m omnia_amd.facade``) and the single-node launcher.  Env contract
(set by the operator's deployment builder):

  OMNIA_AGENT_NAME / OMNIA_NAMESPACE / OMNIA_FACADE_PORT / OMNIA_RUNTIME_ADDRESS
  OMNIA_MODE (agent|function), OMNIA_FACADE_TYPES (websocket,rest,a2a,mcp)
  OMNIA_GRACE_WINDOW_SECONDS / OMNIA_ROUTE_REDIS_URL / POD_IP (realtime blip-resume)
  OMNIA_HANDLER_MODE (runtime|echo|demo), OMNIA_INPUT_SCHEMA / OMNIA_OUTPUT_SCHEMA
  OMNIA_A2A_TASK_STORE_URL (redis://...: A2A tasks + state pub/sub across replicas)
  auth: OMNIA_AUTH_SHARED_TOKEN, OMNIA_AUTH_CLIENT_KEYS (json {id: sha256}),
        OMNIA_OIDC_ISSUER / OMNIA_OIDC_AUDIENCE / OMNIA_OIDC_HS256_SECRET /
        OMNIA_OIDC_JWKS_FILE, OMNIA_EDGE_TRUST=true,
        OMNIA_AUTH_ALLOW_ANONYMOUS (default true when no validator is configured)
  management-plane twin (cmd/agent/websocket.go:148-153, mgmt_plane.go:46-71):
        OMNIA_INTERNAL_FACADE_PORT (18080) / OMNIA_INTERNAL_A2A_PORT (19999) /
        OMNIA_INTERNAL_MCP_PORT (19998): the same routes served a second time
        behind a chain holding ONLY the mgmt-plane validator (RS256 JWTs from
        OMNIA_MGMT_PLANE_JWKS_URL, agent / workspace claims checked against
        OMNIA_AGENT_NAME / OMNIA_WORKSPACE_NAME); never anonymous.  The public
        chain never accepts mgmt-plane tokens.
  recording: OMNIA_SESSION_API_URL (+ OMNIA_RECORDING_WORKERS / _QUEUE)
  media: OMNIA_MEDIA_STORAGE=local|s3|gcs|azure (+ OMNIA_MEDIA_ROOT / _BUCKET / ...)
  limits: OMNIA_MAX_CONNECTIONS, OMNIA_MSG_RATE, OMNIA_MSG_BURST, OMNIA_DRAIN_TIMEOUT
"""
from __future__ import annotations

import json
import os

from .auth import (AuthChain, ClientKeyValidator, EdgeTrustValidator, JWKSResolver,
                   MgmtPlaneValidator, OIDCValidator, SharedTokenValidator)
from .server import FacadeConfig, FacadeServer


def auth_from_env(env) -> AuthChain:
    """The public listener's chain: data-plane validators only."""
    vs = []
    if env.get("OMNIA_AUTH_SHARED_TOKEN"):
        vs.append(SharedTokenValidator(env["OMNIA_AUTH_SHARED_TOKEN"]))
    if env.get("OMNIA_AUTH_CLIENT_KEYS"):
        vs.append(ClientKeyValidator(json.loads(env["OMNIA_AUTH_CLIENT_KEYS"])))
    if env.get("OMNIA_OIDC_ISSUER") or env.get("OMNIA_OIDC_HS256_SECRET"):
        jwks = None
        if env.get("OMNIA_OIDC_JWKS_FILE"):
            with open(env["OMNIA_OIDC_JWKS_FILE"]) as f:
                jwks = json.load(f)
        hs = env.get("OMNIA_OIDC_HS256_SECRET")
        vs.append(OIDCValidator(env.get("OMNIA_OIDC_ISSUER"), env.get("OMNIA_OIDC_AUDIENCE"),
                                jwks=jwks, hs_key=hs.encode() if hs else None))
    if env.get("OMNIA_EDGE_TRUST", "").lower() == "true":
        et = json.loads(env.get("OMNIA_EDGE_TRUST_CONFIG", "{}") or "{}")
        hm = et.get("headerMapping") or {}
        peers = env.get("OMNIA_EDGE_TRUST_PEERS", "127.0.0.1,::1")
        vs.append(EdgeTrustValidator(hm.get("subject", ""), hm.get("endUser", ""),
                                     hm.get("email", ""),
                                     claims_from_headers=et.get("claimsFromHeaders") or {},
                                     trusted_peers=[p for p in peers.split(",") if p]
                                     if peers != "*" else None))
    anon = env.get("OMNIA_AUTH_ALLOW_ANONYMOUS", "true" if not vs else "false").lower() == "true"
    return AuthChain(vs, allow_anonymous=anon)


def mgmt_auth_from_env(env, resolver: JWKSResolver | None = None) -> AuthChain:
    """The twin listeners' chain: the mgmt-plane validator alone, strict."""
    url = env.get("OMNIA_MGMT_PLANE_JWKS_URL", "")
    vs = []
    if url or resolver is not None:
        vs.append(MgmtPlaneValidator(resolver or JWKSResolver(url),
                                     expected_agent=env.get("OMNIA_AGENT_NAME", ""),
                                     expected_workspace=env.get("OMNIA_WORKSPACE_NAME", "")))
    return AuthChain(vs, allow_anonymous=False, strict=True)


def internal_ports(env) -> list[int]:
    """Twin listener ports the operator allocated (0 / unset = none)."""
    out = []
    for k in ("OMNIA_INTERNAL_FACADE_PORT", "OMNIA_INTERNAL_A2A_PORT", "OMNIA_INTERNAL_MCP_PORT"):
        try:
            p = int(env.get(k, "") or 0)
        except ValueError:
            p = 0
        if p > 0 and p not in out:
            out.append(p)
    return out


def public_ports(env, port: int) -> list[int]:
    out = [port]
    for k in ("OMNIA_A2A_PORT", "OMNIA_MCP_PORT"):
        try:
            p = int(env.get(k, "") or 0)
        except ValueError:
            p = 0
        if p > 0 and p not in out:
            out.append(p)
    return out


def config_from_env(env) -> FacadeConfig:
    funcs = {}
    if env.get("OMNIA_MODE") == "function":
        funcs["*"] = {"input_schema": json.loads(env.get("OMNIA_INPUT_SCHEMA", "null")),
                      "output_schema": json.loads(env.get("OMNIA_OUTPUT_SCHEMA", "null"))}
    c = FacadeConfig(agent=env.get("OMNIA_AGENT_NAME", "agent"),
                     namespace=env.get("OMNIA_NAMESPACE", "default"),
                     port=int(env.get("OMNIA_FACADE_PORT", 8080)), functions=funcs)
    for k, f, t in (("OMNIA_MAX_CONNECTIONS", "max_connections", int),
                    ("OMNIA_MSG_RATE", "msg_rate", float), ("OMNIA_MSG_BURST", "msg_burst", float),
                    ("OMNIA_DRAIN_TIMEOUT", "drain_timeout_s", float),
                    ("OMNIA_MEDIA_ENABLED", "media_enabled", lambda v: v.lower() == "true")):
        if env.get(k):
            setattr(c, f, t(env[k]))
    try:  # cmd/agent/websocket.go:218-225: positive integer seconds, default 15
        g = int(env.get("OMNIA_GRACE_WINDOW_SECONDS", "") or 0)
    except ValueError:
        g = 0
    if g > 0:
        c.grace_window_s = float(g)
    c.pod_addr = f"{env.get('POD_IP', '')}:{c.port}"
    return c


def build_facade(env, runtime_client, recorder=None, mgmt_resolver=None) -> FacadeServer:
    """The public facade; ``.internal`` is its management-plane twin (or None)."""
    handler = None
    mode = env.get("OMNIA_HANDLER_MODE", "runtime")
    if mode in ("echo", "demo"):
        from .handlers import DemoHandler, EchoHandler

        handler = EchoHandler() if mode == "echo" else DemoHandler()
    cfg = config_from_env(env)
    if recorder is None and env.get("OMNIA_SESSION_API_URL"):
        from ..session.httpclient import RecordingPolicyCache, RecordingPool, SessionHTTPClient

        client = SessionHTTPClient(env["OMNIA_SESSION_API_URL"])
        # recording gate: session-api's effective privacy policy for this agent
        # (GET /api/v1/privacy-policy), cached, fail-open
        policy = RecordingPolicyCache(client.get_privacy_policy, cfg.namespace, cfg.agent,
                                      ttl_s=float(env.get("OMNIA_PRIVACY_POLICY_TTL_S", 60)))
        recorder = RecordingPool(client, workers=int(env.get("OMNIA_RECORDING_WORKERS", 100)),
                                 queue=int(env.get("OMNIA_RECORDING_QUEUE", 1000)),
                                 policy=policy)
    media = None
    if env.get("OMNIA_MEDIA_STORAGE"):
        from ..media import build_media_storage

        media = build_media_storage(env)
    cfg.media_enabled = cfg.media_enabled or media is not None
    from .realtime import route_store_from_env

    routes = route_store_from_env(env)  # OMNIA_ROUTE_REDIS_URL
    types = set(filter(None, env.get("OMNIA_FACADE_TYPES", "").split(",")))

    a2a_store: dict = {}  # one task store for the public listener and its twin

    def make(auth: AuthChain) -> FacadeServer:
        f = FacadeServer(cfg, handler=handler, runtime_client=runtime_client, auth=auth,
                         recorder=recorder, media_store=media, routes=routes)
        if media is not None:
            from ..media import mount_media

            mount_media(f.app, media)
        if "a2a" in types:
            from .a2a import RedisTaskStore, mount_a2a

            store = None
            if env.get("OMNIA_A2A_TASK_STORE_URL"):  # redis://... shared by the replicas
                from ..utils.resp import RedisClient

                store = a2a_store.setdefault("s", RedisTaskStore(
                    RedisClient(env["OMNIA_A2A_TASK_STORE_URL"])))
            mount_a2a(f, runtime_client, task_store=store)
        if "mcp" in types or env.get("OMNIA_MCP_ENABLED", "").lower() == "true":
            from .mcp import mount_mcp

            mount_mcp(f, runtime_client)
        return f

    fac = make(auth_from_env(env))
    fac.internal = make(mgmt_auth_from_env(env, mgmt_resolver)) if internal_ports(env) else None
    return fac


async def dial_runtime(address: str, attempts: int = 30, delay_s: float = 1.0):
    """``runtime_dial.go:47-120``: wait for the runtime's gRPC channel to be ready."""
    import asyncio

    import grpc

    from .runtime_client import GrpcRuntimeClient

    client = GrpcRuntimeClient(address)
    for i in range(attempts):
        try:
            await asyncio.wait_for(client.ch.channel_ready(), timeout=delay_s * 2)
            return client
        except (asyncio.TimeoutError, grpc.aio.AioRpcError):
            await asyncio.sleep(delay_s)
    raise RuntimeError(f"runtime at {address} not reachable after {attempts} attempts")


def env() -> dict:
    return dict(os.environ)


async def start_facade(fac: FacadeServer, env, host: str = "0.0.0.0") -> dict:
    """Bind the public listener(s) and the twin's; returns {name: bound port}."""
    port = int(env.get("OMNIA_FACADE_PORT", 8080))
    bound = {"facade": await fac.start(host, port, extra_ports=public_ports(env, port)[1:])}
    if getattr(fac, "internal", None) is not None:
        ports = internal_ports(env)
        bound["facade-mgmt"] = await fac.internal.start(host, ports[0], extra_ports=ports[1:])
    return bound


async def stop_facade(fac: FacadeServer) -> None:
    await fac.drain()
    if getattr(fac, "internal", None) is not None:
        await fac.internal.drain()
        await fac.internal.stop()
    await fac.stop()
