"""Policy broker sidecar (``ee/cmd/policy-broker``, ``ee/pkg/policy``).

``POST /v1/decision`` with ``{"headers": {...}, "body": {...}, "identity": {...}}``
evaluates every ToolPolicy whose selector matches the call's
``x-omnia-tool-registry`` / ``x-omnia-tool-name``:

1. required claims: each ``x-omnia-claim-<claim>`` header must be present;
2. rules in order: a rule's CEL ``deny`` expression over ``headers``, ``body``,
   ``identity`` returning true denies; evaluation errors follow ``onFailure``
   (``deny`` = fail closed, the default; ``allow``);
3. ``mode: audit`` turns a deny into ``allow`` + ``wouldDeny`` (logged);
4. on allow, header injection: static ``value`` or CEL-computed value per header.

Decisions are cached per (policy generation, call) nowhere: CEL is compiled once
per policy version (``utils.cel``), evaluation is microseconds.  Policies come
from the API server (list + poll watcher, ``ee/pkg/policy/watcher.go``) or a file.

``python -m omnia_amd.ee.policy_broker --port 8090 --policies policies.yaml``
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import time
from dataclasses import dataclass, field

from aiohttp import web

from ..observability import metrics as M
from ..utils import cel
from ..observability.logging import configure as configure_logging

log = logging.getLogger("omnia.policy_broker")

HEADER_TOOL_NAME = "x-omnia-tool-name"
HEADER_TOOL_REGISTRY = "x-omnia-tool-registry"
HEADER_CLAIM_PREFIX = "x-omnia-claim-"
MAX_REQUEST_BYTES = 1 << 20


@dataclass
class Decision:
    allowed: bool = True
    denied_by: str = ""
    message: str = ""
    mode: str = "enforce"
    would_deny: bool = False
    policy: str = ""
    error: str = ""

    def to_json(self, injected=None) -> dict:
        d = {"allow": self.allowed, "deniedBy": self.denied_by, "message": self.message,
             "mode": self.mode, "wouldDeny": self.would_deny}
        if injected:
            d["injectedHeaders"] = injected
        return d


@dataclass
class CompiledPolicy:
    name: str
    namespace: str
    registry: str
    tools: list
    rules: list  # (name, program, message)
    required_claims: list  # (claim, message)
    injections: list  # (header, static value | None, program | None)
    mode: str = "enforce"
    on_failure: str = "deny"
    generation: int = 0


def compile_policy(obj: dict) -> CompiledPolicy:
    """ToolPolicy object (CRD shape) -> compiled policy; raises on bad CEL."""
    md, spec = obj.get("metadata", {}), obj.get("spec", {})
    sel = spec.get("selector") or {}
    rules = []
    for r in spec.get("rules") or []:
        deny = r.get("deny") or {}
        rules.append((r.get("name", ""), cel.compile(deny.get("cel", "false")),
                      deny.get("message", "")))
    inj = []
    for h in spec.get("headerInjection") or []:
        has_v, has_c = bool(h.get("value")), bool(h.get("cel"))
        if has_v == has_c:
            raise ValueError(f"header {h.get('header')!r}: exactly one of value / cel")
        inj.append((h["header"], h.get("value") if has_v else None,
                    cel.compile(h["cel"]) if has_c else None))
    return CompiledPolicy(
        name=md.get("name", ""), namespace=md.get("namespace", "default"),
        registry=sel.get("registry", ""), tools=list(sel.get("tools") or []), rules=rules,
        required_claims=[(c["claim"], c.get("message", "")) for c in
                         spec.get("requiredClaims") or []],
        injections=inj, mode=(spec.get("mode") or "enforce").lower(),
        on_failure=(spec.get("onFailure") or "deny").lower(),
        generation=int(md.get("generation") or 0))


def _identity(payload: dict | None) -> dict:
    p = payload or {}
    return {"origin": p.get("origin", ""), "subject": p.get("subject", ""),
            "endUser": p.get("endUser", ""), "workspace": p.get("workspace", ""),
            "agent": p.get("agent", ""), "claims": dict(p.get("claims") or {})}


class Evaluator:
    def __init__(self):
        self.policies: dict[str, CompiledPolicy] = {}

    def set_policy(self, obj: dict) -> CompiledPolicy:
        p = compile_policy(obj)
        self.policies[f"{p.namespace}/{p.name}"] = p
        return p

    def remove_policy(self, namespace: str, name: str):
        self.policies.pop(f"{namespace}/{name}", None)

    def matching(self, headers: dict) -> list[CompiledPolicy]:
        tool, reg = headers.get(HEADER_TOOL_NAME, ""), headers.get(HEADER_TOOL_REGISTRY, "")
        return [p for _, p in sorted(self.policies.items())
                if p.registry == reg and (not p.tools or tool in p.tools)]

    @staticmethod
    def _apply_mode(p: CompiledPolicy, d: Decision) -> Decision:
        d.mode, d.policy = p.mode, p.name
        if p.mode == "audit" and not d.allowed:
            d.allowed, d.would_deny = True, True
        return d

    def _eval_policy(self, p: CompiledPolicy, headers, body, identity) -> Decision:
        for claim, msg in p.required_claims:
            if HEADER_CLAIM_PREFIX + claim.lower() not in headers:
                return self._apply_mode(p, Decision(False, f"required-claim:{claim}",
                                                    msg or f"missing required claim {claim}"))
        act = {"headers": headers, "body": body, "identity": identity}
        for name, prog, msg in p.rules:
            try:
                out = prog.eval(act)
                if not isinstance(out, bool):
                    raise cel.CELError(f"rule returned non-bool {type(out).__name__}")
            except cel.CELError as e:
                if p.on_failure == "allow":
                    return Decision(True, name, "", p.mode, policy=p.name, error=str(e))
                return self._apply_mode(p, Decision(False, name, f"rule evaluation failed: {e}",
                                                    error=str(e)))
            if out:
                return self._apply_mode(p, Decision(False, name, msg))
        return Decision(True, policy=p.name, mode=p.mode)

    def evaluate(self, headers: dict, body: dict | None, identity: dict | None) -> Decision:
        headers = {str(k).lower(): str(v) for k, v in (headers or {}).items()}
        body = body if isinstance(body, dict) else {}
        ident = _identity(identity)
        audit = None
        for p in self.matching(headers):
            d = self._eval_policy(p, headers, body, ident)
            if not d.allowed:
                return d
            if audit is None and d.denied_by:
                audit = d
        return audit or Decision(True)

    def inject(self, headers: dict, body: dict | None, identity: dict | None) -> dict:
        headers = {str(k).lower(): str(v) for k, v in (headers or {}).items()}
        act = {"headers": headers, "body": body if isinstance(body, dict) else {},
               "identity": _identity(identity)}
        out = {}
        for p in self.matching(headers):
            for h, value, prog in p.injections:
                if prog is None:
                    out[h] = value
                    continue
                try:
                    v = prog.eval(act)
                    out[h] = ("true" if v else "false") if isinstance(v, bool) else str(v)
                except cel.CELError:
                    if p.on_failure != "allow":
                        raise
        return out


def build_app(ev: Evaluator) -> web.Application:
    async def decision(request):
        if request.content_length and request.content_length > MAX_REQUEST_BYTES:
            return web.json_response({"error": "request too large"}, status=413)
        try:
            req = await request.json()
            if not isinstance(req, dict):
                raise ValueError
        except (ValueError, json.JSONDecodeError):
            return web.json_response({"error": "malformed decision request"}, status=400)
        t0 = time.perf_counter()
        d = ev.evaluate(req.get("headers") or {}, req.get("body"), req.get("identity"))
        injected = None
        if d.allowed:
            try:
                injected = ev.inject(req.get("headers") or {}, req.get("body"),
                                     req.get("identity"))
            except cel.CELError as e:
                log.error("header injection failed: %s", e)
        M.TOOLPOLICY_LATENCY.observe(time.perf_counter() - t0)
        M.TOOLPOLICY_DECISIONS.labels("allow" if d.allowed else "deny").inc()
        if d.denied_by:
            log.info("policy decision allowed=%s deniedBy=%s mode=%s policy=%s tool=%s",
                     d.allowed, d.denied_by, d.mode, d.policy,
                     (req.get("headers") or {}).get(HEADER_TOOL_NAME))
        return web.json_response(d.to_json(injected))

    async def healthz(_):
        return web.json_response({"status": "ok", "policies": len(ev.policies)})

    async def metrics(_):
        return web.Response(body=M.exposition(), content_type="text/plain")

    app = web.Application(client_max_size=MAX_REQUEST_BYTES)
    app.router.add_post("/v1/decision", decision)
    app.router.add_get("/healthz", healthz)
    app.router.add_get("/readyz", healthz)
    app.router.add_get("/metrics", metrics)
    return app


class PolicyWatcher:
    """List-and-poll ToolPolicy objects from the in-memory API store or the
    operator's K8s-style REST API; (re)compiles changed generations."""

    def __init__(self, ev: Evaluator, source, namespace: str | None = None,
                 interval: float = 5.0):
        self.ev, self.source, self.ns, self.interval = ev, source, namespace, interval
        self.errors: dict[str, str] = {}

    async def _list(self) -> list[dict]:
        if hasattr(self.source, "list"):
            return [o for o in self.source.list("ToolPolicy", self.ns)]
        import aiohttp

        path = (f"/apis/omnia.altairalabs.ai/v1alpha1/namespaces/{self.ns}/toolpolicies"
                if self.ns else "/apis/omnia.altairalabs.ai/v1alpha1/toolpolicies")
        async with aiohttp.ClientSession() as s:
            async with s.get(self.source.rstrip("/") + path) as r:
                return (await r.json()).get("items", [])

    async def sync_once(self):
        items = await self._list()
        seen = set()
        for o in items:
            md = o.get("metadata", {})
            key = f"{md.get('namespace', 'default')}/{md.get('name')}"
            seen.add(key)
            cur = self.ev.policies.get(key)
            if cur is not None and cur.generation == int(md.get("generation") or 0):
                continue
            try:
                self.ev.set_policy(o)
                self.errors.pop(key, None)
            except (cel.CELError, ValueError, KeyError) as e:
                self.errors[key] = str(e)
                log.error("ToolPolicy %s rejected: %s", key, e)
        for key in list(self.ev.policies):
            if key not in seen:
                ns, name = key.split("/", 1)
                self.ev.remove_policy(ns, name)

    async def run(self):
        while True:
            try:
                await self.sync_once()
            except Exception as e:  # noqa: BLE001
                log.warning("policy sync failed: %s", e)
            await asyncio.sleep(self.interval)


def main(argv=None):
    import yaml

    ap = argparse.ArgumentParser(description="omnia policy broker")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8090)
    ap.add_argument("--policies", default="", help="YAML/JSON file of ToolPolicy objects")
    ap.add_argument("--api-server", default="", help="operator REST base URL to watch")
    ap.add_argument("--namespace", default=None)
    a = ap.parse_args(argv)
    ev = Evaluator()
    if a.policies:
        for o in yaml.safe_load_all(open(a.policies)):
            if o and o.get("kind") == "ToolPolicy":
                ev.set_policy(o)
    app = build_app(ev)
    if a.api_server:
        w = PolicyWatcher(ev, a.api_server, a.namespace)

        async def start(app):
            app["watch"] = asyncio.create_task(w.run())

        app.on_startup.append(start)
    configure_logging()
    web.run_app(app, host=a.host, port=a.port)


if __name__ == "__main__":
    main()
