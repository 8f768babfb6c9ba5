"""SessionPrivacyPolicy watcher + the privacy middleware of session-api and
memory-api (``ee/pkg/privacy/watcher.go``, ``middleware.go``, ``redact_body.go``).

:class:`PolicyWatcher` keeps, by polling, the SessionPrivacyPolicies of its own
namespace plus the global default ``omnia-system/default``, its own Workspace
and the AgentRuntimes of its namespace (the reference narrowed its informers to
exactly that set).  The effective policy of a write, most specific first: the
agent's ``privacyPolicyRef`` -> the agent's service group's ``privacyPolicyRef``
in the Workspace -> the global default -> none.  ``on_change(old, new)`` fires
when a policy is added, changed or evicted.  Objects come from a *source*:
:class:`StoreSource` (an in-process ``APIStore``) or :class:`HTTPSource` (the
operator's API server).

:func:`session_privacy_middleware` (aiohttp) enforces it on session-api writes
that name a session: recording disabled -> 204 and nothing stored; assistant /
system / tool messages from the runtime need ``recording.runtimeData``
(``X-Omnia-Source: facade`` writes always pass); a user who opted out (privacy
store, ``X-Omnia-User-ID``) -> 204; ``recording.pii.redact`` -> the body is
redacted field by field per endpoint (messages: content; tool calls: arguments
and result; provider calls: request and response; events: data; eval results:
explanation) before the handler sees it; a redaction failure blocks the write
(500).  Drops are counted in ``omnia_session_api_writes_dropped_total{reason}``.
:func:`memory_privacy_middleware` applies the same PII redaction to memory-api
saves / updates (content, title, summary) under the policy of the writing agent.
"""
from __future__ import annotations

import asyncio
import json
import logging
import re

from aiohttp import web

from ...observability import metrics as M

log = logging.getLogger("omnia.privacy.policy")

GLOBAL_NS, GLOBAL_NAME = "omnia-system", "default"
API = "/apis/omnia.altairalabs.ai/v1alpha1"


class StoreSource:
    def __init__(self, store):
        self.store = store

    async def list(self, kind: str, namespace: str | None = None) -> list[dict]:
        return list(self.store.list(kind, namespace) if namespace else self.store.list(kind))

    async def get(self, kind: str, name: str, namespace: str | None) -> dict | None:
        return self.store.try_get(kind, name, namespace)


class HTTPSource:
    PLURAL = {"SessionPrivacyPolicy": "sessionprivacypolicies", "Workspace": "workspaces",
              "AgentRuntime": "agentruntimes"}

    def __init__(self, base_url: str, token: str = ""):
        self.base, self.token = base_url.rstrip("/"), token

    async def _get(self, path: str):
        import aiohttp

        h = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        async with aiohttp.ClientSession() as s:
            async with s.get(self.base + path, headers=h) as r:
                if r.status == 404:
                    return None
                if r.status != 200:
                    raise RuntimeError(f"GET {path}: HTTP {r.status}")
                return await r.json()

    async def list(self, kind, namespace=None):
        p = self.PLURAL[kind]
        path = f"{API}/namespaces/{namespace}/{p}" if namespace else f"{API}/{p}"
        return ((await self._get(path)) or {}).get("items", [])

    async def get(self, kind, name, namespace):
        p = self.PLURAL[kind]
        path = f"{API}/namespaces/{namespace}/{p}/{name}" if namespace else f"{API}/{p}/{name}"
        return await self._get(path)


class PrivacyPrefsClient:
    """privacy-api opt-out lookups for the middleware (``GET
    /api/v1/privacy/preferences/{user}``), cached for ``ttl_s``."""

    def __init__(self, base_url: str, ttl_s: float = 30.0):
        self.base, self.ttl_s = base_url.rstrip("/"), ttl_s
        self.cache: dict[str, tuple[float, bool]] = {}

    async def is_opted_out(self, user: str, agent: str = "") -> bool:
        import time

        import aiohttp

        hit = self.cache.get(user)
        if hit and time.time() - hit[0] < self.ttl_s:
            return hit[1]
        try:
            async with aiohttp.ClientSession() as s:
                async with s.get(f"{self.base}/api/v1/privacy/preferences/{user}") as r:
                    out = bool((await r.json()).get("optedOut")) if r.status == 200 else False
        except Exception:  # noqa: BLE001 - an unreachable privacy-api records (fail open)
            return False
        self.cache[user] = (time.time(), out)
        return out


class PolicyWatcher:
    def __init__(self, source, own_workspace: str = "", own_namespace: str = "",
                 poll_s: float = 30.0):
        self.source = source
        self.own_workspace, self.own_namespace = own_workspace, own_namespace
        self.poll_s = poll_s
        self.policies: dict[str, dict] = {}  # "ns/name" -> spec
        self.workspaces: dict[str, dict] = {}
        self.agents: dict[str, dict] = {}
        self.on_change = None
        self.synced = False

    async def load_all(self):
        seen: dict[str, dict] = {}
        if self.own_namespace:
            for p in await self.source.list("SessionPrivacyPolicy", self.own_namespace):
                seen[f"{self.own_namespace}/{p['metadata']['name']}"] = p.get("spec") or {}
        g = await self.source.get("SessionPrivacyPolicy", GLOBAL_NAME, GLOBAL_NS)
        if g is not None:
            seen[f"{GLOBAL_NS}/{GLOBAL_NAME}"] = g.get("spec") or {}
        for k in set(self.policies) | set(seen):
            old, new = self.policies.get(k), seen.get(k)
            if old != new and self.on_change is not None:
                self.on_change(old, new)
        self.policies = seen
        ws = {}
        if self.own_workspace:
            w = await self.source.get("Workspace", self.own_workspace, None)
            if w is not None:
                ws[self.own_workspace] = w
        self.workspaces = ws
        ags = {}
        if self.own_namespace:
            for a in await self.source.list("AgentRuntime", self.own_namespace):
                ags[f"{self.own_namespace}/{a['metadata']['name']}"] = a
        self.agents = ags
        self.synced = True

    async def run(self):
        while True:
            try:
                await self.load_all()
            except Exception as e:  # noqa: BLE001 - keep the last good snapshot
                log.warning("privacy policy reload failed: %s", e)
            await asyncio.sleep(self.poll_s)

    def effective(self, namespace: str, agent: str) -> dict | None:
        if namespace and agent:
            ar = self.agents.get(f"{namespace}/{agent}")
            ref = ((ar or {}).get("spec") or {}).get("privacyPolicyRef") or {}
            if ref.get("name") and f"{namespace}/{ref['name']}" in self.policies:
                return self.policies[f"{namespace}/{ref['name']}"]
        if namespace:
            group = "default"
            ar = self.agents.get(f"{namespace}/{agent}") if agent else None
            if ar and (ar.get("spec") or {}).get("serviceGroup"):
                group = ar["spec"]["serviceGroup"]
            for w in self.workspaces.values():
                if ((w.get("spec") or {}).get("namespace") or {}).get("name") != namespace:
                    continue
                for sg in (w.get("spec") or {}).get("services") or []:
                    name = (sg.get("privacyPolicyRef") or {}).get("name")
                    if sg.get("name") == group and name and \
                            f"{namespace}/{name}" in self.policies:
                        return self.policies[f"{namespace}/{name}"]
        return self.policies.get(f"{GLOBAL_NS}/{GLOBAL_NAME}")


# ------------------------------------------------------------------ body redaction
_FIELDS = [(re.compile(r"/messages$"), ("content",)),
           (re.compile(r"/tool-calls$"), ("arguments", "result")),
           (re.compile(r"/provider-calls$"), ("request", "response")),
           (re.compile(r"/events$"), ("data",)),
           (re.compile(r"/eval-results|/evaluate$"), ("explanation", "details"))]


def redact_body(body: bytes, path: str, redactor) -> bytes:
    """Redact the endpoint's free-text fields; strings in nested JSON values are
    redacted recursively.  Raises ValueError on a body that is not JSON."""
    if not body:
        return body
    fields = next((f for rx, f in _FIELDS if rx.search(path)), None)
    if fields is None:
        return body
    from ..redaction import redact_json

    doc = json.loads(body)
    items = doc if isinstance(doc, list) else [doc]
    for it in items:
        if not isinstance(it, dict):
            continue
        for f in fields:
            if f in it and it[f] is not None:
                it[f] = redactor(it[f]) if isinstance(it[f], str) else redact_json(it[f],
                                                                                   redactor)
    return json.dumps(doc).encode()


def _redactor_for(policy: dict):
    from ..redaction import Redactor

    pii = (policy.get("recording") or {}).get("pii") or {}
    if not pii.get("redact"):
        return None
    return Redactor(pii.get("patterns") or None, pii.get("strategy") or "replace")


_SESSION = re.compile(r"/api/v1/sessions/([^/]+)")
_MESSAGES = re.compile(r"/api/v1/sessions/[^/]+/messages$")
_WRITE = ("POST", "PUT", "PATCH")


def _drop(reason: str):
    M.SESSION_API_WRITES_DROPPED.labels(reason).inc()
    return web.Response(status=204)


def session_privacy_middleware(watcher: PolicyWatcher, resolve_session, prefs=None):
    """``resolve_session(session_id) -> (namespace, agent) | None``; ``prefs``: an
    object with ``is_opted_out(user, agent)`` (the privacy store or a client)."""

    @web.middleware
    async def mw(request, handler):
        if request.method not in _WRITE:
            return await handler(request)
        m = _SESSION.search(request.path)
        if not m or m.group(1) in ("search",):
            return await handler(request)
        who = resolve_session(m.group(1))
        if who is None:
            return await handler(request)
        ns, agent = who
        policy = watcher.effective(ns, agent)
        if policy is None:
            return await handler(request)
        rec = policy.get("recording") or {}
        if not rec.get("enabled", True):
            return _drop("recording-disabled")
        if _MESSAGES.search(request.path):
            src = request.headers.get("X-Omnia-Source", "")
            body = await request.read()
            if src != "facade" and not rec.get("runtimeData", False):
                try:
                    role = (json.loads(body or b"{}") or {}).get("role", "")
                    meta = (json.loads(body or b"{}") or {}).get("metadata") or {}
                except ValueError:
                    role, meta = "", {}
                rich = role in ("assistant", "system") or meta.get("type") in (
                    "tool_call", "tool_result")
                if src == "runtime" or rich:
                    return _drop("runtime-data-disabled")
        oo = policy.get("userOptOut") or {}
        user = request.headers.get("X-Omnia-User-ID", "")
        if oo.get("enabled") and user and prefs is not None:
            out = prefs.is_opted_out(user, agent)
            if asyncio.iscoroutine(out):
                out = await out
            if out:
                return _drop("user-opted-out")
        red = _redactor_for(policy)
        if red is not None:
            try:
                new = redact_body(await request.read(), request.path, red)
            except (ValueError, TypeError) as e:
                M.SESSION_API_WRITES_DROPPED.labels("redaction-failed").inc()
                log.error("body redaction failed, blocking write: %s", e)
                return web.json_response({"error": "redaction failed"}, status=500)
            # read() cached the body; the handler's request.json() reads the cache
            request._read_bytes = new
        return await handler(request)

    return mw


def memory_privacy_middleware(watcher: PolicyWatcher, default_namespace: str = ""):
    """Redact memory-api writes (content / title / summary) under the policy of
    the writing agent (``x-omnia-agent-name`` / ``x-omnia-namespace`` headers)."""

    @web.middleware
    async def mw(request, handler):
        if request.method not in _WRITE or not request.path.startswith("/api/v1/memories") \
                and not request.path.startswith("/api/v1/agent-memories"):
            return await handler(request)
        ns = request.headers.get("x-omnia-namespace", default_namespace)
        policy = watcher.effective(ns, request.headers.get("x-omnia-agent-name", ""))
        red = _redactor_for(policy or {})
        if red is None:
            return await handler(request)
        try:
            doc = json.loads(await request.read() or b"{}")
        except ValueError:
            return web.json_response({"error": "redaction failed"}, status=500)
        if isinstance(doc, dict):
            for f in ("content", "title", "summary"):
                if isinstance(doc.get(f), str):
                    doc[f] = red(doc[f])
        request._read_bytes = json.dumps(doc).encode()  # read() cache -> handler
        return await handler(request)

    return mw
