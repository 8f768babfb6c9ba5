"""Doctor checks (``internal/doctor/checks/*.go`` semantics, re-derived).

Each checker returns :class:`~.runner.Check` objects named like the reference's
so dashboards and runbooks match:

* Infrastructure -- ``<Service>Healthy`` (``/healthz``), ``<Name>Reachable``
  (TCP), ``RedisReachable`` (PING over RESP), ``GPUKernelsLoaded`` (the gfx950
  kernel extension + a visible device: the in-node engine replaces the
  reference's Ollama probe)
* Agent          -- ``WebSocketConnect``, ``SendMessageGetResponse``,
  ``AgentUsesTools`` (session-api tool-call rows of the doctor's session)
* Sessions       -- ``SessionAPIDocsServed``, ``SessionCreated``,
  ``SessionSearch``, ``MessagesRecorded``, ``ProviderCallsTracked``
* Memory         -- ``MemoryAPIDocsServed``, ``MemorySave``, ``MemoryRetrieve``,
  ``MemoryList``, ``MemoryDelete``, ``MemoryExport``, ``MemoryUserOwnership``,
  ``MemoryUserIsolation``, ``ConsolidationWorkerRunning`` (the memory-api's
  ``omnia_memory_worker_running`` gauge)
* Privacy        -- ``PrivacyAPIHealthy``, ``MemoryOptOutRespected``,
  ``MemoryDeletionCascade``
* CRDs           -- ``AgentRuntimesExist``, ``MemoryEnabled``,
  ``PromptPacksCompiled``, ``ToolRegistriesDiscovered``, ``WorkspacesConfigured``
  read from the operator's API server; ``CRDManifestsValid`` offline
* Workspace      -- ``WorkspaceResolved``: the Workspace owning the agent
  namespace and its service group's session / memory URLs (the doctor fills
  the Sessions / Memory URLs from it when not given explicitly)
* Observability  -- ``<Service> metrics``: ``/metrics`` carries samples with the
  service's ``omnia_<snake>_`` prefix
"""
from __future__ import annotations

import json
import re
import uuid

from .result import FAIL, PASS, SKIP, TestResult, failed, passed, skipped
from .runner import Check

API = "/apis/omnia.altairalabs.ai/v1alpha1"
TIMEOUT_S = 10.0


def _session(timeout: float = TIMEOUT_S):
    import aiohttp

    return aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout))


async def _get(url: str, **kw):
    async with _session() as s:
        async with s.get(url, **kw) as r:
            body = await r.text()
            return r.status, body


def _json(body: str):
    try:
        return json.loads(body)
    except ValueError:
        return None


class State:
    """What one run's checks share: the agent check's session id, the resolved
    workspace service URLs."""

    def __init__(self):
        self.session_id = ""
        self.workspace = ""
        self.session_url = ""
        self.memory_url = ""


# ------------------------------------------------------------------ infrastructure
def probe_check(name: str, base, path: str = "/healthz", suffix: str = "Healthy") -> Check:
    """``base``: a URL, or a callable returning one when the check runs (URLs the
    Workspace check resolves)."""
    async def run():
        url = base() if callable(base) else base
        if not url:
            return skipped(f"no {name} URL configured")
        st, body = await _get(url.rstrip("/") + path)
        return passed(f"HTTP {st}") if st == 200 else failed(f"HTTP {st}: {body[:200]}")

    return Check(name + suffix, "Infrastructure", run)


def tcp_check(name: str, addr: str) -> Check:
    async def run():
        import asyncio

        if not addr:
            return skipped(f"no {name} address configured")
        host, _, port = addr.rpartition(":")
        _, w = await asyncio.wait_for(asyncio.open_connection(host or "127.0.0.1", int(port)),
                                      TIMEOUT_S)
        w.close()
        return passed(f"{addr} accepts connections")

    return Check(name + "Reachable", "Infrastructure", run)


def redis_check(url: str) -> Check:
    async def run():
        if not url:
            return skipped("no redis URL configured")
        from ..utils.resp import RedisClient

        r = RedisClient(url)
        try:
            pong = await r.ping()
        finally:
            r.close()
        return passed("PONG") if pong in (b"PONG", "PONG", True) else failed(repr(pong))

    return Check("RedisReachable", "Infrastructure", run)


def gpu_check() -> Check:
    async def run():
        import torch

        if not torch.cuda.is_available():
            return skipped("no GPU visible to the doctor")
        from .. import ops

        k = ops.kernels()
        free, total = torch.cuda.mem_get_info()
        return passed(f"{torch.cuda.get_device_name(0)}, kernels {k.arch}, "
                      f"{free / 2**30:.0f}/{total / 2**30:.0f} GiB free")

    return Check("GPUKernelsLoaded", "Infrastructure", run)


# ------------------------------------------------------------------ agent
class AgentChecker:
    def __init__(self, facade_url: str, state: State, token: str = "",
                 headers: dict | None = None, prompt: str = "doctor ping"):
        self.url, self.state, self.token = facade_url, state, token
        self.headers = dict(headers or {})
        self.prompt = prompt
        self.connected = False

    def checks(self) -> list[Check]:
        return [Check("WebSocketConnect", "Agent", self.connect),
                Check("SendMessageGetResponse", "Agent", self.chat),
                Check("AgentUsesTools", "Agent", self.tools)]

    def _url(self) -> str:
        u = self.url
        if self.token:
            u += ("&" if "?" in u else "?") + f"token={self.token}"
        return u

    async def connect(self) -> TestResult:
        if not self.url:
            return skipped("no facade URL configured")
        async with _session() as s:
            async with s.ws_connect(self._url(), headers=self.headers) as ws:
                hello = await ws.receive_json(timeout=TIMEOUT_S)
        if hello.get("type") != "connected":
            return failed(f"unexpected handshake frame {hello.get('type')!r}")
        self.connected = True
        return passed(f"session {hello.get('session_id', '')}")

    async def chat(self) -> TestResult:
        if not self.url:
            return skipped("no facade URL configured")
        async with _session(120) as s:
            async with s.ws_connect(self._url(), headers=self.headers) as ws:
                hello = await ws.receive_json(timeout=TIMEOUT_S)
                sid = hello.get("session_id", "")
                await ws.send_json({"type": "message", "content": self.prompt})
                while True:
                    m = await ws.receive_json(timeout=110)
                    t = m.get("type")
                    if t == "tool_call":  # client tools: answer so the turn completes
                        tc = m["tool_call"]
                        await ws.send_json({"type": "tool_result", "tool_result": {
                            "call_id": tc["id"], "result": {"doctor": True}}})
                    elif t == "done":
                        self.state.session_id = sid
                        return passed(f"response of {len(m.get('content') or '')} chars")
                    elif t == "error":
                        return failed(json.dumps(m.get("error")))

    async def tools(self) -> TestResult:
        if not self.state.session_id:
            return skipped("no agent chat session available")
        if not self.state.session_url:
            return skipped("no session-api URL to read tool calls from")
        st, body = await _get(f"{self.state.session_url}/api/v1/sessions/"
                              f"{self.state.session_id}/tool-calls")
        rows = (_json(body) or {}).get("tool-calls", []) if st == 200 else []
        done = [r for r in rows if r.get("status") in ("success", "error")]
        if not done:
            return skipped("the agent made no tool call on the doctor's turn")
        ok = [r for r in done if r.get("status") == "success"]
        names = sorted({r.get("name", "") for r in done})
        return passed(f"{len(ok)}/{len(done)} tool calls succeeded: {names}") if ok else \
            failed(f"every tool call failed: {names}")


# ------------------------------------------------------------------ sessions
class SessionChecker:
    def __init__(self, state: State, namespace: str = "doctor"):
        self.state, self.namespace = state, namespace
        self.own = ""

    def checks(self) -> list[Check]:
        return [Check("SessionAPIDocsServed", "Sessions", self.docs),
                Check("SessionCreated", "Sessions", self.created),
                Check("SessionSearch", "Sessions", self.search),
                Check("MessagesRecorded", "Sessions", self.messages),
                Check("ProviderCallsTracked", "Sessions", self.provider_calls)]

    @property
    def base(self) -> str:
        return self.state.session_url.rstrip("/")

    def _sid(self) -> str:
        return self.state.session_id or self.own

    async def docs(self) -> TestResult:
        if not self.base:
            return skipped("no session-api URL configured")
        st, body = await _get(self.base + "/api/v1/openapi.json")
        doc = _json(body) or {}
        if st != 200 or "paths" not in doc:
            return failed(f"HTTP {st}")
        return passed(f"{len(doc['paths'])} paths documented")

    async def created(self) -> TestResult:
        if not self.base:
            return skipped("no session-api URL configured")
        if not self.state.session_id:
            # no agent turn ran: create and populate a doctor session ourselves
            self.own = "doctor-" + uuid.uuid4().hex[:10]
            async with _session() as s:
                r = await s.post(self.base + "/api/v1/sessions",
                                 json={"id": self.own, "namespace": self.namespace,
                                       "agentName": "doctor"})
                if r.status >= 300:
                    return failed(f"create HTTP {r.status}")
                await s.post(f"{self.base}/api/v1/sessions/{self.own}/messages",
                             json={"role": "user", "content": "doctor ping"})
        st, body = await _get(f"{self.base}/api/v1/sessions/{self._sid()}")
        return passed(f"session {self._sid()}") if st == 200 else failed(f"HTTP {st}")

    async def search(self) -> TestResult:
        if not self.base:
            return skipped("no session-api URL configured")
        st, body = await _get(self.base + "/api/v1/sessions/search", params={"q": "doctor"})
        if st != 200:
            return failed(f"HTTP {st}")
        return passed(f"{len((_json(body) or {}).get('sessions', []))} sessions matched")

    async def messages(self) -> TestResult:
        if not self.base or not self._sid():
            return skipped("no agent chat session available")
        st, body = await _get(f"{self.base}/api/v1/sessions/{self._sid()}/messages")
        n = len((_json(body) or {}).get("messages", [])) if st == 200 else 0
        return passed(f"{n} messages") if n else failed(f"no messages (HTTP {st})")

    async def provider_calls(self) -> TestResult:
        if not self.base or not self.state.session_id:
            return skipped("no agent chat session available")
        st, body = await _get(f"{self.base}/api/v1/sessions/{self.state.session_id}/"
                              f"provider-calls")
        rows = (_json(body) or {}).get("provider-calls", []) if st == 200 else []
        return passed(f"{len(rows)} provider calls") if rows else \
            skipped("no provider calls recorded (runtime without a session-api sink)")


# ------------------------------------------------------------------ memory
class MemoryChecker:
    MARKER = "smoke-42"

    def __init__(self, state: State, workspace: str = ""):
        self.state = state
        self.workspace = workspace
        self.user = "doctor-" + uuid.uuid4().hex[:8]
        self.other = self.user + "-other"
        self.mem_id = ""

    def checks(self) -> list[Check]:
        return [Check("MemoryAPIDocsServed", "Memory", self.docs),
                Check("MemorySave", "Memory", self.save),
                Check("MemoryRetrieve", "Memory", self.retrieve),
                Check("MemoryList", "Memory", self.list),
                Check("MemoryExport", "Memory", self.export),
                Check("MemoryUserOwnership", "Memory", self.ownership),
                Check("MemoryUserIsolation", "Memory", self.isolation),
                Check("MemoryDelete", "Memory", self.delete),
                Check("ConsolidationWorkerRunning", "Memory", self.worker),
                Check("ConsolidationPassesHealthy", "Memory", self.passes)]

    @property
    def base(self) -> str:
        return self.state.memory_url.rstrip("/")

    @property
    def ws(self) -> str:
        return self.workspace or self.state.workspace or "doctor"

    def _need(self):
        return None if self.base else skipped("no memory-api URL configured")

    async def docs(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        st, body = await _get(self.base + "/api/v1/openapi.yaml")
        return passed("OpenAPI served") if st == 200 and "openapi" in body else \
            failed(f"HTTP {st}")

    async def save(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        async with _session() as s:
            r = await s.post(self.base + "/api/v1/memories", json={
                "content": f"{self.MARKER} doctor marker", "type": "fact",
                "scope": {"workspace_id": self.ws, "virtual_user_id": self.user}})
            body = await r.json()
        if r.status != 201:
            return failed(f"HTTP {r.status}: {body}")
        self.mem_id = body["memory"]["id"]
        return passed(f"memory {self.mem_id}")

    async def retrieve(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        async with _session() as s:
            r = await s.post(self.base + "/api/v1/memories/retrieve", json={
                "workspace_id": self.ws, "virtual_user_id": self.user, "query": self.MARKER})
            got = await r.json()
        ok = any(self.MARKER in m.get("content", "") for m in got.get("memories", []))
        return passed(f"{self.MARKER} recalled") if ok else failed("marker not recalled")

    async def _list(self, user: str) -> list:
        st, body = await _get(self.base + "/api/v1/memories",
                              params={"workspace": self.ws, "virtual_user_id": user})
        return (_json(body) or {}).get("memories", []) if st == 200 else []

    async def list(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        mems = await self._list(self.user)
        return passed(f"{len(mems)} memories") if any(m["id"] == self.mem_id for m in mems) \
            else failed("saved memory missing from the list")

    async def export(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        st, body = await _get(self.base + "/api/v1/memories/export",
                              params={"workspace": self.ws, "virtual_user_id": self.user})
        mems = (_json(body) or {}).get("memories", []) if st == 200 else []
        return passed(f"{len(mems)} exported") if mems else failed(f"HTTP {st}, nothing exported")

    async def ownership(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        mems = [m for m in await self._list(self.user) if m["id"] == self.mem_id]
        if not mems:
            return failed("saved memory not found")
        owner = (mems[0].get("scope") or {}).get("virtual_user_id")
        return passed("scoped to its user") if owner == self.user else \
            failed(f"owner {owner!r} != {self.user!r}")

    async def isolation(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        leaked = [m for m in await self._list(self.other) if m["id"] == self.mem_id]
        return failed("another user can list the memory") if leaked else \
            passed("invisible to another user")

    async def delete(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        async with _session() as s:
            r = await s.delete(self.base + "/api/v1/memories",
                               params={"workspace": self.ws, "virtual_user_id": self.user})
        left = await self._list(self.user)
        return passed("deleted") if r.status < 300 and not left else \
            failed(f"HTTP {r.status}, {len(left)} left")

    async def worker(self) -> TestResult:
        if (r := self._need()) is not None:
            return r
        st, body = await _get(self.base + "/metrics")
        if st != 200:
            return failed(f"metrics HTTP {st}")
        vals = {}
        for m in re.finditer(r'^omnia_memory_worker_running\{name="([a-z_]+)"\} ([0-9.]+)$',
                             body, re.M):
            vals[m.group(1)] = float(m.group(2))
        for name in ("consolidation", "compaction"):
            if name in vals:
                return passed(f"{name} worker running") if vals[name] == 1 else \
                    failed(f"{name} worker not running (gauge={vals[name]:g})")
        return skipped("consolidation worker not enabled (gauge series absent)")

    async def passes(self) -> TestResult:
        """Consolidation pass outcomes (``omnia_memory_consolidation_passes_total``
        by status): failing passes with no successful one mean the function or
        the applier is broken for every workspace."""
        if (r := self._need()) is not None:
            return r
        st, body = await _get(self.base + "/metrics")
        if st != 200:
            return failed(f"metrics HTTP {st}")
        by: dict = {}
        for m in re.finditer(r'^omnia_memory_consolidation_passes_total\{([^}]*)\} ([0-9.e+]+)$',
                             body, re.M):
            sm = re.search(r'status="([a-z_]+)"', m.group(1))
            if sm:
                by[sm.group(1)] = by.get(sm.group(1), 0.0) + float(m.group(2))
        if not by:
            return skipped("no consolidation passes yet")
        good = by.get("ok", 0) + by.get("empty", 0)
        bad = {k: v for k, v in by.items() if k not in ("ok", "empty") and v}
        if bad and not good:
            return failed("every pass failed: " + ", ".join(f"{k}={v:g}" for k, v in bad.items()))
        return passed(f"{good:g} good passes" + (f", failures {bad}" if bad else ""))


# ------------------------------------------------------------------ privacy
class PrivacyChecker:
    def __init__(self, privacy_url: str, state: State, workspace: str = ""):
        self.base = privacy_url.rstrip("/")
        self.state = state
        self.workspace = workspace
        self.user = "doctor-privacy-" + uuid.uuid4().hex[:6]

    def checks(self) -> list[Check]:
        return [Check("PrivacyAPIHealthy", "Privacy", self.healthy),
                Check("MemoryOptOutRespected", "Privacy", self.opt_out),
                Check("MemoryDeletionCascade", "Privacy", self.cascade)]

    async def healthy(self) -> TestResult:
        if not self.base:
            return skipped("no privacy-api URL configured")
        st, _ = await _get(self.base + "/healthz")
        return passed("healthy") if st == 200 else failed(f"HTTP {st}")

    async def opt_out(self) -> TestResult:
        if not self.base:
            return skipped("no privacy-api URL configured")
        async with _session() as s:
            r = await s.post(self.base + "/api/v1/privacy/opt-out",
                             json={"userId": self.user, "scope": "all"})
            if r.status >= 300:
                return failed(f"opt-out HTTP {r.status}")
        st, body = await _get(f"{self.base}/api/v1/privacy/preferences/{self.user}")
        prefs = _json(body) or {}
        opted = prefs.get("optedOut")
        return passed("opt-out recorded") if st == 200 and opted else \
            failed(f"preferences do not show the opt-out: {body[:200]}")

    async def cascade(self) -> TestResult:
        mem = self.state.memory_url.rstrip("/")
        if not mem:
            return skipped("no memory-api URL configured")
        ws = self.workspace or self.state.workspace or "doctor"
        scope = {"workspace_id": ws, "virtual_user_id": self.user}
        async with _session() as s:
            r = await s.post(mem + "/api/v1/memories", json={"content": "deletion cascade test",
                                                              "scope": scope})
            if r.status != 201:
                return failed(f"save HTTP {r.status}")
            r = await s.delete(mem + "/api/v1/memories",
                               params={"workspace": ws, "virtual_user_id": self.user})
            st, body = r.status, await r.text()
        left = (_json((await _get(mem + "/api/v1/memories", params={
            "workspace": ws, "virtual_user_id": self.user}))[1]) or {}).get("memories", [])
        return passed("user erasure removed every memory") if st < 300 and not left else \
            failed(f"HTTP {st}, {len(left)} memories left")


# ------------------------------------------------------------------ CRDs / workspace
class CRDChecker:
    def __init__(self, operator_url: str, namespace: str = "default"):
        self.base = operator_url.rstrip("/")
        self.ns = namespace

    def checks(self) -> list[Check]:
        if not self.base:
            return [Check("CRDManifestsValid", "CRDs", self.manifests)]
        return [Check("AgentRuntimesExist", "CRDs", self.agent_runtimes),
                Check("MemoryEnabled", "CRDs", self.memory_enabled),
                Check("PromptPacksCompiled", "CRDs", self.prompt_packs),
                Check("ToolRegistriesDiscovered", "CRDs", self.tool_registries),
                Check("WorkspacesConfigured", "CRDs", self.workspaces)]

    async def manifests(self) -> TestResult:
        from ..api import crds

        bad = [k.kind for k in crds.KINDS.values()
               if crds.crd_manifest(k).get("kind") != "CustomResourceDefinition"]
        return passed(f"{len(crds.KINDS)} kinds render") if not bad else failed(f"invalid {bad}")

    async def _items(self, plural: str, namespaced: bool = True) -> list:
        path = f"{API}/namespaces/{self.ns}/{plural}" if namespaced else f"{API}/{plural}"
        st, body = await _get(self.base + path)
        if st != 200:
            raise RuntimeError(f"GET {path}: HTTP {st}")
        return (_json(body) or {}).get("items", [])

    async def agent_runtimes(self) -> TestResult:
        items = await self._items("agentruntimes")
        if not items:
            return failed(f"no AgentRuntimes in {self.ns}")
        ready = [i["metadata"]["name"] for i in items
                 if (i.get("status") or {}).get("phase") in ("Running", "Ready")]
        return passed(f"{len(items)} AgentRuntimes, {len(ready)} running")

    async def memory_enabled(self) -> TestResult:
        items = await self._items("agentruntimes")
        on = [i["metadata"]["name"] for i in items
              if ((i.get("spec") or {}).get("memory") or {}).get("enabled")]
        return passed(f"memory on for {on}") if on else skipped("no AgentRuntime enables memory")

    async def prompt_packs(self) -> TestResult:
        items = await self._items("promptpacks")
        if not items:
            return skipped(f"no PromptPacks in {self.ns}")
        bad = [i["metadata"]["name"] for i in items
               if (i.get("status") or {}).get("phase") not in ("Active", "Ready", "Compiled")]
        return failed(f"not compiled: {bad}") if bad else passed(f"{len(items)} compiled")

    async def tool_registries(self) -> TestResult:
        items = await self._items("toolregistries")
        if not items:
            return skipped(f"no ToolRegistries in {self.ns}")
        n = sum(len((i.get("status") or {}).get("discoveredTools") or []) for i in items)
        return passed(f"{len(items)} registries, {n} tools discovered")

    async def workspaces(self) -> TestResult:
        items = await self._items("workspaces", namespaced=False)
        if not items:
            return skipped("no Workspaces")
        ready = [i["metadata"]["name"] for i in items
                 if (i.get("status") or {}).get("phase") == "Ready"]
        return passed(f"{len(ready)}/{len(items)} ready") if ready else \
            failed("no Workspace is Ready")


class WorkspaceChecker:
    """Resolve the Workspace that owns the agent namespace
    (``checks/workspace.go`` ResolveWorkspaceUID) and, from its status, the
    service group's session-api / memory-api URLs."""

    def __init__(self, operator_url: str, namespace: str, state: State,
                 service_group: str = "default", resolve=None):
        self.base = operator_url.rstrip("/")
        self.ns, self.state, self.group = namespace, state, service_group
        self.resolve = resolve  # optional url rewriter (single-node endpoints)

    def checks(self) -> list[Check]:
        return [Check("WorkspaceResolved", "Workspace", self.run)]

    async def run(self) -> TestResult:
        if not self.base:
            return skipped("no operator URL configured")
        st, body = await _get(self.base + f"{API}/workspaces")
        if st != 200:
            return failed(f"HTTP {st}")
        for ws in (_json(body) or {}).get("items", []):
            if ((ws.get("spec") or {}).get("namespace") or {}).get("name") != self.ns:
                continue
            self.state.workspace = ws["metadata"]["name"]
            for sg in (ws.get("status") or {}).get("services") or []:
                if sg.get("name") == self.group:
                    fix = self.resolve or (lambda u: u)
                    self.state.session_url = self.state.session_url or fix(
                        sg.get("sessionURL", ""))
                    self.state.memory_url = self.state.memory_url or fix(
                        sg.get("memoryURL", ""))
            return passed(f"workspace {self.state.workspace}")
        return skipped(f"no Workspace owns namespace {self.ns}")


# ------------------------------------------------------------------ observability
def metrics_prefix(name: str) -> str:
    """``SessionAPI`` -> ``omnia_session_api_`` (checks/observability.go)."""
    out = []
    for i, ch in enumerate(name):
        if i and ch.isupper():
            prev, nxt = name[i - 1], name[i + 1] if i + 1 < len(name) else ""
            if prev.islower() or (prev.isupper() and nxt.islower()):
                out.append("_")
        out.append(ch.lower())
    return "omnia_" + "".join(out) + "_"


def metrics_check(name: str, url: str, prefix: str | None = None) -> Check:
    async def run():
        if not url:
            return skipped("no metrics URL configured")
        p = prefix or metrics_prefix(name)
        st, body = await _get(url.rstrip("/") + ("" if url.endswith("/metrics") else "/metrics"))
        if st != 200:
            return failed(f"HTTP {st}")
        n = sum(1 for line in body.splitlines() if line.startswith(p))
        return passed(f"{n} metrics found") if n else failed(f"no metrics with prefix {p!r}")

    return Check(f"{name} metrics", "Observability", run)


__all__ = ["State", "AgentChecker", "SessionChecker", "MemoryChecker", "PrivacyChecker",
           "CRDChecker", "WorkspaceChecker", "probe_check", "tcp_check", "redis_check",
           "gpu_check", "metrics_check", "metrics_prefix", "PASS", "FAIL", "SKIP"]
