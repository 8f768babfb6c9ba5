"""Runtime side of memory: HTTP client + composite retriever.

* :class:`MemoryHTTPClient` -- ``internal/memory/httpclient/store.go`` (list /
  search / save / delete / retrieve / semantic), bearer token optional.
* :class:`CompositeRetriever` -- ``internal/runtime/memory_retriever.go:105-436``:
  an always-included, cached "profile" pull (identity / preferences / health,
  cap 20, TTL 30 s) merged with a per-turn episodic search (cap 10) by strategy
  ``keyword`` (FTS with OR semantics), ``semantic`` (server-side hybrid +
  CEL deny-filter) or ``composite`` (both legs, RRF k=60).  No user in scope ->
  nothing injected.
* :class:`HTTPMemoryRetriever` -- the adapter the agent loop calls per turn.
"""
from __future__ import annotations

import logging
import time

from ..utils.cel import DenyFilter
from .fts import to_or_query
from .model import META_CONSENT_CATEGORY, PROFILE_CATEGORIES, SCOPE_AGENT, SCOPE_USER, \
    SCOPE_WORKSPACE
from .retrieval import RRF_K, rrf_fuse

log = logging.getLogger("omnia.memory.retriever")

STRATEGY_KEYWORD, STRATEGY_SEMANTIC, STRATEGY_COMPOSITE = "keyword", "semantic", "composite"
PROFILE_LIMIT = 20
EPISODIC_LIMIT = 10
PROFILE_TTL = 30.0
LIST_FETCH_LIMIT = 200


class MemoryHTTPClient:
    def __init__(self, base_url: str, token: str = "", timeout: float = 10.0, session=None):
        self.base = base_url.rstrip("/")
        self.token = token
        self.timeout = timeout
        self._session = session

    async def _req(self, method: str, path: str, params=None, body=None):
        import aiohttp

        headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        own = self._session is None
        s = self._session or aiohttp.ClientSession(
            timeout=aiohttp.ClientTimeout(total=self.timeout))
        try:
            async with s.request(method, self.base + path, params=params, json=body,
                                 headers=headers) as r:
                if r.status == 204:
                    return None
                data = await r.json(content_type=None)
                if r.status >= 400:
                    raise RuntimeError(f"memory-api {method} {path}: {r.status} "
                                       f"{(data or {}).get('error')}")
                return data
        finally:
            if own:
                await s.close()

    @staticmethod
    def _params(scope: dict, **extra) -> dict:
        p = {"workspace": scope.get(SCOPE_WORKSPACE, "")}
        if scope.get(SCOPE_USER):
            p["virtual_user_id"] = scope[SCOPE_USER]
        if scope.get(SCOPE_AGENT):
            p["agent"] = scope[SCOPE_AGENT]
        p.update({k: str(v) for k, v in extra.items() if v not in (None, "")})
        return p

    async def list(self, scope: dict, limit: int = 50, types=None) -> list[dict]:
        d = await self._req("GET", "/api/v1/memories", self._params(
            scope, limit=limit, type=",".join(types or [])))
        return d.get("memories", [])

    async def search(self, scope: dict, query: str, limit: int = 10) -> list[dict]:
        d = await self._req("GET", "/api/v1/memories/search",
                            self._params(scope, q=query, limit=limit))
        return d.get("memories", [])

    async def save(self, scope: dict, content: str, type_: str = "fact", confidence: float = 0.7,
                   metadata: dict | None = None, about: dict | None = None, **kw) -> dict:
        body = {"scope": scope, "content": content, "type": type_, "confidence": confidence,
                "metadata": metadata or {}}
        if about:
            body["about"] = about
        body.update(kw)
        return await self._req("POST", "/api/v1/memories", body=body)

    async def open(self, entity_id: str, workspace: str) -> dict:
        d = await self._req("GET", f"/api/v1/memories/{entity_id}", {"workspace": workspace})
        return d.get("memory", {})

    async def forget(self, entity_id: str, workspace: str):
        await self._req("DELETE", f"/api/v1/memories/{entity_id}", {"workspace": workspace})

    async def delete_all(self, scope: dict) -> int:
        d = await self._req("DELETE", "/api/v1/memories", self._params(scope))
        return int((d or {}).get("deleted", 0))

    async def retrieve(self, workspace: str, user: str = "", agent: str = "", query: str = "",
                       limit: int = 15, **kw) -> list[dict]:
        body = {"workspace_id": workspace, "virtual_user_id": user, "agent_id": agent,
                "query": query, "limit": limit, **kw}
        d = await self._req("POST", "/api/v1/memories/retrieve", body=body)
        return d.get("memories", [])

    async def retrieve_semantic(self, workspace: str, query: str, deny_cel: str = "",
                                limit: int = 10) -> list[dict]:
        d = await self._req("POST", "/api/v1/memories/retrieve/semantic",
                            body={"workspace_id": workspace, "query": query,
                                  "deny_cel": deny_cel, "limit": limit})
        return d.get("memories", [])


def _is_profile(m: dict) -> bool:
    return (m.get("metadata") or {}).get(META_CONSENT_CATEGORY) in PROFILE_CATEGORIES


class CompositeRetriever:
    def __init__(self, client: MemoryHTTPClient, strategy: str = STRATEGY_KEYWORD,
                 deny_cel: str = "", workspace: str = "", limit: int = EPISODIC_LIMIT,
                 profile_limit: int = PROFILE_LIMIT, profile_ttl: float = PROFILE_TTL):
        self.client = client
        self.strategy = strategy
        self.deny_cel = deny_cel
        self.deny = DenyFilter(deny_cel)
        self.workspace = workspace
        self.limit = limit or EPISODIC_LIMIT
        self.profile_limit = profile_limit
        self.profile_ttl = profile_ttl
        self._cache: dict[str, tuple[float, list]] = {}

    async def retrieve_context(self, scope: dict, query: str) -> list[dict]:
        if not scope.get(SCOPE_USER):
            return []
        profile = await self._profile(scope)
        q = (query or "").strip()
        if not q:
            return profile
        try:
            episodic = await self._episodic(scope, q)
        except Exception as e:  # noqa: BLE001 - profile alone is still useful
            log.debug("episodic retrieve failed: %s", e)
            return profile
        seen = {m.get("id") for m in profile}
        out = list(profile)
        for m in episodic:
            if not _is_profile(m) and m.get("id") not in seen:
                seen.add(m.get("id"))
                out.append(m)
        return out

    async def _profile(self, scope: dict) -> list[dict]:
        key = f"{scope.get(SCOPE_WORKSPACE)}|{scope.get(SCOPE_USER)}"
        hit = self._cache.get(key)
        if hit and hit[0] > time.monotonic():
            return hit[1]
        try:
            allm = await self.client.list(scope, LIST_FETCH_LIMIT)
        except Exception as e:  # noqa: BLE001
            log.debug("profile list failed: %s", e)
            return []
        prof = [m for m in allm if _is_profile(m)][: self.profile_limit]
        self._cache[key] = (time.monotonic() + self.profile_ttl, prof)
        return prof

    def _ws(self, scope):
        return self.workspace or scope.get(SCOPE_WORKSPACE, "")

    async def _keyword(self, scope, q):
        fetch = min(self.limit * 3, LIST_FETCH_LIMIT) if self.deny_cel else self.limit
        mems = await self.client.search(scope, to_or_query(q), fetch)
        return [m for m in mems if self.deny.allowed(m.get("metadata"))][: self.limit]

    async def _episodic(self, scope, q):
        if self.strategy == STRATEGY_SEMANTIC:
            return await self.client.retrieve_semantic(self._ws(scope), q, self.deny_cel,
                                                       self.limit)
        if self.strategy == STRATEGY_COMPOSITE:
            kw = sem = None
            kerr = serr = None
            try:
                kw = await self._keyword(scope, q)
            except Exception as e:  # noqa: BLE001
                kerr = e
            try:
                sem = await self.client.retrieve_semantic(self._ws(scope), q, self.deny_cel,
                                                          self.limit)
            except Exception as e:  # noqa: BLE001
                serr = e
            if kerr is not None and serr is not None:
                raise kerr
            return rrf_fuse([kw or [], sem or []], RRF_K, self.limit, key=lambda m: m.get("id"))
        return await self._keyword(scope, q)


def format_memories(mems: list[dict]) -> str:
    lines = []
    for m in mems:
        c = (m.get("content") or "").strip()
        if c:
            suffix = " (more: memory__open)" if m.get("has_full_body") else ""
            lines.append(f"- {c}{suffix}")
    return "\n".join(lines)


class HTTPMemoryRetriever:
    """Adapter for :class:`omnia_amd.runtime.agent.Agent` (``memory.retrieve``)."""

    def __init__(self, base_url: str, workspace: str = "", agent: str = "",
                 strategy: str = STRATEGY_COMPOSITE, deny_cel: str = "", limit: int = 10,
                 token: str = "", client: MemoryHTTPClient | None = None):
        self.client = client or MemoryHTTPClient(base_url, token)
        self.workspace = workspace
        self.agent = agent
        self.retriever = CompositeRetriever(self.client, strategy, deny_cel, workspace, limit)

    async def retrieve(self, session_id: str, content: str, ctx=None) -> str:
        user = getattr(ctx, "user_id", "") if ctx is not None else ""
        ws = self.workspace or (getattr(ctx, "workspace", "") if ctx is not None else "")
        scope = {SCOPE_WORKSPACE: ws}
        if user:
            scope[SCOPE_USER] = user
        mems = await self.retriever.retrieve_context(scope, content)
        return format_memories(mems)
