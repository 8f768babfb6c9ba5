"""memory-api HTTP service (``cmd/memory-api``, ``internal/memory/api/handler.go:405-447``).

Same routes and JSON shapes as the reference: scope from ``workspace`` /
``virtual_user_id`` (legacy ``user_id``) / ``agent`` query params, list
responses ``{memories:[...], total}`` with a derived ``tier``, recall responses
swap bodies > 2 KiB for a 240-rune preview, enterprise-only routes return 403
unless started with ``--enterprise``.

``python -m omnia_amd.memory.api --port 8400 --db /var/lib/omnia/memory.db
[--embedding local|hash|openai] [--enterprise]``
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import time

from aiohttp import web

from ..observability import metrics as M
from ..utils.cel import CELError
from . import retrieval as R
from .model import (META_ABOUT_KEY, META_ABOUT_KIND, META_CONSENT_CATEGORY, PII_CATEGORIES,
                    SCOPE_AGENT, SCOPE_USER, SCOPE_WORKSPACE, Memory, Tier, normalize_scope,
                    parse_time)
from .service import MemoryService
from .store import MultiTierRequest, NotFound
from ..observability.logging import configure as configure_logging

log = logging.getLogger("omnia.memory.api")

MAX_BODY = 16 << 20
DEFAULT_LIST_LIMIT = 50
MAX_LIST_LIMIT = 1000
DEFAULT_BATCH_DELETE = 500
MAX_BATCH_DELETE = 10000
MAX_PARAM = 256
SVC_KEY = web.AppKey("memory_service", MemoryService)


def _err(status: int, msg: str):
    return web.json_response({"error": msg}, status=status)


def _trunc(v: str | None) -> str:
    return (v or "")[:MAX_PARAM]


def _scope_from_query(q) -> dict:
    ws = _trunc(q.get("workspace"))
    if not ws:
        raise web.HTTPBadRequest(text=json.dumps({"error": "workspace is required"}),
                                 content_type="application/json")
    s = {SCOPE_WORKSPACE: ws}
    uid = q.get("virtual_user_id") or q.get("user_id")
    if uid:
        s[SCOPE_USER] = _trunc(uid)
    if q.get("agent"):
        s[SCOPE_AGENT] = _trunc(q.get("agent"))
    return s


def _int(q, name, default):
    try:
        return int(q.get(name, default))
    except (TypeError, ValueError):
        return default


def _types(s: str | None) -> list[str]:
    return [t.strip() for t in (s or "").split(",") if t.strip()]


def _list_json(mems, preview=False, related=None) -> dict:
    related = related or {}
    out = [m.to_json(inline_preview=preview, related=related.get(m.id)) for m in mems]
    return {"memories": out, "total": len(out)}


async def _body(request) -> dict:
    if request.content_length and request.content_length > MAX_BODY:
        raise web.HTTPRequestEntityTooLarge(max_size=MAX_BODY, actual_size=request.content_length)
    try:
        d = await request.json()
    except (json.JSONDecodeError, ValueError):
        raise web.HTTPBadRequest(text=json.dumps({"error": "invalid JSON body"}),
                                 content_type="application/json")
    if not isinstance(d, dict):
        raise web.HTTPBadRequest(text=json.dumps({"error": "body must be an object"}),
                                 content_type="application/json")
    for k, v in d.items():
        t = _BODY_TYPES.get(k)
        if v is None or t is None:
            continue
        ok = (isinstance(v, t) and not (isinstance(v, bool) and t is not bool)) if t in (
            int, bool) else isinstance(v, t) and not (isinstance(v, bool) and t == (int, float))
        if not ok:
            raise web.HTTPBadRequest(text=json.dumps({"error": f"{k} has the wrong type"}),
                                     content_type="application/json")
        if isinstance(v, list) and k in _STR_LISTS and not all(isinstance(x, str) for x in v):
            raise web.HTTPBadRequest(text=json.dumps({"error": f"{k} must be strings"}),
                                     content_type="application/json")
    return d


# JSON types of the body fields the handlers read (null = absent)
_BODY_TYPES = {"scope": dict, "metadata": dict, "about": dict, "content": str, "query": str,
               "text": str, "type": str, "title": str, "summary": str, "category": str,
               "purpose": str, "relation_type": str, "source_id": str, "target_id": str,
               "session_id": str, "workspace": str, "user_id": str, "agent_id": str, "id": str,
               "ids": list, "source_ids": list, "types": list, "turn_range": list,
               "documents": list, "limit": int, "weight": (int, float),
               "confidence": (int, float), "min_confidence": (int, float), "granted": bool}
_STR_LISTS = {"ids", "source_ids", "types"}


_MEM_FIELDS = {"id": str, "type": str, "content": str, "metadata": dict, "category": str,
               "about": dict, "session_id": str, "title": str, "summary": str,
               "turn_range": list, "scope": dict}


def _bad(msg: str):
    return web.HTTPBadRequest(text=json.dumps({"error": msg}), content_type="application/json")


def _memory_from_request(d: dict, scope: dict | None = None) -> Memory:
    for k, t in _MEM_FIELDS.items():
        v = d.get(k)
        if v is not None and not isinstance(v, t):
            raise _bad(f"{k} must be {'an object' if t is dict else 'a ' + t.__name__}")
    c = d.get("confidence")
    if c is not None and (isinstance(c, bool) or not isinstance(c, (int, float))
                          or not 0.0 <= float(c) <= 1.0):
        raise _bad("confidence must be a number in [0, 1]")
    tr = d.get("turn_range")
    if tr is not None and not all(isinstance(x, int) and not isinstance(x, bool) for x in tr):
        raise _bad("turn_range must be integers")
    ea = d.get("expires_at")
    if ea is not None and not isinstance(ea, (str, int, float)) or isinstance(ea, bool):
        raise _bad("expires_at must be a timestamp")
    meta = dict(d.get("metadata") or {})
    if d.get("category"):
        meta.setdefault(META_CONSENT_CATEGORY, d["category"])
    about = d.get("about") or {}
    if about.get("kind") and about.get("key"):
        meta[META_ABOUT_KIND] = about["kind"]
        meta[META_ABOUT_KEY] = about["key"]
    tr = d.get("turn_range")
    return Memory(id=d.get("id", ""), type=d.get("type") or "fact", content=d.get("content", ""),
                  confidence=float(d.get("confidence") or 0.7),
                  scope=normalize_scope(scope if scope is not None else d.get("scope")),
                  metadata=meta, session_id=d.get("session_id", ""),
                  turn_range=list(tr) if tr and any(tr) else None, title=d.get("title", ""),
                  summary=d.get("summary", ""), expires_at=parse_time(d.get("expires_at")))


def chunk_text(text: str, size: int = 200, overlap: int = 40) -> list[str]:
    """Ingestion ChunkStrategy: word windows of ``size`` with ``overlap``."""
    words = text.split()
    if not words:
        return []
    step = max(1, size - overlap)
    out = []
    for i in range(0, len(words), step):
        out.append(" ".join(words[i:i + size]))
        if i + size >= len(words):
            break
    return out


def build_app(svc: MemoryService, enterprise: bool = False, chunk_size: int = 200,
              chunk_overlap: int = 40, tokens: set | None = None) -> web.Application:
    @web.middleware
    async def mw(request, handler):
        if tokens and request.path != "/healthz":
            auth = request.headers.get("Authorization", "")
            if not auth.startswith("Bearer ") or auth[7:] not in tokens:
                return _err(401, "unauthorized")
        status = 500
        try:
            resp = await handler(request)
            status = resp.status
            return resp
        except web.HTTPException as e:
            status = e.status
            raise
        except NotFound as e:
            status = 404
            return _err(404, f"memory not found: {e}")
        except (ValueError, KeyError) as e:
            status = 400
            return _err(400, str(e))
        except PermissionError as e:
            status = 403
            return _err(403, str(e))
        finally:
            M.MEMORY_OPS.labels(op=request.method, status=str(status)).inc()

    app = web.Application(middlewares=[mw], client_max_size=MAX_BODY)
    r = app.router

    def ee(fn):
        async def wrapped(request):
            if not enterprise:
                return _err(403, "enterprise feature not enabled")
            return await fn(request)
        return wrapped

    async def healthz(_):
        return web.json_response({"status": "ok"})

    async def metrics(_):
        return web.Response(body=M.exposition(), content_type="text/plain")

    async def list_memories(request):
        q = request.query
        scope = _scope_from_query(q)
        limit = min(max(_int(q, "limit", DEFAULT_LIST_LIMIT), 1), MAX_LIST_LIMIT)
        shared = q.get("include_shared") == "true"
        if shared:
            req = MultiTierRequest(workspace_id=scope[SCOPE_WORKSPACE],
                                   user_id=scope.get(SCOPE_USER, ""),
                                   agent_id=scope.get(SCOPE_AGENT, ""), types=_types(q.get("type")),
                                   limit=limit)
            mems = svc.store.retrieve_multi_tier(req)
        else:
            mems = await svc.list_cached(scope, _types(q.get("type")), limit,
                                         _int(q, "offset", 0))
        return web.json_response(_list_json(mems))

    async def search(request):
        q = request.query
        scope = _scope_from_query(q)
        if not q.get("q"):
            return _err(400, "query parameter q is required")
        limit = min(max(_int(q, "limit", DEFAULT_LIST_LIMIT), 1), MAX_LIST_LIMIT)
        mems = await svc.search_cached(scope, q["q"], limit)
        mc = float(q.get("min_confidence") or 0)
        mems = [m for m in mems if m.confidence >= mc]
        return web.json_response(_list_json(mems, preview=True,
                                            related=svc.store.related([m.id for m in mems])))

    async def export(request):
        scope = _scope_from_query(request.query)
        return web.json_response(_list_json(svc.store.export_all(scope)))

    async def save(request):
        d = await _body(request)
        mem = _memory_from_request(d)
        if not mem.content:
            return _err(400, "content is required")
        res = await svc.save(mem)
        m = svc.store.get(res["id"])
        out = {"memory": m.to_json() if m else {"id": res["id"]}, "action": res["action"]}
        for k in ("supersedes", "supersede_reason", "potential_duplicates"):
            if res.get(k):
                out[k] = res[k]
        return web.json_response(out, status=201)

    async def open_memory(request):
        ws = request.query.get("workspace")
        m = svc.store.get(request.match_info["id"], ws, touch=True)
        if m is None:
            return _err(404, "memory not found")
        rel = svc.store.related([m.id])
        return web.json_response({"memory": m.to_json(related=rel.get(m.id))})

    async def update(request):
        d = await _body(request)
        m = await svc.update(request.match_info["id"], d.get("content"), d.get("metadata"),
                             d.get("confidence"), request.query.get("workspace"))
        return web.json_response({"memory": m.to_json()})

    async def supersede(request):
        d = await _body(request)
        src = d.get("source_ids") or []
        if not src:
            return _err(400, "source_ids is required")
        mem = _memory_from_request(d)
        res = await svc.supersede(src, mem)
        return web.json_response({"id": res["id"], "supersedes": src}, status=201)

    async def conflicts(request):
        q = request.query
        scope = _scope_from_query(q)
        c = svc.store.conflicts(scope[SCOPE_WORKSPACE], scope.get(SCOPE_USER, ""),
                                _int(q, "limit", 50))
        return web.json_response({"conflicts": c, "total": len(c)})

    async def link(request):
        d = await _body(request)
        scope = normalize_scope(d.get("scope"))
        if not scope.get(SCOPE_WORKSPACE):
            return _err(400, "scope.workspace_id is required")
        for k in ("source_id", "target_id", "relation_type"):
            if not d.get(k):
                return _err(400, f"{k} is required")
        rid = svc.store.link(scope[SCOPE_WORKSPACE], d["source_id"], d["target_id"],
                             d["relation_type"], float(d.get("weight") or 1.0))
        return web.json_response({"id": rid}, status=201)

    async def delete_one(request):
        ok = await svc.forget(request.match_info["id"], request.query.get("workspace"))
        if not ok:
            return _err(404, "memory not found")
        return web.Response(status=204)

    async def delete_batch(request):
        q = request.query
        scope = _scope_from_query(q)
        limit = min(max(_int(q, "limit", DEFAULT_BATCH_DELETE), 1), MAX_BATCH_DELETE)
        return web.json_response({"deleted": await svc.batch_delete(scope, limit)})

    async def delete_all(request):
        scope = _scope_from_query(request.query)
        if SCOPE_USER not in scope:
            return _err(400, "virtual_user_id is required for delete-all")
        return web.json_response({"deleted": await svc.delete_all(scope)})

    async def retrieve(request):
        d = await _body(request)
        ws = d.get("workspace_id")
        if not ws:
            return _err(400, "workspace_id is required")
        hl = d.get("half_life") or {}
        req = MultiTierRequest(
            workspace_id=ws, user_id=d.get("virtual_user_id") or d.get("user_id") or "",
            agent_id=d.get("agent_id") or "", query=d.get("query") or "",
            types=d.get("types") or [], purposes=d.get("purposes") or [],
            min_confidence=float(d.get("min_confidence") or 0),
            limit=int(d.get("limit") or R.DEFAULT_LIMIT), tiers=d.get("tiers") or [],
            seed_entity_ids=d.get("seed_entity_ids") or [],
            relation_types=d.get("relation_types") or [],
            max_graph_hops=int(d.get("max_graph_hops") or 1),
            half_life=R.HalfLife(**{**svc.policy_half_life.__dict__,
                                    **{k: float(v) for k, v in hl.items()
                                       if k in ("user", "agent", "institutional")}}),
            ranker=svc.policy_ranker)
        mems = await svc.retrieve_multi_tier(req)
        return web.json_response(_list_json(mems, preview=True,
                                            related=svc.store.related([m.id for m in mems])))

    async def retrieve_semantic(request):
        d = await _body(request)
        ws = d.get("workspace_id")
        if not ws:
            return _err(400, "workspace_id is required")
        try:
            mems = await svc.retrieve_semantic(ws, d.get("query") or "", d.get("deny_cel") or "",
                                               int(d.get("limit") or 10))
        except CELError as e:
            return _err(500, f"deny_cel: {e}")
        return web.json_response(_list_json(mems, preview=True))

    async def aggregate(request):
        q = request.query
        ws = _trunc(q.get("workspace"))
        if not ws:
            return _err(400, "workspace is required")
        rows = svc.store.aggregate(ws, q.get("groupBy") or "category")
        return web.json_response({"groups": rows, "total": sum(r["count"] for r in rows)})

    async def projection(request):
        q = request.query
        ws = _trunc(q.get("workspace"))
        if not ws:
            return _err(400, "workspace is required")
        return web.json_response(_project(svc, ws, q.get("virtual_user_id") or q.get("user_id")))

    # institutional (workspace-wide) and agent-scoped admin paths
    async def save_inst(request):
        d = await _body(request)
        ws = d.get("workspace_id") or (d.get("scope") or {}).get(SCOPE_WORKSPACE)
        if not ws:
            return _err(400, "workspace_id is required")
        mem = _memory_from_request(d, {SCOPE_WORKSPACE: ws})
        mem.metadata.setdefault("source_type", "operator_curated")
        res = await svc.save(mem, require_user=False)
        return web.json_response({"memory": svc.store.get(res["id"]).to_json(),
                                  "action": res["action"]}, status=201)

    async def list_inst(request):
        q = request.query
        ws = _trunc(q.get("workspace"))
        if not ws:
            return _err(400, "workspace is required")
        mems = svc.store.list({SCOPE_WORKSPACE: ws}, _types(q.get("type")),
                              min(max(_int(q, "limit", DEFAULT_LIST_LIMIT), 1), MAX_LIST_LIMIT),
                              _int(q, "offset", 0))
        return web.json_response(_list_json(mems))

    async def delete_inst(request):
        ws = _trunc(request.query.get("workspace"))
        m = svc.store.get(request.match_info["id"], ws or None)
        if m is None or m.tier != Tier.INSTITUTIONAL:
            return _err(404, "memory not found")
        await svc.forget(m.id, ws or None)
        return web.Response(status=204)

    async def ingest(request):
        d = await _body(request)
        ws = d.get("workspace_id")
        if not ws:
            return _err(400, "workspace_id is required")
        url = d.get("url") or d.get("title") or "doc"
        for i, chunk in enumerate(chunk_text(d.get("text") or "", chunk_size, chunk_overlap)):
            mem = Memory(type="document", content=chunk, confidence=0.9,
                         scope={SCOPE_WORKSPACE: ws}, title=d.get("title", ""),
                         metadata={META_ABOUT_KIND: "sharepoint_doc",
                                   META_ABOUT_KEY: f"{url}#{i}", "url": d.get("url", ""),
                                   "site": d.get("site", ""), "source_type": "operator_curated"})
            # embeddings are backfilled by the re-embed worker (202 semantics)
            svc.store.save(mem, require_user=False)
        return web.Response(status=202)

    async def summary_candidates(request):
        q = request.query
        ws = _trunc(q.get("workspace"))
        if not ws:
            return _err(400, "workspace is required")
        docs = {}
        for m in svc.store.list({SCOPE_WORKSPACE: ws}, ["document"], MAX_LIST_LIMIT):
            url = m.metadata.get("url") or m.metadata.get(META_ABOUT_KEY, "").split("#")[0]
            docs.setdefault(url, []).append({"id": m.id, "content": m.content})
        have = {m.metadata.get("url") for m in svc.store.list({SCOPE_WORKSPACE: ws},
                                                              ["document_summary"], MAX_LIST_LIMIT)}
        cands = [{"url": u, "chunks": c} for u, c in docs.items() if u not in have]
        return web.json_response({"candidates": cands, "total": len(cands)})

    async def save_doc_summary(request):
        d = await _body(request)
        ws = d.get("workspace_id")
        if not ws or not d.get("content"):
            return _err(400, "workspace_id and content are required")
        mem = Memory(type="document_summary", content=d["content"], confidence=0.9,
                     scope={SCOPE_WORKSPACE: ws}, title=d.get("title", ""),
                     metadata={META_ABOUT_KIND: "document_summary",
                               META_ABOUT_KEY: d.get("url", ""), "url": d.get("url", ""),
                               "source_type": "system_generated"})
        res = await svc.save(mem, require_user=False)
        return web.json_response({"id": res["id"]}, status=201)

    async def save_agent(request):
        d = await _body(request)
        scope = normalize_scope(d.get("scope"))
        if not scope.get(SCOPE_WORKSPACE) or not scope.get(SCOPE_AGENT):
            return _err(400, "scope.workspace_id and scope.agent_id are required")
        scope.pop(SCOPE_USER, None)
        mem = _memory_from_request(d, scope)
        mem.metadata.setdefault("source_type", "operator_curated")
        res = await svc.save(mem, require_user=False)
        return web.json_response({"memory": svc.store.get(res["id"]).to_json(),
                                  "action": res["action"]}, status=201)

    async def list_agent(request):
        q = request.query
        ws, agent = _trunc(q.get("workspace")), _trunc(q.get("agent"))
        if not ws or not agent:
            return _err(400, "workspace and agent are required")
        mems = svc.store.list({SCOPE_WORKSPACE: ws, SCOPE_AGENT: agent}, _types(q.get("type")),
                              min(max(_int(q, "limit", DEFAULT_LIST_LIMIT), 1), MAX_LIST_LIMIT),
                              _int(q, "offset", 0))
        return web.json_response(_list_json(mems))

    async def delete_agent(request):
        q = request.query
        m = svc.store.get(request.match_info["id"], q.get("workspace") or None)
        if m is None or m.tier != Tier.AGENT:
            return _err(404, "memory not found")
        await svc.forget(m.id)
        return web.Response(status=204)

    async def compaction_candidates(request):
        q = request.query
        ws = _trunc(q.get("workspace"))
        if not ws:
            return _err(400, "workspace is required")
        c = svc.store.compaction_candidates(ws, float(q.get("older_than_s") or 30 * R.DAY),
                                            _int(q, "min_count", 10), _int(q, "limit", 20))
        return web.json_response({"candidates": c, "total": len(c)})

    async def compaction_summary(request):
        d = await _body(request)
        src = d.get("source_ids") or []
        if not src or not d.get("content"):
            return _err(400, "source_ids and content are required")
        mem = _memory_from_request(d)
        mem.type = d.get("type") or "summary"
        mem.metadata.setdefault("source_type", "system_generated")
        res = await svc.supersede(src, mem)
        return web.json_response({"id": res["id"], "supersedes": src}, status=201)

    async def consent_event(request):
        d = await _body(request)
        # the privacy-api notifier's body is {"userId", "category"} with ?workspace=
        ws = d.get("workspace_id") or request.query.get("workspace") or ""
        user = d.get("virtual_user_id") or d.get("user_id") or d.get("userId")
        cat = d.get("category")
        if not (user and cat):
            return _err(400, "virtual_user_id and category are required")
        if (d.get("action") or "revoked") == "revoked":
            obs = []
            for w in ([ws] if ws else svc.store.list_workspace_ids()):
                obs += svc.store.revoke_consent(w, user, cat)
                await svc._invalidate(w)
            svc._drop_vectors(obs)
            return web.json_response({"deleted_observations": len(obs)})
        if not ws:
            return _err(400, "workspace_id is required to re-grant consent")
        with svc.store.lock:
            svc.store.db.execute("DELETE FROM consent_revocations WHERE workspace_id = ? AND "
                                 "virtual_user_id = ? AND category = ?", (ws, user, cat))
        return web.json_response({"status": "granted"})

    async def dim_change(request):
        d = await _body(request)
        t = int(d.get("target_dim") or 0)
        if not 1 <= t <= 2000:
            return _err(400, "target_dim must be in 1..2000")
        svc.store.record_dim_consent(t)
        return web.json_response({"target_dim": t, "status": "recorded"})

    async def stats(request):
        ws = _trunc(request.query.get("workspace"))
        if not ws:
            return _err(400, "workspace is required")
        return web.json_response(svc.stats(ws))

    async def openapi(_):
        paths = sorted({str(res.canonical) for res in app.router.resources()})
        return web.json_response({"openapi": "3.0.3", "info": {"title": "Omnia Memory API",
                                                               "version": "v1"},
                                  "paths": {p: {} for p in paths}})

    r.add_get("/healthz", healthz)
    r.add_get("/metrics", metrics)
    r.add_get("/api/v1/openapi.yaml", openapi)
    r.add_get("/api/v1/memories", list_memories)
    r.add_get("/api/v1/memories/search", search)
    r.add_get("/api/v1/memories/export", export)
    r.add_post("/api/v1/memories", save)
    r.add_get("/api/v1/memories/aggregate", ee(aggregate))
    r.add_get("/api/v1/memories/projection", ee(projection))
    r.add_get("/api/v1/memories/conflicts", conflicts)
    r.add_get("/api/v1/memories/stats", stats)
    r.add_post("/api/v1/memories/supersede", supersede)
    r.add_post("/api/v1/memories/retrieve", retrieve)
    r.add_post("/api/v1/memories/retrieve/semantic", retrieve_semantic)
    r.add_post("/api/v1/memories/consent-events", ee(consent_event))
    r.add_delete("/api/v1/memories/batch", delete_batch)
    r.add_get("/api/v1/memories/{id}", open_memory)
    r.add_patch("/api/v1/memories/{id}", update)
    r.add_delete("/api/v1/memories/{id}", delete_one)
    r.add_delete("/api/v1/memories", delete_all)
    r.add_post("/api/v1/relations", link)
    r.add_post("/api/v1/institutional/memories", ee(save_inst))
    r.add_get("/api/v1/institutional/memories", ee(list_inst))
    r.add_delete("/api/v1/institutional/memories/{id}", ee(delete_inst))
    r.add_post("/api/v1/institutional/ingest", ee(ingest))
    r.add_get("/api/v1/ingest/summary-candidates", summary_candidates)
    r.add_post("/api/v1/ingest/summaries", save_doc_summary)
    r.add_post("/api/v1/agent-memories", save_agent)
    r.add_get("/api/v1/agent-memories", list_agent)
    r.add_delete("/api/v1/agent-memories/{id}", delete_agent)
    r.add_get("/api/v1/compaction/candidates", compaction_candidates)
    r.add_post("/api/v1/compaction/summaries", compaction_summary)
    r.add_post("/admin/embedding-dimension-change", dim_change)
    app[SVC_KEY] = svc
    return app


def _project(svc: MemoryService, ws: str, user: str | None) -> dict:
    """Memory Galaxy (``ee/pkg/memory/projection``): the stored layout the
    projection worker rendered for this scope when there is one, else a live
    render (dense basis when >= 70 % of the rows carry embeddings, otherwise
    TF-IDF/LSA; PCA below 30 points, t-SNE on the device above).  PII-category
    points are masked server-side before serialisation (SERVICE.md "Memory
    Galaxy")."""
    from ..ee import projection as P

    inputs = P.gather_inputs(svc.store, ws, user)
    if not inputs:
        return {"points": [], "basis": "none"}
    stored = P.ProjectionStore(svc.store).load(P.scope_key(ws, user))
    res = P.from_stored(stored, inputs) if stored else P.project(inputs)
    if stored and not res["points"]:
        res = P.project(inputs, stored.get("coords"))
    cats = {i.entity_id: i.category for i in inputs}
    pts = []
    for p in res["points"]:
        if cats.get(p["id"]) in PII_CATEGORIES:
            pts.append({"x": p["x"], "y": p["y"], "tier": p["tier"],
                        "confidence": p["confidence"], "masked": True})
        else:
            pts.append(p)
    M.MEMORY_OPS.labels(op="projection", status=res["basis"]).inc()
    res["points"] = pts
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description="omnia memory-api")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--db", default=":memory:")
    ap.add_argument("--embedding", default="", help="hash | local | openai | ollama")
    ap.add_argument("--embedding-model", default="")
    ap.add_argument("--embedding-url", default="")
    ap.add_argument("--enterprise", action="store_true")
    ap.add_argument("--ingest-chunk-size", type=int, default=200)
    ap.add_argument("--ingest-chunk-overlap", type=int, default=40)
    ap.add_argument("--redis", default="", help="host:port for omnia:memory-events streams")
    ap.add_argument("--reembed-interval", type=float, default=5.0)
    ap.add_argument("--policy-file", default="",
                    help="MemoryPolicy spec (JSON; the operator's memory-policy-<name> ConfigMap)")
    ap.add_argument("--compaction-interval", default=os.environ.get("COMPACTION_INTERVAL", ""),
                    help="temporal-summarisation worker period (e.g. 6h); empty disables")
    ap.add_argument("--compaction-age", default=os.environ.get("COMPACTION_AGE", ""),
                    help="age threshold of compaction candidates (e.g. 720h)")
    ap.add_argument("--privacy-operator-url", default=os.environ.get("OMNIA_OPERATOR_URL", ""),
                    help="EE: redact writes under the SessionPrivacyPolicy watched here")
    ap.add_argument("--privacy-namespace", default=os.environ.get("OMNIA_NAMESPACE", ""))
    ap.add_argument("--privacy-workspace", default=os.environ.get("OMNIA_WORKSPACE", ""))
    ap.add_argument("--postgres-dsn", default=os.environ.get("MEMORY_POSTGRES_DSN", ""),
                    help="Postgres + pgvector store (needs a DB-API driver); default SQLite --db")
    ap.add_argument("--redis-cache", default=os.environ.get("MEMORY_CACHE_REDIS_URL", ""),
                    help="redis://host:port for the list / search read cache")
    ap.add_argument("--cache-ttl", type=int, default=300)
    ap.add_argument("--tombstone-interval", default=os.environ.get("TOMBSTONE_INTERVAL", ""),
                    help="tombstone GC period (e.g. 1h); empty disables")
    ap.add_argument("--tombstone-min-age", default=os.environ.get("TOMBSTONE_MIN_AGE", "720h"))
    ap.add_argument("--tombstone-min-inactive", type=int, default=20)
    ap.add_argument("--tombstone-keep-recent", type=int, default=5)
    ap.add_argument("--access-touch-interval", type=float,
                    default=float(os.environ.get("ACCESS_TOUCH_INTERVAL", "1.0")),
                    help="seconds per batched access-count flush; 0 = one update per read")
    ap.add_argument("--consolidation-interval",
                    default=os.environ.get("CONSOLIDATION_INTERVAL", ""),
                    help="EE consolidation worker tick (e.g. 1m); per-axis cron schedules "
                         "from the policy decide what runs; empty disables")
    ap.add_argument("--consolidation-function-url",
                    default=os.environ.get("CONSOLIDATION_FUNCTION_URL", ""),
                    help="base URL of the consolidation function facades (default: the "
                         "functionRef's in-cluster Service)")
    ap.add_argument("--projection-interval",
                    default=os.environ.get("PROJECTION_INTERVAL", "5m"),
                    help="Memory Galaxy render check period (policy spec.projection)")
    ap.add_argument("--policy-name", default=os.environ.get("OMNIA_MEMORY_POLICY", "default"))
    a = ap.parse_args(argv)
    from .embedding import build_embedder
    from .store import MemoryStore
    from .workers import ReembedWorker, RetentionWorker

    emb = build_embedder({"type": a.embedding, "model": a.embedding_model,
                          "baseURL": a.embedding_url}) if a.embedding else None
    pub = None
    if a.redis:
        from ..utils.resp import RedisClient

        url = a.redis if "://" in a.redis else f"redis://{a.redis}"
        rc = RedisClient(url)

        async def pub(stream, ev):
            await rc.xadd(stream, {"event": json.dumps(ev)}, maxlen=100_000)

    policy = None
    if a.policy_file:
        with open(a.policy_file) as f:
            policy = json.load(f)
    if a.postgres_dsn:
        from .sqldialect import MemoryPostgres, connect_postgres

        conn = connect_postgres(a.postgres_dsn)
        if conn is None:
            raise SystemExit("--postgres-dsn given but no Postgres DB-API driver is installed")
        store = MemoryStore(dialect=MemoryPostgres(paramstyle="format"), conn=conn)
    else:
        store = MemoryStore(a.db)
    if a.access_touch_interval > 0:
        store.enable_touch_batching(a.access_touch_interval)
    svc = MemoryService(store, emb, publisher=pub, enterprise=a.enterprise)
    if a.enterprise and policy:
        # EE recall bias + per-tier decay from the workspace's MemoryPolicy
        svc.policy_ranker = R.tier_ranker_from_policy(policy)
        svc.policy_half_life = R.half_life_from_policy(policy)
    if a.redis_cache:
        from ..utils.resp import RedisClient
        from .cache import CachedStore

        svc.cache = CachedStore(store, RedisClient(a.redis_cache), a.cache_ttl)
    app = build_app(svc, a.enterprise, a.ingest_chunk_size, a.ingest_chunk_overlap)
    watcher = None
    if a.privacy_operator_url:
        from ..ee.privacy.policy import HTTPSource, PolicyWatcher, memory_privacy_middleware

        watcher = PolicyWatcher(HTTPSource(a.privacy_operator_url), a.privacy_workspace,
                                a.privacy_namespace)
        app.middlewares.append(memory_privacy_middleware(watcher, a.privacy_namespace))
    if a.enterprise and emb is not None:
        from ..ee.privacy.classify import EmbeddingClassifier

        svc.embedding_classifier = EmbeddingClassifier(emb)
    tombstone = None
    if a.tombstone_interval:
        from ..utils.durations import parse_duration
        from .workers import TombstoneWorker

        tombstone = TombstoneWorker(svc, parse_duration(a.tombstone_interval),
                                    min_age_s=parse_duration(a.tombstone_min_age),
                                    min_inactive=a.tombstone_min_inactive,
                                    keep_recent=a.tombstone_keep_recent)
    compaction = None
    if a.compaction_interval:
        from ..utils.durations import parse_duration
        from .workers import CompactionWorker

        try:
            every = parse_duration(a.compaction_interval)
        except ValueError:
            every = 0
        if every > 0:
            kw = {}
            if a.compaction_age:
                try:
                    kw["older_than_s"] = parse_duration(a.compaction_age)
                except ValueError:
                    log.error("invalid compaction age %r, using the default", a.compaction_age)
            compaction = CompactionWorker(svc, interval=every, **kw)
        else:
            log.error("invalid compaction interval %r: worker disabled", a.compaction_interval)

    consolidation = None
    if a.consolidation_interval and a.enterprise and policy:
        from ..ee.consolidation import ConsolidationWorker, FunctionClient
        from ..utils.durations import parse_duration

        consolidation = ConsolidationWorker(
            store, [(a.policy_name, policy)], workspaces=lambda _p: store.list_workspace_ids(),
            client=FunctionClient(base_url=a.consolidation_function_url),
            interval_s=parse_duration(a.consolidation_interval))

    projection = None
    if a.enterprise and policy and (policy.get("projection") or {}).get("enabled"):
        from ..ee.projection import ProjectionWorker
        from ..utils.durations import parse_duration

        projection = ProjectionWorker(store, [(a.policy_name, policy)],
                                      workspaces=lambda _p: store.list_workspace_ids(),
                                      interval_s=parse_duration(a.projection_interval))

    async def start_workers(app):
        app["workers"] = [asyncio.create_task(ReembedWorker(svc, a.reembed_interval).run()),
                          asyncio.create_task(RetentionWorker(svc, policy=policy).run())]
        if watcher is not None:
            app["workers"].append(asyncio.create_task(watcher.run()))
        ec = getattr(svc, "embedding_classifier", None)
        if ec is not None:
            try:
                await ec.prewarm()  # exemplar centroids on the in-node embedder
            except Exception as e:  # noqa: BLE001 - rules-only classification then
                log.warning("embedding classifier prewarm failed: %s", e)
        if compaction is not None:
            app["workers"].append(asyncio.create_task(compaction.run()))
        if tombstone is not None:
            app["workers"].append(asyncio.create_task(tombstone.run()))
        if consolidation is not None:
            app["workers"].append(asyncio.create_task(consolidation.run()))
        if projection is not None:
            app["workers"].append(asyncio.create_task(projection.run()))

    async def stop_workers(app):
        for t in app.get("workers", []):
            t.cancel()
        if store.touch_batcher is not None:
            store.touch_batcher.stop()

    app.on_startup.append(start_workers)
    app.on_cleanup.append(stop_workers)
    configure_logging()
    web.run_app(app, host=a.host, port=a.port)


if __name__ == "__main__":
    main()
