"""session-api service (``cmd/session-api``, ``internal/session/api``).

REST over the tiered store; message appends publish ``message.appended`` events
to Redis Streams ``omnia:eval-events:<namespace>``
(``internal/session/api/event_publisher.go:34,91-98``) for the eval worker;
per-client-IP rate limiting; optional service-account bearer auth with
subject / namespace allowlists (TokenReview stand-in: a static token map);
EE middleware hooks for PII redaction and privacy opt-out.

``python -m omnia_amd.session.api --port 8300 --db /var/lib/omnia/sessions.db``
"""
from __future__ import annotations

import argparse
import os
import asyncio
import json
import logging
import time

from aiohttp import web

from ..observability import metrics as M
from ..utils.ratelimit import KeyedLimiter
from .model import (EvalResult, Message, ProviderCall, RuntimeEvent, Session, ToolCall,
                    STATUS_ACTIVE, TERMINAL)
from .store import ColdArchive, HotCache, LocalBlobStore, TierError, TieredSessionService, WarmStore

log = logging.getLogger("omnia.session.api")


class StreamPublisher:
    """XADD to omnia:eval-events:<ns> (MAXLEN ~ 100k)."""

    def __init__(self, redis_client, maxlen: int = 100_000):
        self.r = redis_client
        self.maxlen = maxlen

    async def __call__(self, ev: dict):
        ns = ev.get("namespace") or "default"
        try:
            await self.r.xadd(f"omnia:eval-events:{ns}", {"event": json.dumps(ev)},
                              maxlen=self.maxlen)
        except Exception as e:  # noqa: BLE001 - publishing is best effort
            log.debug("event publish failed: %s", e)


class MemoryPublisher:
    def __init__(self):
        self.events: list[dict] = []

    async def __call__(self, ev):
        self.events.append(ev)


def session_resolver(svc: TieredSessionService, cache_size: int = 10000):
    """session id -> (namespace, agent) for the privacy middleware (bounded cache,
    ``session_cache.go``)."""
    cache: dict[str, tuple[str, str]] = {}

    def resolve(sid: str):
        hit = cache.get(sid)
        if hit is not None:
            return hit
        try:
            v = svc.get(sid, with_messages=False)
        except Exception:  # noqa: BLE001 - unknown / unreadable: no policy applies
            return None
        if v is None:
            return None
        s = v[0]
        if len(cache) >= cache_size:
            cache.pop(next(iter(cache)))
        cache[sid] = (s.namespace, s.agent_name)
        return cache[sid]

    return resolve


def _bad(msg: str):
    return web.HTTPBadRequest(text=json.dumps({"error": msg}), content_type="application/json")


async def _json_obj(request, lists: bool = False):
    """The request body as a JSON object (or, with ``lists``, an array), or 400."""
    try:
        body = await request.json()
    except (ValueError, UnicodeDecodeError) as e:
        raise _bad(f"invalid JSON body: {e}") from None
    if not isinstance(body, dict) and not (lists and isinstance(body, list)):
        raise _bad("request body must be a JSON object")
    return body


def _num(v, kind, name: str):
    """``kind(v)`` for a query / body field, or 400 (finite values only)."""
    try:
        x = kind(v)
    except (TypeError, ValueError, OverflowError):
        raise _bad(f"{name} must be a number") from None
    if kind is float and (x != x or x in (float("inf"), float("-inf"))):
        raise _bad(f"{name} must be finite")
    return x


def _model(cls, d):
    """``cls.from_json(d)`` with a wrongly typed field answered as 400."""
    try:
        return cls.from_json(d)
    except (ValueError, TypeError) as e:
        raise _bad(str(e)) from None


def build_app(svc: TieredSessionService, rate: float = 200.0, burst: float = 400.0,
              tokens: dict | None = None, allowed_namespaces: set | None = None,
              redactor=None, optout=None, audit_logger=None, media_deleter=None,
              privacy_middleware=None, retention: dict | None = None,
              policy_resolver=None) -> web.Application:
    """``audit_logger`` (EE, :class:`omnia_amd.ee.audit.AuditLogger`): record
    session created/accessed/searched/deleted events and serve them at
    ``/api/v1/audit/sessions`` (reference session-api audit wiring)."""
    limiter = KeyedLimiter(rate, burst)

    def audit(request, event, **kw):
        if audit_logger is None:
            return
        from ..ee.audit import Entry

        audit_logger.log_event(Entry(event, ipAddress=request.remote or "",
                                     userAgent=request.headers.get("User-Agent", ""),
                                     userId=request.headers.get("x-omnia-user-id", ""), **kw))

    @web.middleware
    async def count(request, handler):
        route = request.match_info.route.resource
        name = route.canonical if route is not None else "?"
        status = 500
        try:
            resp = await handler(request)
            status = resp.status
            return resp
        except web.HTTPException as e:
            status = e.status
            raise
        finally:
            M.SESSION_API_REQUESTS.labels(request.method, name, str(status)).inc()

    @web.middleware
    async def guard(request, handler):
        if request.path in ("/healthz", "/metrics"):
            return await handler(request)
        if not limiter.allow(request.remote or "?"):
            return web.json_response({"error": "rate_limited"}, status=429)
        if tokens is not None:
            h = request.headers.get("Authorization", "")
            tok = h[7:] if h.lower().startswith("bearer ") else ""
            ident = tokens.get(tok)
            if ident is None:
                return web.json_response({"error": "unauthorized"}, status=401)
            sa_ns = ident.split(":")[2] if ident.count(":") >= 3 else ""
            if allowed_namespaces is not None and sa_ns not in allowed_namespaces \
                    and ident not in allowed_namespaces:
                return web.json_response({"error": "forbidden"}, status=403)
        return await handler(request)

    mws = [count, guard] + ([privacy_middleware] if privacy_middleware is not None else [])
    app = web.Application(middlewares=mws, client_max_size=32 * 2**20)
    r = app.router

    def nf(sid):
        return web.json_response({"error": "session_not_found", "sessionId": sid}, status=404)

    async def healthz(_):
        return web.json_response({"status": "ok"})

    async def create(request):
        body = await _json_obj(request)
        s = _model(Session, body)
        if optout is not None and optout(s):
            return web.Response(status=204)
        s = svc.create(s)
        audit(request, "session_created", sessionId=s.id, agentName=s.agent_name,
              namespace=s.namespace)
        return web.json_response(s.to_json(), status=201)

    async def list_sessions(request):
        q = request.query
        rows = svc.warm.list_sessions(namespace=q.get("namespace"), agent=q.get("agent"),
                                      status=q.get("status"), user=q.get("user"),
                                      before=_num(q["before"], float, "before") if q.get("before") else None,
                                      after=_num(q["after"], float, "after") if q.get("after") else None,
                                      limit=_num(q.get("limit", 100), int, "limit"),
                                      offset=_num(q.get("offset", 0), int, "offset"), q=q.get("q"))
        return web.json_response({"sessions": [s.to_json() for s in rows],
                                  "total": len(rows)})

    async def search(request):
        q = request.query
        rows = svc.warm.list_sessions(namespace=q.get("namespace"), agent=q.get("agent"),
                                      q=q.get("q", ""), limit=_num(q.get("limit", 50), int, "limit"))
        audit(request, "session_searched", query=q.get("q", ""), resultCount=len(rows),
              namespace=q.get("namespace") or "")
        return web.json_response({"sessions": [s.to_json() for s in rows]})

    async def get(request):
        sid = request.match_info["id"]
        audit(request, "session_accessed", sessionId=sid)
        try:
            v = svc.get(sid, with_messages=False)
        except TierError:
            return web.json_response({"error": "store_unavailable"}, status=503)
        if v is None:
            return nf(sid)
        return web.json_response(v[0].to_json())

    async def get_messages(request):
        sid = request.match_info["id"]
        try:
            v = svc.get(sid)
        except TierError:
            return web.json_response({"error": "store_unavailable"}, status=503)
        if v is None:
            return nf(sid)
        msgs = v[1]
        lim = _num(request.query.get("limit", 1000), int, "limit")
        off = _num(request.query.get("offset", 0), int, "offset")
        return web.json_response({"messages": [m.to_json() for m in msgs[off:off + lim]]})

    async def append(request):
        sid = request.match_info["id"]
        body = await _json_obj(request)
        m = _model(Message, body)
        if redactor is not None:
            m.content = redactor(m.content)
        try:
            m = await svc.append_message(sid, m)
        except KeyError:
            return nf(sid)
        return web.json_response(m.to_json(), status=201)

    def recorder(table, cls):
        async def post(request):
            sid = request.match_info["id"]
            body = await _json_obj(request)
            obj = _model(cls, {**body, "sessionId": sid})
            try:
                svc.record(table, sid, obj)
            except KeyError:
                return nf(sid)
            return web.json_response(obj.to_json(), status=201)

        async def get_(request):
            sid = request.match_info["id"]
            return web.json_response({table.replace("_", "-"): svc.warm.list_rows(table, sid)})

        return post, get_

    async def eval_results_post(request):
        body = await _json_obj(request, lists=True)
        items = body if isinstance(body, list) else body.get("results", [body])
        if not isinstance(items, list):
            raise _bad("results must be an array")
        out = []
        for it in items:
            e = _model(EvalResult, it)
            try:
                svc.record("eval_results", e.session_id, e)
            except KeyError:
                return nf(e.session_id)
            out.append(e.to_json())
        return web.json_response({"results": out}, status=201)

    async def eval_results_list(request):
        """GET /api/v1/eval-results?passed=&evalId=&limit=&offset= across sessions."""
        qs = request.query
        passed = None
        if qs.get("passed") not in (None, ""):
            passed = qs["passed"].lower() in ("1", "true", "yes")
        try:
            limit = max(1, min(1000, _num(qs.get("limit", 100), int, "limit")))
            offset = max(0, _num(qs.get("offset", 0), int, "offset"))
        except ValueError:
            return web.json_response({"error": "invalid limit/offset"}, status=400)
        rows = svc.warm.list_eval_results(passed, qs.get("evalId") or None, limit, offset)
        return web.json_response({"results": rows})

    async def eval_results_summary(request):
        sid = request.match_info["id"]
        rows = svc.warm.list_rows("eval_results", sid)
        total = len(rows)
        passed = sum(1 for r in rows if r.get("passed"))
        return web.json_response({"sessionId": sid, "total": total, "passed": passed,
                                  "passRate": passed / total if total else 0.0})

    async def eval_aggregate(request):
        return web.json_response({"evals": svc.warm.aggregate_evals(
            request.query.get("namespace"))})

    async def provider_aggregate(request):
        return web.json_response({"groups": svc.warm.aggregate_provider_calls(
            request.query.get("namespace"), request.query.get("groupBy", "model"))})

    async def provider_usage(request):
        body = await _json_obj(request)
        ws = body.get("workspace") or ""
        if not isinstance(ws, str):
            raise _bad("workspace must be a string")
        svc.warm.provider_usage(ws, body)
        return web.json_response({"ok": True}, status=201)

    async def ttl(request):
        sid = request.match_info["id"]
        body = await _json_obj(request)
        try:
            s = svc.refresh_ttl(sid, _num(body.get("ttlSeconds", svc.default_ttl_s), float,
                                         "ttlSeconds"))
        except KeyError:
            return nf(sid)
        return web.json_response(s.to_json())

    async def status(request):
        sid = request.match_info["id"]
        body = await _json_obj(request)
        st = body.get("status", STATUS_ACTIVE)
        if st not in TERMINAL | {STATUS_ACTIVE}:
            return web.json_response({"error": "invalid_status"}, status=400)
        prev = svc._get_session_only(sid)
        prev = prev.status if prev is not None else ""  # captured before the in-place update
        try:
            s = svc.update_status(sid, st, body.get("endedAt"))
        except KeyError:
            return nf(sid)
        await svc.publish_completed_if(prev, s)
        return web.json_response(s.to_json())

    async def evaluate(request):
        """POST /api/v1/sessions/{id}/evaluate (handler.go:265): 202 + a
        ``session.evaluate`` event for the eval worker."""
        sid = request.match_info["id"]
        try:
            await svc.publish_evaluate(sid)
        except KeyError:
            return nf(sid)
        except (RuntimeError, ValueError) as e:
            return web.json_response({"error": str(e)}, status=409)
        return web.json_response({"sessionId": sid, "status": "queued"}, status=202)

    async def decorate(request):
        sid = request.match_info["id"]
        body = await _json_obj(request)
        try:
            s = svc.decorate(sid, body.get("tags"), body.get("state"))
        except KeyError:
            return nf(sid)
        return web.json_response(s.to_json())

    async def delete(request):
        sid = request.match_info["id"]
        if svc.delete(sid):
            audit(request, "session_deleted", sessionId=sid)
            return web.Response(status=204)
        return nf(sid)

    async def bulk_delete(request):
        ns = request.query.get("namespace")
        if not ns:
            return web.json_response({"error": "namespace required"}, status=400)
        before = _num(request.query["before"], float, "before") \
            if request.query.get("before") else None
        rows = svc.warm.list_sessions(namespace=ns, agent=request.query.get("agent"),
                                      before=before, limit=100000)
        n = sum(1 for s in rows if svc.delete(s.id))
        M.RETENTION_DELETED.labels("warm").inc(n)
        return web.json_response({"deleted": n})

    async def delete_by_user(request):
        """Session-tier DSAR (``session_erase_handler.go``): the user's sessions,
        optionally one workspace / a created-at range, and their media."""
        from ..ee.privacy.erasure import EraseScope, SessionTierEraser

        body = await _json_obj(request)
        uid = body.get("virtual_user_id", "")
        if not uid:
            return web.json_response({"error": "virtual_user_id required"}, status=400)

        def ts(v):
            if v in (None, ""):
                return None
            if isinstance(v, (int, float)):
                return float(v)
            import datetime as dt

            return dt.datetime.fromisoformat(str(v).replace("Z", "+00:00")).timestamp()

        try:
            scope = EraseScope(uid, body.get("workspace") or "", ts(body.get("date_from")),
                               ts(body.get("date_to")))
        except ValueError as e:
            return web.json_response({"error": f"bad date: {e}"}, status=400)
        res = await SessionTierEraser(svc, media_deleter).erase(scope)
        return web.json_response(res)

    async def metrics(_):
        return web.Response(body=M.exposition(), content_type="text/plain")

    async def compact(request):
        """One compaction run (warm -> cold archival, warm purge, cold expiry) on
        this replica's tiers -- what the workspace's compaction CronJob calls
        (``python -m omnia_amd.session.compaction --session-api URL``).  Body:
        optional ``warmRetentionSeconds`` / ``coldRetentionSeconds`` / ``dryRun``
        overriding the mounted SessionRetentionPolicy."""
        from .compaction import CompactionConfig, CompactionEngine

        try:
            body = await _json_obj(request) if request.can_read_body else {}
        except ValueError:
            return web.json_response({"error": "body must be JSON"}, status=400)
        ret = retention or {}
        try:
            cfg = CompactionConfig(
                float(body.get("warmRetentionSeconds", ret.get("warm_retention_s", 7 * 86400))),
                float(body.get("coldRetentionSeconds",
                               ret.get("cold_retention_s", 365 * 86400))),
                dry_run=bool(body.get("dryRun", False)))
        except (TypeError, ValueError):
            return web.json_response({"error": "retention must be a number"}, status=400)
        if cfg.warm_retention_s < 0 or cfg.cold_retention_s < 0:
            return web.json_response({"error": "retention must be >= 0"}, status=400)
        res = await asyncio.to_thread(CompactionEngine(svc.warm, svc.cold, svc.hot, cfg).run)
        return web.json_response({"archived": res.archived, "purged": res.purged,
                                  "coldExpired": res.cold_expired, "skipped": res.skipped,
                                  "errors": res.errors, "coldArchive": svc.cold is not None},
                                 status=500 if res.errors else 200)

    async def openapi(_):
        routes = sorted({(rt.method, rt.resource.canonical) for rt in app.router.routes()
                         if rt.resource is not None and rt.method != "HEAD"})
        paths: dict = {}
        for method, path in routes:
            paths.setdefault(path, {})[method.lower()] = {"responses": {"200": {
                "description": "ok"}}}
        return web.json_response({"openapi": "3.0.3", "info": {"title": "Omnia Session API",
                                                               "version": "v1"},
                                  "paths": paths})

    r.add_get("/healthz", healthz)
    r.add_get("/metrics", metrics)
    r.add_get("/api/v1/openapi.json", openapi)
    if audit_logger is not None:
        from ..ee.audit import mount_routes

        mount_routes(app, audit_logger)
    r.add_post("/api/v1/sessions", create)
    r.add_get("/api/v1/sessions", list_sessions)
    r.add_delete("/api/v1/sessions", bulk_delete)
    r.add_get("/api/v1/sessions/search", search)
    r.add_get("/api/v1/sessions/{id}", get)
    r.add_delete("/api/v1/sessions/{id}", delete)
    r.add_get("/api/v1/sessions/{id}/messages", get_messages)
    r.add_post("/api/v1/sessions/{id}/messages", append)
    for path, table, cls in (("tool-calls", "tool_calls", ToolCall),
                             ("provider-calls", "provider_calls", ProviderCall),
                             ("events", "events", RuntimeEvent)):
        p, g = recorder(table, cls)
        r.add_post(f"/api/v1/sessions/{{id}}/{path}", p)
        r.add_get(f"/api/v1/sessions/{{id}}/{path}", g)
    async def privacy_policy(request):
        # GET /api/v1/privacy-policy?namespace=&agent= (internal/session/api/handler.go
        # handleGetPrivacyPolicy): the facade-visible subset -- the recording block
        # -- of the effective SessionPrivacyPolicy; 204 when none applies or no
        # resolver is wired (non-enterprise), never 404
        if policy_resolver is None:
            return web.Response(status=204)
        ns = request.query.get("namespace", "")
        agent = request.query.get("agent", "")
        eff = policy_resolver(ns, agent)
        if not eff:
            return web.Response(status=204)
        rec = dict(eff.get("recording") or {})
        out = {"enabled": bool(rec.get("enabled", True)),
               "facadeData": bool(rec.get("facadeData", True)),
               "runtimeData": bool(rec.get("runtimeData", True))}
        for k, v in rec.items():  # any further recording fields, never encryption
            out.setdefault(k, v)
        return web.json_response({"recording": out})

    r.add_get("/api/v1/privacy-policy", privacy_policy)
    r.add_post("/api/v1/eval-results", eval_results_post)
    r.add_get("/api/v1/eval-results", eval_results_list)
    r.add_post("/api/v1/sessions/{id}/evaluate", evaluate)
    r.add_get("/api/v1/eval-results/aggregate", eval_aggregate)
    r.add_get("/api/v1/sessions/{id}/eval-results",
              lambda req: _rows(svc, "eval_results", req))
    r.add_get("/api/v1/sessions/{id}/eval-results/summary", eval_results_summary)
    r.add_get("/api/v1/provider-calls/aggregate", provider_aggregate)
    r.add_post("/api/v1/provider-usage", provider_usage)
    r.add_post("/api/v1/sessions/{id}/ttl", ttl)
    r.add_patch("/api/v1/sessions/{id}/status", status)
    r.add_patch("/api/v1/sessions/{id}/stats", status)
    r.add_patch("/api/v1/sessions/{id}/decorate", decorate)
    r.add_post("/api/v1/privacy/sessions/delete-by-user", delete_by_user)
    r.add_post("/api/v1/admin/compaction", compact)
    return app


async def _rows(svc, table, request):
    sid = request.match_info["id"]
    return web.json_response({"results": svc.warm.list_rows(table, sid)})


def main(argv=None):
    ap = argparse.ArgumentParser("session-api")
    ap.add_argument("--port", type=int, default=8300)
    ap.add_argument("--db", default=":memory:")
    ap.add_argument("--cold-dir", default=os.environ.get("OMNIA_SESSION_COLD_DIR", ""),
                    help="local-directory cold archive (single-node deployments)")
    # cmd/session-api/main.go:120-155: object-store cold archive (env fallbacks)
    ap.add_argument("--cold-backend", default=os.environ.get("COLD_BACKEND", ""),
                    help="s3 | gcs | azure")
    ap.add_argument("--cold-bucket", default=os.environ.get("COLD_BUCKET", ""))
    ap.add_argument("--cold-region", default=os.environ.get("COLD_REGION", ""))
    ap.add_argument("--cold-endpoint", default=os.environ.get("COLD_ENDPOINT", ""))
    ap.add_argument("--cold-prefix", default=os.environ.get("COLD_PREFIX", "sessions/"))
    ap.add_argument("--redis-url", default="")
    ap.add_argument("--ttl", type=float, default=24 * 3600)
    ap.add_argument("--audit-db", default="", help="EE: enable the audit log (SQLite path)")
    ap.add_argument("--audit-retention-days", type=int, default=0)
    ap.add_argument("--audit-hub", default="", help="EE: privacy-api URL to forward audit to")
    ap.add_argument("--retention-config", default="",
                    help="retention.yaml of a SessionRetentionPolicy: hot-cache sizing and "
                         "an in-process compaction loop with its warm/cold retention")
    ap.add_argument("--compaction-interval", type=float, default=3600.0)
    ap.add_argument("--otlp-enabled", action="store_true",
                    default=os.environ.get("OTLP_ENABLED", "").lower() == "true")
    ap.add_argument("--otlp-grpc-port", type=int,
                    default=int(os.environ.get("OTLP_GRPC_PORT", 4317)))
    ap.add_argument("--otlp-http-port", type=int,
                    default=int(os.environ.get("OTLP_HTTP_PORT", 4318)))
    ap.add_argument("--encryption-provider", default=os.environ.get("ENCRYPTION_PROVIDER", ""),
                    help="EE: encrypt message content/metadata at rest (local | vault | ...)")
    ap.add_argument("--encryption-key-id", default=os.environ.get("ENCRYPTION_KEY_ID", "local"))
    ap.add_argument("--encryption-key-file", default=os.environ.get("ENCRYPTION_KEY_FILE", ""),
                    help="local provider: versioned KEK ring (rotated by the key-rotation "
                         "controller)")
    ap.add_argument("--media-root", default=os.environ.get("OMNIA_MEDIA_ROOT", ""),
                    help="local media store root: DSAR erasure deletes each session's media")
    ap.add_argument("--privacy-operator-url", default=os.environ.get("OMNIA_OPERATOR_URL", ""),
                    help="EE: watch SessionPrivacyPolicies through this API server and "
                         "enforce them on writes")
    ap.add_argument("--privacy-namespace", default=os.environ.get("OMNIA_NAMESPACE", ""))
    ap.add_argument("--privacy-workspace", default=os.environ.get("OMNIA_WORKSPACE", ""))
    ap.add_argument("--privacy-api-url", default=os.environ.get("OMNIA_PRIVACY_API_URL", ""),
                    help="EE: opt-out lookups for the privacy middleware")
    ap.add_argument("--tokens-file", default=os.environ.get("OMNIA_SESSION_API_TOKENS_FILE", ""),
                    help="JSON {bearer token: service-account identity}; enables auth on the "
                         "REST and both OTLP listeners")
    a = ap.parse_args(argv)
    tokens = None
    if a.tokens_file:
        with open(a.tokens_file) as f:
            tokens = {str(k): str(v) for k, v in json.load(f).items()}
    cold = ColdArchive(LocalBlobStore(a.cold_dir)) if a.cold_dir else None
    if a.cold_backend and a.cold_bucket:
        from .blobstores import build_cold_blobstore

        cold = ColdArchive(build_cold_blobstore(a.cold_backend, a.cold_bucket, a.cold_region,
                                                a.cold_endpoint, a.cold_prefix))
    pub = None
    if a.redis_url:
        from ..utils.resp import RedisClient

        pub = StreamPublisher(RedisClient(a.redis_url))
    if a.db.startswith(("postgres://", "postgresql://")):
        warm = WarmStore.postgres(a.db)  # weekly-partitioned tables (sqldialect.py)
        from .sqldialect import PartitionManager

        def _pg(sql):
            with warm.lock:
                return warm._run(sql, ())

        PartitionManager(_pg, warm.d).ensure_ahead(2)
    else:
        warm = WarmStore(a.db)
    retention = {}
    if a.retention_config:
        import yaml

        from ..operator.policies import retention_from_config

        with open(a.retention_config) as f:
            retention = retention_from_config(yaml.safe_load(f) or {})
    hot = HotCache(max_sessions=retention.get("hot_max_sessions", 10000),
                   ttl_s=retention.get("hot_ttl_s", 3600),
                   max_messages=retention.get("hot_max_messages", 200))
    svc = TieredSessionService(hot, warm, cold, a.ttl, pub)
    if a.encryption_provider:
        from ..ee.encryption import Encryptor, build_provider

        svc.encryptor = Encryptor(build_provider({"type": a.encryption_provider,
                                                  "keyID": a.encryption_key_id,
                                                  "keyFile": a.encryption_key_file or None}))
    audit_logger = None
    app_kw = {"tokens": tokens}
    if a.audit_db:
        from ..ee.audit import AuditLogger, Forwarder

        audit_logger = AuditLogger(a.audit_db, retention_days=a.audit_retention_days)
        app_kw["audit_logger"] = audit_logger
    if a.media_root:
        from ..ee.privacy.erasure import LocalMediaDeleter

        app_kw["media_deleter"] = LocalMediaDeleter(a.media_root)
    watcher = None
    if a.privacy_operator_url:
        from ..ee.privacy.policy import (HTTPSource, PolicyWatcher, PrivacyPrefsClient,
                                         session_privacy_middleware)

        watcher = PolicyWatcher(HTTPSource(a.privacy_operator_url), a.privacy_workspace,
                                a.privacy_namespace)
        app_kw["privacy_middleware"] = session_privacy_middleware(
            watcher, session_resolver(svc),
            PrivacyPrefsClient(a.privacy_api_url) if a.privacy_api_url else None)
        app_kw["policy_resolver"] = watcher.effective
    app = build_app(svc, retention=retention, **app_kw)
    if watcher is not None:
        async def watch(_app):
            import asyncio

            task = asyncio.create_task(watcher.run())
            yield
            task.cancel()

        app.cleanup_ctx.append(watch)
    if audit_logger is not None and a.audit_hub:
        fw = Forwarder(audit_logger, a.audit_hub)

        async def forward_loop(_app):
            async def loop():
                import asyncio

                while True:
                    await fw.drain_once()
                    audit_logger.delete_expired()
                    await asyncio.sleep(10)

            import asyncio

            task = asyncio.create_task(loop())
            yield
            task.cancel()

        app.cleanup_ctx.append(forward_loop)
    if retention:
        async def compaction_loop(_app):
            from .compaction import CompactionConfig, CompactionEngine

            eng = CompactionEngine(warm, cold, hot, CompactionConfig(
                retention.get("warm_retention_s", 7 * 86400),
                retention.get("cold_retention_s", 365 * 86400)))

            async def loop():
                while True:
                    await asyncio.sleep(a.compaction_interval)
                    try:
                        await asyncio.to_thread(eng.run)
                    except Exception as e:  # noqa: BLE001
                        logging.getLogger("omnia.session").warning("compaction failed: %s", e)

            task = asyncio.create_task(loop())
            yield
            task.cancel()

        app.cleanup_ctx.append(compaction_loop)
    if a.otlp_enabled:
        async def otlp_servers(_app):
            from .otlp import Transformer, build_otlp_app, serve_otlp_grpc

            tr = Transformer(svc)
            runner = web.AppRunner(build_otlp_app(tr, tokens=tokens))
            await runner.setup()
            await web.TCPSite(runner, "0.0.0.0", a.otlp_http_port).start()
            grpc_srv, _ = await serve_otlp_grpc(tr, a.otlp_grpc_port, tokens=tokens)
            yield
            await grpc_srv.stop(1)
            await runner.cleanup()

        app.cleanup_ctx.append(otlp_servers)
    web.run_app(app, port=a.port)


if __name__ == "__main__":
    main()
