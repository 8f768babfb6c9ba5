"""Operator dashboard (minimal).

The reference dashboard is a ~124K-line Next.js app (``dashboard/``): workspace
resource browser, agent status, session viewer, a WebSocket console to an
agent's facade, arena and consent UIs.  This is the serving-side core of it as
one dependency-free page plus a small aiohttp backend:

* ``GET /api/resources/{plural}`` proxies the operator REST API (K8s-style);
* ``GET /api/sessions`` proxies session-api search (``/api/v1/sessions``) and
  ``GET /api/sessions/{id}/messages`` one session's transcript;
* ``GET /api/overview`` -- AgentRuntime phase / replicas / engine summary;
* ``GET /api/arena/jobs`` -- ArenaJobs with type, phase and result summary;
* ``GET /api/consent/{user}`` -- the privacy API's consent record (read-only);
* costs, quality, memories, memory analytics, privacy stats (workspace-scoped
  ``/api/workspaces/{ws}/...``), topology, tools, skills and settings views:
  ``dashboard_views.py``;
* ``/`` -- the page: resource tables, session list, and a chat console;
* ``GET /api/auth/jwks`` -- the management-plane signing key set (public, the
  agents' facades fetch it: ``OMNIA_MGMT_PLANE_JWKS_URL``);
* ``GET /api/agents/{ns}/{name}/ws`` -- the console's WebSocket, proxied to the
  agent's management-plane twin (``status.managementEndpoints.ws``, port 18080)
  with a freshly minted RS256 JWT (origin ``management-plane``, the agent /
  workspace claims, the caller's subject): the browser never holds a token the
  agent's public listener would accept (``dashboard/SERVICE.md``, WS proxy).
  The browser's ``Origin`` must be the dashboard's own (or ``--allowed-origin``).
  Under OIDC the page first ``POST``s ``/api/agents/{ns}/{name}/ws-ticket`` with
  its bearer and connects with the one-time ``?ticket=``; without OIDC the
  console is closed unless ``--open-console`` (loopback only).
  The signing key's ``kid`` is its RFC 7638 thumbprint by default.

Management writes (``--allow-writes``; off by default):

* ``POST /api/resources/{plural}`` -- create an object from a JSON or YAML body
  (the API server's admission -- schemas, CEL rules, webhooks -- applies);
* ``DELETE /api/resources/{plural}/{ns}/{name}``;
* ``POST /api/agents/{ns}/{name}/scale`` ``{"replicas": n}`` -- merge-patches
  ``spec.runtime.replicas``;
* ``POST /api/arena/jobs/{ns}/{name}/cancel`` -- sets ``spec.cancelled``.

With ``--oidc-jwks-file`` every ``/api/*`` route requires an IdP-issued bearer
JWT (RS256, issuer / audience checked) and the caller's bearer is forwarded to
the API server -- the dashboard holds no credentials of its own to lend to
callers.  Write routes are guarded independently of the API server:

* ``--allow-writes`` refuses to start without OIDC (``--insecure-dev-writes``
  lifts that for a dashboard bound to loopback only);
* the caller's token must carry a write group (``--oidc-write-group``, default
  ``omnia-admin``) in its ``groups`` or ``roles`` claim -- an authenticated
  read-only user cannot write;
* a write must be ``application/json`` / ``application/yaml`` (a cross-site
  form or ``text/plain`` POST cannot be sent without a CORS preflight, which the
  dashboard never answers) and, when the browser sends ``Origin``, it must be
  the dashboard's own origin (or ``--allowed-origin``).
Run: ``python -m omnia_amd.operator.dashboard --port 3000 --api http://operator:8090``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import urllib.parse

import aiohttp
from aiohttp import web

from ..api import crds

PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>Omnia (MI355X)</title>
<style>body{font:14px system-ui;margin:24px;color:#222}table{border-collapse:collapse;margin:8px 0}
td,th{border:1px solid #ccc;padding:4px 8px}th{background:#f3f3f3}#log{height:240px;overflow:auto;
border:1px solid #ccc;padding:6px;white-space:pre-wrap}</style></head><body>
<h1>Omnia &mdash; MI355X agent platform</h1>
<h2>Agents</h2><table id="agents"><tr><th>namespace</th><th>name</th><th>phase</th>
<th>replicas</th><th>provider</th></tr></table>
<h2>Resources</h2><select id="kind"></select><table id="res"></table>
<h3>Apply</h3><textarea id="yaml" rows="8" cols="80" placeholder="YAML or JSON object"></textarea><br>
<button onclick="applyObj()">create</button> <span id="applied"></span>
<h2>Sessions</h2><table id="sess"><tr><th>id</th><th>agent</th><th>messages</th></tr></table>
<pre id="msgs"></pre>
<h2>Arena</h2><table id="arena"><tr><th>namespace</th><th>name</th><th>type</th><th>phase</th>
<th>result</th></tr></table>
<h2>Consent</h2><input id="cuser" placeholder="user id"><button onclick="consent()">lookup</button>
<pre id="cons"></pre>
<h2>Console</h2><input id="ws" size="40" value="/api/agents/default/agent/ws">
<button onclick="conn()">connect</button><br><input id="msg" size="60">
<button onclick="send()">send</button><div id="log"></div>
<script>
const KINDS=__KINDS__;let sock;
async function j(u){const r=await fetch(u);return r.json()}
async function applyObj(){const k=document.getElementById('kind').value;
 const r=await fetch('/api/resources/'+k,{method:'POST',headers:{'Content-Type':'application/yaml'},body:document.getElementById('yaml').value});
 const o=await r.json();document.getElementById('applied').textContent=r.status+' '+(o.error||o.message||(o.metadata||{}).name||'')}
async function agents(){const o=await j('/api/overview');const t=document.getElementById('agents');
 for(const a of o.agents){const r=t.insertRow();for(const v of [a.namespace,a.name,a.phase,a.replicas,a.provider])
 r.insertCell().textContent=v??''}}
async function res(){const k=document.getElementById('kind').value;const o=await j('/api/resources/'+k);
 const t=document.getElementById('res');t.innerHTML='<tr><th>namespace</th><th>name</th><th>phase</th></tr>';
 for(const it of (o.items||[])){const r=t.insertRow();r.insertCell().textContent=it.metadata.namespace||'';
 r.insertCell().textContent=it.metadata.name;r.insertCell().textContent=(it.status||{}).phase||''}}
async function msgs(id){const o=await j('/api/sessions/'+encodeURIComponent(id)+'/messages');
 document.getElementById('msgs').textContent=(o.messages||[]).map(m=>m.role+': '+m.content).join('\\n')}
async function sess(){const o=await j('/api/sessions');const t=document.getElementById('sess');
 for(const s of (o.sessions||[])){const r=t.insertRow();for(const v of [s.id,s.agent_name,s.message_count])
 r.insertCell().textContent=v;r.onclick=()=>msgs(s.id)}}
async function arena(){const o=await j('/api/arena/jobs');const t=document.getElementById('arena');
 for(const a of o.jobs){const r=t.insertRow();for(const v of [a.namespace,a.name,a.type,a.phase,
 JSON.stringify(a.result||{})])r.insertCell().textContent=v??''}}
async function consent(){const u=document.getElementById('cuser').value;
 document.getElementById('cons').textContent=JSON.stringify(
 await j('/api/consent/'+encodeURIComponent(u)),null,1)}
function log(x){const l=document.getElementById('log');l.textContent+=x+'\\n';l.scrollTop=1e9}
async function conn(){let v=document.getElementById('ws').value;
 if(/^\/api\/agents\/[^/]+\/[^/]+\/ws$/.test(v)){const r=await fetch(v+'-ticket',{method:'POST'});
  if(r.ok){v+='?ticket='+encodeURIComponent((await r.json()).ticket)}}
 sock=new WebSocket(v.startsWith('/')?(location.protocol==='https:'?'wss://':'ws://')+location.host+v:v);
 sock.onmessage=e=>{const m=JSON.parse(e.data);log(m.type+': '+(m.content||m.error?.message||''))}}
function send(){sock.send(JSON.stringify({type:'message',content:document.getElementById('msg').value}))}
const sel=document.getElementById('kind');for(const k of KINDS){const o=document.createElement('option');
 o.value=k;o.textContent=k;sel.appendChild(o)};sel.onchange=res;agents();res();sess();arena();
</script>__VIEWS__</body></html>"""


WRITE_TYPES = ("application/json", "application/yaml", "application/x-yaml")


def _claim_set(claims: dict, *names) -> set:
    out = set()
    for n in names:
        v = claims.get(n)
        if isinstance(v, str):
            out.update(v.replace(",", " ").split())
        elif isinstance(v, (list, tuple)):
            out.update(str(x) for x in v)
    return out


def _console_ws_path(path: str) -> bool:
    p = path.split("/")
    return len(p) == 6 and p[1] == "api" and p[2] == "agents" and p[5] == "ws"


def oidc_middleware(jwks: dict, issuer: str = "", audience: str = ""):
    """401 on ``/api/*`` without a valid IdP bearer token; the verified claims
    ride on the request (``request["claims"]``) for the write guard.  The
    console WebSocket is the one exception: a browser cannot put a bearer on a
    WebSocket, so it presents a one-time ``ticket`` minted by the authenticated
    ``POST .../ws-ticket`` route instead (checked by the route itself)."""
    from ..facade.auth import AuthError, bearer, jwt_decode

    @web.middleware
    async def mw(request, handler):
        if _console_ws_path(request.path) and request.query.get("ticket") and \
                not request.headers.get("Authorization"):
            return await handler(request)
        if request.path.startswith("/api/") and request.path != "/api/auth/jwks":
            tok = bearer(request.headers)
            if not tok:
                return web.json_response({"error": "missing bearer token"}, status=401)
            try:
                claims = jwt_decode(tok, jwks=jwks, issuer=issuer or None,
                                    audience=audience or None)
            except AuthError:
                return web.json_response({"error": "invalid token"}, status=401)
            if "exp" not in claims:
                return web.json_response({"error": "token without exp"}, status=401)
            request["claims"] = claims
        return await handler(request)

    return mw


def build_app(api: str, session_api: str = "", privacy_api: str = "",
              oidc: dict | None = None, allow_writes: bool = False,
              insecure_dev_writes: bool = False,
              allowed_origins: tuple = (), mgmt_key=None, mgmt_kid: str = "",
              twin_resolver=None, token_ttl_s: int = 300,
              open_console: bool = False, memory_api: str = "") -> web.Application:
    """``oidc``: ``{"jwks": {...}, "issuer": ..., "audience": ...,
    "write_groups": [...]}`` gates the API; ``allow_writes`` enables the
    management routes, which need OIDC unless ``insecure_dev_writes`` (module doc).
    ``mgmt_kid`` defaults to the signing key's RFC 7638 thumbprint.  The agent
    console mints management-plane tokens only for an OIDC-authenticated caller
    (one-time ticket) or, without OIDC, when ``open_console`` opts in."""
    if mgmt_key is not None and not mgmt_kid:
        from ..facade.auth import jwk_thumbprint

        mgmt_kid = jwk_thumbprint(mgmt_key)
    if allow_writes and not oidc and not insecure_dev_writes:
        raise ValueError("--allow-writes needs OIDC (--oidc-jwks-file); use "
                         "--insecure-dev-writes only for a loopback-bound dev dashboard")
    write_groups = set((oidc or {}).get("write_groups") or ["omnia-admin"])
    mws = [oidc_middleware(oidc["jwks"], oidc.get("issuer", ""), oidc.get("audience", ""))] \
        if oidc else []
    app = web.Application(middlewares=mws)
    plurals = sorted(k.plural for k in crds.KINDS.values())

    async def _get(url):
        async with aiohttp.ClientSession() as s:
            async with s.get(url, timeout=aiohttp.ClientTimeout(total=10)) as r:
                return r.status, await r.json(content_type=None)

    async def _send(request, method, url, body=None, ctype="application/json"):
        hdrs = {"Content-Type": ctype}
        auth = request.headers.get("Authorization")
        if auth:
            hdrs["Authorization"] = auth  # the API server authorises the caller
        data = None if body is None else (body if isinstance(body, (bytes, str))
                                          else json.dumps(body))
        async with aiohttp.ClientSession() as s:
            async with s.request(method, url, data=data, headers=hdrs,
                                 timeout=aiohttp.ClientTimeout(total=10)) as r:
                return r.status, await r.json(content_type=None)

    def _writes_on(request):
        if not allow_writes:
            return web.json_response({"error": "dashboard is read-only "
                                               "(start it with --allow-writes)"}, status=403)
        ctype = (request.headers.get("Content-Type") or "").split(";")[0].strip().lower()
        if request.method != "DELETE" and ctype not in WRITE_TYPES:
            return web.json_response({"error": "writes must be application/json or "
                                               "application/yaml"}, status=415)
        origin = request.headers.get("Origin")
        if origin:
            own = {f"{request.scheme}://{request.host}", f"http://{request.host}",
                   f"https://{request.host}"}
            if origin not in own and origin not in allowed_origins:
                return web.json_response({"error": "cross-origin write refused"}, status=403)
        if oidc:
            have = _claim_set(request.get("claims") or {}, "groups", "roles")
            if not have & write_groups:
                return web.json_response({"error": "caller lacks a write group "
                                                   f"({', '.join(sorted(write_groups))})"},
                                         status=403)
        return None

    base = f"{api}/apis/{crds.GROUP}/{crds.VERSION}"

    def _ns_url(plural, ns, name=""):
        kind = next(k for k in crds.KINDS.values() if k.plural == plural)
        root = f"{base}/namespaces/{ns}/{plural}" if kind.scope == "Namespaced" else \
            f"{base}/{plural}"
        return root + (f"/{urllib.parse.quote(name, safe='')}" if name else "")

    async def create(request):
        if (deny := _writes_on(request)) is not None:
            return deny
        plural = request.match_info["plural"]
        if plural not in plurals:
            return web.json_response({"error": "unknown resource"}, status=404)
        raw = await request.text()
        try:
            import yaml

            obj = yaml.safe_load(raw) if raw.strip() else None
        except Exception as e:  # noqa: BLE001 - yaml.YAMLError and friends
            return web.json_response({"error": f"unparsable body: {e}"}, status=400)
        if not isinstance(obj, dict) or not (obj.get("metadata") or {}).get("name"):
            return web.json_response({"error": "body must be one object with metadata.name"},
                                     status=400)
        ns = obj["metadata"].get("namespace") or "default"
        st, body = await _send(request, "POST", _ns_url(plural, ns), obj)
        return web.json_response(body, status=st)

    async def delete(request):
        if (deny := _writes_on(request)) is not None:
            return deny
        plural, ns, name = (request.match_info[k] for k in ("plural", "ns", "name"))
        if plural not in plurals:
            return web.json_response({"error": "unknown resource"}, status=404)
        st, body = await _send(request, "DELETE", _ns_url(plural, ns, name))
        return web.json_response(body, status=st)

    async def scale(request):
        if (deny := _writes_on(request)) is not None:
            return deny
        try:
            n = int((await request.json())["replicas"])
            if n < 0:
                raise ValueError
        except (KeyError, ValueError, TypeError, json.JSONDecodeError):
            return web.json_response({"error": "body must be {\"replicas\": n >= 0}"},
                                     status=400)
        ns, name = request.match_info["ns"], request.match_info["name"]
        st, body = await _send(request, "PATCH", _ns_url("agentruntimes", ns, name),
                               {"spec": {"runtime": {"replicas": n}}},
                               "application/merge-patch+json")
        return web.json_response(body, status=st)

    async def cancel_job(request):
        if (deny := _writes_on(request)) is not None:
            return deny
        ns, name = request.match_info["ns"], request.match_info["name"]
        st, body = await _send(request, "PATCH", _ns_url("arenajobs", ns, name),
                               {"spec": {"cancelled": True}}, "application/merge-patch+json")
        return web.json_response(body, status=st)

    async def page(_):
        from .dashboard_views import PAGE_SECTIONS

        return web.Response(text=PAGE.replace("__KINDS__", json.dumps(plurals)).replace(
            "__VIEWS__", PAGE_SECTIONS), content_type="text/html")

    async def resources(request):
        plural = request.match_info["plural"]
        if plural not in plurals:
            return web.json_response({"error": "unknown resource"}, status=404)
        st, body = await _get(f"{api}/apis/{crds.GROUP}/{crds.VERSION}/{plural}")
        return web.json_response(body, status=st)

    async def sessions(request):
        if not session_api:
            return web.json_response({"sessions": []})
        st, body = await _get(f"{session_api}/api/v1/sessions?limit="
                              f"{int(request.query.get('limit', 50))}")
        return web.json_response(body, status=st)

    async def session_messages(request):
        if not session_api:
            return web.json_response({"messages": []})
        sid = urllib.parse.quote(request.match_info["id"], safe="")
        st, body = await _get(f"{session_api}/api/v1/sessions/{sid}/messages")
        return web.json_response(body, status=st)

    async def arena_jobs(_):
        st, body = await _get(f"{api}/apis/{crds.GROUP}/{crds.VERSION}/arenajobs")
        jobs = []
        for it in (body or {}).get("items", []):
            spec, status = it.get("spec", {}), it.get("status", {})
            jobs.append({"namespace": it["metadata"].get("namespace"),
                         "name": it["metadata"]["name"], "type": spec.get("type"),
                         "phase": status.get("phase"),
                         "result": status.get("result") or status.get("results")})
        return web.json_response({"jobs": jobs})

    async def consent(request):
        if not privacy_api:
            return web.json_response({"error": "privacy api not configured"}, status=404)
        user = urllib.parse.quote(request.match_info["user"], safe="")
        st, body = await _get(f"{privacy_api}/api/v1/privacy/preferences/{user}/consent")
        return web.json_response(body, status=st)

    async def overview(_):
        st, body = await _get(f"{api}/apis/{crds.GROUP}/{crds.VERSION}/agentruntimes")
        out = []
        for it in (body or {}).get("items", []):
            spec, status = it.get("spec", {}), it.get("status", {})
            provs = spec.get("providers") or []
            out.append({"namespace": it["metadata"].get("namespace"),
                        "name": it["metadata"]["name"], "phase": status.get("phase"),
                        "replicas": (status.get("replicas") or {}).get("ready"),
                        "provider": ",".join(p.get("providerRef", {}).get("name", "")
                                             for p in provs)})
        return web.json_response({"agents": out})

    async def healthz(_):
        return web.json_response({"status": "ok"})

    # ------------------------------------------------ management plane
    from ..facade.auth import jwk_from_private, mint_mgmt_token

    async def jwks(_):
        keys = [jwk_from_private(mgmt_key, mgmt_kid)] if mgmt_key is not None else []
        return web.json_response({"keys": keys})

    async def _twin(ns: str, name: str):
        """ws:// URL of an agent's mgmt twin + its workspace, from its status."""
        if twin_resolver is not None:
            return await twin_resolver(ns, name)
        st, body = await _get(_ns_url("agentruntimes", ns, name))
        if st != 200:
            return None, ""
        status = body.get("status") or {}
        port = (status.get("managementEndpoints") or {}).get("ws")
        ep = status.get("serviceEndpoint") or f"{name}.{ns}.svc.cluster.local"
        if not port:
            return None, ""
        ws = ((body.get("spec") or {}).get("workspaceRef") or {}).get("name", "")
        return f"ws://{ep.rsplit(':', 1)[0]}:{port}/ws", ws

    tickets: dict = {}  # one-time console tickets: ticket -> (ns, name, claims, expiry)

    def _origin_ok(request) -> bool:
        origin = request.headers.get("Origin")
        if not origin:
            return True  # not a browser (a browser always sends Origin on a WebSocket)
        own = {f"{request.scheme}://{request.host}", f"http://{request.host}",
               f"https://{request.host}"}
        return origin in own or origin in allowed_origins

    async def ws_ticket(request):
        """One-time, 30 s ticket for the console WebSocket of one agent: the
        bearer-authenticated half of the browser console flow under OIDC."""
        if mgmt_key is None:
            return web.json_response({"error": "management plane not configured"}, status=503)
        if not oidc:
            return web.json_response({"error": "tickets need OIDC"}, status=404)
        if not _origin_ok(request):
            return web.json_response({"error": "cross-origin request refused"}, status=403)
        import secrets
        import time as _time

        now = _time.monotonic()
        for k, v in list(tickets.items()):
            if v[3] < now:
                tickets.pop(k, None)
        t = secrets.token_urlsafe(24)
        tickets[t] = (request.match_info["ns"], request.match_info["name"],
                      request.get("claims") or {}, now + 30.0)
        return web.json_response({"ticket": t, "expires_in": 30})

    async def agent_ws(request):
        """Browser <-> dashboard <-> agent twin, frame for frame."""
        if mgmt_key is None:
            return web.json_response({"error": "management plane not configured"}, status=503)
        ns, name = request.match_info["ns"], request.match_info["name"]
        # cross-site WebSocket hijacking: browsers do not apply same-origin rules
        # to WebSockets, so the Origin a browser sends must be the dashboard's
        if not _origin_ok(request):
            return web.json_response({"error": "cross-origin console refused"}, status=403)
        if oidc:
            claims = request.get("claims")
            if claims is None:  # no bearer (middleware let it through): a ticket
                import time as _time

                rec = tickets.pop(request.query.get("ticket", ""), None)
                if rec is None or rec[3] < _time.monotonic() or rec[:2] != (ns, name):
                    return web.json_response({"error": "invalid or expired console ticket"},
                                             status=401)
                claims = rec[2]
        elif open_console:
            claims = {}
        else:
            return web.json_response({"error": "the agent console needs OIDC "
                                               "(--oidc-jwks-file) or --open-console"},
                                     status=403)
        url, workspace = await _twin(ns, name)
        if not url:
            return web.json_response({"error": "agent has no management endpoint"}, status=404)
        tok = mint_mgmt_token(mgmt_key, mgmt_kid, str(claims.get("sub") or "dashboard"),
                              agent=name, workspace=workspace, ttl_s=token_ttl_s)
        q = {k: v for k, v in request.query.items() if k in ("session", "binary", "resume")}
        if q:
            url += "?" + urllib.parse.urlencode(q)
        down = web.WebSocketResponse(heartbeat=30.0)
        await down.prepare(request)
        async with aiohttp.ClientSession() as s:
            try:
                up = await s.ws_connect(url, headers={"Authorization": f"Bearer {tok}"},
                                        heartbeat=30.0)
            except aiohttp.WSServerHandshakeError as e:
                await down.send_json({"type": "error", "error": {
                    "code": "upstream_rejected", "message": f"agent twin: {e.status}"}})
                await down.close()
                return down

            async def pump(src, dst):
                async for m in src:
                    if m.type == aiohttp.WSMsgType.TEXT:
                        await dst.send_str(m.data)
                    elif m.type == aiohttp.WSMsgType.BINARY:
                        await dst.send_bytes(m.data)
                    else:
                        break
                await dst.close()

            async with up:
                t1 = asyncio.ensure_future(pump(up, down))
                t2 = asyncio.ensure_future(pump(down, up))
                await asyncio.wait({t1, t2}, return_when=asyncio.FIRST_COMPLETED)
                for t in (t1, t2):
                    t.cancel()
        return down

    app.router.add_get("/", page)
    app.router.add_get("/api/resources/{plural}", resources)
    app.router.add_get("/api/sessions", sessions)
    app.router.add_get("/api/overview", overview)
    app.router.add_get("/api/sessions/{id}/messages", session_messages)
    app.router.add_get("/api/arena/jobs", arena_jobs)
    app.router.add_get("/api/consent/{user}", consent)
    app.router.add_get("/healthz", healthz)
    app.router.add_get("/api/auth/jwks", jwks)
    app.router.add_get("/api/agents/{ns}/{name}/ws", agent_ws)
    app.router.add_post("/api/agents/{ns}/{name}/ws-ticket", ws_ticket)
    app.router.add_post("/api/resources/{plural}", create)
    app.router.add_delete("/api/resources/{plural}/{ns}/{name}", delete)
    app.router.add_post("/api/agents/{ns}/{name}/scale", scale)
    app.router.add_post("/api/arena/jobs/{ns}/{name}/cancel", cancel_job)
    # costs / quality / memories / memory analytics / topology / tools / skills /
    # settings (dashboard_views.py)
    from . import dashboard_views

    dashboard_views.mount(app, _get, api, session_api, memory_api, privacy_api, settings={
        "auth": "oidc" if oidc else "none", "writes": bool(allow_writes),
        "console": "ticket" if oidc else ("open" if open_console else "closed"),
        "kinds": plurals})
    return app


def main(argv=None):
    ap = argparse.ArgumentParser("omnia-dashboard")
    ap.add_argument("--port", type=int, default=3000)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--api", default="http://127.0.0.1:8090")
    ap.add_argument("--session-api", default="")
    ap.add_argument("--privacy-api", default="")
    ap.add_argument("--memory-api", default="")
    ap.add_argument("--oidc-jwks-file", default="", help="IdP JWKS; gates /api/* when set")
    ap.add_argument("--oidc-issuer", default="")
    ap.add_argument("--oidc-audience", default="")
    ap.add_argument("--allow-writes", action="store_true",
                    help="enable create / delete / scale / cancel routes (needs OIDC)")
    ap.add_argument("--oidc-write-group", action="append", default=[],
                    help="group / role claim allowed to write (repeatable; default omnia-admin)")
    ap.add_argument("--allowed-origin", action="append", default=[])
    ap.add_argument("--insecure-dev-writes", action="store_true",
                    help="allow writes without OIDC; only with a loopback --host")
    ap.add_argument("--mgmt-signing-key", default="",
                    help="PEM RSA key that signs management-plane JWTs (default: an "
                         "ephemeral key generated at start; facades re-fetch the JWKS)")
    ap.add_argument("--mgmt-kid", default="",
                    help="kid of the signing key (default: its RFC 7638 thumbprint, so a "
                         "restarted dashboard with a new ephemeral key gets a new kid)")
    ap.add_argument("--open-console", action="store_true",
                    help="without OIDC: let any same-origin caller open the agent console "
                         "(only with a loopback --host)")
    a = ap.parse_args(argv)
    from ..utils.rsa import generate_private_key, load_private_key

    if a.mgmt_signing_key:
        with open(a.mgmt_signing_key) as f:
            mgmt_key = load_private_key(f.read())
    else:
        mgmt_key = generate_private_key(2048)
    oidc = None
    if a.oidc_jwks_file:
        with open(a.oidc_jwks_file) as f:
            oidc = {"jwks": json.load(f), "issuer": a.oidc_issuer, "audience": a.oidc_audience,
                    "write_groups": a.oidc_write_group or ["omnia-admin"]}
    if a.insecure_dev_writes and a.host not in ("127.0.0.1", "localhost", "::1"):
        ap.error("--insecure-dev-writes needs --host 127.0.0.1")
    if a.open_console and a.host not in ("127.0.0.1", "localhost", "::1"):
        ap.error("--open-console needs --host 127.0.0.1")

    async def run():
        runner = web.AppRunner(build_app(a.api, a.session_api, a.privacy_api, oidc,
                                         allow_writes=a.allow_writes,
                                         insecure_dev_writes=a.insecure_dev_writes,
                                         allowed_origins=tuple(a.allowed_origin),
                                         mgmt_key=mgmt_key, mgmt_kid=a.mgmt_kid,
                                         open_console=a.open_console,
                                         memory_api=a.memory_api))
        await runner.setup()
        await web.TCPSite(runner, a.host, a.port).start()
        await asyncio.Event().wait()

    asyncio.run(run())


if __name__ == "__main__":
    main()
