"""Dashboard analysis views: the data behind the
reference dashboard's costs, quality, memories, memory-analytics, topology,
tools, skills and settings pages (``dashboard/src/app/{costs,quality,memories,
memory-analytics,topology,tools,skills,settings}/page.tsx`` and their hooks:
``hooks/costs.ts``, ``use-eval-quality.ts``, ``use-memory-aggregate.ts``,
``use-memory-projection.ts``, ``use-consolidation-stats.ts``,
``use-consent-stats.ts``, ``use-enforcement-stats.ts``).

Same shape as the reference's backend-for-frontend: workspace-scoped routes
``/api/workspaces/{ws}/...`` resolve the Workspace to its namespace (the
Workspace CR's ``spec.namespace.name``) and proxy session-api, memory-api and
the privacy API; the cluster views (topology, tools, skills) are computed from
the operator REST API's objects.  The page fragments render them as tables and
an SVG dependency graph, without any front-end build.
"""
from __future__ import annotations

import urllib.parse

from aiohttp import web

from ..api import crds


def _q(v: str) -> str:
    return urllib.parse.quote(v or "", safe="")


def _meta(o: dict) -> tuple[str, str]:
    m = o.get("metadata") or {}
    return m.get("namespace") or "", m.get("name") or ""


def topology(objs: dict[str, list]) -> dict:
    """Nodes / edges of the agent dependency graph: AgentRuntime -> PromptPack,
    Provider, ToolRegistry (and the registry's handlers), PromptPack -> the
    SkillSources of its namespace, Workspace -> its agents."""
    nodes, edges, seen = [], [], set()

    def node(kind, ns, name, **kw):
        nid = f"{kind}/{ns}/{name}"
        if nid not in seen:
            seen.add(nid)
            nodes.append({"id": nid, "kind": kind, "namespace": ns, "name": name, **kw})
        return nid

    for pp in objs.get("promptpacks", []):
        ns, name = _meta(pp)
        node("PromptPack", ns, name, phase=(pp.get("status") or {}).get("phase"))
    for pv in objs.get("providers", []):
        ns, name = _meta(pv)
        node("Provider", ns, name, type=(pv.get("spec") or {}).get("type"),
             phase=(pv.get("status") or {}).get("phase"))
    for tr in objs.get("toolregistries", []):
        ns, name = _meta(tr)
        tid = node("ToolRegistry", ns, name, phase=(tr.get("status") or {}).get("phase"))
        for h in (tr.get("spec") or {}).get("handlers") or []:
            hid = node("ToolHandler", ns, f"{name}/{h.get('name')}", type=h.get("type"))
            edges.append({"from": tid, "to": hid, "rel": "handler"})
    for ss in objs.get("skillsources", []):
        ns, name = _meta(ss)
        node("SkillSource", ns, name, phase=(ss.get("status") or {}).get("phase"))
    for ar in objs.get("agentruntimes", []):
        ns, name = _meta(ar)
        spec, st = ar.get("spec") or {}, ar.get("status") or {}
        aid = node("AgentRuntime", ns, name, phase=st.get("phase"))
        ref = (spec.get("promptPackRef") or {}).get("name")
        if ref:
            edges.append({"from": aid, "to": node("PromptPack", ns, ref), "rel": "promptpack"})
            for ss in objs.get("skillsources", []):
                sns, sname = _meta(ss)
                if sns == ns:
                    edges.append({"from": node("PromptPack", ns, ref),
                                  "to": node("SkillSource", ns, sname), "rel": "skills"})
        for p in spec.get("providers") or []:
            pref = (p.get("providerRef") or {}).get("name")
            if pref:
                edges.append({"from": aid, "to": node("Provider", ns, pref),
                              "rel": p.get("name") or "provider"})
        tref = (spec.get("toolRegistryRef") or {}).get("name")
        if tref:
            edges.append({"from": aid, "to": node("ToolRegistry", ns, tref), "rel": "tools"})
    for ws in objs.get("workspaces", []):
        _, name = _meta(ws)
        wns = (((ws.get("spec") or {}).get("namespace") or {}).get("name")) or ""
        wid = node("Workspace", "", name)
        for n in list(nodes):
            if n["kind"] == "AgentRuntime" and n["namespace"] == wns:
                edges.append({"from": wid, "to": n["id"], "rel": "contains"})
    return {"nodes": nodes, "edges": edges}


def tools_view(registries: list) -> list[dict]:
    out = []
    for tr in registries:
        ns, name = _meta(tr)
        st = tr.get("status") or {}
        for t in st.get("discoveredTools") or []:
            out.append({"namespace": ns, "registry": name, "tool": t.get("name"),
                        "handler": t.get("handlerName"), "endpoint": t.get("endpoint"),
                        "status": t.get("status"), "description": t.get("description", "")})
        if not st.get("discoveredTools"):
            for h in (tr.get("spec") or {}).get("handlers") or []:
                out.append({"namespace": ns, "registry": name,
                            "tool": (h.get("tool") or {}).get("name") or h.get("name"),
                            "handler": h.get("name"), "endpoint": h.get("endpoint", ""),
                            "status": st.get("phase") or "Pending",
                            "description": (h.get("tool") or {}).get("description", "")})
    return out


def skills_view(sources: list) -> list[dict]:
    out = []
    for ss in sources:
        ns, name = _meta(ss)
        spec, st = ss.get("spec") or {}, ss.get("status") or {}
        src = spec.get("source") or {}
        out.append({"namespace": ns, "name": name, "type": src.get("type"),
                    "phase": st.get("phase"),
                    "skills": st.get("skillCount", len(st.get("skills") or [])),
                    "lastSync": st.get("lastSyncTime") or st.get("lastSyncedAt"),
                    "revision": st.get("revision") or st.get("lastRevision")})
    return out


def mount(app: web.Application, get, api: str, session_api: str = "", memory_api: str = "",
          privacy_api: str = "", settings: dict | None = None) -> None:
    """Add the view routes; ``get(url) -> (status, json)`` is the dashboard's
    proxy GET (it forwards the caller's bearer)."""
    base = f"{api}/apis/{crds.GROUP}/{crds.VERSION}"

    async def _list(plural):
        st, body = await get(f"{base}/{plural}")
        return (body or {}).get("items", []) if st == 200 else []

    async def _ns_of(ws: str) -> str:
        for w in await _list("workspaces"):
            if _meta(w)[1] == ws:
                return (((w.get("spec") or {}).get("namespace") or {}).get("name")) or ws
        return ws

    def _need(url, what):
        if not url:
            raise web.HTTPNotFound(text=f'{{"error": "{what} not configured"}}',
                                   content_type="application/json")

    async def costs(request):
        _need(session_api, "session api")
        ns = await _ns_of(request.match_info["ws"])
        by = request.query.get("groupBy", "model")
        st, body = await get(f"{session_api}/api/v1/provider-calls/aggregate?namespace="
                             f"{_q(ns)}&groupBy={_q(by)}")
        groups = (body or {}).get("groups", []) if st == 200 else []
        total = sum(float(g.get("costUsd", g.get("cost_usd", 0.0)) or 0.0) for g in groups)
        toks = sum(int(g.get("inputTokens", 0) or 0) + int(g.get("outputTokens", 0) or 0)
                   for g in groups)
        return web.json_response({"namespace": ns, "groupBy": by, "groups": groups,
                                  "totalCostUsd": round(total, 6), "totalTokens": toks},
                                 status=200 if st == 200 else st)

    async def quality(request):
        _need(session_api, "session api")
        ns = await _ns_of(request.match_info["ws"])
        st, body = await get(f"{session_api}/api/v1/eval-results/aggregate?namespace={_q(ns)}")
        evals = (body or {}).get("evals", []) if st == 200 else []
        n = sum(int(e.get("total", 0) or 0) for e in evals)
        p = sum(int(e.get("passed", 0) or 0) for e in evals)
        return web.json_response({"namespace": ns, "evals": evals, "total": n, "passed": p,
                                  "passRate": (p / n) if n else None},
                                 status=200 if st == 200 else st)

    async def memory_proxy(request, path, extra=""):
        _need(memory_api, "memory api")
        ws = request.match_info["ws"]
        qs = urllib.parse.urlencode({**request.query, "workspace": ws})
        st, body = await get(f"{memory_api}{path}?{qs}{extra}")
        return web.json_response(body, status=st)

    async def memories(request):
        return await memory_proxy(request, "/api/v1/memories")

    async def memory_aggregate(request):
        return await memory_proxy(request, "/api/v1/memories/aggregate")

    async def memory_projection(request):
        return await memory_proxy(request, "/api/v1/memories/projection")

    async def memory_stats(request):
        return await memory_proxy(request, "/api/v1/memories/stats")

    async def privacy_proxy(request, path):
        _need(privacy_api, "privacy api")
        st, body = await get(f"{privacy_api}{path}")
        return web.json_response(body, status=st)

    async def consent_stats(request):
        return await privacy_proxy(request, "/api/v1/privacy/consent/stats")

    async def enforcement_stats(request):
        return await privacy_proxy(request, "/api/v1/privacy/enforcement-stats")

    async def topo(_):
        objs = {p: await _list(p) for p in ("agentruntimes", "promptpacks", "providers",
                                            "toolregistries", "skillsources", "workspaces")}
        return web.json_response(topology(objs))

    async def tools(_):
        return web.json_response({"tools": tools_view(await _list("toolregistries"))})

    async def skills(_):
        return web.json_response({"sources": skills_view(await _list("skillsources"))})

    async def settings_view(_):
        return web.json_response({"endpoints": {
            "operator": api, "sessionApi": session_api or None, "memoryApi": memory_api or None,
            "privacyApi": privacy_api or None}, **(settings or {})})

    r = app.router
    r.add_get("/api/workspaces/{ws}/costs", costs)
    r.add_get("/api/workspaces/{ws}/eval-results/aggregate", quality)
    r.add_get("/api/workspaces/{ws}/memories", memories)
    r.add_get("/api/workspaces/{ws}/memory/aggregate", memory_aggregate)
    r.add_get("/api/workspaces/{ws}/memory/projection", memory_projection)
    r.add_get("/api/workspaces/{ws}/memory/stats", memory_stats)
    r.add_get("/api/workspaces/{ws}/privacy/consent/stats", consent_stats)
    r.add_get("/api/workspaces/{ws}/privacy/enforcement-stats", enforcement_stats)
    r.add_get("/api/topology", topo)
    r.add_get("/api/tools", tools)
    r.add_get("/api/skills", skills)
    r.add_get("/api/settings", settings_view)


PAGE_SECTIONS = """
<h2>Workspace views</h2>workspace <input id="wsname" value="default" size="16">
<button onclick="wsviews()">load</button>
<h3>Costs</h3><table id="costs"></table><div id="costsum"></div>
<h3>Quality</h3><table id="quality"></table><div id="qsum"></div>
<h3>Memories</h3><table id="mems"></table>
<h3>Memory analytics</h3><table id="memagg"></table><pre id="memproj"></pre>
<h3>Privacy</h3><pre id="privstats"></pre>
<h2>Topology</h2><svg id="topo" width="900" height="420" style="border:1px solid #ccc"></svg>
<h2>Tools</h2><table id="tools"></table>
<h2>Skills</h2><table id="skills"></table>
<h2>Settings</h2><pre id="settings"></pre>
<script>
function table(id,rows,cols){const t=document.getElementById(id);
 t.innerHTML='<tr>'+cols.map(c=>'<th>'+c+'</th>').join('')+'</tr>';
 for(const r of rows){const tr=t.insertRow();for(const c of cols){const v=r[c];
 tr.insertCell().textContent=(v!==null&&typeof v==='object')?JSON.stringify(v):(v??'')}}}
async function jj(u){const r=await fetch(u);return r.ok?r.json():{}}
async function wsviews(){const w=encodeURIComponent(document.getElementById('wsname').value);
 const c=await jj('/api/workspaces/'+w+'/costs');const g=c.groups||[];
 table('costs',g,Object.keys(g[0]||{key:1}));document.getElementById('costsum').textContent=
 'total $'+(c.totalCostUsd??0)+', '+(c.totalTokens??0)+' tokens';
 const q=await jj('/api/workspaces/'+w+'/eval-results/aggregate');const e=q.evals||[];
 table('quality',e,Object.keys(e[0]||{evalId:1}));document.getElementById('qsum').textContent=
 q.passRate==null?'no eval results':'pass rate '+(100*q.passRate).toFixed(1)+'%';
 const m=await jj('/api/workspaces/'+w+'/memories');table('mems',(m.memories||m.items||[]).slice(0,50),
 ['id','category','content','confidence']);
 const a=await jj('/api/workspaces/'+w+'/memory/aggregate?groupBy=tier');table('memagg',a.groups||[],
 Object.keys((a.groups||[])[0]||{key:1}));
 document.getElementById('memproj').textContent=JSON.stringify(await jj('/api/workspaces/'+w+
 '/memory/projection'),null,1);
 document.getElementById('privstats').textContent=JSON.stringify({consent:await jj('/api/workspaces/'+
 w+'/privacy/consent/stats'),enforcement:await jj('/api/workspaces/'+w+'/privacy/enforcement-stats')},null,1)}
async function topo(){const g=await jj('/api/topology');const s=document.getElementById('topo');
 const kinds=['Workspace','AgentRuntime','PromptPack','Provider','ToolRegistry','ToolHandler','SkillSource'];
 const pos={},col={};for(const n of (g.nodes||[])){const k=kinds.indexOf(n.kind);col[k]=(col[k]||0)+1;
 pos[n.id]=[20+k*125,20+col[k]*34]}
 let h='';for(const e of (g.edges||[])){const a=pos[e.from],b=pos[e.to];if(a&&b)
 h+='<line x1="'+(a[0]+110)+'" y1="'+a[1]+'" x2="'+b[0]+'" y2="'+b[1]+'" stroke="#999"/>'}
 for(const n of (g.nodes||[])){const p=pos[n.id];h+='<text x="'+p[0]+'" y="'+(p[1]+4)+
 '" font-size="11">'+n.kind[0]+': '+n.name.replace(/</g,'')+'</text>'}s.innerHTML=h}
async function cluster(){table('tools',(await jj('/api/tools')).tools||[],['namespace','registry','tool',
 'handler','status','endpoint']);table('skills',(await jj('/api/skills')).sources||[],['namespace','name',
 'type','phase','skills','lastSync']);document.getElementById('settings').textContent=
 JSON.stringify(await jj('/api/settings'),null,1);topo()}
cluster();
</script>"""
