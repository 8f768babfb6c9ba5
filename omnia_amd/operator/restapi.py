"""Operator REST extras (``internal/tooltest``, ``internal/api/deploy``,
``internal/api/content``):

* ``POST /api/v1/namespaces/{ns}/toolregistries/{name}/test`` -- execute one
  tool of a ToolRegistry through the real tool executor (handlers, auth,
  retries, breaker) and return the result, latency and error
  (``internal/tooltest/server.go:50-182``);
* ``POST /api/v1/namespaces/{ns}/deploy[?dryRun=true]`` -- translate a
  DeployIntent into PromptPack + pack ConfigMap (+ ToolRegistry, AgentPolicy)
  + one AgentRuntime per agent and apply them (``deploy/{translate,apply}.go``);
* ``GET|PUT|DELETE /api/v1/workspaces/{ws}/content/{path}`` -- the workspace
  content tree (pack bundles, skills) with path-traversal guards
  (``internal/api/content``).
"""
from __future__ import annotations

import json
import os
import tempfile
import time
from pathlib import Path

import yaml
from aiohttp import web

from .apistore import APIStore, Conflict, Invalid

API = "omnia.altairalabs.ai/v1alpha1"


def _err(status, msg):
    return web.json_response({"error": msg}, status=status)


# ------------------------------------------------------------------ deploy intent
def translate(intent: dict, ns: str) -> list[dict]:
    """DeployIntent -> ordered list of objects (ConfigMap, PromptPack, ToolRegistry,
    AgentPolicy, AgentRuntime...)."""
    pack = intent.get("pack") or {}
    if not pack.get("name") or not pack.get("content"):
        raise ValueError("pack.name and pack.content are required")
    if not intent.get("agents"):
        raise ValueError("at least one agent is required")
    labels = {"omnia.altairalabs.ai/deployed-by": "deploy-api", **(intent.get("labels") or {})}
    version = pack.get("version") or "1.0.0"
    cm_name = f"{pack['name']}-pack"
    content = pack["content"]
    if not isinstance(content, str):
        content = json.dumps(content)
    objs = [{"apiVersion": "v1", "kind": "ConfigMap",
             "metadata": {"name": cm_name, "namespace": ns, "labels": labels},
             "data": {"pack.json": content}},
            {"apiVersion": API, "kind": "PromptPack",
             "metadata": {"name": pack["name"], "namespace": ns, "labels": labels},
             "spec": {"packName": pack["name"], "version": version,
                      "source": {"type": "configmap", "configMapRef": {"name": cm_name}}}}]
    tools = intent.get("tools")
    if tools:
        objs.append({"apiVersion": API, "kind": "ToolRegistry",
                     "metadata": {"name": tools.get("name", pack["name"] + "-tools"),
                                  "namespace": ns, "labels": labels},
                     "spec": {"handlers": tools.get("handlers", [])}})
    pol = intent.get("policy")
    if pol:
        objs.append({"apiVersion": API, "kind": "AgentPolicy",
                     "metadata": {"name": pol.get("name", pack["name"] + "-policy"),
                                  "namespace": ns, "labels": labels},
                     "spec": {k: v for k, v in pol.items() if k != "name"}})
    for a in intent["agents"]:
        spec = {"promptPackRef": {"name": pack["name"]},
                "providers": [{"name": p.get("name", p["ref"]), "providerRef": {"name": p["ref"]},
                               **({"role": p["role"]} if p.get("role") else {})}
                              for p in a.get("providers") or []],
                "facades": [{"type": f.get("type", "websocket")} for f in
                            a.get("facades") or [{"type": "websocket"}]]}
        if a.get("promptName"):
            spec["promptPackRef"]["prompt"] = a["promptName"]
        if a.get("useTools") and tools:
            spec["toolRegistryRef"] = {"name": tools.get("name", pack["name"] + "-tools")}
        rt = a.get("runtime") or {}
        if rt:
            spec["runtime"] = {"replicas": rt.get("replicas", 1)}
            if rt.get("cpu") or rt.get("memory"):
                spec["runtime"]["resources"] = {"requests": {k: v for k, v in (
                    ("cpu", rt.get("cpu")), ("memory", rt.get("memory"))) if v}}
        mem = a.get("memory") or {}
        if mem.get("enabled"):
            spec["memory"] = {"enabled": True, **({"retrieval": mem["retrieval"]}
                                                  if mem.get("retrieval") else {})}
        if a.get("externalAuth"):
            spec["externalAuth"] = a["externalAuth"]
        if a.get("rollout"):
            spec["rollout"] = a["rollout"]
        if a.get("evals"):
            spec["evals"] = a["evals"]
        objs.append({"apiVersion": API, "kind": "AgentRuntime",
                     "metadata": {"name": a["name"], "namespace": ns, "labels": labels},
                     "spec": spec})
    return objs


def apply_objects(store: APIStore, objs: list[dict], dry_run: bool = False) -> list[dict]:
    from ..api import crds

    out = []
    for o in objs:
        if o["kind"] in crds.KINDS:
            errs = crds.validate_object(json.loads(json.dumps(o)))
            if errs:
                raise Invalid(errs)
        if dry_run:
            out.append({"kind": o["kind"], "name": o["metadata"]["name"], "action": "validated"})
            continue
        cur = store.try_get(o["kind"], o["metadata"]["name"], o["metadata"].get("namespace"))
        if cur is None:
            store.create(o)
            out.append({"kind": o["kind"], "name": o["metadata"]["name"], "action": "created"})
        else:
            cur.update({k: v for k, v in o.items() if k not in ("metadata", "status")})
            cur["metadata"].setdefault("labels", {}).update(o["metadata"].get("labels") or {})
            store.update(cur)
            out.append({"kind": o["kind"], "name": o["metadata"]["name"], "action": "updated"})
    return out


# ------------------------------------------------------------------ routes
def mount(app: web.Application, store: APIStore, content_root: str | None = None):
    root = Path(content_root or os.environ.get("OMNIA_CONTENT_ROOT",
                                               tempfile.gettempdir() + "/omnia-content"))

    async def tool_test(request):
        from ..tools.executor import CallContext, OmniaExecutor

        ns, name = request.match_info["ns"], request.match_info["name"]
        reg = store.try_get("ToolRegistry", name, ns)
        if reg is None:
            return _err(404, f"ToolRegistry {ns}/{name} not found")
        body = await request.json()
        tool = body.get("tool") or body.get("name")
        handlers = [h for h in reg["spec"].get("handlers", [])
                    if h.get("type") != "client"]
        ex = OmniaExecutor({"handlers": handlers})
        try:
            await ex.discover()
        except Exception as e:  # noqa: BLE001
            return web.json_response({"ok": False, "error": f"discovery failed: {e}"})
        if tool not in ex.tools:
            return _err(404, f"tool {tool!r} not in registry (have {sorted(ex.tools)})")
        t0 = time.perf_counter()
        try:
            res, is_err = await ex.execute(tool, body.get("arguments") or {},
                                           CallContext(session_id="tool-test", namespace=ns))
            try:
                res = json.loads(res)
            except (TypeError, ValueError):
                pass
            return web.json_response({"ok": not is_err, "result": res,
                                      "latencyMs": round((time.perf_counter() - t0) * 1e3, 2)})
        except Exception as e:  # noqa: BLE001
            return web.json_response({"ok": False, "error": str(e),
                                      "latencyMs": round((time.perf_counter() - t0) * 1e3, 2)})

    async def deploy(request):
        ns = request.match_info["ns"]
        try:
            raw = await request.text()
            intent = yaml.safe_load(raw) if raw.strip() else {}
            objs = translate(intent or {}, ns)
            res = apply_objects(store, objs, request.query.get("dryRun") == "true")
        except (ValueError, KeyError) as e:
            return _err(400, str(e))
        except Invalid as e:
            return _err(422, str(e))
        except Conflict as e:
            return _err(409, str(e))
        return web.json_response({"applied": res}, status=200 if request.query.get(
            "dryRun") == "true" else 201)

    def _path(ws: str, rel: str) -> Path:
        base = (root / "workspaces" / ws).resolve()
        p = (base / rel).resolve()
        if not str(p).startswith(str(base) + os.sep) and p != base:
            raise PermissionError("path escapes the workspace")
        return p

    async def content(request):
        try:
            p = _path(request.match_info["ws"], request.match_info.get("path", ""))
        except PermissionError as e:
            return _err(403, str(e))
        if request.method == "GET":
            if p.is_dir():
                return web.json_response({"entries": sorted(
                    [{"name": c.name, "dir": c.is_dir(),
                      "size": c.stat().st_size if c.is_file() else 0} for c in p.iterdir()],
                    key=lambda e: e["name"])})
            if not p.exists():
                return _err(404, "not found")
            return web.Response(body=p.read_bytes())
        if request.method == "PUT":
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(await request.read())
            return web.json_response({"written": p.stat().st_size}, status=201)
        if request.method == "DELETE":
            if not p.exists():
                return _err(404, "not found")
            if p.is_dir():
                return _err(400, "refusing to delete a directory")
            p.unlink()
            return web.Response(status=204)
        return _err(405, "method not allowed")

    app.router.add_post("/api/v1/namespaces/{ns}/toolregistries/{name}/test", tool_test)
    app.router.add_post("/api/v1/namespaces/{ns}/deploy", deploy)
    app.router.add_route("*", "/api/v1/workspaces/{ws}/content/{path:.*}", content)
    return app

