"""Kubernetes-style REST front for the in-memory API store.

It lets ``omnia`` CLI, the dashboard, ``kubectl --server`` style clients, and
the operator's own :class:`~omnia_amd.operator.kube.KubeClient` (real-cluster
mode, tested against this server) talk to a running single-node operator.
The wire behaviour follows the kube-apiserver conventions the client relies on:

  /api/v1/namespaces/{ns}/{plural}[/{name}[/status]]             core kinds
  /apis/{group}/{version}/namespaces/{ns}/{plural}[/{name}]        namespaced kinds
  /apis/{group}/{version}/{plural}[/{name}]                        cluster kinds / all-ns list

* LIST returns ``metadata.resourceVersion`` (the store's current revision) and
  honours ``labelSelector`` (``k=v``, ``k!=v``, ``k in (a,b)``, ``k notin (..)``,
  ``k``, ``!k``) and ``fieldSelector`` on ``metadata.name``/``metadata.namespace``;
* ``?watch=1&resourceVersion=N`` replays the retained history after N then
  streams live events; a compacted N yields an ``ERROR`` event with a 410
  ``Expired`` Status; ``allowWatchBookmarks`` emits periodic BOOKMARKs;
  ``timeoutSeconds`` ends the stream;
* PUT/PATCH on ``/status`` touch only the status subresource; PATCH accepts
  ``merge-patch+json`` (RFC 7386), ``json-patch+json`` (RFC 6902),
  ``strategic-merge-patch+json`` (as merge) and ``apply-patch+yaml`` (server-side
  apply, ``fieldManager`` required);
* optional bearer-token authentication (401 with a Status body);
* errors are ``Status`` objects (404 NotFound, 409 Conflict/AlreadyExists,
  422 Invalid with ``details.causes``, 410 Expired).
"""
from __future__ import annotations

import asyncio
import copy
import json
import os
import re

import yaml
from aiohttp import web

from ..api import crds
from .apistore import APIStore, Conflict, Gone, Invalid, NotFound
from .kube import BUILTIN

CORE = {plural: kind for kind, (_, plural, _) in BUILTIN.items()}


def kind_of(plural: str) -> str:
    if plural in crds.PLURAL:
        return crds.PLURAL[plural]
    if plural in CORE:
        return CORE[plural]
    raise KeyError(plural)


_SEL = re.compile(r"\s*(!?)([A-Za-z0-9_./-]+)\s*(?:(=|==|!=)\s*([^,]*)|"
                  r"\s+(in|notin)\s*\(([^)]*)\))?\s*(?:,|$)")


def parse_label_selector(s: str) -> dict:
    """labelSelector query string -> LabelSelector dict."""
    ml, exprs = {}, []
    pos = 0
    while pos < len(s):
        m = _SEL.match(s, pos)
        if not m or m.end() == pos:
            raise ValueError(f"bad labelSelector {s!r}")
        neg, key, op, val, setop, vals = m.groups()
        if op in ("=", "=="):
            ml[key] = val.strip()
        elif op == "!=":
            exprs.append({"key": key, "operator": "NotIn", "values": [val.strip()]})
        elif setop:
            exprs.append({"key": key, "operator": "In" if setop == "in" else "NotIn",
                          "values": [v.strip() for v in vals.split(",") if v.strip()]})
        else:
            exprs.append({"key": key, "operator": "DoesNotExist" if neg else "Exists"})
        pos = m.end()
    out = {"matchLabels": ml}
    if exprs:
        out["matchExpressions"] = exprs
    return out


def merge_patch(target, patch):
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = dict(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def _ptr(path: str) -> list:
    if path == "":
        return []
    if not path.startswith("/"):
        raise ValueError(f"bad JSON pointer {path!r}")
    return [p.replace("~1", "/").replace("~0", "~") for p in path[1:].split("/")]


def _walk(doc, parts):
    for p in parts:
        doc = doc[int(p)] if isinstance(doc, list) else doc[p]
    return doc


def json_patch(doc, ops: list):
    """RFC 6902 JSON patch (add / remove / replace / move / copy / test)."""
    doc = copy.deepcopy(doc)

    def add(parts, value):
        nonlocal doc
        if not parts:
            doc = value
            return
        parent = _walk(doc, parts[:-1])
        last = parts[-1]
        if isinstance(parent, list):
            parent.insert(len(parent) if last == "-" else int(last), value)
        else:
            parent[last] = value

    def remove(parts):
        parent = _walk(doc, parts[:-1])
        last = parts[-1]
        if isinstance(parent, list):
            return parent.pop(int(last))
        return parent.pop(last)

    for op in ops:
        kind, parts = op["op"], _ptr(op["path"])
        try:
            if kind == "add":
                add(parts, copy.deepcopy(op["value"]))
            elif kind == "remove":
                remove(parts)
            elif kind == "replace":
                remove(parts)
                add(parts, copy.deepcopy(op["value"]))
            elif kind == "move":
                v = remove(_ptr(op["from"]))
                add(parts, v)
            elif kind == "copy":
                add(parts, copy.deepcopy(_walk(doc, _ptr(op["from"]))))
            elif kind == "test":
                if _walk(doc, parts) != op["value"]:
                    raise ValueError(f"test failed at {op['path']}")
            else:
                raise ValueError(f"unknown op {kind}")
        except (KeyError, IndexError, TypeError) as e:
            raise ValueError(f"json patch {kind} {op['path']}: {e}") from None
    return doc


def _status(code: int, reason: str, msg: str, causes: list[str] | None = None) -> dict:
    st = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
          "message": msg, "reason": reason, "code": code}
    if causes:
        st["details"] = {"causes": [{"message": c} for c in causes]}
    return st


def build_app(store: APIStore, token: str | None = None,
              bookmark_interval: float = 30.0) -> web.Application:
    from .restapi import mount

    middlewares = []
    token = token or os.environ.get("OMNIA_APISERVER_TOKEN") or None
    jwks_path = os.environ.get("OMNIA_DASHBOARD_JWKS_FILE", "")
    if jwks_path:
        # dashboard-minted identity tokens guard the workspace content API (C18 authz)
        from .authz import IdentityVerifier, authz_middleware

        with open(jwks_path) as f:
            jwks = json.load(f)
        middlewares.append(authz_middleware(IdentityVerifier(
            jwks, issuer=os.environ.get("OMNIA_DASHBOARD_ISSUER", ""),
            audience=os.environ.get("OMNIA_DASHBOARD_AUDIENCE", "")), store))
    app = web.Application(middlewares=middlewares)
    mount(app, store)  # specific routes first: the generic resource routes below are greedy

    def err(status, reason, msg, causes=None):
        return web.json_response(_status(status, reason, msg, causes), status=status)

    def authed(request) -> bool:
        if not token:
            return True
        return request.headers.get("Authorization", "") == f"Bearer {token}"

    def list_filter(request, kind, ns):
        sel = None
        if request.query.get("labelSelector"):
            sel = parse_label_selector(request.query["labelSelector"])
        items = store.list(kind, ns, sel)
        fs = request.query.get("fieldSelector")
        if fs:
            for term in fs.split(","):
                k, _, v = term.partition("=")
                v = v.lstrip("=")
                field = k.strip().split(".", 1)[-1]
                items = [o for o in items if o["metadata"].get(field, "") == v]
        return sel, items

    async def watch(request, kind, ns, sel):
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        await resp.prepare(request)
        q = store.watch(kind)  # register first: no gap between replay and live events
        bookmarks = request.query.get("allowWatchBookmarks") in ("1", "true")
        timeout = float(request.query.get("timeoutSeconds") or 1800)
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        sent_rv = 0

        def visible(o):
            from .apistore import match_labels

            if ns and o["metadata"].get("namespace") != ns:
                return False
            return match_labels(o["metadata"].get("labels", {}), sel)

        async def send(et, o):
            await resp.write((json.dumps({"type": et, "object": o}) + "\n").encode())

        try:
            rv = request.query.get("resourceVersion", "")
            if rv in ("", "0"):
                for o in store.list(kind, ns, sel):
                    await send("ADDED", o)
                sent_rv = int(store.current_rv())
            else:
                try:
                    hist = store.events_since(int(rv), kind)
                except Gone as e:
                    await send("ERROR", _status(410, "Expired", str(e)))
                    return resp
                sent_rv = int(rv)
                for r, (et, o) in hist:
                    if visible(o):
                        await send(et, o)
                    sent_rv = max(sent_rv, r)
            while True:
                left = deadline - loop.time()
                if left <= 0:
                    break
                try:
                    et, o = await asyncio.wait_for(q.get(), min(left, bookmark_interval))
                except asyncio.TimeoutError:
                    if bookmarks and loop.time() < deadline:
                        gv = crds.API_VERSION if kind in crds.KINDS else BUILTIN.get(
                            kind, ("v1",))[0]
                        await send("BOOKMARK", {"kind": kind, "apiVersion": gv, "metadata": {
                            "resourceVersion": store.current_rv()}})
                    continue
                r = int(o["metadata"].get("resourceVersion") or 0)
                if r <= sent_rv:
                    continue  # already replayed from history
                sent_rv = r
                if visible(o):
                    await send(et, o)
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            store.unwatch(q)
        return resp

    def json_ok(obj, status=200):
        headers = {}
        if store.warnings:  # Warn-mode pruning surfaces as HTTP Warning headers
            headers["Warning"] = ", ".join(f'299 - "{w}"' for w in store.warnings[:10])
        return web.json_response(obj, status=status, headers=headers)

    async def handle(request):
        if not authed(request):
            return err(401, "Unauthorized", "Unauthorized")
        fv = request.query.get("fieldValidation") or None
        if fv not in (None, "Strict", "Warn", "Ignore"):
            return err(400, "BadRequest", f"invalid fieldValidation {fv!r}")
        mi = request.match_info
        try:
            kind = kind_of(mi["plural"])
        except KeyError:
            return err(404, "NotFound", f"the server could not find the requested resource "
                       f"({mi['plural']})")
        ns = mi.get("ns")
        name = mi.get("name")
        sub = mi.get("sub")
        if sub not in (None, "status"):
            return err(404, "NotFound", f"subresource {sub} not found")
        try:
            if request.method == "GET":
                if name:
                    return web.json_response(store.get(kind, name, ns))
                try:
                    sel, items = list_filter(request, kind, ns)
                except ValueError as e:
                    return err(400, "BadRequest", str(e))
                if request.query.get("watch") in ("1", "true"):
                    return await watch(request, kind, ns, sel)
                gv = crds.API_VERSION if kind in crds.KINDS else BUILTIN.get(kind, ("v1",))[0]
                return web.json_response({"kind": kind + "List", "apiVersion": gv,
                                          "metadata": {"resourceVersion": store.current_rv()},
                                          "items": items})
            if request.method == "POST":
                body = await request.json()
                body.setdefault("kind", kind)
                if ns:
                    body.setdefault("metadata", {})["namespace"] = ns
                return json_ok(store.create(body, fv), status=201)
            if request.method == "PUT":
                body = await request.json()
                body.setdefault("kind", kind)
                if sub == "status":
                    return web.json_response(store.update_status(body))
                return json_ok(store.update(body, field_validation=fv))
            if request.method == "PATCH":
                ctype = request.headers.get("Content-Type", "").split(";")[0].strip()
                raw = await request.read()
                if ctype == "application/apply-patch+yaml":
                    if not request.query.get("fieldManager"):
                        return err(422, "Invalid", "fieldManager is required for apply "
                                   "patch", ["fieldManager: Required value"])
                    body = yaml.safe_load(raw.decode()) or {}
                    body.setdefault("kind", kind)
                    body.setdefault("metadata", {}).update(
                        {"name": name, **({"namespace": ns} if ns else {})})
                    if sub == "status":
                        cur = store.get(kind, name, ns)
                        cur["status"] = merge_patch(cur.get("status") or {},
                                                    body.get("status") or {})
                        return web.json_response(store.update_status(cur))
                    return json_ok(store.apply(body, fv))
                patch = json.loads(raw or b"{}")
                cur = store.get(kind, name, ns)
                if ctype == "application/json-patch+json":
                    try:
                        new = json_patch(cur, patch)
                    except ValueError as e:
                        return err(422, "Invalid", str(e), [str(e)])
                elif ctype in ("application/merge-patch+json",
                               "application/strategic-merge-patch+json"):
                    new = merge_patch(cur, patch)
                else:
                    return err(415, "UnsupportedMediaType", f"unsupported patch type {ctype}")
                # a patch without an explicit resourceVersion is unconditional
                if "resourceVersion" not in ((patch if isinstance(patch, dict) else {})
                                             .get("metadata") or {}):
                    new["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
                if sub == "status":
                    return web.json_response(store.update_status(new))
                return json_ok(store.update(new, field_validation=fv))
            if request.method == "DELETE":
                existed = store.delete(kind, name, ns)
                if not existed:
                    raise NotFound(f"{kind} {name} not found")
                return web.json_response({"kind": "Status", "apiVersion": "v1",
                                          "status": "Success",
                                          "details": {"name": name, "kind": mi["plural"]}})
        except NotFound as e:
            return err(404, "NotFound", str(e))
        except Conflict as e:
            reason = "AlreadyExists" if "already exists" in str(e) else "Conflict"
            return err(409, reason, str(e))
        except Invalid as e:
            return err(422, "Invalid", str(e), e.errors)
        return err(405, "MethodNotAllowed", "method not allowed")

    r = app.router
    for base in ("/api/v1", "/apis/{group}/{version}"):
        r.add_route("*", base + "/namespaces/{ns}/{plural}", handle)
        r.add_route("*", base + "/namespaces/{ns}/{plural}/{name}", handle)
        r.add_route("*", base + "/namespaces/{ns}/{plural}/{name}/{sub}", handle)
        r.add_route("*", base + "/{plural}", handle)
        r.add_route("*", base + "/{plural}/{name}", handle)
        r.add_route("*", base + "/{plural}/{name}/{sub}", handle)

    async def healthz(_):
        return web.json_response({"status": "ok"})

    r.add_get("/healthz", healthz)
    return app
