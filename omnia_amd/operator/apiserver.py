"""Kubernetes-style REST front for the in-memory API store (so ``omnia`` CLI,
the dashboard or ``kubectl --server`` style clients can talk to a running
single-node operator).  Paths follow the K8s conventions:

  /api/v1/namespaces/{ns}/{plural}[/{name}[/status]]             core kinds
  /apis/{group}/{version}/namespaces/{ns}/{plural}[/{name}]        namespaced CRDs
  /apis/{group}/{version}/{plural}[/{name}]                        cluster CRDs
  ?watch=1 streams newline-delimited JSON watch events.
"""
from __future__ import annotations

import os

import json

from aiohttp import web

from ..api import crds
from .apistore import APIStore, Conflict, Invalid, NotFound

CORE = {"configmaps": "ConfigMap", "secrets": "Secret", "services": "Service",
        "namespaces": "Namespace", "serviceaccounts": "ServiceAccount",
        "persistentvolumeclaims": "PersistentVolumeClaim", "deployments": "Deployment",
        "horizontalpodautoscalers": "HorizontalPodAutoscaler", "scaledobjects": "ScaledObject",
        "poddisruptionbudgets": "PodDisruptionBudget", "rolebindings": "RoleBinding",
        "networkpolicies": "NetworkPolicy", "leases": "Lease", "httproutes": "HTTPRoute"}


def kind_of(plural: str) -> str:
    if plural in crds.PLURAL:
        return crds.PLURAL[plural]
    if plural in CORE:
        return CORE[plural]
    raise KeyError(plural)


def build_app(store: APIStore) -> web.Application:
    from .restapi import mount

    middlewares = []
    jwks_path = os.environ.get("OMNIA_DASHBOARD_JWKS_FILE", "")
    if jwks_path:
        # dashboard-minted identity tokens guard the workspace content API (C18 authz)
        import json

        from .authz import IdentityVerifier, authz_middleware

        with open(jwks_path) as f:
            jwks = json.load(f)
        middlewares.append(authz_middleware(IdentityVerifier(
            jwks, issuer=os.environ.get("OMNIA_DASHBOARD_ISSUER", ""),
            audience=os.environ.get("OMNIA_DASHBOARD_AUDIENCE", "")), store))
    app = web.Application(middlewares=middlewares)
    mount(app, store)  # specific routes first: the generic resource routes below are greedy

    def err(status, msg):
        return web.json_response({"kind": "Status", "status": "Failure", "message": msg,
                                  "code": status}, status=status)

    async def handle(request):
        mi = request.match_info
        try:
            kind = kind_of(mi["plural"])
        except KeyError:
            return err(404, f"unknown resource {mi['plural']}")
        ns = mi.get("ns")
        name = mi.get("name")
        sub = mi.get("sub")
        try:
            if request.method == "GET":
                if name:
                    return web.json_response(store.get(kind, name, ns))
                if request.query.get("watch"):
                    resp = web.StreamResponse()
                    await resp.prepare(request)
                    q = store.watch(kind)
                    try:
                        for o in store.list(kind, ns):
                            await resp.write((json.dumps({"type": "ADDED", "object": o})
                                              + "\n").encode())
                        while True:
                            et, o = await q.get()
                            if ns and o["metadata"].get("namespace") != ns:
                                continue
                            await resp.write((json.dumps({"type": et, "object": o})
                                              + "\n").encode())
                    finally:
                        store.unwatch(q)
                sel = None
                if request.query.get("labelSelector"):
                    sel = {"matchLabels": dict(kv.split("=", 1) for kv in
                                               request.query["labelSelector"].split(","))}
                return web.json_response({"kind": kind + "List",
                                          "items": store.list(kind, ns, sel)})
            if request.method == "POST":
                body = await request.json()
                body.setdefault("kind", kind)
                if ns:
                    body.setdefault("metadata", {})["namespace"] = ns
                return web.json_response(store.create(body), status=201)
            if request.method == "PUT":
                body = await request.json()
                if sub == "status":
                    return web.json_response(store.update_status(body))
                return web.json_response(store.update(body))
            if request.method == "PATCH":
                body = await request.json()
                body.setdefault("kind", kind)
                body.setdefault("metadata", {}).update({"name": name, **({"namespace": ns}
                                                                          if ns else {})})
                return web.json_response(store.apply(body))
            if request.method == "DELETE":
                return web.json_response({"deleted": store.delete(kind, name, ns)})
        except NotFound as e:
            return err(404, str(e))
        except Conflict as e:
            return err(409, str(e))
        except Invalid as e:
            return err(422, str(e))
        return err(405, "method not allowed")

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
