"""Canary traffic routing for AgentRuntime rollouts (SURVEY §2.1 C11;
reference ``internal/controller/rollout_{routing,mesh,istio}.go``).

Modes (``spec.rollout.trafficRouting.mode``), resolved like the reference:
* ``mesh``     -- the operator OWNS an Istio VirtualService + DestinationRule
  (``<agent>-rollout``): stable / candidate subsets selected by the
  ``omnia.altairalabs.ai/track`` pod label, route weights = rollout weight,
  and a ``x-omnia-variant`` response header per subset.  Requested but no mesh
  installed -> degraded to ``replica-weighted`` (status says so);
* ``external`` -- legacy ``istio:`` form: the user's VirtualService routes
  named in ``virtualService.routes`` get their stable/candidate weights patched,
  and the DestinationRule gets a consistent-hash on the session header so a
  session sticks to one track;
* ``replica-weighted`` -- no mesh: traffic follows replica counts, so the
  candidate Deployment gets ``ceil(replicas * weight / 100)`` replicas (at
  least 1 while weight > 0) and stable the rest.
Resetting (promotion / rollback) returns 100 % to stable.
"""
from __future__ import annotations

import math
import os

ISTIO_API = "networking.istio.io/v1"
TRACK_LABEL = "omnia.altairalabs.ai/track"
SESSION_HEADER = "x-omnia-session-id"


def mesh_available() -> bool:
    return os.environ.get("OMNIA_MESH_ENABLED", "").lower() in ("1", "true", "yes")


def resolve_mode(cfg: dict | None, mesh: bool) -> tuple[str, bool]:
    """(mode, degraded)."""
    if not cfg:
        return ("mesh" if mesh else "replica-weighted"), False
    mode = cfg.get("mode", "")
    if mode == "mesh":
        return ("mesh", False) if mesh else ("replica-weighted", True)
    if mode in ("replica-weighted", "external"):
        return mode, False
    if cfg.get("istio"):
        return "external", False
    return ("mesh" if mesh else "replica-weighted"), False


def service_dns(name: str, ns: str) -> str:
    return f"{name}.{ns}.svc.cluster.local"


def owned_objects(name: str, ns: str, mesh_cfg: dict | None, weight: int) -> list[dict]:
    m = mesh_cfg or {}
    stable, cand = m.get("stableSubset") or "stable", m.get("candidateSubset") or "canary"
    host = service_dns(name, ns)
    hosts = m.get("hosts") or [host]
    dr = {"apiVersion": ISTIO_API, "kind": "DestinationRule",
          "metadata": {"name": f"{name}-rollout", "namespace": ns},
          "spec": {"host": host, "subsets": [
              {"name": stable, "labels": {TRACK_LABEL: "stable"}},
              {"name": cand, "labels": {TRACK_LABEL: "candidate"}}]}}
    vs = {"apiVersion": ISTIO_API, "kind": "VirtualService",
          "metadata": {"name": f"{name}-rollout", "namespace": ns},
          "spec": {"hosts": hosts, "http": [{"name": "rollout", "route": [
              {"destination": {"host": host, "subset": stable}, "weight": 100 - weight,
               "headers": {"response": {"set": {"x-omnia-variant": "stable"}}}},
              {"destination": {"host": host, "subset": cand}, "weight": weight,
               "headers": {"response": {"set": {"x-omnia-variant": "candidate"}}}}]}]}}
    if m.get("waypoint"):
        vs["metadata"]["labels"] = {"istio.io/use-waypoint": m["waypoint"]}
    return [dr, vs]


def patch_route_weights(vs: dict, routes: list[str], stable: str, cand: str, weight: int) -> int:
    """Patch the named http routes of a user VirtualService; returns routes hit."""
    hit = 0
    for r in (vs.get("spec") or {}).get("http") or []:
        if routes and r.get("name") not in routes:
            continue
        for dst in r.get("route") or []:
            sub = (dst.get("destination") or {}).get("subset")
            if sub == stable:
                dst["weight"] = 100 - weight
            elif sub == cand:
                dst["weight"] = weight
        hit += 1
    return hit


def patch_destination_rule(dr: dict, sticky: bool, header: str = SESSION_HEADER) -> None:
    tp = dr.setdefault("spec", {}).setdefault("trafficPolicy", {})
    if sticky:
        tp["loadBalancer"] = {"consistentHash": {"httpHeaderName": header}}
    else:
        tp.pop("loadBalancer", None)


def split_replicas(total: int, weight: int) -> tuple[int, int]:
    """(stable, candidate) replica counts for replica-weighted routing."""
    total = max(1, total)
    if weight <= 0:
        return total, 0
    if weight >= 100:
        return 0, total
    cand = min(total, max(1, math.ceil(total * weight / 100)))
    return max(1, total - cand) if cand < total else 0, cand


def apply(store, ar: dict, weight: int, active: bool) -> dict:
    """Reconcile routing objects for ``weight``; returns the status block."""
    spec, md = ar["spec"], ar["metadata"]
    ns, name = md["namespace"], md["name"]
    cfg = (spec.get("rollout") or {}).get("trafficRouting")
    mode, degraded = resolve_mode(cfg, mesh_available())
    w = weight if active else 0
    status = {"trafficRoutingMode": mode, "deliveredWeight": w, "degraded": degraded}
    if mode == "mesh":
        for obj in owned_objects(name, ns, (cfg or {}).get("mesh"), w):
            obj["metadata"]["ownerReferences"] = [{
                "apiVersion": ar["apiVersion"], "kind": ar["kind"], "name": name,
                "uid": md.get("uid", ""), "controller": True}]
            store.apply(obj)
    elif mode == "external":
        ist = (cfg or {}).get("istio") or {}
        vref, dref = ist.get("virtualService") or {}, ist.get("destinationRule") or {}
        stable = dref.get("stableSubset") or "stable"
        cand = dref.get("candidateSubset") or "canary"
        vs = store.try_get("VirtualService", vref.get("name", ""), ns)
        if vs is not None:
            status["routesPatched"] = patch_route_weights(vs, vref.get("routes") or [],
                                                          stable, cand, w)
            store.apply(vs)
        else:
            status["degraded"] = True
            status["message"] = f"VirtualService {vref.get('name')!r} not found"
        dr = store.try_get("DestinationRule", dref.get("name", ""), ns)
        if dr is not None:
            # spec.rollout.stickySession.hashOn (rollout_types.go:150): the header a
            # session's requests hash on, so one conversation stays on one track
            ss = (spec.get("rollout") or {}).get("stickySession") or {}
            patch_destination_rule(dr, active, ss.get("hashOn") or SESSION_HEADER)
            store.apply(dr)
    else:
        total = int((spec.get("runtime") or {}).get("replicas", 1) or 1)
        s, c = split_replicas(total, w)
        status["stableReplicas"], status["candidateReplicas"] = s, c
    return status
