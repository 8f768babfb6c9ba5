"""AgentRuntime sub-resources and reconciler probes.

Each function is idempotent and takes the store (APIStore or KubeClient):

* :func:`reconcile_facade_route` -- operator-owned Gateway API ``HTTPRoute``
  ``<agent>-facade`` when a default-exposure Gateway is configured and the
  primary facade opts in via ``expose.enabled``; never adopts or deletes a
  route it does not control (``internal/controller/facade_route.go:61-173``).
* :func:`reconcile_facade_rbac` -- ``<agent>-facade`` ServiceAccount, Role
  (agentruntimes/providers get, agentruntimes/status get+patch, secrets get --
  widened to list/watch only for client-key auth --, namespaces get,
  toolpolicies get/list/watch), RoleBinding to the *effective* facade SA, and
  the workspace-reader ClusterRoleBinding scoped to the agent's own Workspace
  (``facade_rbac.go:50-304``).
* :func:`policy_broker_container` -- the policy-broker sidecar (decision port
  8090, metrics/health 8091, ToolPolicy watch scoped to the namespace) injected
  when the operator is configured with a broker image
  (``policy_broker_sidecar.go:46-137``, ``deployment_builder.go:202-210``).
* :func:`reconcile_eval_workers` -- one ``arena-eval-worker-<group>``
  Deployment (+ SA/Role/RoleBinding) per service group that has an eval-enabled
  agent whose framework does not self-evaluate inline (or whose group opts in),
  REDIS_URL resolved like the group's session-api; stale groups are deleted
  (``eval_worker.go:60-459``).
* :func:`reconcile_oidc_jwks` -- fetch ``{issuer}/.well-known/openid-configuration``
  -> ``jwks_uri`` and mirror the JWKS into Secret ``agent-<name>-oidc-jwks``
  (``jwks.json``), stamped with a fetched-at annotation so reconciles inside the
  6 h refresh window skip the HTTP round-trip; failures set ``OIDCJWKSReady``
  False and never block bring-up (``agentruntime_oidc_jwks.go:107-388``).
* :func:`probe_tools` -- bounded-concurrency TCP reachability probes of a
  ToolRegistry's network endpoints (``toolregistry_probe.go:53-155``).
* :func:`provider_health_url` / :func:`check_endpoint_health` -- Provider
  endpoint liveness: any HTTP response (even 401) is reachable; only
  connection failures are unhealthy (``provider_controller.go:701-769``).
"""
from __future__ import annotations

import concurrent.futures as cf
import datetime as _dt
import json
import os
import socket
import time
import urllib.error
import urllib.parse
import urllib.request
from dataclasses import dataclass, field

from .apistore import owner_ref, set_condition

LABEL_NAME = "app.kubernetes.io/name"
LABEL_INSTANCE = "app.kubernetes.io/instance"
LABEL_MANAGED_BY = "app.kubernetes.io/managed-by"
LABEL_COMPONENT = "app.kubernetes.io/component"
LABEL_OMNIA_COMPONENT = "omnia.altairalabs.ai/component"
LABEL_SERVICE_GROUP = "omnia.altairalabs.ai/service-group"
LABEL_READER_FOR = "omnia.altairalabs.ai/workspace-reader-for"
LABEL_CREDENTIAL_KIND = "omnia.altairalabs.ai/credential-kind"
OMNIA_AGENT, OMNIA_OPERATOR = "omnia-agent", "omnia-operator"
EVAL_WORKER = "arena-eval-worker"

POLICY_BROKER_PORT, POLICY_BROKER_HEALTH_PORT = 8090, 8091
EVAL_WORKER_METRICS_PORT = 9090
OIDC_JWKS_KEY = "jwks.json"
OIDC_FETCHED_AT = "omnia.altairalabs.ai/oidc-jwks-fetched-at"
OIDC_REFRESH_S = 6 * 3600
OIDC_TIMEOUT_S = 5.0
OIDC_MOUNT = "/etc/omnia/oidc"
PROBE_INTERVAL_S, PROBE_TIMEOUT_S, MAX_CONCURRENT_PROBES = 60.0, 5.0, 8
HEALTH_TIMEOUT_S, HEALTH_REQUEUE_S = 5.0, 60.0
DEFAULT_PROVIDER_ENDPOINTS = {"claude": "https://api.anthropic.com",
                              "openai": "https://api.openai.com",
                              "gemini": "https://generativelanguage.googleapis.com"}


def _http_get(url: str, timeout: float) -> tuple[int, bytes]:
    req = urllib.request.Request(url, headers={"Accept": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, r.read(1 << 20)
    except urllib.error.HTTPError as e:
        return e.code, e.read(1 << 20)


@dataclass
class OperatorConfig:
    """Operator-wide settings (the reference's manager flags / chart values)."""

    expose_base_domain: str = ""
    expose_gateway_name: str = ""
    expose_gateway_namespace: str = ""
    expose_gateway_section: str = ""
    policy_broker_image: str = ""
    license_api_url: str = ""
    eval_worker_image: str = "ghcr.io/omnia-mi355x/omnia-eval-worker:latest"
    workspace_reader_rbac: bool = False
    session_redis_url: str = ""
    namespace: str = "omnia-system"  # the operator's own namespace (policy ConfigMaps)
    istio: bool | None = None  # None: discover AuthorizationPolicy support from the API
    http_get: object = field(default=_http_get, repr=False)  # (url, timeout) -> (status, body)
    clock: object = field(default=time.time, repr=False)
    dial: object = field(default=None, repr=False)  # (host, port, timeout) -> None | raises

    @classmethod
    def from_env(cls, env=None) -> "OperatorConfig":
        e = os.environ if env is None else env
        return cls(expose_base_domain=e.get("OMNIA_EXPOSE_BASE_DOMAIN", ""),
                   expose_gateway_name=e.get("OMNIA_EXPOSE_GATEWAY", ""),
                   expose_gateway_namespace=e.get("OMNIA_EXPOSE_GATEWAY_NAMESPACE", ""),
                   expose_gateway_section=e.get("OMNIA_EXPOSE_GATEWAY_SECTION", ""),
                   policy_broker_image=e.get("OMNIA_POLICY_BROKER_IMAGE", ""),
                   license_api_url=e.get("OMNIA_LICENSE_API_URL", ""),
                   eval_worker_image=e.get("OMNIA_EVAL_WORKER_IMAGE",
                                           cls.eval_worker_image),
                   workspace_reader_rbac=e.get("OMNIA_WORKSPACE_READER_RBAC", "").lower()
                   in ("1", "true"),
                   session_redis_url=e.get("OMNIA_SESSION_REDIS_URL", ""),
                   namespace=e.get("POD_NAMESPACE", "") or e.get("OMNIA_OPERATOR_NAMESPACE",
                                                                 "omnia-system"),
                   istio={"true": True, "1": True, "false": False, "0": False}.get(
                       e.get("OMNIA_ISTIO_ENABLED", "").lower()))

    @property
    def exposure_configured(self) -> bool:
        return bool(self.expose_gateway_name and self.expose_base_domain)


def _agent_labels(ar: dict) -> dict:
    return {LABEL_NAME: OMNIA_AGENT, LABEL_INSTANCE: ar["metadata"]["name"],
            LABEL_MANAGED_BY: OMNIA_OPERATOR}


def _controlled_by(obj: dict, owner: dict) -> bool:
    uid = owner["metadata"].get("uid")
    return any(r.get("uid") == uid and r.get("controller")
               for r in obj["metadata"].get("ownerReferences") or [])


# ------------------------------------------------------------------ facades
PRIMARY_ORDER = ("websocket", "rest", "a2a", "custom")


def primary_facade(ar: dict) -> dict | None:
    by_type = {f.get("type"): f for f in ar["spec"].get("facades") or []}
    for t in PRIMARY_ORDER:
        if t in by_type:
            return by_type[t]
    return None


def primary_facade_port(ar: dict, default: int = 8080) -> int:
    f = primary_facade(ar)
    return int(f["port"]) if f and f.get("port") else default


def reconcile_facade_route(store, ar: dict, cfg: OperatorConfig) -> dict | None:
    """Returns the route's (host, port) decision, or None when not exposed."""
    ns, name = ar["metadata"]["namespace"], ar["metadata"]["name"]
    rname = name + "-facade"
    existing = store.try_get("HTTPRoute", rname, ns)
    if existing is not None and not _controlled_by(existing, ar):
        return None  # hand-written route: never adopt or delete
    f = primary_facade(ar)
    want = cfg.exposure_configured and f is not None and bool((f.get("expose") or {}).get(
        "enabled"))
    if not want:
        if existing is not None:
            store.delete("HTTPRoute", rname, ns)
        return None
    host = (f.get("expose") or {}).get("host") or f"{name}.{ns}.{cfg.expose_base_domain}"
    port = primary_facade_port(ar)
    parent = {"name": cfg.expose_gateway_name}
    if cfg.expose_gateway_namespace:
        parent["namespace"] = cfg.expose_gateway_namespace
    if cfg.expose_gateway_section:
        parent["sectionName"] = cfg.expose_gateway_section
    store.apply({"apiVersion": "gateway.networking.k8s.io/v1", "kind": "HTTPRoute",
                 "metadata": {"name": rname, "namespace": ns, "labels": _agent_labels(ar),
                              "ownerReferences": [owner_ref(ar)]},
                 "spec": {"parentRefs": [parent], "hostnames": [host],
                          "rules": [{"matches": [{"path": {"type": "PathPrefix",
                                                           "value": "/"}}],
                                     "backendRefs": [{"name": name, "port": port}]}]}})
    return {"host": host, "port": port}


# ------------------------------------------------------------------ RBAC
def workspace_for_namespace(store, ns: str) -> dict | None:
    for ws in store.list("Workspace"):
        if ((ws.get("spec") or {}).get("namespace") or {}).get("name") == ns:
            return ws
    return None


def effective_facade_sa(store, ar: dict) -> str:
    """podOverrides SA > Workspace runtime-default SA > ``<name>-facade``
    (``workspace_runtime_identity.go``)."""
    po = ar["spec"].get("podOverrides") or {}
    if po.get("serviceAccountName"):
        return po["serviceAccountName"]
    ws = workspace_for_namespace(store, ar["metadata"]["namespace"])
    sa = (((ws or {}).get("spec") or {}).get("runtime") or {}).get("serviceAccountName")
    return sa or ar["metadata"]["name"] + "-facade"


def reconcile_facade_rbac(store, ar: dict, cfg: OperatorConfig) -> str:
    ns, name = ar["metadata"]["namespace"], ar["metadata"]["name"]
    sa_name = name + "-facade"
    own = [owner_ref(ar)]
    labels = _agent_labels(ar)
    store.apply({"apiVersion": "v1", "kind": "ServiceAccount",
                 "metadata": {"name": sa_name, "namespace": ns, "labels": labels,
                              "ownerReferences": own}})
    secret_verbs = ["get", "list", "watch"] if (ar["spec"].get("externalAuth") or {}).get(
        "clientKeys") else ["get"]
    store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                 "metadata": {"name": sa_name, "namespace": ns, "labels": labels,
                              "ownerReferences": own},
                 "rules": [
                     {"apiGroups": ["omnia.altairalabs.ai"],
                      "resources": ["agentruntimes", "providers"], "verbs": ["get"]},
                     {"apiGroups": ["omnia.altairalabs.ai"],
                      "resources": ["agentruntimes/status"], "verbs": ["get", "patch"]},
                     {"apiGroups": [""], "resources": ["secrets"], "verbs": secret_verbs},
                     {"apiGroups": [""], "resources": ["namespaces"], "verbs": ["get"]},
                     {"apiGroups": ["omnia.altairalabs.ai"], "resources": ["toolpolicies"],
                      "verbs": ["get", "list", "watch"]}]})
    eff = effective_facade_sa(store, ar)
    store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                 "metadata": {"name": sa_name, "namespace": ns, "labels": labels,
                              "ownerReferences": own},
                 "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role",
                             "name": sa_name},
                 "subjects": [{"kind": "ServiceAccount", "name": eff, "namespace": ns}]})
    if cfg.workspace_reader_rbac:
        ws = workspace_for_namespace(store, ns)
        if ws is not None:  # unresolved workspace: skip, never delete (transient errors)
            crb_name = f"{ns}-{name}-workspace-reader"
            role = f"omnia-workspace-{ws['metadata']['name']}-reader"
            cur = store.try_get("ClusterRoleBinding", crb_name, None)
            if cur is not None and (cur.get("roleRef") or {}).get("name") != role:
                store.delete("ClusterRoleBinding", crb_name, None)  # roleRef is immutable
            store.apply({"apiVersion": "rbac.authorization.k8s.io/v1",
                         "kind": "ClusterRoleBinding",
                         "metadata": {"name": crb_name,
                                      "labels": {**labels, LABEL_READER_FOR: ns}},
                         "roleRef": {"apiGroup": "rbac.authorization.k8s.io",
                                     "kind": "ClusterRole", "name": role},
                         "subjects": [{"kind": "ServiceAccount", "name": eff,
                                       "namespace": ns}]})
    return eff


# ------------------------------------------------------------------ policy broker
def policy_broker_container(ar: dict, cfg: OperatorConfig) -> dict:
    env = [{"name": "OMNIA_AGENT_NAME", "valueFrom": {"fieldRef": {
               "fieldPath": f"metadata.labels['{LABEL_INSTANCE}']"}}},
           {"name": "OMNIA_NAMESPACE", "value": ar["metadata"]["namespace"]},
           {"name": "POLICY_BROKER_LISTEN_ADDR", "value": f":{POLICY_BROKER_PORT}"},
           {"name": "POLICY_BROKER_HEALTH_ADDR", "value": f":{POLICY_BROKER_HEALTH_PORT}"}]
    if cfg.license_api_url:
        env.append({"name": "OPERATOR_API_URL", "value": cfg.license_api_url})
    return {"name": "policy-broker", "image": cfg.policy_broker_image,
            "imagePullPolicy": "IfNotPresent",
            "ports": [{"name": "policy-broker", "containerPort": POLICY_BROKER_PORT,
                       "protocol": "TCP"},
                      {"name": "metrics", "containerPort": POLICY_BROKER_HEALTH_PORT,
                       "protocol": "TCP"}],
            "env": env,
            "readinessProbe": {"httpGet": {"path": "/readyz",
                                           "port": POLICY_BROKER_HEALTH_PORT},
                               "initialDelaySeconds": 3, "periodSeconds": 10},
            "livenessProbe": {"httpGet": {"path": "/healthz",
                                          "port": POLICY_BROKER_HEALTH_PORT},
                              "initialDelaySeconds": 5, "periodSeconds": 20}}


# ------------------------------------------------------------------ eval worker
INLINE_EVAL_FRAMEWORKS = ("promptkit", "omnia-mi355x")


def _self_evaluates(spec: dict) -> bool:
    return (spec.get("framework") or {}).get("type", "omnia-mi355x") in INLINE_EVAL_FRAMEWORKS


def find_service_group(store, ns: str, group: str) -> dict | None:
    ws = workspace_for_namespace(store, ns)
    for sg in ((ws or {}).get("spec") or {}).get("services") or []:
        if sg.get("name", "default") == group:
            return sg
    return None


def resolve_group_redis(sg: dict | None, default: str) -> str:
    """per-component session.redis > group redis > operator default."""
    sg = sg or {}
    return ((sg.get("session") or {}).get("redis") or {}).get("url") or \
        (sg.get("redis") or {}).get("url") or default


def eval_worker_groups(store, ns: str) -> dict[str, dict]:
    needed: dict[str, dict] = {}
    for rt in store.list("AgentRuntime", ns):
        spec = rt["spec"]
        if rt["metadata"].get("deletionTimestamp") or not (spec.get("evals") or {}).get(
                "enabled"):
            continue
        group = spec.get("serviceGroup") or "default"
        sg = find_service_group(store, ns, group)
        if _self_evaluates(spec) and not ((sg or {}).get("evalWorker") or {}).get("enabled"):
            continue
        if group not in needed:
            po = ((sg or {}).get("evalWorker") or {}).get("podOverrides") or \
                (spec.get("evals") or {}).get("podOverrides") or {}
            needed[group] = {"podOverrides": po, "serviceGroup": sg}
    return needed


def eval_worker_deployment(store, ns: str, group: str, info: dict,
                           cfg: OperatorConfig) -> dict:
    name = f"{EVAL_WORKER}-{group}"
    labels = {LABEL_NAME: EVAL_WORKER, LABEL_INSTANCE: name, LABEL_MANAGED_BY: OMNIA_OPERATOR,
              LABEL_OMNIA_COMPONENT: "eval-worker", LABEL_SERVICE_GROUP: group}
    env = [{"name": "NAMESPACE", "value": ns}, {"name": "OMNIA_SERVICE_GROUP", "value": group}]
    redis = resolve_group_redis(info.get("serviceGroup"), cfg.session_redis_url)
    if redis:
        env.append({"name": "REDIS_URL", "value": redis})
    ws = workspace_for_namespace(store, ns)
    if ws is not None:
        env.append({"name": "OMNIA_WORKSPACE_NAME", "value": ws["metadata"]["name"]})
    po = info.get("podOverrides") or {}
    container = {"name": "eval-worker", "image": cfg.eval_worker_image,
                 "command": ["python", "-m", "omnia_amd.ee.eval_worker"],
                 "ports": [{"name": "metrics", "containerPort": EVAL_WORKER_METRICS_PORT}],
                 "env": env + [{"name": e["name"], "value": e.get("value", "")}
                               for e in po.get("extraEnv") or []]}
    if po.get("resources"):
        container["resources"] = po["resources"]
    pod_spec = {"serviceAccountName": po.get("serviceAccountName") or name,
                "containers": [container]}
    for f in ("nodeSelector", "tolerations", "priorityClassName", "imagePullSecrets"):
        if po.get(f):
            pod_spec[f] = po[f]
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": ns, "labels": labels},
            "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                     "template": {"metadata": {
                         "labels": {**labels, LABEL_COMPONENT: "eval-worker",
                                    **(po.get("labels") or {})},
                         "annotations": {"prometheus.io/scrape": "true",
                                         "prometheus.io/port": str(EVAL_WORKER_METRICS_PORT),
                                         "prometheus.io/path": "/metrics",
                                         **(po.get("annotations") or {})}},
                         "spec": pod_spec}}}


def reconcile_eval_workers(store, ns: str, cfg: OperatorConfig) -> list[str]:
    needed = eval_worker_groups(store, ns)
    for group, info in needed.items():
        name = f"{EVAL_WORKER}-{group}"
        labels = {LABEL_NAME: EVAL_WORKER, LABEL_MANAGED_BY: OMNIA_OPERATOR,
                  LABEL_SERVICE_GROUP: group}
        store.apply({"apiVersion": "v1", "kind": "ServiceAccount",
                     "metadata": {"name": name, "namespace": ns, "labels": labels}})
        store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                     "metadata": {"name": name, "namespace": ns, "labels": labels},
                     "rules": [{"apiGroups": ["omnia.altairalabs.ai"],
                                "resources": ["agentruntimes", "providers"],
                                "verbs": ["get", "list", "watch"]},
                               {"apiGroups": [""], "resources": ["secrets"],
                                "verbs": ["get"]}]})
        store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                     "metadata": {"name": name, "namespace": ns, "labels": labels},
                     "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role",
                                 "name": name},
                     "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": ns}]})
        store.apply(eval_worker_deployment(store, ns, group, info, cfg))
    sel = {"matchLabels": {LABEL_NAME: EVAL_WORKER, LABEL_MANAGED_BY: OMNIA_OPERATOR}}
    for kind in ("Deployment", "ServiceAccount", "Role", "RoleBinding"):
        for o in store.list(kind, ns, sel):
            if (o["metadata"].get("labels") or {}).get(LABEL_SERVICE_GROUP) not in needed:
                store.delete(kind, o["metadata"]["name"], ns)
    return sorted(needed)


# ------------------------------------------------------------------ OIDC JWKS mirror
def oidc_secret_name(agent: str) -> str:
    return f"agent-{agent}-oidc-jwks"


def _rfc3339(t: float) -> str:
    return _dt.datetime.fromtimestamp(t, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _parse_rfc3339(s: str) -> float:
    return _dt.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(
        tzinfo=_dt.timezone.utc).timestamp()


def fetch_jwks(issuer: str, cfg: OperatorConfig) -> bytes:
    disc_url = issuer.rstrip("/") + "/.well-known/openid-configuration"
    try:
        code, body = cfg.http_get(disc_url, OIDC_TIMEOUT_S)
    except (OSError, ValueError) as e:
        raise RuntimeError(f"fetch discovery: GET {disc_url}: {e}") from None
    if code != 200:
        raise RuntimeError(f"fetch discovery: GET {disc_url}: status {code}")
    try:
        jwks_uri = json.loads(body).get("jwks_uri", "")
    except ValueError as e:
        raise RuntimeError(f"parse discovery: {e}") from None
    if not jwks_uri:
        raise RuntimeError("discovery document missing jwks_uri")
    try:
        code, blob = cfg.http_get(jwks_uri, OIDC_TIMEOUT_S)
    except (OSError, ValueError) as e:
        raise RuntimeError(f"fetch jwks: GET {jwks_uri}: {e}") from None
    if code != 200:
        raise RuntimeError(f"fetch jwks: GET {jwks_uri}: status {code}")
    try:
        keys = json.loads(blob).get("keys")
    except (ValueError, AttributeError) as e:
        raise RuntimeError(f"jwks is not valid JSON: {e}") from None
    if not keys:
        raise RuntimeError("jwks has no keys")
    return blob


def reconcile_oidc_jwks(store, ar: dict, st: dict, cfg: OperatorConfig) -> float | None:
    """Returns the requeue delay for the next refresh (None: OIDC not configured)."""
    import base64

    ns, name = ar["metadata"]["namespace"], ar["metadata"]["name"]
    gen = ar["metadata"].get("generation")
    oidc = (ar["spec"].get("externalAuth") or {}).get("oidc")
    sname = oidc_secret_name(name)
    if not oidc:
        if store.try_get("Secret", sname, ns) is not None:
            store.delete("Secret", sname, ns)
        return None
    issuer = oidc.get("issuer", "")
    if not issuer:
        set_condition(st, "OIDCJWKSReady", False, "MissingIssuer",
                      "spec.externalAuth.oidc.issuer is empty", gen)
        return None
    now = cfg.clock()
    cur = store.try_get("Secret", sname, ns)
    if cur is not None:
        at = ((cur["metadata"].get("annotations") or {}).get(OIDC_FETCHED_AT))
        if at and OIDC_JWKS_KEY in (cur.get("data") or {}):
            try:
                elapsed = now - _parse_rfc3339(at)
            except ValueError:
                elapsed = OIDC_REFRESH_S
            if elapsed < OIDC_REFRESH_S:
                set_condition(st, "OIDCJWKSReady", True, "JWKSUpdated",
                              f"JWKS mirrored from {issuer} (cached)", gen)
                return OIDC_REFRESH_S - elapsed
    try:
        blob = fetch_jwks(issuer, cfg)
    except RuntimeError as e:
        set_condition(st, "OIDCJWKSReady", False, "DiscoveryFailed", str(e)[:300], gen)
        return OIDC_REFRESH_S if cur is not None else 60.0
    store.apply({"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                 "metadata": {"name": sname, "namespace": ns,
                              "labels": {LABEL_CREDENTIAL_KIND: "agent-oidc-jwks",
                                         LABEL_INSTANCE: name,
                                         LABEL_MANAGED_BY: OMNIA_OPERATOR},
                              "annotations": {OIDC_FETCHED_AT: _rfc3339(now)},
                              "ownerReferences": [owner_ref(ar)]},
                 "data": {OIDC_JWKS_KEY: base64.b64encode(blob).decode()}})
    set_condition(st, "OIDCJWKSReady", True, "JWKSUpdated", f"JWKS mirrored from {issuer}", gen)
    return OIDC_REFRESH_S


# ------------------------------------------------------------------ probes
def is_network_endpoint(ep: str) -> bool:
    return bool(ep) and not ep.startswith(("client://", "stdio://"))


def probe_address(ep: str) -> tuple[str, int] | None:
    u = urllib.parse.urlsplit(ep)
    if u.scheme and u.netloc:
        try:
            port = u.port
        except ValueError:
            return None
        return u.hostname or "", port or (443 if u.scheme == "https" else 80)
    host, sep, port = ep.rpartition(":")
    if sep and host and port.isdigit():
        return host.strip("[]"), int(port)
    return None


def _tcp_dial(host: str, port: int, timeout: float) -> None:
    socket.create_connection((host, port), timeout=timeout).close()


def probe_tools(tools: list[dict], timeout: float, dial=None) -> None:
    """TCP-dial every network endpoint concurrently (bounded); marks each tool
    Available/Unavailable with lastChecked + error.  No tool invocation."""
    dial = dial or _tcp_dial
    now = _rfc3339(time.time())

    def one(t):
        t["lastChecked"] = now
        addr = probe_address(t["endpoint"])
        if addr is None:
            t["status"] = "Unavailable"
            t["error"] = f"probe: unrecognized endpoint address {t['endpoint']!r}"
            return
        try:
            dial(addr[0], addr[1], timeout)
        except OSError as e:
            t["status"] = "Unavailable"
            t["error"] = f"probe failed: {e}"
            return
        t["status"] = "Available"
        t.pop("error", None)

    targets = [t for t in tools if is_network_endpoint(t.get("endpoint", ""))]
    if not targets:
        return
    with cf.ThreadPoolExecutor(min(MAX_CONCURRENT_PROBES, len(targets))) as ex:
        list(ex.map(one, targets))


def provider_health_url(spec: dict) -> str:
    t = spec.get("type")
    if t in ("mock", "local") or spec.get("platform"):
        return ""  # no endpoint / cloud-SDK auth
    if spec.get("role", "llm") in ("tts", "stt", "image"):
        return ""  # no liveness endpoint; synthesis endpoints cost money
    base = spec.get("baseURL") or DEFAULT_PROVIDER_ENDPOINTS.get(t, "")
    if not base:
        return ""
    return base.rstrip("/") + "/api/tags" if t == "ollama" else base


def check_endpoint_health(url: str, cfg: OperatorConfig) -> str | None:
    """None when reachable (any HTTP status counts), else the error text."""
    try:
        cfg.http_get(url, HEALTH_TIMEOUT_S)
    except (OSError, ValueError) as e:
        return str(e) or type(e).__name__
    return None
