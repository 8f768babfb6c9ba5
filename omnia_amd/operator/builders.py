"""Pod/Service/autoscaling object builders for an AgentRuntime.

Mirrors ``internal/controller/deployment_builder*.go``, ``autoscaling.go``,
``pdb.go``, ``tools_config.go``: two containers (``facade`` + ``runtime``),
ports facade 8080 / health 8081 / runtime gRPC 9000 / metrics 9001 / A2A 9999 /
MCP 9998 (+ mgmt twins 18080/19999/19998), pack at /etc/omnia/pack, tools at
/etc/omnia/tools, tool secrets at /etc/omnia/tool-secrets, labels
``app.kubernetes.io/{name,instance,managed-by}`` + ``omnia.altairalabs.ai/
{component,track,mode}``, a config-hash pod annotation that rolls pods on any
config change, HPA (memory 70 % / CPU 90 %, 300 s scale-down stabilisation) or a
KEDA ScaledObject on ``sum(omnia_agent_connections_active{...})`` (threshold
200, scale-to-zero allowed), and a PDB (minAvailable 1).

MI355X addition: a ``local`` Provider puts ``amd.com/gpu: <tp>`` on the runtime
container and passes the engine block as ``OMNIA_ENGINE_*`` env.
"""
from __future__ import annotations

import hashlib
import json
import os

import yaml

from ..runtime.config import RuntimeConfig
from ..runtime.context_store import parse_ttl
from .apistore import owner_ref

LABEL_NAME = "app.kubernetes.io/name"
LABEL_INSTANCE = "app.kubernetes.io/instance"
LABEL_MANAGED_BY = "app.kubernetes.io/managed-by"
LABEL_COMPONENT = "omnia.altairalabs.ai/component"
LABEL_TRACK = "omnia.altairalabs.ai/track"
LABEL_MODE = "omnia.altairalabs.ai/mode"
LABEL_PACK_NAME = "omnia.altairalabs.ai/pack-name"
FINALIZER = "agentruntime.omnia.altairalabs.ai/finalizer"
ANN_CONFIG_HASH = "omnia.altairalabs.ai/config-hash"

FACADE_PORT, FACADE_HEALTH_PORT = 8080, 8081
RUNTIME_GRPC_PORT, RUNTIME_HEALTH_PORT = 9000, 9001
A2A_PORT, MCP_PORT = 9999, 9998
MGMT_PORTS = {"facade-mgmt": 18080, "a2a-mgmt": 19999, "mcp-mgmt": 19998}
FACADE_IMAGE = "ghcr.io/omnia-mi355x/omnia-facade:latest"
RUNTIME_IMAGE = "ghcr.io/omnia-mi355x/omnia-runtime-rocm:latest"
KEDA_DEFAULT_THRESHOLD = 200


def selector_labels(ar: dict, track: str = "stable") -> dict:
    return {LABEL_NAME: "omnia-agent", LABEL_INSTANCE: ar["metadata"]["name"],
            LABEL_TRACK: track}


def pod_labels(ar: dict, track: str = "stable") -> dict:
    return {**selector_labels(ar, track), LABEL_MANAGED_BY: "omnia-operator",
            LABEL_COMPONENT: "agent", LABEL_MODE: ar["spec"].get("mode", "agent")}


def tools_configmap(ar: dict, registry: dict | None, tool_access: list | None = None) -> dict:
    """The runtime's tool config: the registry's handlers, the registry name and
    the compiled AgentPolicy tool access (``operator/policies.py``)."""
    handlers = []
    for h in (registry or {}).get("spec", {}).get("handlers", []):
        e = {k: v for k, v in h.items() if k in ("name", "type", "endpoint", "tool", "httpConfig",
                                                 "grpcConfig", "mcpConfig", "openAPIConfig",
                                                 "clientConfig", "timeout", "auth")}
        handlers.append(e)
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": ar["metadata"]["name"] + "-tools",
                         "namespace": ar["metadata"]["namespace"],
                         "labels": pod_labels(ar), "ownerReferences": [owner_ref(ar)]},
            "data": {"tools.yaml": yaml.safe_dump(
                {"handlers": handlers,
                 **({"registry": registry["metadata"]["name"]} if registry else {}),
                 **({"toolAccess": tool_access} if tool_access else {})}, sort_keys=True)}}


def runtime_config(ar: dict, pack: dict, providers: list[dict], registry: dict | None) -> RuntimeConfig:
    spec = ar["spec"]
    md = ar["metadata"]
    ctx = spec.get("context") or {}
    llm = next((p for p in providers if p["spec"].get("role", "llm") == "llm"), None)
    pspec = dict((llm or {}).get("spec") or {"type": "mock"})
    pspec["name"] = (llm or {}).get("metadata", {}).get("name", "mock")
    c = RuntimeConfig(
        agent_name=md["name"], namespace=md["namespace"], promptpack_path="/etc/omnia/pack",
        promptpack_name=pack["spec"]["packName"], promptpack_version=pack["spec"]["version"],
        mode=spec.get("mode", "agent"), output_format=spec.get("outputFormat", ""),
        output_schema=spec.get("outputSchema"), context_type=ctx.get("type", "memory"),
        context_url=(ctx.get("storeRef") or {}).get("url", ""),
        context_ttl_s=parse_ttl(ctx.get("ttl", "24h")) or 86400, provider=pspec,
        extra_providers=[dict(p["spec"], name=p["metadata"]["name"]) for p in providers
                         if p is not llm],
        tools_config_path="/etc/omnia/tools")
    if (spec.get("duplex") or {}).get("enabled"):
        c.duplex = dict(spec["duplex"])
    d = pspec.get("defaults") or {}
    c.context_window = int(d.get("contextWindow", 0) or 0)
    c.truncation = d.get("truncationStrategy", "sliding")
    if pspec.get("type") == "local":
        eng = dict(pspec.get("engine") or {})
        c.engine = {"model": eng.get("model") or pspec.get("model"), "tp": eng.get("tp", 1),
                    "max_batch": eng.get("maxBatch", 256),
                    "kv_fraction": eng.get("kvFraction", 0.85),
                    "max_model_len": eng.get("maxModelLen", 8192),
                    "block_size": eng.get("blockSize", 32), "dtype": eng.get("dtype",
                                                                             "bfloat16")}
        extra = {"swapGiB": "swap_gib", "mixedBudget": "mixed_budget", "epMode": "ep_mode",
                 "ep": "ep",
                 "numBlocks": "num_blocks", "useGraphs": "use_graphs", "device": "device",
                 "cpThreshold": "cp_threshold", "tokenizer": "tokenizer",
                 "checkpoint": "checkpoint"}
        for k, v in eng.items():  # the engine knobs beyond the core sizing fields
            if k in extra and v is not None:
                c.engine[extra[k]] = v
    mem = spec.get("memory") or {}
    c.memory_enabled = bool(mem.get("enabled"))
    ret = mem.get("retrieval") or {}
    if ret.get("strategy"):
        c.memory_strategy = ret["strategy"]
    if ret.get("limit"):
        c.memory_limit = int(ret["limit"])
    if (ret.get("accessFilter") or {}).get("denyCEL"):
        c.memory_deny_cel = ret["accessFilter"]["denyCEL"]
    c.eval_enabled = bool((spec.get("evals") or {}).get("enabled"))
    c.eval_inline_groups = list(((spec.get("evals") or {}).get("inline") or {}).get("groups")
                                or [])
    return c


def _env_list(env: dict) -> list[dict]:
    return [{"name": k, "value": str(v)} for k, v in sorted(env.items())]


def _mgmt_enabled(f: dict | None) -> bool:
    """facades[].managementPlane, default true (agentruntime_types.go:186-192)."""
    return f is not None and f.get("managementPlane") is not False


def management_endpoints(ar: dict) -> dict | None:
    """Twin listener ports per surface (``deployment_builder_management.go:84-103``):
    the primary facade's WS twin, the A2A twin of a dual-protocol pod, the MCP twin;
    published as ``status.managementEndpoints`` and allocated on the facade."""
    facs = ar["spec"].get("facades", [])
    by = {f["type"]: f for f in facs}
    primary = facs[0] if facs else None
    me = {}
    if _mgmt_enabled(primary):
        me["ws"] = MGMT_PORTS["facade-mgmt"]
    if primary is not None and primary.get("type") != "a2a" and _mgmt_enabled(by.get("a2a")):
        me["a2a"] = MGMT_PORTS["a2a-mgmt"]
    if _mgmt_enabled(by.get("mcp")):
        me["mcp"] = MGMT_PORTS["mcp-mgmt"]
    return me or None


def facade_env(ar: dict, mgmt_jwks_url: str | None = None) -> dict:
    spec, md = ar["spec"], ar["metadata"]
    fac = {f["type"]: f for f in spec.get("facades", [])}
    env = {"OMNIA_AGENT_NAME": md["name"], "OMNIA_NAMESPACE": md["namespace"],
           "OMNIA_FACADE_PORT": str(FACADE_PORT),
           "OMNIA_RUNTIME_ADDRESS": f"127.0.0.1:{RUNTIME_GRPC_PORT}",
           "OMNIA_MODE": spec.get("mode", "agent"),
           "OMNIA_FACADE_TYPES": ",".join(sorted(fac))}
    h = next((f.get("handler") for f in spec.get("facades", []) if f.get("handler")), None)
    if h:
        env["OMNIA_HANDLER_MODE"] = h
    if "a2a" in fac:
        env["OMNIA_A2A_PORT"] = str(fac["a2a"].get("port", A2A_PORT))
    if "mcp" in fac:
        env["OMNIA_MCP_ENABLED"] = "true"
        env["OMNIA_MCP_PORT"] = str(fac["mcp"].get("port", MCP_PORT))
    if spec.get("inputSchema") is not None:
        env["OMNIA_INPUT_SCHEMA"] = json.dumps(spec["inputSchema"])
    if spec.get("outputSchema") is not None:
        env["OMNIA_OUTPUT_SCHEMA"] = json.dumps(spec["outputSchema"])
    ea = spec.get("externalAuth") or {}
    oidc = ea.get("oidc") or {}
    if oidc:
        env["OMNIA_OIDC_ISSUER"] = oidc.get("issuer", "")
        if oidc.get("audience"):
            env["OMNIA_OIDC_AUDIENCE"] = oidc["audience"]
        env["OMNIA_OIDC_JWKS_FILE"] = "/etc/omnia/oidc/jwks.json"
    if ea.get("edgeTrust") is not None:  # presence enables it (external_auth_types.go:59)
        env["OMNIA_EDGE_TRUST"] = "true"
        if ea["edgeTrust"]:
            env["OMNIA_EDGE_TRUST_CONFIG"] = json.dumps(ea["edgeTrust"], sort_keys=True)
    # blip-resume route hints share the Redis of a Redis context store
    # (internal/controller/deployment_builder_env.go:147-162)
    ctx = spec.get("context") or {}
    if ctx.get("type") == "redis" and (ctx.get("storeRef") or {}).get("url"):
        env["OMNIA_ROUTE_REDIS_URL"] = ctx["storeRef"]["url"]
    # management-plane twin listeners + the dashboard JWKS their chain trusts
    # (deployment_builder_env.go:124-134; empty URL = no dashboard installed)
    me = management_endpoints(ar) or {}
    for surface, key in (("ws", "OMNIA_INTERNAL_FACADE_PORT"), ("a2a", "OMNIA_INTERNAL_A2A_PORT"),
                         ("mcp", "OMNIA_INTERNAL_MCP_PORT")):
        if surface in me:
            env[key] = str(me[surface])
    url = os.environ.get("OMNIA_MGMT_PLANE_JWKS_URL", "") if mgmt_jwks_url is None \
        else mgmt_jwks_url
    if url:
        env["OMNIA_MGMT_PLANE_JWKS_URL"] = url
    ws = (spec.get("workspaceRef") or {}).get("name") or md.get("labels", {}).get(
        "omnia.altairalabs.ai/workspace", "")
    if ws:
        env["OMNIA_WORKSPACE_NAME"] = ws
    return env


def config_hash(*parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(json.dumps(p, sort_keys=True, default=str).encode())
    return h.hexdigest()[:16]


def deployment(ar: dict, rc: RuntimeConfig, pack_cm: str, track: str = "stable",
               replicas: int | None = None, extra_hash=None,
               facade_extra: dict | None = None, sidecars: list | None = None,
               sa_name: str | None = None) -> dict:
    spec, md = ar["spec"], ar["metadata"]
    rt = spec.get("runtime") or {}
    po = spec.get("podOverrides") or {}
    name = md["name"] + ("" if track == "stable" else "-candidate")
    fenv = facade_env(ar)
    fenv.update(facade_extra or {})
    renv = rc.to_env()
    for e in rt.get("extraEnv") or []:
        renv[e["name"]] = e.get("value", "")
    for e in po.get("extraEnv") or []:
        fenv[e["name"]] = e.get("value", "")
        renv[e["name"]] = e.get("value", "")
    ports = [{"name": "facade", "containerPort": FACADE_PORT},
             {"name": "facade-health", "containerPort": FACADE_HEALTH_PORT}]
    types = {f["type"] for f in spec.get("facades", [])}
    if "a2a" in types:
        ports.append({"name": "a2a", "containerPort": A2A_PORT})
    if "mcp" in types:
        ports.append({"name": "mcp", "containerPort": MCP_PORT})
    me = management_endpoints(ar) or {}
    for surface, n in (("ws", "facade-mgmt"), ("a2a", "a2a-mgmt"), ("mcp", "mcp-mgmt")):
        if surface in me:
            ports.append({"name": n, "containerPort": MGMT_PORTS[n]})
    resources = dict(rt.get("resources") or {})
    if rc.provider.get("type") == "local" and rc.engine.get("device", "cuda") != "cpu":
        n = int(rc.engine.get("tp", 1))
        if rc.engine.get("ep_mode") == "a2a":  # one GPU per EP rank
            n = max(n, int(rc.engine.get("ep", 1) or 1))
        resources.setdefault("limits", {})["amd.com/gpu"] = str(n)
        resources.setdefault("requests", {})["amd.com/gpu"] = str(n)
    fw = spec.get("framework") or {}
    containers = [
        {"name": "facade", "image": FACADE_IMAGE, "ports": ports, "env": _env_list(fenv),
         "readinessProbe": {"httpGet": {"path": "/readyz", "port": FACADE_PORT},
                            "periodSeconds": 5},
         "livenessProbe": {"httpGet": {"path": "/healthz", "port": FACADE_PORT},
                           "periodSeconds": 20},
         "securityContext": {"runAsNonRoot": True, "allowPrivilegeEscalation": False,
                             "capabilities": {"drop": ["ALL"]}}},
        {"name": "runtime", "image": fw.get("image") or RUNTIME_IMAGE,
         "ports": [{"name": "grpc", "containerPort": RUNTIME_GRPC_PORT},
                   {"name": "metrics", "containerPort": RUNTIME_HEALTH_PORT}],
         "env": _env_list(renv), "resources": resources,
         "volumeMounts": [{"name": "promptpack-config", "mountPath": "/etc/omnia/pack"},
                          {"name": "tools-config", "mountPath": "/etc/omnia/tools"},
                          {"name": "pack-cache", "mountPath": "/var/run/omnia/pack-cache"},
                          *(rt.get("volumeMounts") or [])],
         "readinessProbe": {"httpGet": {"path": "/healthz", "port": RUNTIME_HEALTH_PORT},
                            "initialDelaySeconds": 5, "periodSeconds": 10},
         "livenessProbe": {"httpGet": {"path": "/healthz", "port": RUNTIME_HEALTH_PORT},
                           "initialDelaySeconds": 15, "periodSeconds": 20}},
    ]
    volumes = [{"name": "promptpack-config", "configMap": {"name": pack_cm}},
               {"name": "tools-config", "configMap": {"name": md["name"] + "-tools"}},
               {"name": "pack-cache", "emptyDir": {}}, *(rt.get("volumes") or [])]
    if (spec.get("externalAuth") or {}).get("oidc"):
        # the operator-mirrored JWKS Secret (agentruntime_oidc_jwks.go); optional so
        # the pod starts before the first fetch lands (OIDC tokens 401 until then)
        volumes.append({"name": "oidc-jwks", "secret": {
            "secretName": f"agent-{md['name']}-oidc-jwks", "optional": True}})
        containers[0].setdefault("volumeMounts", []).append(
            {"name": "oidc-jwks", "mountPath": "/etc/omnia/oidc", "readOnly": True})
    containers += list(sidecars or [])
    labels = {**pod_labels(ar, track), **(po.get("labels") or {})}
    ann = {ANN_CONFIG_HASH: config_hash(fenv, renv, extra_hash),
           **(po.get("annotations") or {}), **(spec.get("extraPodAnnotations") or {})}
    pod_spec = {"containers": containers, "volumes": volumes,
                "terminationGracePeriodSeconds": 45,
                "serviceAccountName": sa_name or po.get("serviceAccountName") or
                md["name"] + "-facade"}
    for f in ("nodeSelector", "tolerations", "affinity"):
        v = po.get(f) or rt.get(f)
        if v:
            pod_spec[f] = v
    if po.get("priorityClassName"):
        pod_spec["priorityClassName"] = po["priorityClassName"]
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": md["namespace"], "labels": labels,
                         "ownerReferences": [owner_ref(ar)]},
            "spec": {"replicas": rt.get("replicas", 1) if replicas is None else replicas,
                     "selector": {"matchLabels": selector_labels(ar, track)},
                     "template": {"metadata": {"labels": labels, "annotations": ann},
                                  "spec": pod_spec}}}


def service(ar: dict) -> dict:
    md = ar["metadata"]
    types = {f["type"] for f in ar["spec"].get("facades", [])}
    ports = [{"name": "facade", "port": FACADE_PORT, "targetPort": FACADE_PORT,
              "appProtocol": "http"}]
    if "a2a" in types:
        ports.append({"name": "a2a", "port": A2A_PORT, "targetPort": A2A_PORT})
    if "mcp" in types:
        ports.append({"name": "mcp", "port": MCP_PORT, "targetPort": MCP_PORT})
    me = management_endpoints(ar) or {}
    for surface, n in (("ws", "facade-mgmt"), ("a2a", "a2a-mgmt"), ("mcp", "mcp-mgmt")):
        if surface in me:  # appendManagementServicePorts (deployment_builder_management.go)
            ports.append({"name": n, "port": MGMT_PORTS[n], "targetPort": MGMT_PORTS[n],
                          "appProtocol": "http"})
    ports.append({"name": "metrics", "port": RUNTIME_HEALTH_PORT,
                  "targetPort": RUNTIME_HEALTH_PORT})
    sel = {LABEL_NAME: "omnia-agent", LABEL_INSTANCE: md["name"]}
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": md["name"], "namespace": md["namespace"],
                         "labels": pod_labels(ar), "ownerReferences": [owner_ref(ar)]},
            "spec": {"selector": sel, "ports": ports, "type": "ClusterIP"}}


def pdb(ar: dict) -> dict:
    md = ar["metadata"]
    return {"apiVersion": "policy/v1", "kind": "PodDisruptionBudget",
            "metadata": {"name": md["name"], "namespace": md["namespace"],
                         "ownerReferences": [owner_ref(ar)]},
            "spec": {"minAvailable": 1, "selector": {"matchLabels": selector_labels(ar)}}}


def hpa(ar: dict, a: dict) -> dict:
    md = ar["metadata"]
    return {"apiVersion": "autoscaling/v2", "kind": "HorizontalPodAutoscaler",
            "metadata": {"name": md["name"], "namespace": md["namespace"],
                         "ownerReferences": [owner_ref(ar)]},
            "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment",
                                        "name": md["name"]},
                     "minReplicas": max(1, a.get("minReplicas", 1)),
                     "maxReplicas": a.get("maxReplicas", 10),
                     "metrics": [
                         {"type": "Resource", "resource": {"name": "memory", "target": {
                             "type": "Utilization",
                             "averageUtilization": a.get("targetMemoryUtilizationPercentage",
                                                         70)}}},
                         {"type": "Resource", "resource": {"name": "cpu", "target": {
                             "type": "Utilization",
                             "averageUtilization": a.get("targetCPUUtilizationPercentage",
                                                         90)}}}],
                     "behavior": {"scaleDown": {"stabilizationWindowSeconds": a.get(
                         "scaleDownStabilizationSeconds", 300)}}}}


def scaled_object(ar: dict, a: dict, prometheus: str = "http://prometheus:9090") -> dict:
    md = ar["metadata"]
    k = a.get("keda") or {}
    triggers = k.get("triggers") or [{
        "type": "prometheus", "metadata": {
            "serverAddress": prometheus,
            "query": (f'sum(omnia_agent_connections_active{{agent="{md["name"]}",'
                      f'namespace="{md["namespace"]}"}})'),
            "threshold": str(k.get("connectionThreshold") or KEDA_DEFAULT_THRESHOLD)}}]
    return {"apiVersion": "keda.sh/v1alpha1", "kind": "ScaledObject",
            "metadata": {"name": md["name"], "namespace": md["namespace"],
                         "ownerReferences": [owner_ref(ar)]},
            "spec": {"scaleTargetRef": {"name": md["name"]},
                     "minReplicaCount": a.get("minReplicas", 0),
                     "maxReplicaCount": a.get("maxReplicas", 10),
                     "pollingInterval": k.get("pollingInterval", 30),
                     "cooldownPeriod": k.get("cooldownPeriod", 300), "triggers": triggers}}
