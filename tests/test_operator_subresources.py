"""AgentRuntime sub-resources (facade route, facade RBAC, policy-broker sidecar,
eval workers, OIDC JWKS mirror) and reconciler probes (ToolRegistry TCP probe,
Provider endpoint health), mirroring the reference's unit/envtest cases in
``internal/controller/{facade_route,facade_rbac,eval_worker,agentruntime_oidc_jwks,
toolregistry_probe,provider_controller}_test.go``."""
import base64
import json
import os
import socket

import pytest

from omnia_amd.api import crds
from omnia_amd.cli import load_manifests
from omnia_amd.operator import subresources as SR
from omnia_amd.operator.apistore import get_condition
from omnia_amd.operator.controllers import (AgentRuntimeReconciler, PromptPackReconciler,
                                            ProviderReconciler, ToolRegistryReconciler)
from omnia_amd.operator.manager import new_store

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "examples", "echo-function", "manifests.yaml")


class FakeIdP:
    def __init__(self, issuer="https://idp.example.com", keys=None):
        self.issuer = issuer
        self.keys = keys if keys is not None else [{"kty": "RSA", "kid": "k1", "n": "AQ",
                                                    "e": "AQAB"}]
        self.calls = []
        self.down = False

    def get(self, url, timeout):
        self.calls.append(url)
        if self.down:
            raise OSError("connection refused")
        if url == self.issuer + "/.well-known/openid-configuration":
            return 200, json.dumps({"issuer": self.issuer,
                                    "jwks_uri": self.issuer + "/keys"}).encode()
        if url == self.issuer + "/keys":
            return 200, json.dumps({"keys": self.keys}).encode()
        return 404, b"{}"


def setup_store(mutate=None, cfg=None):
    """Echo-function manifests reconciled in dependency order."""
    store = new_store()
    docs = load_manifests([ECHO])
    for d in docs:
        if d["kind"] == "AgentRuntime" and mutate:
            mutate(d)
        store.apply(d)
    cfg = cfg or SR.OperatorConfig()
    for pp in store.list("PromptPack"):
        PromptPackReconciler().reconcile(store, "default", pp["metadata"]["name"])
    for pv in store.list("Provider"):
        ProviderReconciler(None, cfg).reconcile(store, "default", pv["metadata"]["name"])
    r = AgentRuntimeReconciler(None, cfg)
    return store, r


def reconcile(store, r, name="echo"):
    return r.reconcile(store, "default", name)


def test_facade_rbac_objects_and_effective_sa():
    store, r = setup_store()
    reconcile(store, r)
    sa = store.get("ServiceAccount", "echo-facade")
    ar = store.get("AgentRuntime", "echo")
    assert sa["metadata"]["ownerReferences"][0]["uid"] == ar["metadata"]["uid"]
    role = store.get("Role", "echo-facade")
    res = {tuple(x["resources"]): x["verbs"] for x in role["rules"]}
    assert res[("agentruntimes", "providers")] == ["get"]
    assert res[("agentruntimes/status",)] == ["get", "patch"]
    assert res[("secrets",)] == ["get"]
    rb = store.get("RoleBinding", "echo-facade")
    assert rb["subjects"][0]["name"] == "echo-facade"
    dep = store.get("Deployment", "echo")
    assert dep["spec"]["template"]["spec"]["serviceAccountName"] == "echo-facade"

    # podOverrides SA wins and the binding follows it; client keys widen secrets
    def mut(d):
        d["spec"]["podOverrides"] = {"serviceAccountName": "wi-sa"}
        d["spec"]["externalAuth"] = {"clientKeys": {"defaultRole": "viewer"}}

    store, r = setup_store(mut)
    reconcile(store, r)
    assert store.get("RoleBinding", "echo-facade")["subjects"][0]["name"] == "wi-sa"
    role = store.get("Role", "echo-facade")
    assert {tuple(x["resources"]): x["verbs"] for x in role["rules"]}[("secrets",)] == \
        ["get", "list", "watch"]
    assert store.get("Deployment", "echo")["spec"]["template"]["spec"][
        "serviceAccountName"] == "wi-sa"


def test_workspace_reader_binding_scoped_to_own_workspace():
    cfg = SR.OperatorConfig(workspace_reader_rbac=True)
    store, r = setup_store(cfg=cfg)
    reconcile(store, r)
    assert store.try_get("ClusterRoleBinding", "default-echo-workspace-reader", None) is None
    store.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "team"},
                 "spec": {"displayName": "T", "namespace": {"name": "default"},
                          "runtime": {"serviceAccountName": "team-runtime"}}})
    reconcile(store, r)
    crb = store.get("ClusterRoleBinding", "default-echo-workspace-reader", None)
    assert crb["roleRef"]["name"] == "omnia-workspace-team-reader"
    assert crb["subjects"][0]["name"] == "team-runtime"  # workspace runtime-default SA
    assert crb["metadata"]["labels"][SR.LABEL_READER_FOR] == "default"


def test_facade_route_exposure_and_ownership():
    def mut(d):
        d["spec"]["facades"][0]["expose"] = {"enabled": True}

    off = SR.OperatorConfig()
    store, r = setup_store(mut, off)
    reconcile(store, r)
    assert store.try_get("HTTPRoute", "echo-facade") is None  # platform not configured
    cfg = SR.OperatorConfig(expose_base_domain="agents.example.com",
                            expose_gateway_name="omnia-gw", expose_gateway_namespace="gw",
                            expose_gateway_section="https")
    store, r = setup_store(mut, cfg)
    reconcile(store, r)
    rt = store.get("HTTPRoute", "echo-facade")
    assert rt["spec"]["hostnames"] == ["echo.default.agents.example.com"]
    assert rt["spec"]["parentRefs"] == [{"name": "omnia-gw", "namespace": "gw",
                                         "sectionName": "https"}]
    be = rt["spec"]["rules"][0]["backendRefs"][0]
    assert be == {"name": "echo", "port": 8080}
    assert store.get("AgentRuntime", "echo")["status"]["externalURL"] == \
        "https://echo.default.agents.example.com"
    # opt out -> the owned route is removed
    ar = store.get("AgentRuntime", "echo")
    ar["spec"]["facades"][0]["expose"] = {"enabled": False}
    store.update(ar)
    reconcile(store, r)
    assert store.try_get("HTTPRoute", "echo-facade") is None
    # a hand-written route of the same name is never touched
    store.create({"apiVersion": "gateway.networking.k8s.io/v1", "kind": "HTTPRoute",
                  "metadata": {"name": "echo-facade", "namespace": "default"},
                  "spec": {"hostnames": ["mine.example.com"]}})
    ar = store.get("AgentRuntime", "echo")
    ar["spec"]["facades"][0]["expose"] = {"enabled": True, "host": "x.example.com"}
    store.update(ar)
    reconcile(store, r)
    assert store.get("HTTPRoute", "echo-facade")["spec"]["hostnames"] == ["mine.example.com"]


def test_policy_broker_sidecar_injection():
    store, r = setup_store()
    reconcile(store, r)
    names = [c["name"] for c in store.get("Deployment", "echo")["spec"]["template"]["spec"][
        "containers"]]
    assert "policy-broker" not in names
    cfg = SR.OperatorConfig(policy_broker_image="registry/omnia-policy-broker:1",
                            license_api_url="http://operator:8082")
    store, r = setup_store(cfg=cfg)
    reconcile(store, r)
    cs = {c["name"]: c for c in store.get("Deployment", "echo")["spec"]["template"]["spec"][
        "containers"]}
    pb = cs["policy-broker"]
    assert pb["image"] == "registry/omnia-policy-broker:1"
    assert {p["name"]: p["containerPort"] for p in pb["ports"]} == {"policy-broker": 8090,
                                                                   "metrics": 8091}
    env = {e["name"]: e for e in pb["env"]}
    assert env["OMNIA_NAMESPACE"]["value"] == "default"
    assert env["OPERATOR_API_URL"]["value"] == "http://operator:8082"
    assert "fieldRef" in env["OMNIA_AGENT_NAME"]["valueFrom"]
    renv = {e["name"]: e["value"] for e in cs["runtime"]["env"]}
    assert renv["OMNIA_POLICY_BROKER_URL"] == "http://127.0.0.1:8090"


def test_eval_worker_per_service_group_and_cleanup():
    def custom_evals(d):
        d["spec"]["framework"] = {"type": "custom", "image": "x"}
        d["spec"]["evals"] = {"enabled": True}

    cfg = SR.OperatorConfig(session_redis_url="redis://default-redis:6379")
    store, r = setup_store(custom_evals, cfg)
    reconcile(store, r)
    dep = store.get("Deployment", "arena-eval-worker-default")
    env = {e["name"]: e["value"] for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert env["REDIS_URL"] == "redis://default-redis:6379"
    assert env["OMNIA_SERVICE_GROUP"] == "default" and env["NAMESPACE"] == "default"
    ann = dep["spec"]["template"]["metadata"]["annotations"]
    assert ann["prometheus.io/port"] == "9090"
    assert store.get("RoleBinding", "arena-eval-worker-default")["subjects"][0]["name"] == \
        "arena-eval-worker-default"
    assert get_condition(store.get("AgentRuntime", "echo"), "EvalWorkerReady")["reason"] == \
        "WorkerDeployed"
    # group redis override wins over the operator default
    store.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "w"},
                 "spec": {"displayName": "W", "namespace": {"name": "default"},
                          "services": [{"name": "default",
                                        "memory": {"database": {"secretRef": {"name": "m"}}},
                                        "session": {"database": {"secretRef": {"name": "s"}},
                                                    "redis": {"url": "redis://grp:6379"}}}]}})
    reconcile(store, r)
    dep = store.get("Deployment", "arena-eval-worker-default")
    env = {e["name"]: e["value"] for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert env["REDIS_URL"] == "redis://grp:6379" and env["OMNIA_WORKSPACE_NAME"] == "w"
    # evals disabled -> worker + RBAC garbage-collected
    ar = store.get("AgentRuntime", "echo")
    ar["spec"]["evals"] = {"enabled": False}
    store.update(ar)
    reconcile(store, r)
    assert store.try_get("Deployment", "arena-eval-worker-default") is None
    assert store.try_get("Role", "arena-eval-worker-default") is None


def test_inline_evaluating_framework_needs_no_worker_unless_group_opts_in():
    def evals(d):
        d["spec"]["evals"] = {"enabled": True}

    store, r = setup_store(evals)
    reconcile(store, r)
    assert store.try_get("Deployment", "arena-eval-worker-default") is None
    assert get_condition(store.get("AgentRuntime", "echo"), "EvalWorkerReady")["reason"] == \
        "InlineEvals"
    store.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "w"},
                 "spec": {"displayName": "W", "namespace": {"name": "default"},
                          "services": [{"name": "default", "mode": "external",
                                        "external": {"sessionURL": "http://s:8080",
                                                     "memoryURL": "http://m:8080"},
                                        "evalWorker": {
                              "enabled": True, "podOverrides": {"serviceAccountName": "wi"}}}]}})
    reconcile(store, r)
    dep = store.get("Deployment", "arena-eval-worker-default")
    assert dep["spec"]["template"]["spec"]["serviceAccountName"] == "wi"


def test_oidc_jwks_mirror_fetch_cache_and_cleanup():
    idp = FakeIdP()
    now = [1_800_000_000.0]
    cfg = SR.OperatorConfig(http_get=idp.get, clock=lambda: now[0])

    def oidc(d):
        d["spec"]["externalAuth"] = {"oidc": {"issuer": idp.issuer, "audience": "agents"}}

    store, r = setup_store(oidc, cfg)
    after = reconcile(store, r)
    sec = store.get("Secret", "agent-echo-oidc-jwks")
    blob = json.loads(base64.b64decode(sec["data"]["jwks.json"]))
    assert blob["keys"][0]["kid"] == "k1"
    assert sec["metadata"]["labels"][SR.LABEL_CREDENTIAL_KIND] == "agent-oidc-jwks"
    ar = store.get("AgentRuntime", "echo")
    assert get_condition(ar, "OIDCJWKSReady")["status"] == "True"
    assert after is not None and after <= SR.OIDC_REFRESH_S
    dep = store.get("Deployment", "echo")
    fac = dep["spec"]["template"]["spec"]["containers"][0]
    fenv = {e["name"]: e["value"] for e in fac["env"]}
    assert fenv["OMNIA_OIDC_JWKS_FILE"] == "/etc/omnia/oidc/jwks.json"
    assert fenv["OMNIA_OIDC_ISSUER"] == idp.issuer and fenv["OMNIA_OIDC_AUDIENCE"] == "agents"
    assert any(v.get("secret", {}).get("secretName") == "agent-echo-oidc-jwks"
               for v in dep["spec"]["template"]["spec"]["volumes"])
    # within the refresh window: no HTTP round-trip
    n = len(idp.calls)
    now[0] += 3600
    reconcile(store, r)
    assert len(idp.calls) == n
    assert "(cached)" in get_condition(store.get("AgentRuntime", "echo"),
                                       "OIDCJWKSReady")["message"]
    # past the window with the IdP down: condition False, old Secret kept
    now[0] += SR.OIDC_REFRESH_S
    idp.down = True
    reconcile(store, r)
    c = get_condition(store.get("AgentRuntime", "echo"), "OIDCJWKSReady")
    assert c["status"] == "False" and c["reason"] == "DiscoveryFailed"
    assert store.try_get("Secret", "agent-echo-oidc-jwks") is not None
    # OIDC removed -> mirror deleted
    ar = store.get("AgentRuntime", "echo")
    ar["spec"].pop("externalAuth")
    store.update(ar)
    reconcile(store, r)
    assert store.try_get("Secret", "agent-echo-oidc-jwks") is None


def test_oidc_jwks_rejects_empty_keyset():
    idp = FakeIdP(keys=[])
    with pytest.raises(RuntimeError, match="no keys"):
        SR.fetch_jwks(idp.issuer, SR.OperatorConfig(http_get=idp.get))


def _listener():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(8)
    return s


def test_toolregistry_validation_probe_and_phases():
    live = _listener()
    dead = socket.socket()
    dead.bind(("127.0.0.1", 0))
    dead_port = dead.getsockname()[1]
    dead.close()  # nothing listens here
    store = new_store()
    tool = {"name": "t", "description": "d", "inputSchema": {"type": "object"}}
    store.apply({"apiVersion": crds.API_VERSION, "kind": "ToolRegistry",
                 "metadata": {"name": "reg", "namespace": "default"},
                 "spec": {"probe": {"enabled": True, "interval": "30s", "timeout": "1s"},
                          "handlers": [
                              {"name": "up", "type": "http", "tool": tool,
                               "httpConfig": {"endpoint":
                                              f"http://127.0.0.1:{live.getsockname()[1]}/x"}},
                              {"name": "down", "type": "grpc", "tool": {**tool, "name": "t2"},
                               "grpcConfig": {"endpoint": f"127.0.0.1:{dead_port}"}},
                              {"name": "browser", "type": "client",
                               "tool": {**tool, "name": "t3"}},
                              {"name": "stdio", "type": "mcp",
                               "mcpConfig": {"transport": "stdio", "command": "srv"}}]}})
    rr = ToolRegistryReconciler(SR.OperatorConfig())
    after = rr.reconcile(store, "default", "reg")
    assert after == 30.0
    st = store.get("ToolRegistry", "reg")["status"]
    by = {t["handlerName"]: t for t in st["discoveredTools"]}
    assert by["up"]["status"] == "Available"
    assert by["down"]["status"] == "Unavailable" and "probe failed" in by["down"]["error"]
    assert by["browser"]["endpoint"] == "client://browser"
    assert by["stdio"]["endpoint"] == "stdio://srv" and by["stdio"]["status"] == "Available"
    assert st["phase"] == "Degraded" and st["discoveredToolsCount"] == 4
    # an invalid retry policy fails validation
    tr = store.get("ToolRegistry", "reg")
    tr["spec"]["handlers"][0]["httpConfig"]["retryPolicy"] = {"maxAttempts": 3, "initialBackoff": "5s",
                                                             "maxBackoff": "1s"}
    store.update(tr)
    rr.reconcile(store, "default", "reg")
    st = store.get("ToolRegistry", "reg")["status"]
    assert st["phase"] == "Failed"
    assert get_condition(store.get("ToolRegistry", "reg"), "HandlersValid")["status"] == "False"
    live.close()


def test_probe_address_forms():
    assert SR.probe_address("https://api.x.com/v1") == ("api.x.com", 443)
    assert SR.probe_address("http://h:81") == ("h", 81)
    assert SR.probe_address("svc.ns:50051") == ("svc.ns", 50051)
    assert SR.probe_address("nonsense") is None
    assert not SR.is_network_endpoint("client://browser")
    assert not SR.is_network_endpoint("stdio://x")


def test_provider_endpoint_health():
    assert SR.provider_health_url({"type": "mock"}) == ""
    assert SR.provider_health_url({"type": "local"}) == ""
    assert SR.provider_health_url({"type": "claude", "platform": {"type": "bedrock"}}) == ""
    assert SR.provider_health_url({"type": "openai", "role": "tts"}) == ""
    assert SR.provider_health_url({"type": "claude"}) == "https://api.anthropic.com"
    assert SR.provider_health_url({"type": "ollama", "baseURL": "http://o:11434"}) == \
        "http://o:11434/api/tags"
    store = new_store()
    store.apply({"apiVersion": "v1", "kind": "Secret",
                 "metadata": {"name": "k", "namespace": "default"},
                 "stringData": {"api-key": "x"}})
    store.apply({"apiVersion": crds.API_VERSION, "kind": "Provider",
                 "metadata": {"name": "o", "namespace": "default"},
                 "spec": {"type": "ollama", "model": "llama3", "baseURL": "http://o:11434"}})
    seen = []

    def unauthorized(url, timeout):
        seen.append(url)
        return 401, b"{}"  # still proves the server is up

    ProviderReconciler(None, SR.OperatorConfig(http_get=unauthorized)).reconcile(
        store, "default", "o")
    pv = store.get("Provider", "o")
    assert seen == ["http://o:11434/api/tags"]
    assert pv["status"]["phase"] == "Ready"
    assert get_condition(pv, "EndpointReachable")["status"] == "True"

    def refused(url, timeout):
        raise OSError("connection refused")

    after = ProviderReconciler(None, SR.OperatorConfig(http_get=refused)).reconcile(
        store, "default", "o")
    pv = store.get("Provider", "o")
    assert pv["status"]["phase"] == "Unavailable" and after == SR.HEALTH_REQUEUE_S
    assert get_condition(pv, "EndpointReachable")["reason"] == "EndpointUnreachable"


def test_owner_references_garbage_collect_subresources():
    store, r = setup_store()
    reconcile(store, r)
    uid = store.get("AgentRuntime", "echo")["metadata"]["uid"]
    for kind, name in (("ServiceAccount", "echo-facade"), ("Role", "echo-facade"),
                       ("RoleBinding", "echo-facade")):
        refs = store.get(kind, name)["metadata"]["ownerReferences"]
        assert refs[0]["uid"] == uid and refs[0]["controller"] is True
    ar = store.get("AgentRuntime", "echo")
    ar["metadata"]["finalizers"] = []
    store.update(ar)
    store.delete("AgentRuntime", "echo")
    assert store.try_get("Role", "echo-facade") is None
    assert store.try_get("ServiceAccount", "echo-facade") is None
