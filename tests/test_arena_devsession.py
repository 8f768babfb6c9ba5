"""ArenaDevSession reconciler (``ee/internal/controller/arenadevsession_controller_test.go``):
finalizer, Pending -> Starting (SA / Role / RoleBinding / Deployment / Service,
owned, provider credentials as env, pod overrides) -> Ready (endpoint) ->
idle-timeout cleanup -> Stopped, deletion with cleanup, long-name hashing, and
the single-node launcher running the console as a real process."""
import asyncio
import json
import time
import urllib.request

from omnia_amd.ee.arena.devsession import (ACTIVITY_ANNOTATION, FINALIZER,
                                           ArenaDevSessionReconciler, resource_name)
from omnia_amd.operator.apistore import APIStore

API = "omnia.altairalabs.ai/v1alpha1"


def _session(store, name="dev1", **spec):
    store.create({"apiVersion": API, "kind": "ArenaDevSession",
                  "metadata": {"name": name, "namespace": "default"},
                  "spec": {"projectId": "proj", "workspace": "ws", **spec}})


def _get(store, name="dev1"):
    return store.try_get("ArenaDevSession", name, "default")


def _mark_ready(store, rn):
    d = store.get("Deployment", rn, "default")
    d["status"] = {"readyReplicas": 1}
    store.update_status(d)


def test_resource_name_truncates_with_hash():
    assert resource_name("short") == "adc-short"
    long = "x" * 70
    rn = resource_name(long)
    assert len(rn) == 63 and rn.startswith("adc-" + "x" * 50 + "-")
    assert rn != resource_name("x" * 71)


def test_lifecycle_start_ready_idle_stop_delete():
    store = APIStore()
    store.create({"apiVersion": "v1", "kind": "Secret",
                  "metadata": {"name": "oai", "namespace": "default"},
                  "stringData": {"api-key": "k"}})
    now = [1_800_000_000.0]
    r = ArenaDevSessionReconciler(now=lambda: now[0])
    _session(store, idleTimeout="10m", podOverrides={"nodeSelector": {"gpu": "mi355x"},
                                                      "labels": {"team": "a"}})
    assert r.reconcile(store, "default", "dev1") == 1.0  # finalizer first
    assert FINALIZER in _get(store)["metadata"]["finalizers"]
    assert r.reconcile(store, "default", "dev1") == 2.0
    s = _get(store)
    assert s["status"]["phase"] == "Starting"
    rn = "adc-dev1"
    for kind in ("ServiceAccount", "Role", "RoleBinding", "Deployment", "Service"):
        o = store.get(kind, rn, "default")
        assert o["metadata"]["ownerReferences"][0]["kind"] == "ArenaDevSession", kind
    dep = store.get("Deployment", rn, "default")
    pod = dep["spec"]["template"]["spec"]
    c = pod["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["POD_NAMESPACE"] == "default" and env["OMNIA_WORKSPACE_NAME"] == "ws"
    assert c["args"] == ["--port", "8080"] and pod["nodeSelector"] == {"gpu": "mi355x"}
    assert dep["spec"]["template"]["metadata"]["labels"]["team"] == "a"
    role = store.get("Role", rn, "default")
    assert any("providers" in rule["resources"] for rule in role["rules"])
    # not ready yet
    assert r.reconcile(store, "default", "dev1") == 2.0
    assert _get(store)["status"]["message"].startswith("Waiting")
    _mark_ready(store, rn)
    assert r.reconcile(store, "default", "dev1") == 60.0
    st = _get(store)["status"]
    assert st["phase"] == "Ready" and st["endpoint"] == "ws://adc-dev1.default.svc:8080/ws"
    assert st["serviceName"] == rn
    # activity annotation pushes the idle deadline out
    now[0] += 540
    s = _get(store)
    s["metadata"]["annotations"] = {ACTIVITY_ANNOTATION: time.strftime(
        "%Y-%m-%dT%H:%M:%SZ", time.gmtime(now[0]))}
    s.pop("status")
    store.update(s)
    now[0] += 300  # 14 min after start, 5 after the last activity
    assert r.reconcile(store, "default", "dev1") == 60.0
    assert _get(store)["status"]["phase"] == "Ready"
    now[0] += 601
    assert r.reconcile(store, "default", "dev1") is None
    st = _get(store)["status"]
    assert st["phase"] == "Stopped" and st["endpoint"] == ""
    for kind in ("ServiceAccount", "Role", "RoleBinding", "Deployment", "Service"):
        assert store.try_get(kind, rn, "default") is None, kind
    # deletion drops the finalizer after cleanup
    store.delete("ArenaDevSession", "dev1", "default")
    r.reconcile(store, "default", "dev1")
    assert _get(store) is None


def test_delete_while_ready_cleans_up():
    store = APIStore()
    r = ArenaDevSessionReconciler()
    _session(store)
    r.reconcile(store, "default", "dev1")
    r.reconcile(store, "default", "dev1")
    _mark_ready(store, "adc-dev1")
    r.reconcile(store, "default", "dev1")
    store.delete("ArenaDevSession", "dev1", "default")
    r.reconcile(store, "default", "dev1")
    assert _get(store) is None and store.try_get("Deployment", "adc-dev1", "default") is None


def test_provider_secrets_become_env():
    store = APIStore()
    store.objs[("Provider", "default", "claude")] = {
        "kind": "Provider", "metadata": {"name": "claude", "namespace": "default"},
        "spec": {"type": "claude", "secretRef": {"name": "anthropic"}}}
    env = ArenaDevSessionReconciler._provider_env(store, "default")
    assert env == [{"name": "CLAUDE_API_KEY", "valueFrom": {"secretKeyRef": {
        "name": "anthropic", "key": "api-key", "optional": True}}}]


def test_launcher_runs_the_console_process():
    """Single-node mode: the launcher starts the Deployment as a process, reports
    it ready, and the session's local endpoint answers /healthz."""
    from omnia_amd.operator.launcher import LocalLauncher

    store = APIStore()
    r = ArenaDevSessionReconciler()
    _session(store)
    r.reconcile(store, "default", "dev1")
    r.reconcile(store, "default", "dev1")
    launcher = LocalLauncher(store, mode="process")

    async def go():
        try:
            await launcher.sync()
            assert r.reconcile(store, "default", "dev1") == 60.0
            st = _get(store)["status"]
            assert st["phase"] == "Ready" and st["localEndpoint"].startswith("ws://127.0.0.1:")
            url = st["localEndpoint"].replace("ws://", "http://")[: -len("/ws")] + "/healthz"
            with urllib.request.urlopen(url, timeout=10) as resp:
                assert resp.status == 200
        finally:
            for sp, _ in list(getattr(launcher, "services", {}).values()):
                sp.stop()

    asyncio.run(go())
