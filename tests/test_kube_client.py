"""Real-cluster mode: KubeClient (REST, SSA, patches, reflector watch with
bookmarks / 410 re-list), Lease leader election, and the unchanged controllers
reconciling through the client against the kube-style apiserver
(cf. the reference's envtest suites, ``internal/controller/suite_test.go:81-135``)."""
import asyncio
import os
import socket
import threading
import time

import pytest
from aiohttp import web

from omnia_amd.api import crds
from omnia_amd.cli import load_manifests
from omnia_amd.operator.apiserver import build_app, json_patch, merge_patch, \
    parse_label_selector
from omnia_amd.operator.apistore import APIStore, Conflict, Invalid, NotFound, get_condition
from omnia_amd.operator.kube import Gone, KubeClient, KubeConfig, KubeError, LeaseLock, \
    _Reflector, micro_time, parse_time, resource_path, selector_string
from omnia_amd.operator.manager import WEBHOOKS, Manager

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "examples", "echo-function", "manifests.yaml")
TOKEN = "s3cret-sa-token"


class Server:
    """The kube-style apiserver on a private loop thread."""

    def __init__(self, history=10000, bookmark_interval=30.0):
        self.store = APIStore(webhooks=dict(WEBHOOKS), history=history)
        self.loop = asyncio.new_event_loop()
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        self.port = s.getsockname()[1]
        s.close()
        app = build_app(self.store, token=TOKEN, bookmark_interval=bookmark_interval)
        self.runner = web.AppRunner(app)
        ready = threading.Event()

        def run():
            asyncio.set_event_loop(self.loop)
            self.loop.run_until_complete(self.runner.setup())
            self.loop.run_until_complete(web.TCPSite(self.runner, "127.0.0.1",
                                                     self.port).start())
            ready.set()
            self.loop.run_forever()

        self.t = threading.Thread(target=run, daemon=True)
        self.t.start()
        ready.wait(10)
        self.url = f"http://127.0.0.1:{self.port}"

    def client(self, token=TOKEN, **kw):
        return KubeClient(KubeConfig(self.url, token=token), **kw)

    def close(self):
        asyncio.run_coroutine_threadsafe(self.runner.cleanup(), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(5)


@pytest.fixture
def srv():
    s = Server()
    yield s
    s.close()


def cm(name, ns="default", labels=None, **data):
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": name, "namespace": ns, "labels": labels or {}},
            "data": data}


def test_paths_and_selectors():
    assert resource_path("Deployment", "x", "d") == "/apis/apps/v1/namespaces/x/deployments/d"
    assert resource_path("ConfigMap", "x") == "/api/v1/namespaces/x/configmaps"
    assert resource_path("Workspace", None, "w", "status") == \
        "/apis/omnia.altairalabs.ai/v1alpha1/workspaces/w/status"
    assert resource_path("AgentRuntime") == "/apis/omnia.altairalabs.ai/v1alpha1/agentruntimes"
    sel = {"matchLabels": {"a": "1"}, "matchExpressions": [
        {"key": "b", "operator": "In", "values": ["x", "y"]},
        {"key": "c", "operator": "Exists"}, {"key": "d", "operator": "DoesNotExist"}]}
    s = selector_string(sel)
    assert s == "a=1,b in (x,y),c,!d"
    back = parse_label_selector(s)
    assert back["matchLabels"] == {"a": "1"} and len(back["matchExpressions"]) == 3
    assert parse_label_selector("x!=1")["matchExpressions"][0]["operator"] == "NotIn"
    t = time.time()
    assert abs(parse_time(micro_time(t)) - t) < 1e-3


def test_patch_algorithms():
    doc = {"a": {"b": 1, "c": [1, 2]}, "d": "x"}
    assert merge_patch(doc, {"a": {"b": None, "e": 2}, "d": None}) == {"a": {"c": [1, 2], "e": 2}}
    out = json_patch(doc, [{"op": "add", "path": "/a/c/-", "value": 3},
                           {"op": "replace", "path": "/d", "value": "y"},
                           {"op": "move", "from": "/a/b", "path": "/f"},
                           {"op": "copy", "from": "/f", "path": "/g"},
                           {"op": "remove", "path": "/a/c/0"},
                           {"op": "test", "path": "/g", "value": 1}])
    assert out == {"a": {"c": [2, 3]}, "d": "y", "f": 1, "g": 1}
    with pytest.raises(ValueError):
        json_patch(doc, [{"op": "test", "path": "/d", "value": "nope"}])


def test_crud_auth_and_errors(srv):
    c = srv.client()
    with pytest.raises(KubeError) as ei:
        srv.client(token="wrong").list("ConfigMap", "default")
    assert ei.value.code == 401
    o = c.create(cm("one", labels={"tier": "a"}, k="v"))
    assert o["metadata"]["resourceVersion"] and o["apiVersion"] == "v1"
    c.create(cm("two", labels={"tier": "b"}))
    with pytest.raises(Conflict):
        c.create(cm("one"))
    assert [x["metadata"]["name"] for x in c.list("ConfigMap", "default",
                                                  {"matchLabels": {"tier": "a"}})] == ["one"]
    assert len(c.list("ConfigMap", "default", {"matchExpressions": [
        {"key": "tier", "operator": "In", "values": ["a", "b"]}]})) == 2
    items, rv = c.list_with_rv("ConfigMap")
    assert len(items) == 2 and int(rv) >= 2
    # optimistic concurrency
    stale = dict(o)
    o["data"]["k"] = "v2"
    c.update(o)
    stale["data"] = {"k": "v3"}
    with pytest.raises(Conflict):
        c.update(stale)
    # merge + json patch
    p = c.patch("ConfigMap", "one", "default", {"data": {"x": "1", "k": None}})
    assert p["data"] == {"x": "1"}
    p = c.patch("ConfigMap", "one", "default",
                [{"op": "add", "path": "/metadata/labels/new", "value": "l"}], "json")
    assert p["metadata"]["labels"]["new"] == "l"
    # server-side apply: create then update, status untouched
    a = c.apply(cm("applied", z="1"))
    a2 = c.apply(cm("applied", z="2"))
    assert a2["data"]["z"] == "2" and int(a2["metadata"]["resourceVersion"]) > int(
        a["metadata"]["resourceVersion"])
    assert c.delete("ConfigMap", "applied") is True
    assert c.delete("ConfigMap", "applied") is False
    with pytest.raises(NotFound):
        c.get("ConfigMap", "applied")
    assert c.try_get("ConfigMap", "applied") is None


def test_crd_admission_and_status_subresource(srv):
    c = srv.client()
    with pytest.raises(Invalid) as ei:
        c.create({"apiVersion": crds.API_VERSION, "kind": "Provider",
                  "metadata": {"name": "bad", "namespace": "default"},
                  "spec": {"type": "claude", "role": "embedding"}})
    assert any("requires type in" in e for e in ei.value.errors)
    pv = c.create({"apiVersion": crds.API_VERSION, "kind": "Provider",
                   "metadata": {"name": "m", "namespace": "default"},
                   "spec": {"type": "mock"}})
    pv["status"] = {"phase": "Ready"}
    pv["spec"]["model"] = "ignored-by-status-write"
    s = c.update_status(pv)
    assert s["status"]["phase"] == "Ready" and "model" not in s["spec"]
    assert s["metadata"]["generation"] == 1
    s2 = c.patch("Provider", "m", "default", {"status": {"phase": "Error"}}, subresource="status")
    assert s2["status"]["phase"] == "Error"
    # cluster-scoped kind
    ws = c.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "w"},
                  "spec": {"displayName": "W", "namespace": {"name": "w-ns"}}})
    assert "namespace" not in ws["metadata"]
    assert c.get("Workspace", "w", None)["spec"]["environment"] == "development"


def test_watch_stream_bookmarks_and_gone():
    s = Server(history=4, bookmark_interval=0.2)
    try:
        c = s.client()
        o = c.create(cm("w0"))
        rv0 = o["metadata"]["resourceVersion"]
        c.create(cm("w1"))
        evs = list(c.watch_stream("ConfigMap", "default", rv0, timeout_s=1))
        types = [t for t, _ in evs]
        assert types[0] == "ADDED" and evs[0][1]["metadata"]["name"] == "w1"
        assert "BOOKMARK" in types  # idle stream still advances the client's rv
        for i in range(2, 8):
            c.create(cm(f"w{i}"))
        with pytest.raises(Gone):
            list(c.watch_stream("ConfigMap", "default", rv0, timeout_s=1))
    finally:
        s.close()


def test_reflector_relist_diff_and_live_events(srv):
    c = srv.client(watch_timeout_s=1)

    async def go():
        loop = asyncio.get_running_loop()
        q = asyncio.Queue()
        r = _Reflector(c, "ConfigMap", "default", loop, q)
        # a stale cache: 'gone' was deleted and 'kept' modified while we were away
        c.create(cm("kept", v="1"))
        r.cache = {("default", "gone"): cm("gone") | {"metadata": {
            "name": "gone", "namespace": "default", "resourceVersion": "1"}},
                   ("default", "kept"): cm("kept") | {"metadata": {
                       "name": "kept", "namespace": "default", "resourceVersion": "0"}}}
        await asyncio.to_thread(r._relist)
        got = {(await q.get())[0] for _ in range(2)}
        assert got == {"MODIFIED", "DELETED"}
        # live reflector: ADDED for the list, then watch events
        q2 = c.watch("ConfigMap")
        first = await asyncio.wait_for(q2.get(), 5)
        assert first[0] == "ADDED"
        await asyncio.to_thread(c.create, cm("live"))
        seen = []
        deadline = time.time() + 10
        while time.time() < deadline and ("ADDED", "live") not in seen:
            et, o = await asyncio.wait_for(q2.get(), 10)
            seen.append((et, o["metadata"]["name"]))
        assert ("ADDED", "live") in seen
        await asyncio.to_thread(c.delete, "ConfigMap", "live")
        while True:
            et, o = await asyncio.wait_for(q2.get(), 10)
            if o["metadata"]["name"] == "live" and et == "DELETED":
                break
        c.unwatch(q2)

    asyncio.run(go())


def test_lease_leader_election(srv):
    c1, c2 = srv.client(), srv.client()
    now = [1000.0]
    clock = lambda: now[0]  # noqa: E731
    a = LeaseLock(c1, "leader", "omnia-system", "a", lease_duration_s=15, clock=clock)
    b = LeaseLock(c2, "leader", "omnia-system", "b", lease_duration_s=15, clock=clock)
    assert a.try_acquire_or_renew()
    assert not b.try_acquire_or_renew()
    now[0] += 10
    assert a.try_acquire_or_renew()  # renew
    now[0] += 14
    assert not b.try_acquire_or_renew()  # renewed 14 s ago: still held
    now[0] += 2
    assert b.try_acquire_or_renew()  # expired: b takes over
    lease = c1.get("Lease", "leader", "omnia-system")
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
    assert not a.try_acquire_or_renew()
    b.release()
    assert a.try_acquire_or_renew()
    # CAS: a stale read cannot overwrite a newer holder
    stale = c1.get("Lease", "leader", "omnia-system")
    now[0] += 1
    assert a.try_acquire_or_renew()
    stale["spec"]["holderIdentity"] = "intruder"
    with pytest.raises(Conflict):
        c2.update(stale)


def test_manager_reconciles_through_kube_client(srv):
    c = srv.client(watch_timeout_s=2)
    docs = load_manifests([ECHO])

    async def go():
        mgr = Manager(c, leader_elect=True, identity="op-1", namespace="omnia-system")
        mgr.lease_duration_s = 3
        await mgr.start()
        try:
            assert mgr.is_leader and mgr.threaded
            for d in docs:
                await asyncio.to_thread(c.apply, d)
            ar = None
            for _ in range(300):  # generous: reconciles go through HTTP on a loaded box
                await asyncio.sleep(0.1)
                ar = srv.store.try_get("AgentRuntime", "echo", "default")
                dep = srv.store.try_get("Deployment", "echo", "default")
                if dep is not None and get_condition(ar, "PromptPackReady"):
                    break
            assert dep is not None, "Deployment never reconciled through the client"
            assert get_condition(ar, "ProviderReady")["status"] == "True"
            assert srv.store.try_get("Service", "echo", "default") is not None
            lease = srv.store.get("Lease", "omnia-operator-leader", "omnia-system")
            assert lease["spec"]["holderIdentity"] == "op-1"
            # a spec change flows watch -> queue -> reconcile -> apply
            def bump():
                # optimistic concurrency: the controller's status writes bump the
                # resourceVersion, so re-read and retry on a conflict
                for _ in range(20):
                    cur = c.get("AgentRuntime", "echo", "default")
                    cur["spec"]["runtime"] = {"replicas": 3}
                    try:
                        return c.update(cur)
                    except Conflict:
                        time.sleep(0.05)
                raise AssertionError("spec update kept conflicting")

            await asyncio.to_thread(bump)
            for _ in range(300):
                await asyncio.sleep(0.1)
                if srv.store.get("Deployment", "echo", "default")["spec"]["replicas"] == 3:
                    break
            assert srv.store.get("Deployment", "echo", "default")["spec"]["replicas"] == 3
        finally:
            await mgr.stop()
            c.close()
        # ReleaseOnCancel: the next candidate does not wait out the lease
        assert srv.store.get("Lease", "omnia-operator-leader",
                             "omnia-system")["spec"]["holderIdentity"] == ""

    asyncio.run(go())


def test_kubeconfig_loading(tmp_path):
    import base64

    kc = tmp_path / "config"
    ca = base64.b64encode(b"not-a-real-ca").decode()
    kc.write_text(f"""
apiVersion: v1
kind: Config
current-context: dev
contexts:
- name: dev
  context: {{cluster: c1, user: u1, namespace: agents}}
clusters:
- name: c1
  cluster: {{server: "https://10.0.0.1:6443", certificate-authority-data: {ca}}}
users:
- name: u1
  user: {{token: abc}}
""")
    cfg = KubeConfig.from_kubeconfig(str(kc))
    assert cfg.server == "https://10.0.0.1:6443" and cfg.bearer() == "abc"
    assert cfg.namespace == "agents" and open(cfg.ca_file, "rb").read() == b"not-a-real-ca"
    sa = tmp_path / "sa"
    sa.mkdir()
    (sa / "token").write_text("tok1\n")
    (sa / "namespace").write_text("omnia-system")
    (sa / "ca.crt").write_text("")
    os.environ["KUBERNETES_SERVICE_HOST"] = "10.96.0.1"
    try:
        ic = KubeConfig.in_cluster(str(sa))
    finally:
        del os.environ["KUBERNETES_SERVICE_HOST"]
    assert ic.server == "https://10.96.0.1:443" and ic.namespace == "omnia-system"
    assert ic.bearer() == "tok1"
    (sa / "token").write_text("tok2")  # projected token rotated on disk
    assert ic.bearer() == "tok2"
