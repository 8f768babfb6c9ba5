"""Control plane: CRD admission (schema + CEL), reconcilers against the
in-memory API store (cf. the reference's envtest suites), single-node launcher
serving a reconciled AgentRuntime end-to-end."""
import asyncio
import copy
import json
import os

import aiohttp
import pytest

from omnia_amd.api import crds
from omnia_amd.cli import load_manifests
from omnia_amd.operator.apistore import Invalid, get_condition
from omnia_amd.operator.launcher import LocalLauncher
from omnia_amd.operator.manager import Manager, new_store

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "examples", "echo-function", "manifests.yaml")
AGENT = os.path.join(ROOT, "examples", "llama3-8b-agent", "manifests.yaml")


# a managed service group needs its memory + session databases (workspace_types.go:634)
DB = {"memory": {"database": {"secretRef": {"name": "memory-db"}}},
      "session": {"database": {"secretRef": {"name": "session-db"}}}}


def ar(name="a", **spec):
    base = {"facades": [{"type": "websocket"}], "promptPackRef": {"name": "p"}}
    base.update(spec)
    return {"apiVersion": crds.API_VERSION, "kind": "AgentRuntime",
            "metadata": {"name": name, "namespace": "default"}, "spec": base}


def test_crd_inventory_matches_reference_surface():
    assert len(crds.KINDS) == 17
    assert {k.kind for k in crds.KINDS.values() if not k.ee} == {
        "AgentRuntime", "Provider", "PromptPack", "ToolRegistry", "Workspace", "AgentPolicy",
        "MemoryPolicy", "SessionRetentionPolicy", "SkillSource"}
    assert crds.resolve_kind("ar") == "AgentRuntime" and crds.resolve_kind("prov") == "Provider"
    assert crds.KINDS["Workspace"].scope == "Cluster"
    m = crds.crd_manifest(crds.KINDS["AgentRuntime"])
    assert m["metadata"]["name"] == "agentruntimes.omnia.altairalabs.ai"


def test_agentruntime_cel_rules():
    st = new_store()
    with pytest.raises(Invalid, match="inputSchema is required"):
        st.create(ar(mode="function", facades=[{"type": "rest"}]))
    with pytest.raises(Invalid, match="only valid when spec.mode is .function."):
        st.create(ar(inputSchema={"type": "object"}))
    with pytest.raises(Invalid, match="must not contain duplicate facade types"):
        st.create(ar(facades=[{"type": "websocket"}, {"type": "websocket"}]))
    with pytest.raises(Invalid, match="requires exactly one .rest. facade"):
        st.create(ar(mode="function", facades=[{"type": "mcp"}], inputSchema={},
                     outputSchema={}))
    with pytest.raises(Invalid, match="does not compile"):
        st.create(ar(mode="function", facades=[{"type": "rest"}],
                     inputSchema={"type": "bogus"}, outputSchema={}))
    o = st.create(ar())
    assert o["spec"]["mode"] == "agent" and o["spec"]["serviceGroup"] == "default"  # defaults


def test_provider_role_type_matrix():
    st = new_store()
    bad = {"apiVersion": crds.API_VERSION, "kind": "Provider",
           "metadata": {"name": "x"}, "spec": {"type": "claude", "role": "embedding"}}
    with pytest.raises(Invalid, match="role 'embedding' requires type in"):
        st.create(bad)
    with pytest.raises(Invalid, match="spec.model is required"):
        st.create({**bad, "spec": {"type": "vllm"}})
    with pytest.raises(Invalid, match="engine.model"):
        st.create({**bad, "spec": {"type": "local"}})
    st.create({**bad, "spec": {"type": "local", "engine": {"model": "llama-3-8b"}}})


def test_generation_and_status_subresource():
    st = new_store()
    o = st.create(ar())
    assert o["metadata"]["generation"] == 1
    o["status"] = {"phase": "X"}
    o2 = st.update_status(o)
    assert o2["metadata"]["generation"] == 1
    o2["spec"]["facades"] = [{"type": "a2a"}]
    o3 = st.update(o2)
    assert o3["metadata"]["generation"] == 2 and o3["status"]["phase"] == "X"


async def _run_operator(manifests, gpu_count=None, launch=False, engine_factory=None):
    store = new_store()
    mgr = Manager(store, gpu_count=gpu_count)
    await mgr.start()
    launcher = None
    if launch:
        launcher = LocalLauncher(store, engine_factory=engine_factory)
        launcher.start()
    for d in manifests:
        store.apply(d)
    await mgr.settle(timeout=15, quiet=0.4)
    return store, mgr, launcher


def test_reconcile_echo_function_end_to_end():
    docs = load_manifests([ECHO])
    for d in docs:
        if d["kind"] == "Provider":
            d["spec"]["mock"] = {"scenarios": {}}

    async def go():
        store, mgr, launcher = await _run_operator(docs, launch=True)
        try:
            for _ in range(50):
                a = store.get("AgentRuntime", "echo")
                if a["status"].get("phase") == "Running":
                    break
                await asyncio.sleep(0.1)
            ep = store.get("Service", "echo")["status"]["endpoint"]
            # point the mock at a JSON answer through the running pod's provider
            pod = launcher.pods[("default", "echo")]
            prov = pod.runtime_svc.agent.provider
            prov.default_response = '{"echo": "hello"}'
            async with aiohttp.ClientSession() as s:
                r = await s.post(f"http://{ep}/functions/echo", json={"message": "hello"})
                body = await r.json()
                r2 = await s.post(f"http://{ep}/functions/echo", json={"nope": 1})
                mcp = await s.post(f"http://{ep}/mcp", json={"jsonrpc": "2.0", "id": 1,
                                                             "method": "tools/list"})
                tools = (await mcp.json())["result"]["tools"]
            return store, a, r.status, body, r2.status, tools
        finally:
            await launcher.stop()
            await mgr.stop()

    store, a, s1, body, s2, tools = asyncio.run(go())
    assert a["status"]["phase"] == "Running"
    assert get_condition(a, "PromptPackReady")["status"] == "True"
    assert get_condition(a, "ProviderReady")["status"] == "True"
    assert s1 == 200 and body == {"echo": "hello"}
    assert s2 == 400
    assert tools[0]["name"] == "echo" and tools[0]["inputSchema"]["required"] == ["message"]
    dep = store.get("Deployment", "echo")
    names = [c["name"] for c in dep["spec"]["template"]["spec"]["containers"]]
    assert names == ["facade", "runtime"]
    assert store.get("ConfigMap", "echo-tools")
    assert store.get("PromptPack", "echo-pack")["status"]["phase"] == "Active"


def test_reconcile_local_provider_agent_objects():
    docs = load_manifests([AGENT])

    async def go():
        store, mgr, _ = await _run_operator(docs, gpu_count=8)
        await mgr.stop()
        return store

    store = asyncio.run(go())
    a = store.get("AgentRuntime", "assistant")
    dep = store.get("Deployment", "assistant")
    rt = [c for c in dep["spec"]["template"]["spec"]["containers"] if c["name"] == "runtime"][0]
    env = {e["name"]: e["value"] for e in rt["env"]}
    assert rt["resources"]["limits"]["amd.com/gpu"] == "1"
    assert env["OMNIA_ENGINE_MODEL"] == "llama-3-8b"
    assert json.loads(env["OMNIA_PROVIDER_JSON"])["type"] == "local"
    so = store.get("ScaledObject", "assistant")
    assert 'omnia_agent_connections_active{agent="assistant"' in \
        so["spec"]["triggers"][0]["metadata"]["query"]
    assert so["spec"]["minReplicaCount"] == 0
    assert store.get("Provider", "llama3-8b")["status"]["phase"] == "Ready"
    assert store.get("ToolRegistry", "weather-tools")["status"]["toolCount"] == 1
    import yaml

    tools = yaml.safe_load(store.get("ConfigMap", "assistant-tools")["data"]["tools.yaml"])
    assert tools["handlers"][0]["name"] == "weather"
    assert a["status"]["activeVersion"] == "1.0.0"


def test_capability_gate_scales_to_zero_without_gpus():
    docs = load_manifests([AGENT])

    async def go():
        store, mgr, _ = await _run_operator(docs, gpu_count=0)
        await mgr.stop()
        return store

    store = asyncio.run(go())
    assert store.get("Provider", "llama3-8b")["status"]["phase"] == "Error"
    a = store.get("AgentRuntime", "assistant")
    assert get_condition(a, "ProviderReady")["status"] == "False"


def test_promptpack_track_resolution_and_version_rollout():
    docs = load_manifests([ECHO])
    cm = copy.deepcopy([d for d in docs if d["kind"] == "ConfigMap"][0])
    pp = [d for d in docs if d["kind"] == "PromptPack"][0]
    extra = []
    for v in ("1.1.0", "2.0.0-rc1"):
        p = copy.deepcopy(pp)
        p["metadata"]["name"] = f"echo-pack-{v.replace('.', '-')}"
        p["spec"]["version"] = v
        extra.append(p)

    async def go():
        store, mgr, _ = await _run_operator(docs + extra)
        a = store.get("AgentRuntime", "echo")
        v_stable = a["status"]["activeVersion"]
        a["spec"]["promptPackRef"] = {"name": "echo-pack", "track": "prerelease"}
        store.update(a)
        await mgr.settle(timeout=10)
        v_pre = store.get("AgentRuntime", "echo")["status"]["activeVersion"]
        phases = {p["metadata"]["name"]: p["status"]["phase"]
                  for p in store.list("PromptPack")}
        await mgr.stop()
        return v_stable, v_pre, phases

    v_stable, v_pre, phases = asyncio.run(go())
    assert v_stable == "1.1.0" and v_pre == "2.0.0-rc1"
    assert phases["echo-pack-2-0-0-rc1"] == "Active" and phases["echo-pack"] == "Superseded"


def test_finalizer_and_garbage_collection():
    docs = load_manifests([ECHO])

    async def go():
        store, mgr, _ = await _run_operator(docs)
        assert "agentruntime.omnia.altairalabs.ai/finalizer" in \
            store.get("AgentRuntime", "echo")["metadata"]["finalizers"]
        store.delete("AgentRuntime", "echo")
        await mgr.settle(timeout=10)
        await mgr.stop()
        return store

    store = asyncio.run(go())
    assert store.try_get("AgentRuntime", "echo") is None
    assert store.try_get("Deployment", "echo") is None  # owned objects collected
    assert store.try_get("Service", "echo") is None


def test_workspace_reconcile():
    ws = {"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "team-a"},
          "spec": {"displayName": "Team A", "namespace": {"name": "team-a"},
                   "networkPolicy": {"isolate": True}, "storage": {"enabled": True},
                   "services": [{"name": "default", **DB}, {"name": "gold", **DB}]}}

    async def go():
        store, mgr, _ = await _run_operator([ws])
        await mgr.stop()
        return store

    store = asyncio.run(go())
    w = store.get("Workspace", "team-a", None)
    assert w["status"]["phase"] == "Ready"
    groups = {g["name"]: g for g in w["status"]["services"]}
    assert set(groups) == {"default", "gold"}
    assert groups["gold"]["sessionURL"] == "http://session-api-team-a-gold.team-a:8080"
    assert not groups["gold"]["ready"]  # no launcher ran the service pods
    assert get_condition(w, "ServicesReady")["status"] == "False"
    assert store.get("Namespace", "team-a", None)
    dep = store.get("Deployment", "session-api-team-a-gold", "team-a")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][-1] == "omnia_amd.session.api" and "--port" in c["args"]
    assert store.get("NetworkPolicy", "workspace-team-a-isolation", "team-a")


def _fake_kubelet(store):
    """Marks every Deployment rolled out (ready replicas, observed generation),
    as the Deployment controller + kubelet would."""
    async def loop():
        while True:
            for d in store.list("Deployment"):
                st = d.get("status") or {}
                want = d["spec"].get("replicas", 1)
                if st.get("observedGeneration") != d["metadata"]["generation"] or \
                        st.get("readyReplicas") != want:
                    d["status"] = {"replicas": want, "readyReplicas": want,
                                   "updatedReplicas": want, "availableReplicas": want,
                                   "observedGeneration": d["metadata"]["generation"]}
                    d["metadata"].pop("resourceVersion", None)
                    store.update_status(d)
            await asyncio.sleep(0.05)
    return asyncio.ensure_future(loop())


def test_canary_rollout_steps_and_promotion():
    docs = load_manifests([ECHO])
    for d in docs:
        if d["kind"] == "AgentRuntime":
            d["spec"]["rollout"] = {"candidate": {"promptPackRef": {"name": "echo-pack",
                                                                    "version": "1.0.0"}},
                                    "steps": [{"setWeight": 20}, {"pause": {"duration": "1s"}},
                                              {"setWeight": 100}]}

    async def go():
        store = new_store()
        kubelet = _fake_kubelet(store)
        mgr = Manager(store)
        await mgr.start()
        for d in docs:
            store.apply(d)
        seen = []
        for _ in range(100):
            c = store.try_get("Deployment", "echo-candidate")
            if c is not None:
                seen.append(c["metadata"]["labels"]["omnia.altairalabs.ai/track"])
            ro = store.get("AgentRuntime", "echo")["status"].get("rollout") or {}
            seen.append(ro.get("currentWeight"))
            if ro.get("message") == "promoted":
                break
            await asyncio.sleep(0.1)
        await mgr.settle(timeout=5)
        a = store.get("AgentRuntime", "echo")
        cand = store.try_get("Deployment", "echo-candidate")
        events = [e["reason"] for e in store.list("Event")]
        await mgr.stop()
        kubelet.cancel()
        return a, cand, seen, events

    a, cand, seen, events = asyncio.run(go())
    assert "candidate" in seen and 20 in seen
    ro = a["status"]["rollout"]
    assert ro["active"] is False and ro["message"] == "promoted"
    assert cand is None  # candidate folded into stable after promotion
    assert a["spec"]["promptPackRef"] == {"name": "echo-pack", "version": "1.0.0"}
    assert "candidate" not in a["spec"]["rollout"]
    for r in ("RolloutStep", "RolloutPromoting", "RolloutPromoted"):
        assert r in events


def test_rollout_traffic_routing_modes(monkeypatch):
    from omnia_amd.operator import rollout_routing as RR

    assert RR.resolve_mode(None, False) == ("replica-weighted", False)
    assert RR.resolve_mode({"mode": "mesh"}, False) == ("replica-weighted", True)
    assert RR.resolve_mode({"istio": {"virtualService": {"name": "v"}}}, True) == \
        ("external", False)
    assert RR.split_replicas(4, 20) == (3, 1) and RR.split_replicas(4, 60) == (1, 3)
    assert RR.split_replicas(3, 0) == (3, 0) and RR.split_replicas(3, 100) == (0, 3)

    def run(routing, mesh):
        if mesh:
            monkeypatch.setenv("OMNIA_MESH_ENABLED", "1")
        else:
            monkeypatch.delenv("OMNIA_MESH_ENABLED", raising=False)
        docs = load_manifests([ECHO])
        for d in docs:
            if d["kind"] == "AgentRuntime":
                d["spec"]["rollout"] = {"candidate": {"promptPackRef": {"name": "echo-pack",
                                                                    "version": "1.0.0"}},
                                        "steps": [{"setWeight": 30}, {"pause": {"duration": "1h"}}],
                                        "trafficRouting": routing}
                d["spec"].setdefault("runtime", {})["replicas"] = 4
        extra = []
        if routing.get("istio"):
            extra = [{"apiVersion": RR.ISTIO_API, "kind": "VirtualService",
                      "metadata": {"name": "echo-vs", "namespace": "default"},
                      "spec": {"http": [{"name": "primary", "route": [
                          {"destination": {"host": "echo", "subset": "stable"}, "weight": 100},
                          {"destination": {"host": "echo", "subset": "canary"}, "weight": 0}]}]}},
                     {"apiVersion": RR.ISTIO_API, "kind": "DestinationRule",
                      "metadata": {"name": "echo-dr", "namespace": "default"}, "spec": {}}]

        async def go():
            store, mgr, _ = await _run_operator(docs + extra)
            for _ in range(60):
                ro = store.get("AgentRuntime", "echo")["status"].get("rollout") or {}
                if ro.get("currentWeight") == 30 and ro.get("traffic"):
                    break
                await asyncio.sleep(0.1)
            await mgr.settle(timeout=5)
            out = (store.get("AgentRuntime", "echo")["status"]["rollout"],
                   store.try_get("VirtualService", "echo-rollout"),
                   store.try_get("VirtualService", "echo-vs"),
                   store.try_get("DestinationRule", "echo-dr"),
                   store.try_get("Deployment", "echo-candidate"))
            await mgr.stop()
            return out

        return asyncio.run(go())

    ro, owned, _, _, cand = run({"mode": "mesh"}, True)
    assert ro["traffic"]["trafficRoutingMode"] == "mesh"
    w = [r["weight"] for r in owned["spec"]["http"][0]["route"]]
    assert w == [70, 30]
    ro, owned, _, _, cand = run({}, False)
    assert ro["traffic"]["trafficRoutingMode"] == "replica-weighted" and owned is None
    assert ro["traffic"]["candidateReplicas"] == 2 and cand["spec"]["replicas"] == 2
    ro, _, vs, dr, _ = run({"istio": {"virtualService": {"name": "echo-vs", "routes": ["primary"]},
                                      "destinationRule": {"name": "echo-dr"}}}, False)
    assert ro["traffic"]["trafficRoutingMode"] == "external"
    assert [r["weight"] for r in vs["spec"]["http"][0]["route"]] == [70, 30]
    assert dr["spec"]["trafficPolicy"]["loadBalancer"]["consistentHash"]["httpHeaderName"] == \
        "x-omnia-session-id"


def test_process_pods_honour_replicas():
    """Process pod model (omnia serve): each replica is facade + runtime OS
    processes on its own ports; the Service lists every ready endpoint."""
    docs = load_manifests([ECHO])
    for d in docs:
        if d["kind"] == "AgentRuntime":
            d["spec"]["runtime"] = {"replicas": 2}

    async def go():
        store = new_store()
        mgr = Manager(store)
        await mgr.start()
        launcher = LocalLauncher(store, mode="process")
        launcher.start()
        try:
            for d in docs:
                store.apply(d)
            await mgr.settle(timeout=15, quiet=0.4)
            eps = []
            for _ in range(400):
                svc = store.try_get("Service", "echo")
                eps = ((svc or {}).get("status") or {}).get("endpoints") or []
                if len(eps) == 2:
                    break
                await asyncio.sleep(0.1)
            codes = []
            async with aiohttp.ClientSession() as s:
                for ep in eps:
                    r = await s.get(f"http://{ep}/healthz")
                    codes.append(r.status)
            pids = [r.pod.runtime.pid for r in launcher.replicas[("default", "echo")]]
            dep = store.get("Deployment", "echo")
            return eps, codes, pids, dep["status"].get("readyReplicas")
        finally:
            await launcher.stop()
            await mgr.stop()

    eps, codes, pids, ready = asyncio.run(go())
    assert len(eps) == 2 and len(set(eps)) == 2 and codes == [200, 200]
    assert len(set(pids)) == 2 and ready == 2


def test_process_mode_workspace_services_record_sessions():
    """Workspace service group -> session-api process; an agent in the
    workspace namespace gets its URL (local DNS) and the facade records turns."""
    from omnia_amd.ee.arena.fleet import FleetSession

    ws = {"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "team-b"},
          "spec": {"displayName": "Team B", "namespace": {"name": "team-b"},
                   "services": [{"name": "default", **DB}]}}
    docs = [ws] + load_manifests([ECHO])
    for d in docs[1:]:
        d["metadata"]["namespace"] = "team-b"
        if d["kind"] == "AgentRuntime":
            d["spec"] = {"facades": [{"type": "websocket"}], "promptPackRef": {"name": "echo-pack"},
                         "providers": [{"name": "llm", "providerRef": {"name": "echo-mock"}}]}

    async def go():
        store = new_store()
        mgr = Manager(store)
        await mgr.start()
        launcher = LocalLauncher(store, mode="process")
        launcher.start()
        try:
            for d in docs:
                store.apply(d)
            ep = None
            for _ in range(600):
                w = store.get("Workspace", "team-b", None)
                svc = store.try_get("Service", "echo", "team-b")
                ep = ((svc or {}).get("status") or {}).get("endpoint")
                sgs = (w.get("status") or {}).get("services") or []
                if ep and sgs and sgs[0]["ready"]:
                    break
                await asyncio.sleep(0.1)
            dep = store.get("Deployment", "echo", "team-b")
            fac = [c for c in dep["spec"]["template"]["spec"]["containers"]
                   if c["name"] == "facade"][0]
            url = {e["name"]: e["value"] for e in fac["env"]}["OMNIA_SESSION_API_URL"]
            async with FleetSession(f"ws://{ep}/ws") as fs:
                await fs.turn("hello")
                sid = fs.session_id
            sess_ep = store.get("Service", "session-api-team-b-default", "team-b")["status"][
                "endpoint"]
            rows = []
            async with aiohttp.ClientSession() as s:
                for _ in range(50):
                    r = await s.get(f"http://{sess_ep}/api/v1/sessions/{sid}/messages")
                    if r.status == 200:
                        rows = (await r.json()).get("messages", [])
                        if len(rows) >= 2:
                            break
                    await asyncio.sleep(0.1)
            return url, rows
        finally:
            await launcher.stop()
            await mgr.stop()

    url, rows = asyncio.run(go())
    assert url == "http://session-api-team-b-default.team-b:8080"
    assert [m["role"] for m in rows][:2] == ["user", "assistant"]
