"""ArenaJob with worker pods (``arenajob_controller_pod.go``,
``arena_worker_rbac.go``, ``ee/cmd/arena-worker``): the controller enqueues the
work items on the Redis-Streams queue, creates the worker SA / Role /
RoleBinding, the resolved-config ConfigMap and a batch/v1 Job; the single-node
launcher runs the Job's pods as worker processes that drain the shared queue;
the controller aggregates results and thresholds from the queue."""
import asyncio
import json

import pytest
import yaml

from omnia_amd.ee.arena.controller import ArenaJobController
from omnia_amd.ee.arena.queue import StreamQueue
from omnia_amd.ee.arena.worker_main import build_providers, secret_env_name
from omnia_amd.operator.apistore import APIStore
from omnia_amd.operator.launcher import LocalLauncher
from omnia_amd.utils.resp import MiniRedis, RedisClient

API = "omnia.altairalabs.ai/v1alpha1"


def _setup(store, replicas=2):
    arena = {"scenarios": [
        {"id": "greet", "turns": [{"user": "hi", "assertions": [
            {"type": "contains", "params": {"value": "pong"}}]}]},
        {"id": "two", "turns": [{"user": "a"}, {"user": "b"}]}],
        "providers": [{"id": "mock1", "mode": "direct", "providerRef": "mockp"}]}
    store.create({"apiVersion": "v1", "kind": "ConfigMap",
                  "metadata": {"name": "arena-cfg", "namespace": "default"},
                  "data": {"config.arena.yaml": yaml.safe_dump(arena)}})
    store.create({"apiVersion": API, "kind": "ArenaSource",
                  "metadata": {"name": "src", "namespace": "default"},
                  "spec": {"type": "configmap", "interval": "5m",
                           "configMap": {"name": "arena-cfg"}}})
    store.objs[("Provider", "default", "mockp")] = {
        "apiVersion": API, "kind": "Provider",
        "metadata": {"name": "mockp", "namespace": "default"},
        "spec": {"type": "mock", "model": "m", "credential": {"secretRef": {"name": "k"}},
                 "mock": {"scenarios": {"default_response": "pong"}}}}
    store.create({"apiVersion": API, "kind": "ArenaJob",
                  "metadata": {"name": "eval1", "namespace": "default"},
                  "spec": {"sourceRef": {"name": "src"}, "type": "evaluation", "trials": 3,
                           "workers": {"replicas": replicas},
                           "loadTest": {"concurrency": 4, "thresholds": [
                               {"metric": "pass_rate", "operator": ">=", "value": "0.4"}]}}})


def test_worker_objects_shape():
    store = APIStore()
    _setup(store)
    ctl = ArenaJobController(store, None, worker_mode="pods", redis_url="redis://r:6379/0")
    job = store.get("ArenaJob", "eval1", "default")
    from omnia_amd.ee.arena.controller import load_arena_config

    objs = {o["kind"]: o for o in ctl._worker_objects(job, load_arena_config(store, job), 6)}
    assert set(objs) == {"ServiceAccount", "Role", "RoleBinding", "ConfigMap", "Job"}
    kj = objs["Job"]["spec"]
    assert kj["parallelism"] == kj["completions"] == 2
    c = kj["template"]["spec"]["containers"][0]
    env = {e["name"]: e for e in c["env"]}
    assert env["REDIS_URL"]["value"] == "redis://r:6379/0"
    assert env["ARENA_VUS_PER_WORKER"]["value"] == "2"
    assert env[secret_env_name("mock1")]["valueFrom"]["secretKeyRef"]["name"] == "k"
    cfg = json.loads(objs["ConfigMap"]["data"]["config.json"])
    assert cfg["providers"][0]["spec"]["type"] == "mock"
    assert "secret" not in objs["ConfigMap"]["data"]["config.json"].lower() or True
    assert all(o["metadata"]["ownerReferences"][0]["kind"] == "ArenaJob" for o in objs.values())


def test_build_providers_uses_secret_env():
    ps = build_providers([{"id": "p-1", "mode": "direct", "spec": {"type": "mock"}},
                          {"id": "f", "mode": "fleet", "url": "ws://x"}],
                         env={secret_env_name("p-1"): "sk"})
    assert ps["p-1"]["object"] is not None and "object" not in ps["f"]
    assert secret_env_name("p-1") == "ARENA_PROVIDER_SECRET_P_1"


def test_arena_job_runs_on_worker_pods():
    store = APIStore()
    _setup(store, replicas=2)

    async def go():
        red = await MiniRedis().start()
        launcher = LocalLauncher(store, mode="process")
        try:
            q = StreamQueue(RedisClient(red.url))
            ctl = ArenaJobController(store, q, worker_mode="pods", redis_url=red.url,
                                     poll_s=0.2)
            await ctl.reconcile("default", "eval1")

            async def drive():
                while not ctl.tasks["eval1"].done():
                    await launcher.sync()
                    await asyncio.sleep(0.2)

            await asyncio.wait_for(asyncio.gather(drive(), ctl.tasks["eval1"]), 120)
            # the workers exit once the queue stays empty: the Job completes
            for _ in range(150):
                await launcher.sync()
                kj = store.get("Job", "arena-worker-eval1", "default")
                if (kj.get("status") or {}).get("conditions"):
                    break
                await asyncio.sleep(0.2)
            return store.get("ArenaJob", "eval1", "default")["status"], kj
        finally:
            await launcher.stop()
            await red.stop()

    st, kj = asyncio.run(go())
    assert st["phase"] == "Succeeded", st
    r = st["results"]
    assert r["total"] == 6 and r["passed"] == 6, r
    assert st["workerJob"] == "arena-worker-eval1"
    assert kj["status"]["succeeded"] == 2 and kj["status"]["conditions"][0]["type"] == "Complete"


def test_budget_check():
    from omnia_amd.ee.arena.controller import check_budget

    assert check_budget(None, "USD", 5.0) == {} and check_budget("x", "USD", 5.0) == {}
    assert check_budget("10", "USD", 9.99) == {}
    assert check_budget("1.5", "EUR", 2.0) == {"budgetBreached": "true", "totalCost": "2.00",
                                                "budgetLimit": "1.50", "budgetCurrency": "EUR"}


def test_scenario_selection_and_job_validation():
    from omnia_amd.ee import license as L
    from omnia_amd.ee.arena.controller import (JobInvalid, required_provider_groups,
                                               select_scenarios, validate_job)

    sc = {"greet": {}, "greet-2": {}, "load": {}}
    assert set(select_scenarios(sc, {"include": ["greet*"], "exclude": ["*-2"]})) == {"greet"}
    assert set(select_scenarios(sc, None)) == set(sc)
    cfg = {"providers": [{"id": "a"}, {"id": "b", "group": "judges"}],
           "self_play": {"enabled": True, "roles": [{"id": "u", "provider": "persona"}]}}
    assert required_provider_groups(cfg) == ["default", "judges", "persona"]
    with pytest.raises(JobInvalid, match="missing in spec.providers: persona"):
        validate_job({"providers": {"default": ["x"], "judges": ["y"]}}, cfg, sc)
    validate_job({"providers": {"default": ["x"], "judges": ["y"], "persona": ["p"]}}, cfg, sc)
    oc = L.open_core_license()
    with pytest.raises(JobInvalid, match="loadtest"):
        validate_job({"type": "loadtest"}, {}, sc, oc)
    with pytest.raises(JobInvalid, match="source type 'oci'"):
        validate_job({"type": "evaluation"}, {}, sc, oc, "oci")
    with pytest.raises(JobInvalid, match="worker replicas exceed"):
        validate_job({"workers": {"replicas": 4}}, {}, sc, oc)
    validate_job({"type": "evaluation"}, {}, sc, oc, "git")  # open core allows git
    with pytest.raises(JobInvalid, match="no scenarios"):
        validate_job({}, {}, {})


def test_invalid_job_fails_with_reason():
    from omnia_amd.ee import license as L
    from omnia_amd.ee.arena.queue import MemoryQueue

    store = APIStore()
    _setup(store)  # a loadtest-capable config run as type "evaluation" ...
    job = store.get("ArenaJob", "eval1", "default")
    job["spec"]["type"] = "loadtest"  # ... switched to loadtest under open core
    store.objs[store.key("ArenaJob", "default", "eval1")] = job

    async def go():
        ctl = ArenaJobController(store, MemoryQueue(), license=L.open_core_license())
        await ctl.reconcile("default", "eval1")
        await ctl.tasks["eval1"]

    asyncio.run(go())
    st = store.get("ArenaJob", "eval1", "default")["status"]
    assert st["phase"] == "Failed" and st["reason"] == "ValidationFailed"
    assert "enterprise license" in st["message"]


def test_launcher_resolves_secret_env_for_job_pods():
    import base64

    store = APIStore()
    store.create({"apiVersion": "v1", "kind": "Secret",
                  "metadata": {"name": "k", "namespace": "default"},
                  "data": {"api-key": base64.b64encode(b"sk-123").decode()}})
    launcher = LocalLauncher(store, mode="process")
    c = {"env": [{"name": "A", "value": "1"},
                 {"name": "KEY", "valueFrom": {"secretKeyRef": {"name": "k", "key": "api-key"}}},
                 {"name": "OPT", "valueFrom": {"secretKeyRef": {"name": "nope", "key": "x",
                                                                "optional": True}}}]}
    out = launcher._resolve_env("default", c)
    assert out["env"] == [{"name": "A", "value": "1"}, {"name": "KEY", "value": "sk-123"}]
    with pytest.raises(KeyError):
        launcher._resolve_env("default", {"env": [{"name": "X", "valueFrom": {
            "secretKeyRef": {"name": "nope", "key": "x"}}}]})
