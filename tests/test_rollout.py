"""Canary rollout engine (``internal/controller/rollout*_test.go``): analysis
steps against Prometheus / web metric providers, automatic and manual failure
handling, progress-deadline auto-rollback, indefinite pauses, two-phase
promotion, version-triggered rollouts and the last-rolled-back guard."""
import asyncio
import copy
import os

import pytest

from omnia_amd.api import crds
from omnia_amd.cli import load_manifests
from omnia_amd.operator import rollout as R
from omnia_amd.operator.apistore import get_condition
from omnia_amd.operator.controllers import AgentRuntimeReconciler, default_reconcilers
from omnia_amd.operator.manager import Manager, new_store

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "examples", "echo-function", "manifests.yaml")


class FakeProm:
    def __init__(self, values):
        self.values = values  # query substring -> value (or Exception)
        self.urls = []

    def __call__(self, url, headers=None):
        self.urls.append(url)
        for k, v in self.values.items():
            if k in url:
                if isinstance(v, Exception):
                    raise v
                if isinstance(v, dict):
                    return v
                return {"status": "success", "data": {"resultType": "vector", "result": [
                    {"metric": {}, "value": [0, str(v)]}]}}
        return {"status": "success", "data": {"resultType": "vector", "result": []}}


def _kubelet(store, hold_candidate=False):
    async def loop():
        while True:
            for d in store.list("Deployment"):
                if hold_candidate and d["metadata"]["name"].endswith("-candidate"):
                    continue
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


def _docs(rollout=None, extra_versions=()):
    docs = load_manifests([ECHO])
    pp = [d for d in docs if d["kind"] == "PromptPack"][0]
    for v in extra_versions:
        p = copy.deepcopy(pp)
        p["metadata"]["name"] = f"echo-pack-{v.replace('.', '-')}"
        p["spec"]["version"] = v
        docs.append(p)
    for d in docs:
        if d["kind"] == "AgentRuntime" and rollout is not None:
            d["spec"]["promptPackRef"] = {"name": "echo-pack", "version": "1.0.0"}
            d["spec"]["rollout"] = rollout
    return docs


def _analysis(name, metrics, args=None):
    return {"apiVersion": crds.API_VERSION, "kind": "RolloutAnalysis",
            "metadata": {"name": name, "namespace": "default"},
            "spec": {"metrics": metrics, **({"args": args} if args else {})}}


def _run(docs, engine, until, kubelet_hold=False, steps=150, after=None):
    async def go():
        store = new_store()
        rs = default_reconcilers()
        for r in rs:
            if isinstance(r, AgentRuntimeReconciler):
                r.rollout_engine = engine
        kubelet = _kubelet(store, kubelet_hold)
        mgr = Manager(store, reconcilers=rs)
        await mgr.start()
        try:
            for d in docs:
                store.apply(d)
            for _ in range(steps):
                await asyncio.sleep(0.1)
                a = store.get("AgentRuntime", "echo")
                if until(a, store):
                    break
            if after is not None:
                after(store)
                for _ in range(steps):
                    await asyncio.sleep(0.1)
                    a = store.get("AgentRuntime", "echo")
                    if until(a, store):
                        break
            return store.get("AgentRuntime", "echo"), store
        finally:
            await mgr.stop()
            kubelet.cancel()

    return asyncio.run(go())


def _events(store):
    return [(e["reason"], e["message"]) for e in store.list("Event")]


PROM = {"prometheus": {"address": "http://prom:9090",
                       "query": 'sum(rate(errors{agent="{{args.agent}}"}[5m]))'}}


def test_analysis_pass_advances_and_promotes():
    prom = FakeProm({"errors": 0.01})
    docs = _docs({"candidate": {"promptPackRef": {"name": "echo-pack", "version": "1.1.0"}},
                  "steps": [{"setWeight": 10},
                            {"analysis": {"templateName": "err-rate",
                                          "args": [{"name": "agent", "value": "echo"}]}},
                            {"setWeight": 50}]}, extra_versions=["1.1.0"])
    docs.append(_analysis("err-rate", [{"name": "errors", "interval": "1s",
                                        "successCondition": "result[0] < 0.05",
                                        "provider": PROM}],
                          args=[{"name": "agent", "value": "default-agent"}]))
    a, store = _run(docs, R.RolloutEngine(http_json=prom),
                    lambda a, s: (a["status"].get("rollout") or {}).get("message") == "promoted")
    assert a["status"]["rollout"]["message"] == "promoted"
    assert a["spec"]["promptPackRef"]["version"] == "1.1.0"
    # step args override the template's
    assert 'agent%3D%22echo%22' in prom.urls[0] or 'agent="echo"' in prom.urls[0]
    reasons = [r for r, _ in _events(store)]
    assert {"RolloutAnalysisPassed", "RolloutPromoting", "RolloutPromoted"} <= set(reasons)


def test_analysis_failure_automatic_rollback_and_no_retrigger():
    prom = FakeProm({"errors": 0.5})
    docs = _docs({"candidate": {"promptPackRef": {"name": "echo-pack", "version": "1.1.0"}},
                  "steps": [{"setWeight": 10}, {"analysis": {"templateName": "err-rate"}}],
                  "rollback": {"mode": "automatic"},
                  "trigger": {"promptPackChannel": "stable"}}, extra_versions=["1.1.0"])
    docs.append(_analysis("err-rate", [{"name": "errors", "interval": "1s",
                                        "successCondition": "result[0] < 0.05",
                                        "provider": {"prometheus": {
                                            "address": "http://prom:9090",
                                            "query": "errors"}}}]))
    a, store = _run(docs, R.RolloutEngine(http_json=prom),
                    lambda a, s: "auto-rollback" in ((a["status"].get("rollout") or {})
                                                     .get("message") or ""))
    ro = a["status"]["rollout"]
    assert ro["active"] is False and "failed metrics: errors" in ro["message"]
    assert a["spec"]["rollout"]["candidate"]["promptPackRef"] == a["spec"]["promptPackRef"]
    assert a["metadata"]["annotations"][R.LAST_ROLLED_BACK] == "1.1.0"
    assert store.try_get("Deployment", "echo-candidate") is None
    assert get_condition(a, "RolloutActive")["status"] == "False"
    assert any(r == "RolloutRolledBack" for r, _ in _events(store))
    # the trigger does not re-propose the version that was just rolled back
    assert not R.RolloutEngine().maybe_trigger(
        store, a, a["status"], lambda n: [p for p in store.list("PromptPack")])


def test_analysis_failure_manual_hold_and_provider_errors():
    docs = _docs({"candidate": {"promptPackRef": {"name": "echo-pack", "version": "1.1.0"}},
                  "steps": [{"analysis": {"templateName": "err-rate"}}],
                  "rollback": {"mode": "manual"}}, extra_versions=["1.1.0"])
    docs.append(_analysis("err-rate", [{"name": "errors", "interval": "1s",
                                        "successCondition": "result >= 1",
                                        "provider": {"prometheus": {"address": "http://p",
                                                                    "query": "up"}}}]))
    a, store = _run(docs, R.RolloutEngine(http_json=FakeProm({"up": 0})),
                    lambda a, s: "analysis failed" in ((a["status"].get("rollout") or {})
                                                       .get("message") or ""))
    ro = a["status"]["rollout"]
    assert ro["active"] is True and ro["currentStep"] == 0
    assert get_condition(a, "RolloutActive")["reason"] == "AnalysisFailed"
    assert store.try_get("Deployment", "echo-candidate") is not None  # held, not removed
    # a provider outage is retried, never treated as a verdict
    a, _ = _run(docs, R.RolloutEngine(http_json=FakeProm({"up": ConnectionError("down")})),
                lambda a, s: "error" in ((a["status"].get("rollout") or {}).get("message") or ""),
                steps=60)
    assert "error" in a["status"]["rollout"]["message"] and a["status"]["rollout"]["active"]


def test_progress_deadline_auto_rollback():
    clock = [1e9]
    docs = _docs({"candidate": {"promptPackRef": {"name": "echo-pack", "version": "1.1.0"}},
                  "steps": [{"setWeight": 10}, {"pause": {}}],
                  "rollback": {"mode": "automatic"}}, extra_versions=["1.1.0"])
    eng = R.RolloutEngine(clock=lambda: clock[0])

    def push_time(store):
        # the candidate never became ready; ten minutes pass
        d = store.get("Deployment", "echo-candidate")
        d["status"] = {"conditions": [{"type": "Progressing", "status": "False",
                                       "reason": "ProgressDeadlineExceeded"}]}
        d["metadata"].pop("resourceVersion", None)
        store.update_status(d)
        ar = store.get("AgentRuntime", "echo")
        ar["metadata"].setdefault("annotations", {})["poke"] = "1"
        store.update(ar)

    a, store = _run(docs, eng,
                    lambda a, s: "pod unhealthy" in ((a["status"].get("rollout") or {})
                                                     .get("message") or ""),
                    kubelet_hold=True, steps=40, after=push_time)
    assert "pod unhealthy" in a["status"]["rollout"]["message"]
    assert store.try_get("Deployment", "echo-candidate") is None


def test_version_trigger_starts_a_rollout():
    docs = _docs({"steps": [{"setWeight": 25}, {"pause": {}}],
                  "trigger": {"promptPackChannel": "stable"}})

    def publish(store):
        pp = copy.deepcopy(store.get("PromptPack", "echo-pack"))
        for k in ("uid", "resourceVersion", "creationTimestamp", "generation"):
            pp["metadata"].pop(k, None)
        pp.pop("status", None)
        for name, v in (("echo-pack-2-0-0", "2.0.0"), ("echo-pack-3-0-0-rc1", "3.0.0-rc1")):
            p = copy.deepcopy(pp)
            p["metadata"]["name"], p["spec"]["version"] = name, v
            store.apply(p)

    a, store = _run(docs, R.RolloutEngine(),
                    lambda a, s: (a["status"].get("rollout") or {}).get("currentWeight") == 25,
                    after=publish)
    # stable channel: the prerelease is ignored, 2.0.0 is proposed
    assert a["spec"]["rollout"]["candidate"]["promptPackRef"] == {"name": "echo-pack",
                                                                  "version": "2.0.0"}
    ro = a["status"]["rollout"]
    assert ro["active"] and ro["candidateVersion"] == "2.0.0" and ro["message"].startswith(
        "step 1: paused indefinitely")
    assert any(r == "RolloutTriggered" for r, _ in _events(store))


def test_primitives():
    assert R.evaluate_condition("result[0] < 0.05", 0.01)
    assert R.evaluate_condition("result >= 1", 1.0)
    assert not R.evaluate_condition("result[0] != 2", 2.0)
    with pytest.raises(R.AnalysisError):
        R.evaluate_condition("value < 3", 1)
    assert R.version_newer("1.10.0", "1.9.3") and not R.version_newer("1.0.0", "1.0.0")
    assert R.version_newer("2.0.0", "2.0.0-rc1") and R.version_newer("2.0.0-rc2", "2.0.0-rc1")
    packs = [{"spec": {"version": v}} for v in ("1.0.0", "1.2.0", "2.0.0-rc1", "junk")]
    assert R.channel_max(packs, "stable")["spec"]["version"] == "1.2.0"
    assert R.channel_max(packs, "prerelease")["spec"]["version"] == "2.0.0-rc1"
    web = R.query_web("http://x/metrics", "$.data.items[1].score",
                      http_json=lambda u, h=None: {"data": {"items": [{"score": 1},
                                                                       {"score": 0.93}]}})
    assert web == 0.93
    tpl = {"spec": {"metrics": [
        {"name": "a", "interval": "10s", "count": 3, "successCondition": "result < 1",
         "provider": {"web": {"url": "http://x/{{args.path}}", "jsonPath": "v"}}},
        {"name": "b", "interval": "10s", "successCondition": "result < 1", "failureLimit": 1,
         "provider": {"web": {"url": "http://y", "jsonPath": "v"}}}],
        "args": [{"name": "path", "value": "m"}]}}
    seen = []

    def hj(url, headers=None):
        seen.append(url)
        return {"v": 0 if url.endswith("/m") else 5}

    st = {}
    assert R.run_analysis(tpl, {}, hj, state=st, now=100.0) == (None, "measuring", 10.0)
    assert R.run_analysis(tpl, {}, hj, state=st, now=105.0)[0] is None  # not due yet
    assert R.run_analysis(tpl, {}, hj, state=st, now=110.0)[0] is None
    assert R.run_analysis(tpl, {}, hj, state=st, now=120.0) == (True, "all metrics passed",
                                                                 None)
    assert seen[0] == "http://x/m" and len(seen) == 4  # 3 x a, 1 x b (count 1)
    bad = {"spec": {"metrics": [{"name": "e", "interval": "1s", "count": 5,
                                 "successCondition": "result < 1",
                                 "failureCondition": "result > 100",
                                 "provider": {"web": {"url": "http://z", "jsonPath": "v"}}}]}}
    assert R.run_analysis(bad, {}, lambda u, h=None: {"v": 500}, state={}, now=0.0) == \
        (False, "failed metrics: e", None)  # fails fast past failureLimit 0
    ev = {"spec": {"metrics": [{"name": "q", "interval": "1s", "successCondition": "result >= 0.9",
                                "provider": {"arenaEval": {"workspace": "w",
                                                           "evalDef": "quality"}}}]}}
    assert R.run_analysis(ev, {}, eval_lookup=lambda w, e: 0.95, state={})[0] is True
    with pytest.raises(R.AnalysisError):
        R.run_analysis(ev, {}, state={})
    spec = {"promptPackRef": {"name": "p"}, "providers": [{"name": "llm",
                                                           "providerRef": {"name": "a"}}],
            "rollout": {"candidate": {"providerRefs": [{"name": "llm",
                                                        "providerRef": {"name": "b"}}]}}}
    assert R.candidate_differs(spec)
    spec["rollout"]["candidate"]["providerRefs"][0]["providerRef"]["name"] = "a"
    assert not R.candidate_differs(spec)
    spec["rollout"]["candidate"] = {"promptPackRef": {"name": "p", "track": "stable"}}
    assert not R.candidate_differs(spec)  # an empty track is the stable track
