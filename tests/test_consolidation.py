"""EE memory consolidation: action decoding, validator reasons, PII gate,
pre-filter buckets on a real MemoryStore (both SQL dialects), the seven store
writes, applier audit outcomes, and the worker's lock / anchor / cron-due /
mark-on-attempt cycle against an HTTP function facade.

Parity: ``ee/pkg/memory/consolidation/{types,validator,pii_gate,applier,client,
worker}_test.go`` and ``internal/memory/consolidation/prefilter_test.go``
(behaviour, not their SQL text)."""
import asyncio
import copy
import json
import time

import numpy as np
import pytest
import yaml
from aiohttp import web

from omnia_amd.api import crds
from omnia_amd.ee import consolidation as C
from omnia_amd.memory.model import Memory
from omnia_amd.memory.sqldialect import MemoryPostgres
from omnia_amd.memory.store import MemoryStore

WS = "ws1"


@pytest.fixture(params=["sqlite", "postgres-emulated"])
def store(request):
    if request.param == "sqlite":
        return MemoryStore()
    return MemoryStore(dialect=MemoryPostgres(emulate=True))


def save(store, content, user="u1", agent=None, title="", meta=None, age_s=0.0):
    scope = {"workspace_id": WS}
    if user:
        scope["virtual_user_id"] = user
    if agent:
        scope["agent_id"] = agent
    res = store.save(Memory(content=content, scope=scope, title=title, metadata=meta or {}),
                     require_user=False)
    if age_s:
        store._q("UPDATE memory_observations SET observed_at = ? WHERE id = ?",
                 [time.time() - age_s, res["observation_id"]])
    return res["id"], res["observation_id"]


def active_oids(store, entity_id):
    now = time.time()
    return [r[0] for r in store._q(
        "SELECT id FROM memory_observations WHERE entity_id = ? AND superseded_by IS NULL AND "
        "(valid_until IS NULL OR valid_until > ?)", [entity_id, now])]


# ------------------------------------------------------------------ decoding
def test_unmarshal_all_kinds_and_errors():
    future = "2099-01-01T00:00:00Z"
    acts = C.unmarshal_actions(json.dumps([
        {"action": "create_summary", "fromIDs": ["a", "b"], "scope": {"workspaceID": WS},
         "content": "sum", "metadata": {"k": "v"}},
        {"action": "supersede", "targetIDs": ["a"], "withID": "s"},
        {"action": "rescope", "targetIDs": ["a"], "newScope": {"workspaceID": WS, "agentID": "x"}},
        {"action": "invalidate", "targetIDs": ["a"], "validUntil": future},
        {"action": "merge_entities", "canonicalID": "c", "mergeIDs": ["d"]},
        {"action": "discard", "targetIDs": ["a"], "reason": "dup"},
        {"action": "rescore", "targetID": "a", "importance": 0.9, "confidence": 0.4}]))
    assert [a.kind for a in acts] == ["create_summary", "supersede", "rescope", "invalidate",
                                      "merge_entities", "discard", "rescore"]
    assert acts[2].f["newScope"].shape() == C.SHAPE_AGENT
    assert acts[3].f["validUntilTs"] > time.time()
    assert acts[4].modifying_targets() == ["d"] and acts[0].modifying_targets() == []
    with pytest.raises(ValueError, match="unknown action kind"):
        C.unmarshal_actions('[{"action": "explode"}]')
    with pytest.raises(ValueError, match="not a JSON array"):
        C.unmarshal_actions('{"action": "discard"}')
    with pytest.raises(ValueError, match="must be an array"):
        C.unmarshal_actions('[{"action": "discard", "targetIDs": "a"}]')


def test_scope_shapes():
    assert C.Scope(WS).shape() == C.SHAPE_INSTITUTIONAL
    assert C.Scope(WS, agentID="a").shape() == C.SHAPE_AGENT
    assert C.Scope(WS, userID="u").shape() == C.SHAPE_USER
    assert C.Scope(WS, "a", "u").shape() == C.SHAPE_USER_FOR_AGENT


# ------------------------------------------------------------------ validator
def _v(acts, gates=None, mut=None, users=0, pii=C.regex_pii_detector):
    ctx = C.ValidationContext(row_mutability=mut if mut is not None else {"r1": "mutable",
                                                                          "r2": "immutable"},
                              distinct_users=users)
    return [(r.accepted, r.reason) for r in C.Validator(WS, gates or {}, pii).validate(
        C.unmarshal_actions(json.dumps(acts)), ctx)]


def test_validator_reasons():
    ok = {"action": "rescope", "targetIDs": ["r1"], "newScope": {"workspaceID": WS,
                                                                 "agentID": "a"}}
    assert _v([ok]) == [(True, "")]
    assert _v([{"action": "discard", "targetIDs": []}]) == [(False, C.R_SHAPE)]
    assert _v([{"action": "invalidate", "targetIDs": ["r1"],
                "validUntil": "2001-01-01T00:00:00Z"}]) == [(False, C.R_SHAPE)]
    assert _v([{"action": "discard", "targetIDs": ["r2"]}]) == [(False, C.R_MUTABILITY)]
    assert _v([{"action": "discard", "targetIDs": ["zz"]}]) == [(False, C.R_UNKNOWN)]
    assert _v([dict(ok, newScope={"workspaceID": WS})]) == [(False, C.R_INSTITUTIONAL)]
    assert _v([dict(ok, newScope={"workspaceID": "other", "agentID": "a"})]) == \
        [(False, C.R_OUTSIDE_WS)]
    assert _v([ok], {"maxScopeWidening": "cluster"}) == [(False, C.R_WIDENING)]
    g = {"minDistinctUserCount": {"agentScoped": 3}}
    assert _v([ok], g, users=2) == [(False, C.R_ANONYMITY)]
    assert _v([ok], g, users=3) == [(True, "")]
    # user-for-agent has no anonymity gate
    assert _v([dict(ok, newScope={"workspaceID": WS, "agentID": "a", "userID": "u"})], g,
              users=0) == [(True, "")]
    # create_summary touches no existing row: no mutability check
    assert _v([{"action": "create_summary", "fromIDs": ["r2"], "content": "x"}]) == [(True, "")]


def test_pii_gate():
    summ = {"action": "create_summary", "fromIDs": ["r1"], "content": "mail bob@example.com"}
    assert _v([summ]) == [(False, C.R_PII)]
    assert _v([summ], {"requirePIIRedaction": False}) == [(True, "")]
    assert _v([summ], pii=None) == [(True, "")]
    assert _v([{"action": "discard", "targetIDs": ["r1"], "reason": "call 555-123-4567"}]) == \
        [(False, C.R_PII)]


# ------------------------------------------------------------------ pre-filters
def test_prefilter_stale_observations(store):
    old = 40 * 86400
    for i in range(6):
        save(store, f"likes tea {i}", user="u1", title="drinks", age_s=old)
    for i in range(2):  # group too small
        save(store, f"has cat {i}", user="u1", title="pets", age_s=old)
    save(store, "fresh", user="u1", title="drinks")  # too new
    save(store, "locked", user="u1", title="drinks", meta={"mutability": "immutable"},
         age_s=old)
    save(store, "regulated", user="u1", title="drinks", meta={"source_type": "regulated"},
         age_s=old)
    b = C.PreFilterRunner(store, "cpu").stale_observations(C.PreFilterOptions(
        WS, older_than=time.time() - 30 * 86400, min_group_size=5))
    assert len(b) == 1 and len(b[0].entries) == 6
    assert {e.content for e in b[0].entries} == {f"likes tea {i}" for i in range(6)}
    assert all(e.mutability == "mutable" and e.scope.userID == "u1" for e in b[0].entries)
    with pytest.raises(ValueError, match="OlderThan"):
        C.validate_prefilter_options(C.AXIS_STALE, C.PreFilterOptions(WS, older_than=0))


def test_prefilter_cross_scope(store):
    for u in ("u1", "u2", "u3"):
        save(store, f"{u}: the office closes at 6pm", user=u, title="office hours")
    save(store, "u1 only", user="u1", title="private")
    save(store, "u9 immutable", user="u9", title="office hours",
         meta={"mutability": "append_only"})
    b = C.PreFilterRunner(store, "cpu").cross_scope_candidates(
        C.PreFilterOptions(WS, min_distinct_users=3))
    assert len(b) == 1 and b[0].stats["distinctUsers"] == 3
    assert {e.scope.userID for e in b[0].entries} == {"u1", "u2", "u3"}
    assert C.PreFilterRunner(store, "cpu").cross_scope_candidates(
        C.PreFilterOptions(WS, min_distinct_users=4)) == []


def test_prefilter_entity_duplicates(store):
    rng = np.random.default_rng(0)
    base = rng.standard_normal(64).astype(np.float32)
    a, ao = save(store, "Acme Corp", title="acme")
    b, bo = save(store, "ACME Corporation", title="acme corp")
    c, co = save(store, "Globex", title="globex")
    store.set_embedding(ao, base, "m")
    store.set_embedding(bo, base + 0.05 * rng.standard_normal(64).astype(np.float32), "m")
    store.set_embedding(co, rng.standard_normal(64).astype(np.float32), "m")
    out = C.PreFilterRunner(store, "cpu").entity_duplicate_candidates(
        C.PreFilterOptions(WS, similarity_floor=0.9))
    assert len(out) == 1
    assert {e.id for e in out[0].entries} == {a, b} and out[0].stats["similarity"] > 0.9
    assert out[0].stats["canonicalID"] == min(a, b)


# ------------------------------------------------------------------ writes
def test_store_writes(store):
    cs = C.ConsolidationStore(store)
    e1, o1 = save(store, "one", user="u1", title="t")
    e2, o2 = save(store, "two", user="u2", title="t")
    e3, o3 = save(store, "three", user="u3", title="t")
    sid = cs.save_summary(WS, C.Scope(WS, agentID="bot"), "summary of one+two", {},
                          [o1, o2], "pack", "now")
    cs.supersede(WS, [o1], sid, "pack", "now")
    assert active_oids(store, e1) == []
    cs.rescope(WS, [o2], C.Scope(WS, agentID="bot"), "shared", "pack", "now")
    g = store.get(e2)
    assert g.scope.get("agent_id") == "bot" and "virtual_user_id" not in g.scope
    assert g.metadata["promoted_by_pack"] == "pack" and g.metadata["rescope_reason"] == "shared"
    cs.invalidate(WS, [o3], time.time() + 3600, "", "pack", "now")
    assert active_oids(store, e3) == [o3]  # still valid for an hour
    cs.discard(WS, [e3], "dup", "pack", "now")  # entity id: its active observations
    assert active_oids(store, e3) == []
    e4, o4 = save(store, "alias", user="u1", title="acme")
    e5, o5 = save(store, "canon", user="u1", title="acme inc")
    cs.merge_entities(WS, e5, [e4], "pack", "now")
    assert store.get(e4) is None
    assert {r[0] for r in store._q("SELECT id FROM memory_observations WHERE entity_id = ?",
                                   [e5])} == {o4, o5}
    cs.rescore(WS, o5, 0.8, 0.33, "pack", "now")
    assert store._q("SELECT confidence FROM memory_observations WHERE id = ?", [o5])[0][0] == \
        pytest.approx(0.33)
    with pytest.raises(LookupError):
        cs.discard("other-ws", [o5], "", "pack", "now")  # workspace confinement


def test_applier_outcomes_and_stop_on_failure(store):
    _, o1 = save(store, "one")
    audit = []
    ap = C.Applier(C.ConsolidationStore(store), audit.append)
    acts = C.unmarshal_actions(json.dumps([
        {"action": "discard", "targetIDs": [o1]},
        {"action": "discard", "targetIDs": ["nope"]},
        {"action": "rescore", "targetID": o1, "confidence": 0.1}]))
    results = [C.Result(acts[0], True), C.Result(acts[1], True), C.Result(acts[2], True)]
    with pytest.raises(RuntimeError, match="apply discard"):
        ap.apply(WS, "run", "pack", results)
    assert [(e["actionKind"], e["outcome"]) for e in audit] == [
        ("discard", C.APPLIED), ("discard", C.APPLY_FAILED)]  # third never attempted
    audit.clear()
    assert ap.apply(WS, "run", "pack", [C.Result(acts[0], False, C.R_PII)]) == {
        C.APPLIED: 0, C.REJECTED: 1, C.APPLY_FAILED: 0}
    assert audit[0]["reason"] == C.R_PII


def test_audit_logger_sink():
    from omnia_amd.ee.audit import AuditLogger

    lg = AuditLogger()
    sink = C.audit_logger_sink(lg)
    sink({"runID": "r", "workspaceID": WS, "packRef": "p", "actionKind": "discard",
          "outcome": C.APPLIED, "reason": "", "targetIDs": ["a", "b"], "now": 0})
    lg.close()  # drains the writer thread
    rows = lg.query(workspace=WS)["entries"]
    assert rows and rows[0]["eventType"] == "memory_consolidated"
    assert rows[0]["metadata"]["actionKind"] == "discard" and rows[0]["resultCount"] == 2


# ------------------------------------------------------------------ worker
POLICY = {"consolidation": {
    "schedule": "0 2 * * *", "schedules": {"crossScopeCandidates": "@every 1h"},
    "functionRefs": {"crossScopeCandidates": {"name": "rescoper", "namespace": "fns"}},
    "safetyGates": {"minDistinctUserCount": {"agentScoped": 3}},
    "timeouts": {"functionCall": "5s", "passWallClock": "30s"}}}


def _function_app(calls, mode="rescope"):
    async def fn(request):
        body = await request.json()
        calls.append((request.match_info["name"], body))
        if mode == "fail":
            return web.json_response({"error": "boom"}, status=500)
        acts = []
        for b in body["buckets"]:
            ids = [e["id"] for e in b["entries"]]
            acts.append({"action": "rescope", "targetIDs": ids,
                         "newScope": {"workspaceID": body["workspaceID"], "agentID": "bot"}})
            # never allowed: institutional destination
            acts.append({"action": "rescope", "targetIDs": ids[:1],
                         "newScope": {"workspaceID": body["workspaceID"]}})
        return web.json_response(acts)

    app = web.Application()
    app.router.add_post("/functions/{name}", fn)
    return app


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


def test_worker_cycle(store):
    for u in ("u1", "u2", "u3"):
        save(store, f"{u}: VPN needs the new client", user=u, title="vpn")

    async def go():
        calls = []
        runner, url = await _serve(_function_app(calls))
        clock = [1_000_000.0]
        audit = []
        w = C.ConsolidationWorker(store, [("pol", POLICY)], workspaces=lambda p: [WS],
                                  client=C.FunctionClient(base_url=url), auditor=audit.append,
                                  now=lambda: clock[0], device="cpu")
        try:
            r = await w.run_once()
            assert [x["status"] for x in r] == ["anchored"] and not calls
            clock[0] += 600
            r = await w.run_once()
            assert [x["status"] for x in r] == ["not_due"] and not calls
            clock[0] += 3600
            r = await w.run_once()
            assert r[0]["status"] == "ok" and len(calls) == 1
            name, body = calls[0]
            assert name == "rescoper" and body["axis"] == C.AXIS_CROSS_SCOPE
            assert body["gates"] == {"minDistinctUserCount": {"agentScoped": 3},
                                     "requirePIIRedaction": True}
            assert r[0]["results"] == [("rescope", True, ""),
                                       ("rescope", False, C.R_INSTITUTIONAL)]
            assert r[0]["counts"] == {C.APPLIED: 1, C.REJECTED: 1, C.APPLY_FAILED: 0}
            assert {a["outcome"] for a in audit} == {C.APPLIED, C.REJECTED}
            mems = store.list({"workspace_id": WS, "agent_id": "bot"}, limit=10)
            assert len(mems) == 3
            # the rescoped rows left the user-scoped pool: the next due pass is empty
            clock[0] += 3600
            r = await w.run_once()
            assert r[0]["status"] == "empty" and len(calls) == 1
            # a second replica cannot run while the lock is held
            other = C.ConsolidationWorker(store, [("pol", POLICY)], workspaces=lambda p: [WS],
                                          client=C.FunctionClient(base_url=url))
            ok, release = w.locks.try_lock(WS, "consolidation")
            assert ok
            assert [x["status"] for x in await other.run_once()] == ["lock_unavailable"]
            release()
        finally:
            await runner.cleanup()

    asyncio.run(go())


def test_worker_marks_on_attempt_when_function_fails(store):
    for u in ("u1", "u2", "u3"):
        save(store, f"{u}: lunch at noon", user=u, title="lunch")

    async def go():
        calls = []
        runner, url = await _serve(_function_app(calls, mode="fail"))
        clock = [2_000_000.0]
        w = C.ConsolidationWorker(store, [("pol", POLICY)], workspaces=lambda p: [WS],
                                  client=C.FunctionClient(base_url=url), now=lambda: clock[0],
                                  device="cpu")
        try:
            await w.run_once()  # anchor
            clock[0] += 3601
            r = await w.run_once()
            assert r[0]["status"] == "function_error" and len(calls) == 1
            r = await w.run_once()  # same instant: marked on attempt, not retried
            assert r[0]["status"] == "not_due" and len(calls) == 1
        finally:
            await runner.cleanup()

    asyncio.run(go())


def test_function_client_urls():
    c = C.FunctionClient()
    assert c.url_for({"name": "f", "namespace": "ns"}) == \
        "http://f.ns.svc.cluster.local:8080/functions/f"
    with pytest.raises(ValueError, match="namespace required"):
        c.url_for({"name": "f"})
    c = C.FunctionClient(resolve=lambda n, ns: "127.0.0.1:9999")
    assert c.url_for({"name": "f", "namespace": "ns"}) == "http://127.0.0.1:9999/functions/f"
    assert C.axis_due("@every 1h", 0.0, 3600.0) and not C.axis_due("@every 1h", 0.0, 3599.0)


def test_consolidation_example_manifests_admitted():
    docs = [d for d in yaml.safe_load_all(open("examples/consolidation/manifests.yaml"))
            if d["apiVersion"].startswith("omnia")]
    assert {d["kind"] for d in docs} == {"Provider", "PromptPack", "AgentRuntime",
                                         "MemoryPolicy"}
    for d in docs:
        assert crds.validate_object(copy.deepcopy(d)) == [], d["metadata"]["name"]
    pol = next(d for d in docs if d["kind"] == "MemoryPolicy")["spec"]
    assert set(pol["consolidation"]["functionRefs"]) == {C.AXIS_CROSS_SCOPE,
                                                         C.AXIS_ENTITY_DUPES}
    assert C.resolved_schedule(pol, C.AXIS_CROSS_SCOPE) == "0 */6 * * *"
    assert C.resolved_schedule(pol, C.AXIS_ENTITY_DUPES) == "0 2 * * *"
    assert C.resolved_timeouts(pol) == (30.0, 600.0)


def test_cluster_listers():
    class FakeClient:
        objs = {("MemoryPolicy", "pol"): {"metadata": {"name": "pol"}, "spec": POLICY},
                ("MemoryPolicy", "plain"): {"metadata": {"name": "plain"}, "spec": {}},
                ("Workspace", "team-a"): {"metadata": {"name": "team-a", "uid": "uid-a"},
                                          "spec": {"services": [
                                              {"name": "default", "memory": {
                                                  "policyRef": {"name": "pol"}}}]}}}

        def list(self, kind, ns=None):
            return [o for (k, _), o in self.objs.items() if k == kind]

        def try_get(self, kind, name, ns=None):
            return self.objs.get((kind, name))

    c = FakeClient()
    pols = C.KubePolicyLister(c)()
    assert [n for n, _ in pols] == ["pol", "plain"]
    assert C.KubeWorkspaceLister(c, "team-a")("pol") == ["uid-a"]
    assert C.KubeWorkspaceLister(c, "team-a")("plain") == []
    assert C.KubeWorkspaceLister(c, "missing")("pol") == []
    assert C.KubeWorkspaceLister(c, "")("pol") == []
    # the worker skips policies without a consolidation block
    w = C.ConsolidationWorker(MemoryStore(), C.KubePolicyLister(c),
                              workspaces=C.KubeWorkspaceLister(c, "team-a"), device="cpu")
    assert asyncio.run(w.run_once()) == [{"workspace": "uid-a", "axis": C.AXIS_CROSS_SCOPE,
                                          "status": "anchored"}]
