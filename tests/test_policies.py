"""Policy reconcilers and their enforcement (``internal/controller/
agentpolicy_controller*_test.go``, ``memorypolicy_*_test.go``,
``sessionretentionpolicy_controller_test.go``): AgentPolicy -> Istio
AuthorizationPolicies + in-node tool access in the runtime executor;
MemoryPolicy validation + retention passes over the memory store;
SessionRetentionPolicy -> retention ConfigMap -> compaction settings."""
import asyncio
import json
import time

import pytest
import yaml

from omnia_amd.memory.model import META_CONSENT_CATEGORY, Memory
from omnia_amd.memory.retention import apply_memory_policy, decay_score, grace_seconds
from omnia_amd.memory.store import MemoryStore
from omnia_amd.operator.apistore import APIStore, get_condition
from omnia_amd.operator.policies import (ISTIO_API, ISTIO_KIND, AgentPolicyReconciler,
                                         MemoryPolicyReconciler, PolicyInvalid,
                                         SessionRetentionPolicyReconciler, compile_tool_access,
                                         desired_authorization_policies, parse_duration,
                                         retention_from_config, validate_agent_policy,
                                         validate_cron, validate_memory_policy)
from omnia_amd.tools.executor import InProcessHandler, OmniaExecutor, ToolAccess


def _ap(name="tools", mode="enforce", access="allowlist", agents=None, on_failure="deny",
        rules=None):
    spec = {"toolAccess": {"mode": access, "rules": rules or [
        {"registry": "reg", "tools": ["get_weather", "search"]}]}, "mode": mode,
        "onFailure": on_failure}
    if agents is not None:
        spec["selector"] = {"agents": agents}
    return {"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "AgentPolicy",
            "metadata": {"name": name, "namespace": "default", "uid": "uid-" + name},
            "spec": spec}


def _agent(store, name):
    store.objs[("AgentRuntime", "default", name)] = {
        "kind": "AgentRuntime", "metadata": {"name": name, "namespace": "default"},
        "spec": {}}


# ------------------------------------------------------------------ AgentPolicy
def test_agent_policy_semantic_validation():
    validate_agent_policy({})  # no toolAccess: nothing to enforce, valid
    for bad, msg in [({"mode": "allowlist", "rules": []}, "rules must not be empty"),
                     ({"mode": "allowlist", "rules": [{"registry": "", "tools": ["x"]}]},
                      "registry must not be empty"),
                     ({"mode": "denylist", "rules": [{"registry": "r", "tools": []}]},
                      "tools must not be empty"),
                     ({"mode": "denylist", "rules": [{"registry": "r", "tools": ["a", ""]}]},
                      "tool name must not be empty")]:
        with pytest.raises(PolicyInvalid, match=msg):
            validate_agent_policy({"toolAccess": bad})


def test_authorization_policies_allowlist_enforce_permissive_denylist():
    pol = _ap(agents=["a1"])
    pol["metadata"]["uid"] = "u"
    allow, deny = desired_authorization_policies(pol)
    assert (allow["apiVersion"], allow["kind"]) == (ISTIO_API, ISTIO_KIND)
    assert allow["metadata"]["name"] == "tools-allow" and allow["spec"]["action"] == "ALLOW"
    when = allow["spec"]["rules"][0]["when"]
    assert when[0] == {"key": "request.headers[X-Omnia-Tool-Name]",
                       "values": ["reg/get_weather", "reg/search"]}
    assert when[1] == {"key": "request.headers[X-Omnia-Agent-Name]", "values": ["a1"]}
    # the DENY catch-all excludes the allowlisted tools (DENY is evaluated first)
    assert deny["spec"]["action"] == "DENY"
    assert deny["spec"]["rules"][0]["when"][0]["notValues"] == ["reg/get_weather", "reg/search"]
    assert allow["metadata"]["ownerReferences"][0]["kind"] == "AgentPolicy"
    (audit,) = desired_authorization_policies(_ap(mode="permissive"))
    assert audit["spec"]["action"] == "AUDIT" and audit["metadata"]["name"] == "tools-allow"
    (d,) = desired_authorization_policies(_ap(access="denylist"))
    assert d["metadata"]["name"] == "tools-deny" and d["spec"]["action"] == "DENY"


def test_agent_policy_reconcile_with_and_without_mesh():
    store = APIStore()
    _agent(store, "a1")
    _agent(store, "a2")
    store.served.add((ISTIO_API, ISTIO_KIND))
    store.create(_ap(agents=["a1"]))
    AgentPolicyReconciler().reconcile(store, "default", "tools")
    p = store.get("AgentPolicy", "tools")
    assert p["status"]["phase"] == "Active" and p["status"]["matchedAgents"] == 1
    assert get_condition(p, "Applied")["message"] == "Policy applied to 1 agent(s)"
    names = {o["metadata"]["name"] for o in store.list(ISTIO_KIND, "default")}
    assert names == {"tools-allow", "tools-deny-all"}
    # switching to a denylist deletes the stale allowlist objects
    cur = store.get("AgentPolicy", "tools")
    cur["spec"]["toolAccess"]["mode"] = "denylist"
    store.update(cur)
    AgentPolicyReconciler().reconcile(store, "default", "tools")
    assert {o["metadata"]["name"] for o in store.list(ISTIO_KIND, "default")} == {"tools-deny"}

    bare = APIStore()  # no Istio: onFailure decides
    bare.create(_ap(name="strict"))
    bare.create(_ap(name="lenient", on_failure="allow", mode="permissive"))
    AgentPolicyReconciler().reconcile(bare, "default", "strict")
    AgentPolicyReconciler().reconcile(bare, "default", "lenient")
    assert bare.get("AgentPolicy", "strict")["status"]["phase"] == "Error"
    assert "cannot enforce" in get_condition(bare.get("AgentPolicy", "strict"),
                                             "Applied")["message"]
    lenient = bare.get("AgentPolicy", "lenient")
    assert lenient["status"]["phase"] == "Active"
    assert "permissive mode" in get_condition(lenient, "Applied")["message"]
    assert "mesh enforcement inactive" in get_condition(lenient, "Applied")["message"]


def _executor(access, registry="reg"):
    async def weather(args, ctx):
        return {"temp": 21}

    async def search(args, ctx):
        return {"hits": []}

    async def admin(args, ctx):
        return {"ok": True}

    ex = OmniaExecutor({"registry": registry, "toolAccess": access,
                        "handlers": [{"name": "h", "type": "inprocess"}]})
    ex.handlers.clear()
    h = InProcessHandler("h", {"get_weather": ("w", {"type": "object"}, weather),
                               "search": ("s", {"type": "object"}, search),
                               "admin_reset": ("a", {"type": "object"}, admin)})
    ex.add_handler(h)
    ex.registry_handlers = {"h"}
    asyncio.run(ex.discover())
    return ex


def test_in_node_tool_access_enforce_and_audit():
    store = APIStore()
    for name, kw in (("allow", {}), ("deny", {"access": "denylist",
                                              "rules": [{"registry": "reg",
                                                         "tools": ["search"]}]}),
                     ("audit", {"mode": "permissive", "access": "denylist",
                                "rules": [{"registry": "reg", "tools": ["get_weather"]}]}),
                     ("other", {"agents": ["someone-else"]})):
        store.create(_ap(name=name, **kw))
        store.served.add((ISTIO_API, ISTIO_KIND))
        AgentPolicyReconciler().reconcile(store, "default", name)
    access = compile_tool_access(store.list("AgentPolicy", "default"), "me")
    assert [a["policy"] for a in access] == ["allow", "audit", "deny"]
    ex = _executor(access)
    out, err = asyncio.run(ex.execute("get_weather", {}))
    assert not err and json.loads(out) == {"temp": 21}
    assert ex.access.audit == [{"tool": "reg/get_weather", "policy": "audit",
                                "decision": "would-deny"}]
    out, err = asyncio.run(ex.execute("search", {}))  # allowlisted but denylisted
    assert err and "denied by AgentPolicy deny" in json.loads(out)["message"]
    out, err = asyncio.run(ex.execute("admin_reset", {}))  # outside the allowlist
    assert err and "denied by AgentPolicy allow" in json.loads(out)["message"]
    # tools of other handlers (skills, memory) are not registry tools
    assert ToolAccess(access, "reg").check("x")[0] is False
    assert ToolAccess(access, "").check("x") == (True, "")


def test_manager_puts_policy_into_the_agents_tool_config():
    import os

    from omnia_amd.operator.manager import Manager, new_store
    from omnia_amd.cli import load_manifests

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    docs = load_manifests([os.path.join(root, "examples", "echo-function", "manifests.yaml")])
    for d in docs:
        if d["kind"] == "AgentRuntime":
            d["spec"]["toolRegistryRef"] = {"name": "reg"}
    docs.append({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "ToolRegistry",
                 "metadata": {"name": "reg", "namespace": "default"},
                 "spec": {"handlers": [{"name": "w", "type": "http",
                                        "httpConfig": {"endpoint": "http://127.0.0.1:1/w"},
                                        "tool": {"name": "get_weather", "description": "d",
                                                 "inputSchema": {"type": "object"}}}]}})
    store = new_store()

    async def go():
        mgr = Manager(store)
        await mgr.start()
        try:
            for d in docs:
                d["metadata"].setdefault("namespace", "default")
                store.apply(d)
            await mgr.settle(8)
            store.create(_ap(name="deny-w", access="denylist", on_failure="allow",
                             rules=[{"registry": "reg", "tools": ["get_weather"]}]))
            doc = {}
            for _ in range(50):
                await mgr.settle(2)
                cm = store.try_get("ConfigMap", "echo-tools", "default")
                doc = yaml.safe_load(cm["data"]["tools.yaml"]) if cm else {}
                if doc.get("toolAccess"):
                    break
            return doc
        finally:
            await mgr.stop()

    doc = asyncio.run(go())
    assert doc["registry"] == "reg"
    assert doc["toolAccess"] == [{"policy": "deny-w", "mode": "denylist", "enforce": True,
                                  "rules": [{"registry": "reg", "tools": ["get_weather"]}]}]


# ------------------------------------------------------------------ MemoryPolicy
def test_durations_cron_and_memory_policy_validation():
    assert parse_duration("30d") == 30 * 86400
    assert parse_duration("1d12h") == 1.5 * 86400
    assert parse_duration("90m") == 5400 and parse_duration("1.5h") == 5400
    for bad in ("", "30", "d", "1x", "5m3"):
        with pytest.raises(PolicyInvalid):
            parse_duration(bad)
    for ok in ("0 3 * * *", "*/15 * * * *", "@daily", "@every 10m", "0 0 1,15 * * 0"):
        validate_cron(ok)
    for bad in ("daily", "* * *", "0 3 * * * * *"):
        with pytest.raises(PolicyInvalid):
            validate_cron(bad)
    validate_memory_policy({"tiers": {"user": {"mode": "TTL",
                                               "ttl": {"default": "30d", "maxAge": "90d"}}}})
    for spec, msg in [
        ({"tiers": {"user": {"ttl": {"default": "90d", "maxAge": "30d"}}}}, "must not exceed"),
        ({"tiers": {"agent": {"decay": {"minScore": "1.5"}}}}, "between 0 and 1"),
        ({"tiers": {"agent": {"decay": {"scoreFormula": {"recencyWeight": "x"}}}}},
         "not a valid decimal"),
        ({"tiers": {"user": {"lru": {"staleAfter": "soon"}}}}, "invalid duration"),
        ({"tiers": {"user": {"perCategory": {"health": {"ttl": {"maxAge": "7x"}}}}}},
         "perCategory"),
        ({"tiers": {}, "schedule": "every day"}, "cron"),
        ({"tiers": {}, "tierPrecedence": {"multiplicative": {"user": "11"}}}, "between 0 and 10"),
    ]:
        with pytest.raises(PolicyInvalid, match=msg):
            validate_memory_policy(spec)


def test_memory_policy_reconciler_publishes_configmap():
    store = APIStore()
    store.create({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "MemoryPolicy",
                  "metadata": {"name": "mp"},
                  "spec": {"tiers": {"user": {"mode": "TTL", "ttl": {"maxAge": "30d"}}}}})
    MemoryPolicyReconciler("ops").reconcile(store, None, "mp")
    p = store.get("MemoryPolicy", "mp", None)
    assert p["status"]["phase"] == "Active"
    cm = store.get("ConfigMap", "memory-policy-mp", "ops")
    assert json.loads(cm["data"]["policy.json"])["tiers"]["user"]["ttl"]["maxAge"] == "30d"


def _mem(store, content, user="", agent="", age_days=0.0, conf=0.7, category=None,
         accessed_days=None):
    scope = {"workspace_id": "ws"}
    if user:
        scope["virtual_user_id"] = user
    if agent:
        scope["agent_id"] = agent
    meta = {META_CONSENT_CATEGORY: category} if category else {}
    r = store.save(Memory(content=content, scope=scope, confidence=conf, metadata=meta),
                   require_user=False)
    t = time.time() - age_days * 86400
    acc = time.time() - accessed_days * 86400 if accessed_days is not None else None
    with store._tx() as db:
        db.execute("UPDATE memory_entities SET created_at = ? WHERE id = ?", (t, r["id"]))
        db.execute("UPDATE memory_observations SET observed_at = ?, accessed_at = ? "
                   "WHERE entity_id = ?", (t, acc, r["id"]))
    return r["id"]


def _live(store):
    return {r[0] for r in store._q("SELECT id FROM memory_entities WHERE forgotten = 0")}


def test_memory_retention_pass_per_tier_and_category():
    st = MemoryStore(":memory:")
    old_user = _mem(st, "old user fact", user="u1", age_days=100)
    new_user = _mem(st, "new user fact", user="u1", age_days=1)
    health = _mem(st, "health fact", user="u1", age_days=10, category="health")
    stale_agent = _mem(st, "stale agent note", agent="a1", age_days=40, accessed_days=40)
    fresh_agent = _mem(st, "fresh agent note", agent="a1", age_days=40, accessed_days=1)
    weak_inst = _mem(st, "weak org fact", age_days=365, conf=0.05)
    strong_inst = _mem(st, "strong org fact", age_days=1, conf=0.95)
    spec = {"tiers": {
        "user": {"mode": "TTL", "ttl": {"maxAge": "90d", "default": "60d"},
                 "softDeleteGraceDays": 3,
                 "perCategory": {"health": {"mode": "TTL", "ttl": {"maxAge": "7d"}}}},
        "agent": {"mode": "LRU", "lru": {"staleAfter": "30d"}},
        "institutional": {"mode": "Decay", "decay": {"minScore": "0.2", "halfLifeDays": 30}}}}
    stats = apply_memory_policy(st, spec)
    assert stats == {"ttl_expired": 2, "ttl_defaulted": 1, "lru_forgotten": 1,
                     "decay_forgotten": 1}
    assert _live(st) == {new_user, fresh_agent, strong_inst}
    exp = st._q("SELECT expires_at, created_at FROM memory_entities WHERE id = ?",
                (new_user,))[0]
    assert abs(exp[0] - exp[1] - 60 * 86400) < 1
    assert grace_seconds(spec) == 3 * 86400
    gone = {old_user, health, stale_agent, weak_inst}
    assert gone.isdisjoint(_live(st))
    # Manual tiers and unconfigured tiers are untouched
    st2 = MemoryStore(":memory:")
    keep = _mem(st2, "x", user="u", age_days=1000)
    assert apply_memory_policy(st2, {"tiers": {"user": {"mode": "Manual"}}})["ttl_expired"] == 0
    assert _live(st2) == {keep}


def test_decay_score_shape():
    fresh = decay_score(0.9, 10, 0, {})
    old = decay_score(0.9, 10, 90 * 86400, {"halfLifeDays": 30})
    assert fresh == pytest.approx(1 / 3 * 0.9 + 1 / 3 + 1 / 3)
    assert old < fresh
    assert decay_score(0.0, 0, 0, {"scoreFormula": {"confidenceWeight": "1",
                                                    "accessFrequencyWeight": "0",
                                                    "recencyWeight": "0"}}) == 0.0


def test_retention_worker_applies_policy():
    from omnia_amd.memory.api import MemoryService
    from omnia_amd.memory.workers import RetentionWorker

    st = MemoryStore(":memory:")
    old = _mem(st, "old", user="u", age_days=100)
    svc = MemoryService(st, None)
    w = RetentionWorker(svc, policy={"tiers": {"user": {"mode": "TTL", "ttl": {"maxAge": "30d"},
                                                        "softDeleteGraceDays": 0}}})
    w.run_once()
    assert w.last_stats["ttl_expired"] == 1
    assert st._q("SELECT count(*) FROM memory_entities WHERE id = ?", (old,))[0][0] == 0


# ------------------------------------------------------------------ SessionRetentionPolicy
def test_session_retention_policy_configmap_lifecycle():
    store = APIStore()
    store.create({"apiVersion": "omnia.altairalabs.ai/v1alpha1",
                  "kind": "SessionRetentionPolicy", "metadata": {"name": "std"},
                  "spec": {"hotCache": {"ttlAfterInactive": "2h", "maxSessions": 500},
                           "warmStore": {"retentionDays": 14},
                           "coldArchive": {"enabled": True, "retentionDays": 400,
                                           "compactionSchedule": "0 2 * * *"}}})
    r = SessionRetentionPolicyReconciler("ops")
    r.reconcile(store, None, "std")
    p = store.get("SessionRetentionPolicy", "std", None)
    assert p["status"]["phase"] == "Active"
    assert "sessionretentionpolicy.omnia.altairalabs.ai/configmap-cleanup" in \
        p["metadata"]["finalizers"]
    doc = yaml.safe_load(store.get("ConfigMap", "retention-policy-std", "ops")["data"]
                         ["retention.yaml"])
    assert doc["warmStore"]["retentionDays"] == 14
    cfg = retention_from_config(doc)
    assert cfg == {"warm_retention_s": 14 * 86400, "cold_retention_s": 400 * 86400,
                   "hot_ttl_s": 7200, "hot_max_sessions": 500}
    store.delete("SessionRetentionPolicy", "std", None)
    r.reconcile(store, None, "std")
    assert store.try_get("ConfigMap", "retention-policy-std", "ops") is None
    assert store.try_get("SessionRetentionPolicy", "std", None) is None
    bad = {"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "SessionRetentionPolicy",
           "metadata": {"name": "bad"},
           "spec": {"coldArchive": {"compactionSchedule": "nightly"}}}
    store.create(bad)
    r.reconcile(store, None, "bad")
    assert store.get("SessionRetentionPolicy", "bad", None)["status"]["phase"] == "Error"


def test_compaction_reads_the_retention_config(tmp_path, monkeypatch):
    from omnia_amd.session import compaction

    cfgf = tmp_path / "retention.yaml"
    cfgf.write_text(yaml.safe_dump({"warmStore": {"retentionDays": 3},
                                    "coldArchive": {"retentionDays": 9}}))
    seen = {}

    class Eng:
        def __init__(self, warm, cold, hot, cfg):
            seen["cfg"] = cfg

        def run(self):
            return {}

    monkeypatch.setattr(compaction, "CompactionEngine", Eng)
    compaction.main(["--db", str(tmp_path / "w.db"), "--retention-config", str(cfgf)])
    assert seen["cfg"].warm_retention_s == 3 * 86400
    assert seen["cfg"].cold_retention_s == 9 * 86400


def test_workspace_services_mount_their_policies():
    from omnia_amd.api import crds
    from omnia_amd.operator.controllers import WorkspaceReconciler

    db = {"session": {"database": {"secretRef": {"name": "db"}}},
          "memory": {"database": {"secretRef": {"name": "db"}}}}
    store = APIStore()
    store.create({"apiVersion": crds.API_VERSION, "kind": "MemoryPolicy",
                  "metadata": {"name": "mp"},
                  "spec": {"tiers": {"user": {"mode": "TTL", "ttl": {"maxAge": "30d"}}}}})
    store.create({"apiVersion": crds.API_VERSION, "kind": "SessionRetentionPolicy",
                  "metadata": {"name": "std"}, "spec": {"warmStore": {"retentionDays": 5}}})
    svc = {"name": "default",
           "session": {**db["session"], "policyRef": {"name": "std"}},
           "memory": {**db["memory"], "policyRef": {"name": "mp"}}}
    store.create({"apiVersion": crds.API_VERSION, "kind": "Workspace",
                  "metadata": {"name": "t"},
                  "spec": {"displayName": "T", "namespace": {"name": "t"}, "services": [svc]}})
    WorkspaceReconciler().reconcile(store, None, "t")
    mem = store.get("Deployment", "memory-api-t-default", "t")["spec"]["template"]["spec"]
    assert "--policy-file" in mem["containers"][0]["args"]
    assert mem["volumes"][0]["configMap"]["name"] == "memory-api-t-default-policy"
    pol = json.loads(store.get("ConfigMap", "memory-api-t-default-policy", "t")["data"]
                     ["policy.json"])
    assert pol["tiers"]["user"]["ttl"]["maxAge"] == "30d"
    ses = store.get("Deployment", "session-api-t-default", "t")["spec"]["template"]["spec"]
    assert "--retention-config" in ses["containers"][0]["args"]
    doc = yaml.safe_load(store.get("ConfigMap", "session-api-t-default-policy", "t")["data"]
                         ["retention.yaml"])
    assert retention_from_config(doc) == {"warm_retention_s": 5 * 86400}
