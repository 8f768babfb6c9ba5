"""CRD schema fidelity: the structural schemas of all 17 kinds (nested blocks,
enums, bounds, patterns, defaults, kubebuilder CEL rules) against the
reference's own manifests (accepted) and a negative suite of invalid nested
fields (rejected), plus field-validation modes, transition rules and the
generated CRD manifests (cf. the reference's ``*_cel_envtest_test.go`` /
``*_types_test.go`` suites)."""
import copy
import os

import pytest
import yaml

from omnia_amd.api import crds
from omnia_amd.api import schema as S
from omnia_amd.operator.apistore import Invalid
from omnia_amd.operator.manager import new_store

REF = "/root/reference"
API = crds.API_VERSION


def obj(kind, spec, name="x", ns="default"):
    md = {"name": name}
    if crds.KINDS[kind].scope == "Namespaced":
        md["namespace"] = ns
    return {"apiVersion": API, "kind": kind, "metadata": md, "spec": copy.deepcopy(spec)}


def errs(kind, spec, **kw):
    return crds.validate_object(obj(kind, spec), **kw)


AR = {"facades": [{"type": "websocket"}], "promptPackRef": {"name": "p"}}
PROV = {"type": "claude", "model": "claude-sonnet-4"}
TR_TOOL = {"name": "get_weather", "description": "d", "inputSchema": {"type": "object"}}
TR = {"handlers": [{"name": "w", "type": "http", "tool": TR_TOOL,
                    "httpConfig": {"endpoint": "http://w:8080/x"}}]}
WS = {"displayName": "Team", "namespace": {"name": "team-ns"}}
DB = {"database": {"secretRef": {"name": "db"}}}


def _reference_docs():
    out = []
    for dp, _, fn in os.walk(REF):
        if "node_modules" in dp or "/.git" in dp:
            continue
        for f in fn:
            if not f.endswith((".yaml", ".yml")):
                continue
            path = os.path.join(dp, f)
            try:
                txt = open(path).read()
                docs = list(yaml.safe_load_all(txt))
            except Exception:  # noqa: BLE001 - helm templates etc. are not YAML
                continue
            for d in docs:
                if isinstance(d, dict) and d.get("kind") in crds.KINDS and \
                        str(d.get("apiVersion", "")).startswith(crds.GROUP):
                    out.append((os.path.relpath(path, REF), d))
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_reference_manifests_are_admitted():
    """Every Omnia-kind manifest shipped in the reference (config/samples,
    examples, charts, docs, test fixtures) is admitted under the apiserver's
    default field validation (Warn: unknown fields pruned with a warning).  The
    one rejection is a sample whose ``spec.type: anthropic`` is outside the
    reference's own Provider enum (``provider_types.go`` ProviderType), i.e.
    the reference apiserver rejects it too."""
    docs = _reference_docs()
    assert len(docs) >= 40 and {d["kind"] for _, d in docs} >= {
        "AgentRuntime", "Provider", "PromptPack", "ToolRegistry", "Workspace", "MemoryPolicy",
        "SkillSource", "ArenaJob", "ArenaSource"}
    rejected, warned = [], []
    for path, d in docs:
        w = []
        e = crds.validate_object(copy.deepcopy(d), field_validation="Warn", warnings=w)
        if e:
            rejected.append((path, d["metadata"]["name"], e))
        if w:
            warned.append((path, w))
    assert [(p, n) for p, n, _ in rejected] == [
        ("examples/echo-function/provider.yaml", "echo-provider")], rejected
    assert "Unsupported value: 'anthropic'" in rejected[0][2][0]
    # kubectl's Strict mode additionally rejects the stale fields the Warn mode pruned
    strict = [p for p, d in docs if crds.validate_object(copy.deepcopy(d))]
    assert len(strict) == 1 + len(warned)
    assert all("unknown field" in x for _, w in warned for x in w)


def test_nested_defaults_applied():
    o = obj("AgentRuntime", {**AR, "runtime": {"autoscaling": {"enabled": True}},
                             "evals": {"enabled": True, "sampling": {}}})
    assert crds.validate_object(o) == []
    sp = o["spec"]
    assert sp["facades"][0]["handler"] == "runtime" and sp["facades"][0]["port"] == 8080
    a = sp["runtime"]["autoscaling"]
    assert (a["type"], a["minReplicas"], a["maxReplicas"], a["targetCPUUtilizationPercentage"],
            a["scaleDownStabilizationSeconds"]) == ("hpa", 1, 100, 90, 300)
    assert sp["evals"]["sampling"] == {"defaultRate": 100, "extendedRate": 10}
    assert sp["serviceGroup"] == "default" and sp["mode"] == "agent"
    w = obj("Workspace", {**WS, "storage": {}})
    assert crds.validate_object(w) == []
    assert w["spec"]["storage"] == {"enabled": True, "size": "10Gi",
                                    "accessModes": ["ReadWriteMany"],
                                    "retentionPolicy": "Delete"}
    m = obj("MemoryPolicy", {"tiers": {"user": {"decay": {}}}})
    assert crds.validate_object(m) == []
    assert m["spec"]["tiers"]["user"]["decay"]["minScore"] == "0.2"
    assert m["spec"]["tiers"]["user"]["decay"]["halfLifeDays"] == 90


NEGATIVE = [
    # (kind, spec, expected substring)
    ("AgentRuntime", {**AR, "facades": [{"type": "websocket", "port": 70000}]},
     "spec.facades[0].port: should be less than or equal to 65535"),
    ("AgentRuntime", {**AR, "facades": [{"type": "grpc"}]}, "spec.facades[0].type: Unsupported"),
    ("AgentRuntime", {**AR, "facades": [{"type": "websocket"}] * 5}, "at most 4 items"),
    ("AgentRuntime", {**AR, "context": {"type": "redis"}},
     "storeRef is required when context.type is 'redis'"),
    ("AgentRuntime", {**AR, "runtime": {"autoscaling": {"targetCPUUtilizationPercentage": 101}}},
     "targetCPUUtilizationPercentage: should be less than or equal to 100"),
    ("AgentRuntime", {**AR, "media": {"storage": {"type": "s3"}}},
     "type s3 requires spec.media.storage.s3"),
    ("AgentRuntime", {**AR, "externalAuth": {"oidc": {"issuer": "https://idp"}}},
     "spec.externalAuth.oidc.audience: Required value"),
    ("AgentRuntime", {**AR, "rollout": {"steps": []}}, "should have at least 1 items"),
    ("AgentRuntime", {**AR, "rollout": {"steps": [{"setWeight": 120}]}},
     "setWeight: should be less than or equal to 100"),
    ("AgentRuntime", {**AR, "promptPackRef": {"name": "p", "version": "1.0.0", "track": "stable"}},
     "mutually exclusive"),
    ("AgentRuntime", {**AR, "rollout": {"steps": [{"setWeight": 10}],
                                        "trigger": {"promptPackChannel": "stable"}}},
     "requires a version-pinned spec.promptPackRef"),
    ("AgentRuntime", {**AR, "serviceGroup": "Bad_Group"}, "spec.serviceGroup: should match"),
    ("AgentRuntime", {**AR, "providers": [{"name": "llm"}]},
     "spec.providers[0].providerRef: Required value"),
    ("AgentRuntime", {**AR, "facades": [{"type": "websocket", "bogus": 1}]},
     "spec.facades[0].bogus: field not declared in schema"),
    ("AgentRuntime", {**AR, "memory": {"retrieval": {"limit": 51}}},
     "limit: should be less than or equal to 50"),
    ("AgentRuntime", {**AR, "duplex": {"enabled": True, "mode": "video"}}, "Unsupported value"),
    ("Provider", {**PROV, "platform": {"type": "vertex"},
                  "auth": {"type": "serviceAccount", "credentialsSecretRef": {"name": "s"}}},
     "project is required when platform.type is vertex"),
    ("Provider", {**PROV, "credential": {"envVar": "K", "filePath": "/k"}},
     "at most one credential method"),
    ("Provider", {**PROV, "credential": {"envVar": "1BAD"}}, "envVar: should match"),
    ("Provider", {"type": "openai", "model": "m", "role": "embedding",
                  "embedding": {"dimensions": 5000}}, "should be less than or equal to 4096"),
    ("Provider", {**PROV, "tts": {"voice": "v"}}, "spec.tts is only valid when spec.role is 'tts'"),
    ("Provider", {**PROV, "platform": {"type": "bedrock", "region": "us-east-1"}},
     "spec.platform and spec.auth must be set together"),
    ("Provider", {"type": "gemini", "model": "m", "platform": {"type": "bedrock"},
                  "auth": {"type": "accessKey", "credentialsSecretRef": {"name": "s"}}},
     "gemini on bedrock is not supported"),
    ("Provider", {"type": "cartesia", "model": "m"}, "cartesia is a tts-only vendor"),
    ("Provider", {"type": "local", "engine": {"model": "llama-3-8b", "tp": 16}},
     "spec.engine.tp: should be less than or equal to 8"),
    ("PromptPack", {"packName": "p", "version": "one", "source": {"type": "configmap"}},
     "spec.version: should match"),
    ("PromptPack", {"packName": "p", "version": "1.0.0", "source": {"type": "git"}},
     "spec.source.type: Unsupported"),
    ("ToolRegistry", {"handlers": []}, "should have at least 1 items"),
    ("ToolRegistry", {"handlers": [{**TR["handlers"][0], "name": "Bad"}]},
     "spec.handlers[0].name: should match"),
    ("ToolRegistry", {"handlers": [{**TR["handlers"][0], "tool": {**TR_TOOL, "name": "Get"}}]},
     "spec.handlers[0].tool.name: should match"),
    ("ToolRegistry", {"handlers": [{**TR["handlers"][0], "httpConfig": {
        "endpoint": "http://w", "retryPolicy": {"maxAttempts": 11}}}]},
     "maxAttempts: should be less than or equal to 10"),
    ("ToolRegistry", {"handlers": [{**TR["handlers"][0], "auth": {"type": "bearer"}}]},
     "auth.type bearer/basic requires secretRef"),
    ("ToolRegistry", {"handlers": [{"name": "m", "type": "mcp",
                                    "mcpConfig": {"transport": "websocket"}}]},
     "transport: Unsupported value"),
    ("ToolRegistry", {"handlers": TR["handlers"] * 2}, "Duplicate value: 'w'"),
    ("Workspace", {**WS, "namespace": {"name": "Team_NS"}}, "spec.namespace.name: should match"),
    ("Workspace", {**WS, "services": [{"name": "default"}]},
     "managed mode requires both memory and session configuration"),
    ("Workspace", {**WS, "services": [{"name": "default", "mode": "external"}]},
     "external mode requires external endpoints"),
    ("Workspace", {**WS, "services": [{"name": "g", "memory": DB, "session": DB,
                                       "redis": {"url": "redis://a", "host": "b"}}]},
     "must use exactly one of existingSecret, url, host, or serviceRef"),
    ("Workspace", {**WS, "roleBindings": [{"role": "admin"}]}, "role: Unsupported value"),
    ("Workspace", {**WS, "costControls": {"alertThresholds": [{"percent": 0}]}},
     "percent: should be greater than or equal to 1"),
    ("MemoryPolicy", {"tiers": {}, "ingestion": {"chunk": {"size": 40, "overlap": 40}}},
     "chunk.overlap must be less than chunk.size"),
    ("MemoryPolicy", {"tiers": {}, "dedup": {"embeddingSimilarity": {
        "autoSupersedeAbove": "0.8", "surfaceDuplicatesAbove": "0.9"}}},
     "surfaceDuplicatesAbove must be strictly less than autoSupersedeAbove"),
    ("MemoryPolicy", {"tiers": {"user": {"decay": {"minScore": "1.5"}}}}, "minScore: should match"),
    ("MemoryPolicy", {"tiers": {"user": {"mode": "Forever"}}}, "mode: Unsupported value"),
    ("MemoryPolicy", {"tiers": {}, "tierPrecedence": {}},
     "spec.tierPrecedence.multiplicative must be set"),
    ("SessionRetentionPolicy", {"coldArchive": {"enabled": True}},
     "retentionDays is required when cold archive is enabled"),
    ("SessionRetentionPolicy", {"warmStore": {"partitionBy": "day"}}, "Unsupported value"),
    ("SkillSource", {"type": "git", "interval": "5m"}, "git source requires spec.git"),
    ("SkillSource", {"type": "git", "interval": "soon", "git": {"url": "https://g"}},
     "spec.interval: should match"),
    ("ArenaJob", {"sourceRef": {"name": "s"}, "loadTest": {"thresholds": [
        {"metric": "latency_p99", "operator": "~", "value": "1s"}]}}, "operator: Unsupported"),
    ("ArenaJob", {"sourceRef": {"name": "s"}, "output": {"type": "gcs"}}, "Unsupported value"),
    ("ArenaJob", {"sourceRef": {"name": "s"}, "schedule": {"cron": "@daily"}},
     "should be at least 9 chars long"),
    ("ArenaSource", {"type": "git", "interval": "1m", "git": {"url": "https://g"},
                     "oci": {"url": "oci://o"}}, "exactly one of git, oci, configMap"),
    ("ArenaSource", {"type": "oci", "interval": "1m", "git": {"url": "https://g"}},
     "the source block must match the chosen type"),
    ("PromptPackSource", {"type": "git", "packName": "p", "interval": "1m",
                          "oci": {"url": "oci://x"}}, "exactly the source block matching type"),
    ("ToolPolicy", {"selector": {"registry": "r"}, "rules": []}, "should have at least 1 items"),
    ("ToolPolicy", {"selector": {"registry": "r"}, "rules": [{"name": "a", "deny": {"cel": "x"}}]},
     "spec.rules[0].deny.message: Required value"),
    ("SessionPrivacyPolicy", {"recording": {"enabled": True},
                              "encryption": {"enabled": True, "keyID": "k"}},
     "kmsProvider is required when encryption is enabled"),
    ("RolloutAnalysis", {"metrics": [{"name": "m", "interval": "1m", "successCondition": "x"}]},
     "spec.metrics[0].provider: Required value"),
    ("ArenaDevSession", {"projectId": "p"}, "spec.workspace: Required value"),
    ("ArenaTemplateSource", {"type": "git", "git": {"url": "https://g"},
                             "syncInterval": "daily"}, "spec.syncInterval: should match"),
    ("AgentPolicy", {"toolAccess": {"mode": "allowlist", "rules": [{"registry": "r", "tools": []}]}},
     "should have at least 1 items"),
]


@pytest.mark.parametrize("kind,spec,want", NEGATIVE,
                         ids=[f"{k}-{i}" for i, (k, _, _) in enumerate(NEGATIVE)])
def test_invalid_nested_fields_rejected(kind, spec, want):
    e = errs(kind, spec)
    assert any(want in x for x in e), e


def test_every_kind_has_a_negative_case():
    assert {k for k, _, _ in NEGATIVE} == set(crds.KINDS)


def test_positive_cases_per_kind():
    good = {
        "AgentRuntime": {**AR, "providers": [{"name": "llm", "providerRef": {"name": "p"}}]},
        "Provider": {**PROV, "credential": {"secretRef": {"name": "k", "key": "api-key"}},
                     "defaults": {"temperature": "0.7", "maxTokens": 512}},
        "PromptPack": {"packName": "p", "version": "v1.2.3-rc.1",
                       "source": {"type": "configmap", "configMapRef": {"name": "cm"}}},
        "ToolRegistry": TR,
        "Workspace": {**WS, "services": [{"name": "default", "memory": DB, "session": DB}]},
        "AgentPolicy": {"toolAccess": {"mode": "denylist", "rules": [
            {"registry": "r", "tools": ["rm_rf"]}]}},
        "MemoryPolicy": {"tiers": {"user": {"mode": "Decay"}},
                         "ingestion": {"chunk": {"size": 200, "overlap": 20}}},
        "SessionRetentionPolicy": {"coldArchive": {"enabled": True, "retentionDays": 365}},
        "SkillSource": {"type": "oci", "interval": "10m", "oci": {"url": "oci://r/skills:v1"}},
        "ArenaJob": {"sourceRef": {"name": "s"}, "type": "loadtest", "loadTest": {
            "thresholds": [{"metric": "ttft_p95", "operator": "<", "value": "500ms"}]}},
        "ArenaSource": {"type": "configmap", "interval": "1m", "configMap": {"name": "c"}},
        "ArenaTemplateSource": {"type": "git", "git": {"url": "https://g/t.git"}},
        "ArenaDevSession": {"projectId": "p", "workspace": "w"},
        "PromptPackSource": {"type": "oci", "packName": "p", "interval": "1h",
                             "oci": {"url": "oci://r/p"}},
        "RolloutAnalysis": {"metrics": [{"name": "m", "interval": "1m", "count": 3,
                                         "successCondition": "result < 0.05",
                                         "provider": {"prometheus": {"address": "http://p",
                                                                     "query": "q"}}}]},
        "SessionPrivacyPolicy": {"recording": {"enabled": True, "pii": {"redact": True}}},
        "ToolPolicy": {"selector": {"registry": "r"}, "rules": [
            {"name": "a", "deny": {"cel": "body.amount > 100", "message": "too much"}}]},
    }
    assert set(good) == set(crds.KINDS)
    for kind, spec in good.items():
        assert errs(kind, spec) == [], (kind, errs(kind, spec))


def test_field_validation_modes_and_store_plumbing():
    spec = {**AR, "runtime": {"replicas": 2, "bogus": True}}
    assert any("runtime.bogus" in e for e in errs("AgentRuntime", spec))
    w = []
    o = obj("AgentRuntime", spec)
    assert crds.validate_object(o, field_validation="Warn", warnings=w) == []
    assert "bogus" not in o["spec"]["runtime"] and w == ['unknown field "spec.runtime.bogus"']
    o = obj("AgentRuntime", spec)
    assert crds.validate_object(o, field_validation="Ignore", warnings=w) == []
    st = new_store()
    with pytest.raises(Invalid, match="runtime.bogus"):
        st.create(obj("AgentRuntime", spec))
    created = st.create(obj("AgentRuntime", spec), field_validation="Warn")
    assert "bogus" not in created["spec"]["runtime"]
    assert st.warnings == ['unknown field "spec.runtime.bogus"']


def test_promptpack_immutable_transition_rule():
    st = new_store()
    pp = st.create(obj("PromptPack", {"packName": "p", "version": "1.0.0",
                                      "source": {"type": "configmap",
                                                 "configMapRef": {"name": "a"}}}))
    pp["spec"]["source"]["configMapRef"]["name"] = "b"
    with pytest.raises(Invalid, match="immutable"):
        st.update(pp)


def test_cel_rule_errors_are_reported_not_raised():
    bad = S.Obj({"a": S.Str()}, rules=[("self.missing.deeper == 1", "needs deeper")])
    e = S.validate(bad, {"a": "x"})
    assert len(e) == 1 and "needs deeper" in e[0]


def test_generated_crds_carry_structural_schemas_and_rules():
    m = crds.crd_manifest(crds.KINDS["AgentRuntime"])
    spec = m["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"]
    rules = [r["message"] for r in spec["x-kubernetes-validations"]]
    assert "mode 'function' requires exactly one 'rest' facade" in rules
    facade = spec["properties"]["facades"]["items"]
    assert facade["properties"]["port"]["maximum"] == 65535
    assert facade["properties"]["a2a"]["properties"]["agentCard"]["required"] == ["name"]
    y = yaml.safe_dump(m)
    assert len(y.splitlines()) > 900  # deep schema, not a stub
    total = sum(len(yaml.safe_dump(crds.crd_manifest(k)).splitlines())
                for k in crds.KINDS.values())
    assert total > 5000
    for k in crds.KINDS.values():  # every node typed or explicitly preserved
        def walk(n, p="spec"):
            if isinstance(n, dict):
                if "properties" in n or "items" in n:
                    assert n.get("type") in ("object", "array"), p
                for key, v in (n.get("properties") or {}).items():
                    walk(v, f"{p}.{key}")
                if isinstance(n.get("items"), dict):
                    walk(n["items"], p + "[]")
        walk(k.spec)
