"""Omnia CRD surface (group ``omnia.altairalabs.ai``, version ``v1alpha1``).

17 kinds -- the 9 core kinds (AgentRuntime, Provider, PromptPack, ToolRegistry,
Workspace, AgentPolicy, MemoryPolicy, SessionRetentionPolicy, SkillSource) and
the 8 enterprise kinds (ArenaJob, ArenaSource, ArenaTemplateSource,
ArenaDevSession, PromptPackSource, RolloutAnalysis, SessionPrivacyPolicy,
ToolPolicy) -- with the reference's names, short names, scope, required
fields, enums, defaults and printer columns (``api/v1alpha1/*_types.go``,
``ee/api/v1alpha1``).  Kubebuilder CEL rules are implemented as Python
validators next to each schema (``agentruntime_types.go:25-62``,
``provider_types.go:289-321``).

The one additive extension (SURVEY §7.1 design choice 3): Provider
``spec.type: local`` + ``spec.engine`` -- the in-node MI355X engine.
"""
from __future__ import annotations

import copy
import re
from dataclasses import dataclass, field

GROUP = "omnia.altairalabs.ai"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"

S = {"type": "string"}
B = {"type": "boolean"}
I = {"type": "integer"}
N = {"type": "number"}
OBJ = {"type": "object"}
ANY_OBJ = {"type": "object", "additionalProperties": True}
SECRET_KEY_REF = {"type": "object", "properties": {"name": S, "key": S}, "required": ["name"]}
GIT = {"type": "object", "properties": {"url": S, "path": S, "ref": ANY_OBJ,
                                        "secretRef": ANY_OBJ}, "required": ["url"]}
OCI = {"type": "object", "properties": {"url": S, "insecure": B, "secretRef": ANY_OBJ},
       "required": ["url"]}
CM_KEY = {"type": "object", "properties": {"name": S, "key": S}, "required": ["name"]}
POD_OVERRIDES = {"type": "object", "properties": {
    "annotations": ANY_OBJ, "labels": ANY_OBJ, "nodeSelector": ANY_OBJ,
    "tolerations": {"type": "array"}, "extraEnv": {"type": "array"},
    "extraEnvFrom": {"type": "array"}, "extraVolumes": {"type": "array"},
    "extraVolumeMounts": {"type": "array"}, "imagePullSecrets": {"type": "array"},
    "priorityClassName": S, "serviceAccountName": S, "resources": ANY_OBJ}}


def enum(*vals, default=None):
    d = {"type": "string", "enum": list(vals)}
    if default is not None:
        d["default"] = default
    return d


def dflt(schema, value):
    d = dict(schema)
    d["default"] = value
    return d


@dataclass
class Kind:
    kind: str
    plural: str
    short: list
    scope: str  # Namespaced | Cluster
    spec: dict
    printer: list = field(default_factory=list)  # (name, jsonPath)
    validators: list = field(default_factory=list)
    ee: bool = False
    status: dict = field(default_factory=lambda: ANY_OBJ)

    @property
    def singular(self) -> str:
        return self.kind.lower()


# ------------------------------------------------------------------ AgentRuntime
FACADE = {"type": "object", "required": ["type"], "properties": {
    "type": enum("websocket", "a2a", "rest", "mcp", "custom"),
    "port": I, "handler": enum("runtime", "echo", "demo"), "image": S,
    "a2a": {"type": "object", "properties": {
        "taskStore": ANY_OBJ, "clients": {"type": "array", "items": {
            "type": "object", "properties": {"name": S, "url": S, "agentRef": ANY_OBJ,
                                             "exposeAsTools": B}}},
        "card": ANY_OBJ}},
    "mcp": ANY_OBJ, "rest": ANY_OBJ, "route": ANY_OBJ}}

AUTOSCALING = {"type": "object", "properties": {
    "enabled": dflt(B, False), "type": enum("hpa", "keda", default="hpa"),
    "minReplicas": dflt(I, 1), "maxReplicas": dflt(I, 10),
    "targetMemoryUtilizationPercentage": dflt(I, 70),
    "targetCPUUtilizationPercentage": dflt(I, 90),
    "scaleDownStabilizationSeconds": dflt(I, 300),
    "keda": {"type": "object", "properties": {
        "pollingInterval": dflt(I, 30), "cooldownPeriod": dflt(I, 300),
        "triggers": {"type": "array"}, "threshold": S}}}}

AGENTRUNTIME = {"type": "object", "required": ["facades", "promptPackRef"], "properties": {
    "mode": enum("agent", "function", default="agent"),
    "facades": {"type": "array", "minItems": 1, "items": FACADE},
    "promptPackRef": {"type": "object", "required": ["name"], "properties": {
        "name": S, "version": S, "track": enum("stable", "prerelease")}},
    "providers": {"type": "array", "items": {"type": "object", "properties": {
        "name": S, "providerRef": {"type": "object", "properties": {"name": S,
                                                                    "namespace": S}},
        "role": S, "requiredCapabilities": {"type": "array", "items": S}}}},
    "toolRegistryRef": {"type": "object", "properties": {"name": S, "namespace": S},
                        "required": ["name"]},
    "context": {"type": "object", "properties": {
        "type": enum("memory", "redis", default="memory"), "ttl": dflt(S, "24h"),
        "storeRef": ANY_OBJ}},
    "runtime": {"type": "object", "properties": {
        "replicas": dflt(I, 1), "resources": ANY_OBJ, "nodeSelector": ANY_OBJ,
        "tolerations": {"type": "array"}, "affinity": ANY_OBJ, "extraEnv": {"type": "array"},
        "volumes": {"type": "array"}, "volumeMounts": {"type": "array"},
        "autoscaling": AUTOSCALING}},
    "framework": {"type": "object", "properties": {
        "type": enum("promptkit", "langchain", "custom", "omnia-mi355x"), "image": S,
        "version": S}},
    "inputSchema": ANY_OBJ, "outputSchema": ANY_OBJ,
    "outputFormat": enum("text", "json", "json_schema"),
    "serviceGroup": dflt(S, "default"),
    "memory": {"type": "object", "properties": {"enabled": B, "retrieval": ANY_OBJ,
                                                "tools": ANY_OBJ}},
    "evals": {"type": "object", "properties": {"enabled": B, "inline": ANY_OBJ,
                                               "sampling": ANY_OBJ, "rateLimit": ANY_OBJ,
                                               "worker": ANY_OBJ, "sessionCompletion": ANY_OBJ,
                                               "podOverrides": POD_OVERRIDES}},
    "externalAuth": {"type": "object", "properties": {"oidc": ANY_OBJ, "clientKeys": ANY_OBJ,
                                                      "edgeTrust": ANY_OBJ}},
    "media": {"type": "object", "properties": {"basePath": S, "storage": ANY_OBJ}},
    "duplex": {"type": "object", "properties": {"enabled": B, "mode": S, "audio": ANY_OBJ}},
    "rollout": {"type": "object", "properties": {
        "candidate": ANY_OBJ, "steps": {"type": "array", "items": {
            "type": "object", "properties": {"setWeight": I, "pause": ANY_OBJ,
                                             "analysis": ANY_OBJ}}},
        "stickySession": ANY_OBJ, "trafficRouting": ANY_OBJ, "rollback": ANY_OBJ,
        "trigger": ANY_OBJ}},
    "podOverrides": POD_OVERRIDES,
    "console": ANY_OBJ, "privacyPolicyRef": {"type": "object", "properties": {"name": S}},
    "extraPodAnnotations": ANY_OBJ,
}}


def _ar_cel(spec: dict) -> list[str]:
    """The AgentRuntime CEL rules (agentruntime_types.go kubebuilder markers)."""
    errs = []
    mode = spec.get("mode", "agent")
    if mode == "function":
        for f in ("inputSchema", "outputSchema"):
            if f not in spec:
                errs.append(f"spec.{f} is required when mode is function")
    else:
        for f in ("inputSchema", "outputSchema", "outputFormat"):
            if f in spec:
                errs.append(f"spec.{f} is only allowed when mode is function")
    facades = spec.get("facades") or []
    types = [f.get("type") for f in facades]
    if len(types) != len(set(types)):
        errs.append("spec.facades: each facade type may appear at most once")
    if mode == "agent" and any(t not in ("websocket", "a2a", "custom") for t in types):
        errs.append("spec.facades: agent mode supports websocket, a2a and custom facades")
    if mode == "function":
        if any(t not in ("rest", "mcp") for t in types):
            errs.append("spec.facades: function mode supports rest and mcp facades")
        if types.count("rest") != 1:
            errs.append("spec.facades: function mode requires exactly one rest facade")
    for f in facades:
        if f.get("type") == "custom" and not f.get("image"):
            errs.append("spec.facades: custom facade requires an image")
    ro = spec.get("rollout") or {}
    if ro.get("trigger") and not (spec.get("promptPackRef") or {}).get("version"):
        errs.append("spec.rollout.trigger requires promptPackRef.version")
    for s in ro.get("steps") or []:
        w = s.get("setWeight")
        if w is not None and not 0 <= w <= 100:
            errs.append("spec.rollout.steps[].setWeight must be within 0..100")
    return errs


# ------------------------------------------------------------------ Provider
PROVIDER_TYPES = ("claude", "openai", "gemini", "ollama", "mock", "vllm", "voyageai",
                  "cartesia", "elevenlabs", "imagen", "huggingface", "local")
PROVIDER = {"type": "object", "required": ["type"], "properties": {
    "type": enum(*PROVIDER_TYPES),
    "role": enum("llm", "embedding", "tts", "stt", "image", "inference", default="llm"),
    "model": S, "baseURL": S, "headers": ANY_OBJ,
    "platform": {"type": "object", "properties": {
        "type": enum("bedrock", "vertex", "azure"), "region": S, "project": S, "endpoint": S}},
    "auth": {"type": "object", "properties": {"type": S, "roleArn": S,
                                              "serviceAccountEmail": S,
                                              "credentialsSecretRef": ANY_OBJ}},
    "credential": {"type": "object", "properties": {"secretRef": SECRET_KEY_REF, "envVar": S,
                                                    "filePath": S}},
    "defaults": {"type": "object", "properties": {
        "temperature": N, "topP": N, "maxTokens": I, "contextWindow": I,
        "truncationStrategy": enum("sliding", "summarize", "custom"),
        "requestTimeout": S, "streamIdleTimeout": S}},
    "pricing": {"type": "object", "properties": {"inputCostPer1K": S, "outputCostPer1K": S,
                                                 "cachedCostPer1K": S}},
    "capabilities": {"type": "array", "items": enum(
        "text", "streaming", "vision", "tools", "json", "audio", "video", "documents",
        "duplex")},
    "embedding": {"type": "object", "properties": {"dimensions": {"type": "integer",
                                                                  "minimum": 1,
                                                                  "maximum": 4096},
                                                   "distance": S}},
    "tts": ANY_OBJ, "stt": ANY_OBJ,
    "engine": {"type": "object", "properties": {
        "model": S, "tp": dflt({"type": "integer", "minimum": 1, "maximum": 8}, 1),
        "dtype": enum("bfloat16", "float16", default="bfloat16"),
        "maxBatch": dflt(I, 256), "kvFraction": dflt(N, 0.85), "maxModelLen": dflt(I, 8192),
        "blockSize": dflt(I, 32), "swapGiB": dflt(N, 0), "tokenizer": S}},
}}

ROLE_TYPES = {
    "llm": {"claude", "openai", "gemini", "ollama", "mock", "vllm", "huggingface", "local"},
    "embedding": {"openai", "gemini", "ollama", "voyageai", "mock", "vllm", "local"},
    "tts": {"openai", "cartesia", "elevenlabs", "mock"},
    "stt": {"openai", "mock"},
    "image": {"openai", "gemini", "imagen", "mock"},
    "inference": {"huggingface", "vllm", "ollama", "mock", "local"},
}
NEEDS_CREDENTIAL = {"claude", "openai", "gemini", "voyageai", "cartesia", "elevenlabs"}


def _provider_cel(spec: dict) -> list[str]:
    errs = []
    t, role = spec.get("type"), spec.get("role", "llm")
    if t and role in ROLE_TYPES and t not in ROLE_TYPES[role]:
        errs.append(f"provider type {t} does not support role {role}")
    if t in ("ollama", "vllm") and not spec.get("baseURL"):
        errs.append(f"spec.baseURL is required for type {t}")
    if t == "local" and not (spec.get("engine") or {}).get("model") and not spec.get("model"):
        errs.append("spec.engine.model (or spec.model) is required for type local")
    if spec.get("platform") and t not in ("claude", "openai", "gemini"):
        errs.append("spec.platform is only valid for claude, openai and gemini")
    if role == "embedding" and spec.get("embedding") is None and t == "local":
        pass
    return errs


# ------------------------------------------------------------------ others
TOOL_HANDLER = {"type": "object", "required": ["name", "type"], "properties": {
    "name": S, "type": enum("http", "openapi", "grpc", "mcp", "client"),
    "endpoint": S, "timeout": S, "tool": {"type": "object", "required": ["name", "description"],
                                          "properties": {"name": S, "description": S,
                                                         "inputSchema": ANY_OBJ,
                                                         "outputSchema": ANY_OBJ}},
    "httpConfig": ANY_OBJ, "grpcConfig": ANY_OBJ, "mcpConfig": ANY_OBJ,
    "openAPIConfig": ANY_OBJ, "clientConfig": ANY_OBJ, "auth": ANY_OBJ,
    "retryPolicy": ANY_OBJ, "selector": ANY_OBJ}}


def _toolregistry_cel(spec):
    errs = []
    names = [h.get("name") for h in spec.get("handlers") or []]
    if len(names) != len(set(names)):
        errs.append("spec.handlers: handler names must be unique")
    for h in spec.get("handlers") or []:
        t = h.get("type")
        if t in ("http", "grpc") and not h.get("tool"):
            errs.append(f"handler {h.get('name')}: {t} handlers require a tool definition")
        if t == "http" and not ((h.get("httpConfig") or {}).get("endpoint") or h.get("endpoint")):
            errs.append(f"handler {h.get('name')}: http handlers require an endpoint")
        if t == "mcp" and not (h.get("mcpConfig") or h.get("endpoint")):
            errs.append(f"handler {h.get('name')}: mcp handlers require mcpConfig")
        if t == "client" and not h.get("tool"):
            errs.append(f"handler {h.get('name')}: client handlers require a tool definition")
    return errs


_SEMVER = re.compile(r"^v?\d+\.\d+\.\d+(-[0-9A-Za-z.-]+)?(\+[0-9A-Za-z.-]+)?$")


def _promptpack_cel(spec):
    errs = []
    if spec.get("version") and not _SEMVER.match(spec["version"]):
        errs.append("spec.version must be a semantic version")
    src = spec.get("source") or {}
    if src.get("type") == "configmap" and not src.get("configMapRef"):
        errs.append("spec.source.configMapRef is required for configmap sources")
    return errs


SOURCE_COMMON = {"interval": S, "suspend": dflt(B, False), "timeout": dflt(S, "60s"),
                 "git": GIT, "oci": OCI, "configMap": CM_KEY, "targetPath": S,
                 "createVersionOnSync": dflt(B, True)}


def _source_cel(spec):
    t = spec.get("type")
    if t in ("git", "oci", "configMap") and t not in spec:
        return [f"spec.{t} is required for type {t}"]
    if t == "configmap" and "configMap" not in spec:
        return ["spec.configMap is required for type configmap"]
    return []


KINDS: dict[str, Kind] = {}


def _reg(k: Kind):
    KINDS[k.kind] = k


_reg(Kind("AgentRuntime", "agentruntimes", ["agent", "ar"], "Namespaced", AGENTRUNTIME,
          [("Phase", ".status.phase"), ("Ready", ".status.replicas.ready"),
           ("Version", ".status.activeVersion"), ("Age", ".metadata.creationTimestamp")],
          [_ar_cel]))
_reg(Kind("Provider", "providers", ["prov"], "Namespaced", PROVIDER,
          [("Type", ".spec.type"), ("Model", ".spec.model"), ("Phase", ".status.phase"),
           ("Age", ".metadata.creationTimestamp")], [_provider_cel]))
_reg(Kind("PromptPack", "promptpacks", ["pp"], "Namespaced", {
    "type": "object", "required": ["packName", "source", "version"], "properties": {
        "packName": S, "version": S,
        "source": {"type": "object", "required": ["type"], "properties": {
            "type": enum("configmap"), "configMapRef": {"type": "object",
                                                        "properties": {"name": S, "key": S}}}},
        "skills": {"type": "array"}, "skillsConfig": ANY_OBJ,
        "rollout": ANY_OBJ}},
    [("Version", ".spec.version"), ("Phase", ".status.phase"),
     ("Age", ".metadata.creationTimestamp")], [_promptpack_cel]))
_reg(Kind("ToolRegistry", "toolregistries", ["tr"], "Namespaced", {
    "type": "object", "required": ["handlers"], "properties": {
        "handlers": {"type": "array", "items": TOOL_HANDLER},
        "probe": {"type": "object", "properties": {"enabled": B, "interval": S,
                                                   "timeout": S}}}},
    [("Tools", ".status.toolCount"), ("Phase", ".status.phase"),
     ("Age", ".metadata.creationTimestamp")], [_toolregistry_cel]))
_reg(Kind("Workspace", "workspaces", ["ws"], "Cluster", {
    "type": "object", "required": ["displayName", "namespace"], "properties": {
        "displayName": S, "description": S,
        "environment": enum("development", "staging", "production", default="development"),
        "namespace": {"type": "object", "required": ["name"], "properties": {
            "name": S, "create": dflt(B, True), "labels": ANY_OBJ, "annotations": ANY_OBJ}},
        "roleBindings": {"type": "array"}, "directGrants": {"type": "array"},
        "anonymousAccess": ANY_OBJ, "costControls": ANY_OBJ, "defaultTags": ANY_OBJ,
        "networkPolicy": ANY_OBJ, "storage": ANY_OBJ, "services": {"type": "array"},
        "runtime": ANY_OBJ, "privacy": ANY_OBJ, "mgmtPlaneMintServiceAccounts": {"type":
                                                                               "array"}}},
    [("Display Name", ".spec.displayName"), ("Environment", ".spec.environment"),
     ("Phase", ".status.phase"), ("Namespace", ".spec.namespace.name"),
     ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("AgentPolicy", "agentpolicies", ["ap"], "Namespaced", {
    "type": "object", "properties": {
        "selector": {"type": "object", "properties": {"agents": {"type": "array"}}},
        "toolAccess": {"type": "object", "properties": {
            "mode": enum("allowlist", "denylist"), "rules": {"type": "array"}}},
        "mode": enum("enforce", "permissive", default="enforce"),
        "onFailure": enum("deny", "allow", default="deny")}},
    [("Mode", ".spec.mode"), ("Phase", ".status.phase"), ("Matched", ".status.matchedCount"),
     ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("MemoryPolicy", "memorypolicies", ["mp"], "Cluster", {
    "type": "object", "required": ["tiers"], "properties": {
        "tiers": {"type": "object", "properties": {"institutional": ANY_OBJ, "agent": ANY_OBJ,
                                                   "user": ANY_OBJ}},
        "schedule": dflt(S, "0 3 * * *"), "batchSize": dflt(I, 1000),
        "consolidation": ANY_OBJ, "dedup": ANY_OBJ, "ingestion": ANY_OBJ, "recall": ANY_OBJ,
        "projection": ANY_OBJ, "supersession": ANY_OBJ, "tierPrecedence": ANY_OBJ,
        "consentRevocation": ANY_OBJ}},
    [("Phase", ".status.phase"), ("Schedule", ".spec.schedule"),
     ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("SessionRetentionPolicy", "sessionretentionpolicies", ["srp"], "Cluster", {
    "type": "object", "properties": {
        "hotCache": {"type": "object", "properties": {
            "enabled": dflt(B, True), "ttlAfterInactive": dflt(S, "24h"),
            "maxSessions": I, "maxMessagesPerSession": I}},
        "warmStore": {"type": "object", "properties": {
            "retentionDays": dflt({"type": "integer", "minimum": 1}, 7),
            "partitionBy": enum("day", "week", "month", default="day")}},
        "coldArchive": {"type": "object", "properties": {
            "enabled": dflt(B, False), "retentionDays": dflt(I, 365),
            "compactionSchedule": dflt(S, "0 2 * * *")}}}},
    [("Phase", ".status.phase"), ("Hot Cache TTL", ".spec.hotCache.ttlAfterInactive"),
     ("Warm Days", ".spec.warmStore.retentionDays"),
     ("Cold Archive", ".spec.coldArchive.enabled"), ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("SkillSource", "skillsources", ["skl"], "Namespaced", {
    "type": "object", "required": ["interval", "type"], "properties": {
        "type": enum("git", "oci", "configmap"), "filter": ANY_OBJ, **SOURCE_COMMON}},
    [("Type", ".spec.type"), ("Phase", ".status.phase"), ("Skills", ".status.skillCount"),
     ("Age", ".metadata.creationTimestamp")], [_source_cel]))
# ---- enterprise
_reg(Kind("ArenaJob", "arenajobs", ["aj"], "Namespaced", {
    "type": "object", "required": ["sourceRef"], "properties": {
        "sourceRef": {"type": "object", "required": ["name"], "properties": {"name": S}},
        "type": enum("evaluation", "loadtest", "datagen", default="evaluation"),
        "arenaFile": dflt(S, "config.arena.yaml"), "scenarios": ANY_OBJ, "providers": ANY_OBJ,
        "toolRegistries": {"type": "array"}, "trials": I, "verbose": B,
        "evaluation": ANY_OBJ, "dataGen": ANY_OBJ, "output": ANY_OBJ, "schedule": ANY_OBJ,
        "workers": ANY_OBJ, "sessionRecording": B, "cancelled": B,
        "ttlSecondsAfterFinished": I,
        "loadTest": {"type": "object", "properties": {
            "concurrency": I, "vusPerWorker": I, "ramp": ANY_OBJ, "budgetLimit": S,
            "budgetCurrency": S, "thresholds": {"type": "array", "items": {
                "type": "object", "properties": {"metric": enum(
                    "latency_avg", "latency_p50", "latency_p90", "latency_p95",
                    "latency_p99", "ttft_avg", "ttft_p50", "ttft_p90", "ttft_p95",
                    "ttft_p99", "error_rate", "pass_rate", "total_cost",
                    "tokens_per_second"), "max": S, "min": S}}}}}}},
    [("Source", ".spec.sourceRef.name"), ("Type", ".spec.type"), ("Phase", ".status.phase"),
     ("Progress", ".status.progress"), ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("ArenaSource", "arenasources", ["as"], "Namespaced", {
    "type": "object", "required": ["interval", "type"], "properties": {
        "type": enum("git", "oci", "configmap", "workspace"), "workspace": ANY_OBJ,
        **SOURCE_COMMON}},
    [("Type", ".spec.type"), ("Phase", ".status.phase"), ("Revision", ".status.revision"),
     ("Age", ".metadata.creationTimestamp")], [_source_cel], ee=True))
_reg(Kind("ArenaTemplateSource", "arenatemplatesources", ["ats"], "Namespaced", {
    "type": "object", "required": ["type"], "properties": {
        "type": enum("git", "oci", "configmap"), "syncInterval": dflt(S, "1h"),
        "templatesPath": dflt(S, "templates/"), "suspend": dflt(B, False),
        "timeout": dflt(S, "60s"), "git": GIT, "oci": OCI, "configMap": CM_KEY}},
    [("Type", ".spec.type"), ("Phase", ".status.phase"), ("Templates",
                                                          ".status.templateCount"),
     ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("ArenaDevSession", "arenadevsessions", ["ads"], "Namespaced", {
    "type": "object", "required": ["projectId", "workspace"], "properties": {
        "projectId": S, "workspace": S, "idleTimeout": dflt(S, "30m"), "image": S,
        "resources": ANY_OBJ, "podOverrides": POD_OVERRIDES}},
    [("Phase", ".status.phase"), ("Project", ".spec.projectId"),
     ("Endpoint", ".status.endpoint"), ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("PromptPackSource", "promptpacksources", ["pps"], "Namespaced", {
    "type": "object", "required": ["interval", "packName", "type"], "properties": {
        "type": enum("git", "oci"), "packName": S, "historyLimit": dflt(I, 10),
        "interval": S, "suspend": dflt(B, False), "timeout": dflt(S, "60s"), "git": GIT,
        "oci": OCI}},
    [("Pack", ".spec.packName"), ("Type", ".spec.type"), ("Phase", ".status.phase"),
     ("Version", ".status.latestVersion"), ("Age", ".metadata.creationTimestamp")],
    [_source_cel], ee=True))
_reg(Kind("RolloutAnalysis", "rolloutanalyses", ["ra"], "Namespaced", {
    "type": "object", "required": ["metrics"], "properties": {
        "args": {"type": "array"},
        "metrics": {"type": "array", "minItems": 1, "items": {
            "type": "object", "required": ["name"], "properties": {
                "name": S, "provider": ANY_OBJ, "successCondition": S, "failureCondition": S,
                "interval": S, "count": I, "failureLimit": I}}}}},
    [("Metrics", ".status.metricCount"), ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("SessionPrivacyPolicy", "sessionprivacypolicies", ["spp"], "Namespaced", {
    "type": "object", "required": ["recording"], "properties": {
        "recording": {"type": "object", "properties": {
            "enabled": dflt(B, True), "facadeData": dflt(B, True),
            "runtimeData": dflt(B, True), "pii": {"type": "object", "properties": {
                "redact": B, "patterns": {"type": "array"}, "strategy": S}}}},
        "retention": ANY_OBJ, "userOptOut": ANY_OBJ, "encryption": ANY_OBJ,
        "auditLog": ANY_OBJ}},
    [("Recording", ".spec.recording.enabled"), ("PII Redact", ".spec.recording.pii.redact"),
     ("Encryption", ".spec.encryption.enabled"), ("Phase", ".status.phase"),
     ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("ToolPolicy", "toolpolicies", ["tp"], "Namespaced", {
    "type": "object", "required": ["rules", "selector"], "properties": {
        "selector": {"type": "object", "required": ["registry"], "properties": {
            "registry": S, "tools": {"type": "array"}}},
        "rules": {"type": "array", "items": {"type": "object", "required": ["name"],
                                             "properties": {"name": S, "description": S,
                                                            "deny": ANY_OBJ}}},
        "requiredClaims": {"type": "array"}, "headerInjection": {"type": "array"},
        "mode": enum("enforce", "audit", default="enforce"),
        "onFailure": enum("deny", "allow", default="deny")}},
    [("Registry", ".spec.selector.registry"), ("Mode", ".spec.mode"),
     ("Phase", ".status.phase"), ("Rules", ".status.ruleCount"),
     ("Age", ".metadata.creationTimestamp")], ee=True))

SHORT = {s: k.kind for k in KINDS.values() for s in k.short}
PLURAL = {k.plural: k.kind for k in KINDS.values()}


def resolve_kind(name: str) -> str:
    n = name.lower()
    for k in KINDS.values():
        if n in (k.kind.lower(), k.plural, k.singular) or n in k.short:
            return k.kind
    raise KeyError(name)


def apply_defaults(schema: dict, obj):
    if not isinstance(obj, dict) or schema.get("type") != "object":
        return obj
    for k, sub in (schema.get("properties") or {}).items():
        if k not in obj and "default" in sub:
            obj[k] = copy.deepcopy(sub["default"])
        if k in obj:
            if sub.get("type") == "object":
                apply_defaults(sub, obj[k])
            elif sub.get("type") == "array" and isinstance(obj[k], list) and "items" in sub:
                for it in obj[k]:
                    apply_defaults(sub["items"], it)
    return obj


def validate_object(obj: dict) -> list[str]:
    """Admission-time validation: apiVersion/kind, metadata, schema + CEL rules."""
    from ..utils import jsonschema

    errs = []
    kind = obj.get("kind")
    k = KINDS.get(kind)
    if k is None:
        return [f"unknown kind {kind}"]
    if obj.get("apiVersion") != API_VERSION:
        errs.append(f"apiVersion must be {API_VERSION}")
    md = obj.get("metadata") or {}
    if not md.get("name"):
        errs.append("metadata.name is required")
    elif not re.match(r"^[a-z0-9]([-a-z0-9.]*[a-z0-9])?$", md["name"]) or len(md["name"]) > 253:
        errs.append("metadata.name must be a DNS subdomain")
    spec = obj.get("spec")
    if spec is None:
        if k.spec.get("required"):
            errs.append("spec is required")
        return errs
    apply_defaults(k.spec, spec)
    errs += [f"spec{('.' + str(e.path)) if e.path else ''}: {e.message}"
             for e in jsonschema.Validator(k.spec).errors(spec)]
    for v in k.validators:
        errs += v(spec)
    return errs


def crd_manifest(k: Kind) -> dict:
    """CustomResourceDefinition object (for ``omnia crds | kubectl apply -f -``)."""
    def strip(s):
        if isinstance(s, dict):
            out = {}
            for kk, vv in s.items():
                if kk == "additionalProperties" and vv is True:
                    out["x-kubernetes-preserve-unknown-fields"] = True
                    continue
                out[kk] = strip(vv)
            if out.get("type") == "object" and "properties" not in out:
                out["x-kubernetes-preserve-unknown-fields"] = True
            return out
        if isinstance(s, list):
            return [strip(x) for x in s]
        return s

    return {
        "apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{k.plural}.{GROUP}"},
        "spec": {"group": GROUP, "scope": k.scope,
                 "names": {"kind": k.kind, "plural": k.plural, "singular": k.singular,
                           "shortNames": k.short, "listKind": k.kind + "List"},
                 "versions": [{"name": VERSION, "served": True, "storage": True,
                               "subresources": {"status": {}},
                               "additionalPrinterColumns": [
                                   {"name": n, "jsonPath": p,
                                    "type": "date" if n == "Age" else "string"}
                                   for n, p in k.printer],
                               "schema": {"openAPIV3Schema": {"type": "object", "properties": {
                                   "apiVersion": S, "kind": S, "metadata": OBJ,
                                   "spec": strip(k.spec),
                                   "status": {"type": "object",
                                              "x-kubernetes-preserve-unknown-fields": True}}}}}]}}
