"""Structural schemas of the 17 Omnia CRD kinds (``spec`` of each).

Authored from the reference's Go API types (``api/v1alpha1/*_types.go``,
``ee/api/v1alpha1/*_types.go``): every nested block, enum, default, bound,
pattern and kubebuilder CEL rule (``+kubebuilder:validation:XValidation``) is
declared, so a manifest the reference's apiserver rejects is rejected here and
an unknown nested field is a strict-validation error instead of being silently
admitted.  Embedded Kubernetes core types (Volume, Affinity, EnvFromSource...)
stay opaque objects, as ``apiextensionsv1.JSON`` fields stay untyped.

MI355X additions (SURVEY §7.1 design choice 3), all additive:
* Provider ``type: local`` + ``spec.engine`` (the in-node engine) and
  ``spec.mock`` (inline mock scenarios);
* AgentRuntime ``framework.type: omnia-mi355x`` (the native runtime, evaluates
  inline like PromptKit);
* ToolRegistry handler-level ``endpoint`` shorthand (resolved like
  ``httpConfig.endpoint`` / ``grpcConfig.endpoint``);
* ``file://`` git source URLs (air-gapped mirrors on the node).
"""
from __future__ import annotations

from .schema import (DURATION, INT_OR_STR, JSON_ANY, OPEN_OBJ, TIME, Arr, Bool, Enum, Int,
                     Map, Obj, Str)

DNS_LABEL = r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$"
SEMVER = (r"^v?(\d+)\.(\d+)\.(\d+)(-[a-zA-Z0-9]+(\.[a-zA-Z0-9]+)*)?"
          r"(\+[a-zA-Z0-9]+(\.[a-zA-Z0-9]+)*)?$")
GO_DURATION = r"^([0-9]+(\.[0-9]+)?(ms|s|m|h))+$"
DAYS_DURATION = r"^([0-9]+d)?([0-9]+h)?([0-9]+m)?([0-9]+s)?$"
UNIT_FRACTION = r"^(0(\.[0-9]+)?|1(\.0+)?)$"
DECIMAL = r"^[0-9]+(\.[0-9]+)?$"

# ------------------------------------------------------------------ core / shared
LOCAL_REF = Obj({"name": Str()})                       # corev1.LocalObjectReference
NAME_REF = Obj({"name": Str(min_len=1)}, ["name"])     # omnia LocalObjectReference
NS_REF = Obj({"name": Str(min_len=1), "namespace": Str()}, ["name"])
SECRET_KEY_REF = Obj({"name": Str(min_len=1), "key": Str()}, ["name"])
SECRET_KEY_SELECTOR = Obj({"name": Str(), "key": Str()}, ["name", "key"])
ENV_VAR = Obj({"name": Str(), "value": Str(), "valueFrom": OPEN_OBJ}, ["name"])
TOLERATION = Obj({"key": Str(), "operator": Str(), "value": Str(), "effect": Str(),
                  "tolerationSeconds": Int(fmt="int64")})
RESOURCES = Obj({"limits": Map(INT_OR_STR), "requests": Map(INT_OR_STR),
                 "claims": Arr(OPEN_OBJ)})
POD_OVERRIDES = Obj({
    "serviceAccountName": Str(), "labels": Map(), "annotations": Map(),
    "nodeSelector": Map(), "tolerations": Arr(TOLERATION), "priorityClassName": Str(),
    "imagePullSecrets": Arr(LOCAL_REF), "extraEnv": Arr(ENV_VAR),
    "extraEnvFrom": Arr(OPEN_OBJ), "extraVolumes": Arr(OPEN_OBJ),
    "extraVolumeMounts": Arr(OPEN_OBJ)})
REDIS = Obj({
    "serviceRef": Obj({"name": Str(min_len=1), "namespace": Str(),
                       "port": Int(minimum=1, maximum=65535)}, ["name"]),
    "existingSecret": Obj({"name": Str(min_len=1), "key": Str(min_len=1)}, ["name", "key"]),
    "url": Str(pattern=r"^rediss?://"), "host": Str(),
    "port": Int(minimum=1, maximum=65535), "db": Int(minimum=0, maximum=15), "user": Str()})


def _one_redis(where: str) -> tuple:
    return ("!has(self.redis) || [has(self.redis.existingSecret), has(self.redis.url) && "
            "size(self.redis.url) > 0, has(self.redis.host) && size(self.redis.host) > 0, "
            "has(self.redis.serviceRef)].exists_one(b, b)",
            f"{where}.redis must use exactly one of existingSecret, url, host, or serviceRef")


GIT_SOURCE = Obj({"url": Str(pattern=r"^(https?|ssh|file)://.*$"),  # + file:// mirrors
                  "ref": Obj({"branch": Str(), "tag": Str(), "commit": Str()}),
                  "path": Str(), "secretRef": SECRET_KEY_REF}, ["url"])
OCI_SOURCE = Obj({"url": Str(pattern=r"^oci://.*$"), "secretRef": SECRET_KEY_REF,
                  "insecure": Bool(False)}, ["url"])
CONFIGMAP_SOURCE = Obj({"name": Str(min_len=1), "key": Str("pack.json")}, ["name"])
WORKSPACE_SOURCE = Obj({"path": Str(min_len=1)}, ["path"])
CONDITIONS = Arr(Obj({"type": Str(), "status": Str(), "reason": Str(), "message": Str(),
                      "lastTransitionTime": TIME, "observedGeneration": Int(fmt="int64")},
                     preserve=True))

# ------------------------------------------------------------------ AgentRuntime
PROVIDER_CAPABILITY = Enum("text", "streaming", "vision", "tools", "json", "audio", "video",
                           "documents", "duplex")
PROVIDER_ROLE = Enum("llm", "embedding", "tts", "stt", "image", "inference")
PROMPTPACK_REF = Obj({"name": Str(min_len=1), "version": Str(),
                      "track": Enum("stable", "prerelease")}, ["name"],
                     [("!(has(self.version) && has(self.track))",
                       "promptPackRef.version and promptPackRef.track are mutually exclusive")])
TOOLREGISTRY_REF = Obj({"name": Str(min_len=1), "namespace": Str()}, ["name"])
NAMED_PROVIDER_REF = Obj({
    "name": Str(min_len=1, pattern=r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$"),
    "providerRef": Obj({"name": Str(min_len=1), "namespace": Str()}, ["name"]),
    "role": Str("llm"), "requiredCapabilities": Arr(PROVIDER_CAPABILITY)},
    ["name", "providerRef"])
A2A_CLIENT = Obj({
    "name": Str(min_len=1),
    "agentRuntimeRef": Obj({"name": Str(min_len=1), "namespace": Str()}, ["name"]),
    "url": Str(), "exposeAsTools": Bool(), "timeout": Str(pattern=GO_DURATION),
    "authentication": Obj({"secretRef": LOCAL_REF})}, ["name"])
AGENT_CARD = Obj({
    "name": Str(min_len=1), "description": Str(), "version": Str(), "organization": Str(),
    "skills": Arr(Obj({"id": Str(min_len=1), "name": Str(min_len=1), "description": Str(),
                       "tags": Arr(Str()), "examples": Arr(Str())}, ["id", "name"])),
    "capabilities": Obj({"streaming": Bool(), "pushNotifications": Bool()}),
    "defaultInputModes": Arr(Str()), "defaultOutputModes": Arr(Str())}, ["name"])
A2A_CONFIG = Obj({
    "enabled": Bool(), "port": Int(9999), "agentCard": AGENT_CARD,
    "taskTTL": Str("1h"), "conversationTTL": Str("30m"),
    "taskStore": Obj({"type": Enum("memory", "redis", default="memory"), "redisURL": Str(),
                      "redisSecretRef": LOCAL_REF}),
    "clients": Arr(A2A_CLIENT)})
FACADE = Obj({
    "type": Enum("websocket", "a2a", "rest", "mcp", "custom", default="websocket"),
    "port": Int(8080, 1, 65535), "drainTimeout": Str(),
    "handler": Enum("echo", "demo", "runtime", default="runtime"), "image": Str(),
    "extraEnv": Arr(ENV_VAR), "clientToolTimeout": DURATION, "a2a": A2A_CONFIG,
    "mcp": Obj({"enabled": Bool(), "port": Int(minimum=1, maximum=65535)}),
    "managementPlane": Bool(),
    "expose": Obj({"enabled": Bool(), "host": Str()})}, ["type"])
CONTEXT = Obj({"type": Enum("memory", "redis", default="memory"), "storeRef": LOCAL_REF,
               "ttl": Str("24h")}, ["type"],
              [("self.type == 'memory' || has(self.storeRef)",
                "spec.context.storeRef is required when context.type is 'redis'")])
KEDA = Obj({"pollingInterval": Int(30, 1), "cooldownPeriod": Int(300, 0),
            "triggers": Arr(Obj({"type": Str(), "metadata": Map()}, ["type", "metadata"])),
            "connectionThreshold": Int(minimum=1)})
AUTOSCALING = Obj({
    "enabled": Bool(False), "type": Enum("hpa", "keda", default="hpa"),
    "minReplicas": Int(1, 0), "maxReplicas": Int(100, 1),
    "targetMemoryUtilizationPercentage": Int(70, 1, 100),
    "targetCPUUtilizationPercentage": Int(90, 1, 100),
    "scaleDownStabilizationSeconds": Int(300, 0, 3600), "keda": KEDA})
RUNTIME = Obj({
    "replicas": Int(1, 0), "autoscaling": AUTOSCALING, "resources": RESOURCES,
    "nodeSelector": Map(), "tolerations": Arr(TOLERATION), "affinity": OPEN_OBJ,
    "volumes": Arr(OPEN_OBJ), "volumeMounts": Arr(OPEN_OBJ), "extraEnv": Arr(ENV_VAR)})
FRAMEWORK = Obj({"type": Enum("promptkit", "langchain", "custom", "omnia-mi355x",
                              default="promptkit"),
                 "version": Str(), "image": Str()}, ["type"])
MEDIA_STORAGE = Obj({
    "type": Enum("none", "local", "s3", "gcs", "azure", default="none"),
    "local": Obj({"basePath": Str(min_len=1), "volumeClaim": Str()}, ["basePath"]),
    "s3": Obj({"bucket": Str(min_len=1), "region": Str(), "prefix": Str(), "endpoint": Str()},
              ["bucket"]),
    "gcs": Obj({"bucket": Str(min_len=1), "prefix": Str()}, ["bucket"]),
    "azure": Obj({"account": Str(min_len=1), "container": Str(min_len=1), "prefix": Str()},
                 ["account", "container"]),
    "defaultTTL": DURATION, "uploadURLTTL": DURATION, "downloadURLTTL": DURATION,
    "maxFileSizeBytes": Int(minimum=1, fmt="int64"), "secretRef": LOCAL_REF}, ["type"],
    [("self.type != 's3' || has(self.s3)", "type s3 requires spec.media.storage.s3"),
     ("self.type != 'gcs' || has(self.gcs)", "type gcs requires spec.media.storage.gcs"),
     ("self.type != 'azure' || has(self.azure)", "type azure requires spec.media.storage.azure"),
     ("self.type != 'local' || has(self.local)", "type local requires spec.media.storage.local")])
DIMENSIONS = Obj({"width": Int(minimum=1), "height": Int(minimum=1)}, ["width", "height"])
AUDIO_REQ = Obj({"maxDurationSeconds": Int(minimum=1), "recommendedSampleRate": Int(minimum=1),
                 "supportsSegmentSelection": Bool(), "channels": Int(), "format": Str(),
                 "chunkDurationMs": Int(minimum=1)})
MEDIA_REQUIREMENTS = Obj({
    "image": Obj({"maxSizeBytes": Int(minimum=1, fmt="int64"), "maxDimensions": DIMENSIONS,
                  "recommendedDimensions": DIMENSIONS, "supportedFormats": Arr(Str()),
                  "preferredFormat": Str(),
                  "compressionGuidance": Enum("none", "lossless", "lossy-high", "lossy-medium",
                                              "lossy-low")}),
    "video": Obj({"maxDurationSeconds": Int(minimum=1), "supportsSegmentSelection": Bool(),
                  "processingMode": Enum("frames", "transcription", "both", "native"),
                  "frameExtractionInterval": Int(minimum=1)}),
    "audio": AUDIO_REQ,
    "document": Obj({"maxPages": Int(minimum=1), "supportsOCR": Bool()})})
CONSOLE = Obj({"allowedAttachmentTypes": Arr(Str()), "allowedExtensions": Arr(Str()),
               "maxFileSize": Int(10485760, 1, fmt="int64"), "maxFiles": Int(5, 1, 20),
               "mediaRequirements": MEDIA_REQUIREMENTS})
EVAL_PATH = Obj({"groups": Arr(Str())})
EVALS = Obj({
    "enabled": Bool(), "inline": EVAL_PATH, "worker": EVAL_PATH,
    "sampling": Obj({"defaultRate": Int(100, 0, 100), "extendedRate": Int(10, 0, 100)}),
    "rateLimit": Obj({"maxEvalsPerSecond": Int(50, 1), "maxConcurrentJudgeCalls": Int(5, 1)}),
    "sessionCompletion": Obj({"inactivityTimeout": Str("5m")}),
    "podOverrides": POD_OVERRIDES})
MEMORY = Obj({
    "enabled": Bool(),
    "retrieval": Obj({"enabled": Bool(), "strategy": Enum("keyword", "semantic", "composite"),
                      "limit": Int(minimum=1, maximum=50),
                      "accessFilter": Obj({"denyCEL": Str()})}),
    "tools": Obj({"enabled": Bool()})})
EXTERNAL_AUTH = Obj({
    "clientKeys": Obj({"defaultRole": Str("viewer"), "trustEndUserHeader": Bool()}),
    "oidc": Obj({"issuer": Str(min_len=1), "audience": Str(min_len=1),
                 "claimMapping": Obj({"subject": Str(), "endUser": Str()})},
                ["issuer", "audience"]),
    "edgeTrust": Obj({"headerMapping": Obj({"subject": Str(), "endUser": Str(), "email": Str()}),
                      "claimsFromHeaders": Map()})})
ROLLOUT = Obj({
    "candidate": Obj({"promptPackRef": PROMPTPACK_REF, "providerRefs": Arr(NAMED_PROVIDER_REF),
                      "toolRegistryRef": TOOLREGISTRY_REF}),
    "steps": Arr(Obj({"setWeight": Int(minimum=0, maximum=100),
                      "pause": Obj({"duration": Str()}),
                      "analysis": Obj({"templateName": Str(min_len=1),
                                       "args": Arr(Obj({"name": Str(min_len=1), "value": Str()},
                                                       ["name", "value"]))},
                                      ["templateName"])}), min_items=1),
    "stickySession": Obj({"hashOn": Str(min_len=1)}, ["hashOn"]),
    "rollback": Obj({"mode": Enum("automatic", "manual", "disabled", default="manual"),
                     "cooldown": Str("5m")}),
    "trafficRouting": Obj({
        "mode": Enum("mesh", "replicaWeighted", "external"),
        "mesh": Obj({"hosts": Arr(Str()), "stableSubset": Str("stable"),
                     "candidateSubset": Str("canary"), "waypoint": Str()}),
        "istio": Obj({"virtualService": Obj({"name": Str(min_len=1),
                                             "routes": Arr(Str(), min_items=1)},
                                            ["name", "routes"]),
                      "destinationRule": Obj({"name": Str(min_len=1),
                                              "stableSubset": Str("stable"),
                                              "candidateSubset": Str("canary")}, ["name"])},
                     ["virtualService", "destinationRule"])}),
    "trigger": Obj({"promptPackChannel": Enum("stable", "prerelease")}, ["promptPackChannel"])},
    ["steps"])
AGENTRUNTIME = Obj({
    "mode": Enum("agent", "function", default="agent"),
    "inputSchema": JSON_ANY, "outputSchema": JSON_ANY,
    "outputFormat": Enum("text", "json", "json_schema"),
    "framework": FRAMEWORK, "promptPackRef": PROMPTPACK_REF,
    "facades": Arr(FACADE, min_items=1, max_items=4),
    "toolRegistryRef": TOOLREGISTRY_REF, "context": CONTEXT, "runtime": RUNTIME,
    "media": Obj({"basePath": Str("/etc/omnia/media"), "storage": MEDIA_STORAGE}),
    "providers": Arr(NAMED_PROVIDER_REF), "evals": EVALS, "console": CONSOLE,
    "duplex": Obj({"enabled": Bool(), "mode": Enum("audio", "audiovideo", default="audio"),
                   "audio": AUDIO_REQ}),
    "externalAuth": EXTERNAL_AUTH, "memory": MEMORY, "extraPodAnnotations": Map(),
    "serviceGroup": Str("default", pattern=r"^[a-z0-9]([a-z0-9-]*[a-z0-9])?$", max_len=63),
    "privacyPolicyRef": LOCAL_REF, "rollout": ROLLOUT, "podOverrides": POD_OVERRIDES},
    ["promptPackRef", "facades"], [
        ("self.mode != 'function' || has(self.inputSchema)",
         "spec.inputSchema is required when spec.mode is 'function'"),
        ("self.mode != 'function' || has(self.outputSchema)",
         "spec.outputSchema is required when spec.mode is 'function'"),
        ("self.mode == 'function' || !has(self.inputSchema)",
         "spec.inputSchema is only valid when spec.mode is 'function'"),
        ("self.mode == 'function' || !has(self.outputSchema)",
         "spec.outputSchema is only valid when spec.mode is 'function'"),
        ("self.mode == 'function' || !has(self.outputFormat)",
         "spec.outputFormat is only valid when spec.mode is 'function'"),
        ("!has(self.facades) || self.facades.all(f, self.facades.exists_one(g, g.type == "
         "f.type))", "spec.facades must not contain duplicate facade types"),
        ("!has(self.facades) || self.mode != 'agent' || self.facades.all(f, f.type == "
         "'websocket' || f.type == 'a2a' || f.type == 'custom')",
         "mode 'agent' allows only 'websocket', 'a2a' and 'custom' facades"),
        ("!has(self.facades) || self.mode != 'function' || self.facades.all(f, f.type == "
         "'rest' || f.type == 'mcp')", "mode 'function' allows only 'rest' and 'mcp' facades"),
        ("!has(self.facades) || self.mode != 'function' || self.facades.exists_one(f, f.type "
         "== 'rest')", "mode 'function' requires exactly one 'rest' facade"),
        ("!has(self.facades) || self.facades.all(f, f.type != 'custom' || (has(f.image) && "
         "size(f.image) > 0))", "facade type 'custom' requires spec.facades[].image"),
        ("!(has(self.rollout) && has(self.rollout.trigger)) || (has(self.promptPackRef) && "
         "has(self.promptPackRef.version) && !has(self.promptPackRef.track))",
         "spec.rollout.trigger requires a version-pinned spec.promptPackRef and is mutually "
         "exclusive with promptPackRef.track")])

# ------------------------------------------------------------------ Provider
PROVIDER_TYPES = ("claude", "openai", "gemini", "ollama", "mock", "vllm", "voyageai",
                  "cartesia", "elevenlabs", "imagen", "huggingface", "local")
ENGINE = Obj({
    "model": Str(), "tp": Int(1, 1, 8), "ep": Int(1, 1, 8),
    "dtype": Enum("bfloat16", "float16", "float32", default="bfloat16"),
    "maxBatch": Int(256, 1), "kvFraction": {"type": "number", "default": 0.85,
                                            "minimum": 0.05, "maximum": 0.98},
    "maxModelLen": Int(8192, 16), "blockSize": Int(32, 8, 256),
    "swapGiB": {"type": "number", "default": 0, "minimum": 0}, "tokenizer": Str(),
    "mixedBudget": Int(minimum=0), "contextParallel": Int(minimum=1, maximum=8),
    # single-node engine knobs (device "cpu" runs the reference ops: tests, dev boxes)
    "device": Enum("cuda", "cpu"), "epMode": Enum("tp", "a2a"),
    "numBlocks": Int(minimum=16), "useGraphs": {"type": "boolean"},
    "cpThreshold": Int(minimum=0),
    # HF safetensors directory on the node (random-init weights when absent)
    "checkpoint": Str()})
PROVIDER = Obj({
    "type": Enum(*PROVIDER_TYPES), "role": Enum("llm", "embedding", "tts", "stt", "image",
                                                "inference", default="llm"),
    "tts": Obj({"voice": Str(), "sampleRate": Int(minimum=8000, maximum=48000),
                "audioFiles": Arr(Str()),
                "format": Enum("pcm", "mp3", "opus", "wav", "flac")}),
    "stt": Obj({"sampleRate": Int(minimum=8000, maximum=48000),
                "language": Str(pattern=r"^[a-z]{2}(-[A-Z]{2})?$")}),
    "embedding": Obj({"dimensions": Int(minimum=1, maximum=4096),
                      "distance": Enum("cosine", "l2", "dot")}),
    "model": Str(), "baseURL": Str(), "headers": Map(),
    "platform": Obj({"type": Enum("bedrock", "vertex", "azure"), "region": Str(),
                     "project": Str(), "endpoint": Str()}, ["type"],
                    [("self.type != 'vertex' || size(self.project) > 0",
                      "project is required when platform.type is vertex"),
                     ("self.type != 'azure' || size(self.endpoint) > 0",
                      "endpoint is required when platform.type is azure")]),
    "auth": Obj({"type": Enum("workloadIdentity", "accessKey", "serviceAccount",
                              "servicePrincipal"),
                 "roleArn": Str(), "serviceAccountEmail": Str(),
                 "credentialsSecretRef": SECRET_KEY_REF}, ["type"],
                [("self.type != 'workloadIdentity' || !has(self.credentialsSecretRef)",
                  "credentialsSecretRef is not used with workloadIdentity auth")]),
    "credential": Obj({"secretRef": SECRET_KEY_REF,
                       "envVar": Str(pattern=r"^[A-Za-z_][A-Za-z0-9_]*$"),
                       "filePath": Str(pattern=r"^/.*")}, (),
                      [("(has(self.secretRef) ? 1 : 0) + (has(self.envVar) ? 1 : 0) + "
                        "(has(self.filePath) ? 1 : 0) <= 1",
                        "at most one credential method may be specified")]),
    "defaults": Obj({"temperature": Str(), "topP": Str(), "maxTokens": Int(),
                     "contextWindow": Int(),
                     "truncationStrategy": Enum("sliding", "summarize", "custom",
                                                default="sliding"),
                     "requestTimeout": Str(), "streamIdleTimeout": Str()}),
    "pricing": Obj({"inputCostPer1K": Str(), "outputCostPer1K": Str(),
                    "cachedCostPer1K": Str()}),
    "capabilities": Arr(PROVIDER_CAPABILITY),
    # MI355X additions
    "engine": ENGINE, "mock": Obj({"path": Str(), "scenarios": JSON_ANY})},
    ["type"], [
        ("(has(self.tts) ? 1 : 0) + (has(self.stt) ? 1 : 0) + (has(self.embedding) ? 1 : 0) "
         "<= 1", "at most one of spec.tts, spec.stt, spec.embedding may be set"),
        ("!has(self.tts) || self.role == 'tts'", "spec.tts is only valid when spec.role is 'tts'"),
        ("!has(self.stt) || self.role == 'stt'", "spec.stt is only valid when spec.role is 'stt'"),
        ("!has(self.embedding) || self.role == 'embedding'",
         "spec.embedding is only valid when spec.role is 'embedding'"),
        ("self.role != 'llm' || self.type in ['claude', 'openai', 'gemini', 'ollama', 'mock', "
         "'vllm', 'local']",
         "role 'llm' requires type in [claude, openai, gemini, ollama, mock, vllm, local]"),
        ("self.role != 'embedding' || self.type in ['openai', 'voyageai', 'gemini', 'ollama', "
         "'local', 'mock']",
         "role 'embedding' requires type in [openai, voyageai, gemini, ollama, local, mock]"),
        ("self.role != 'tts' || self.type in ['openai', 'cartesia', 'elevenlabs', 'mock']",
         "role 'tts' requires type in [openai, cartesia, elevenlabs]"),
        ("self.role != 'stt' || self.type in ['openai', 'mock']",
         "role 'stt' requires type in [openai]"),
        ("self.role != 'image' || self.type in ['imagen', 'mock']",
         "role 'image' requires type in [imagen]"),
        ("self.role != 'inference' || self.type in ['huggingface', 'local', 'mock']",
         "role 'inference' requires type in [huggingface, local]"),
        ("self.type != 'huggingface' || self.role == 'inference'",
         "huggingface is an inference-only vendor; set spec.role to 'inference'"),
        ("self.type != 'voyageai' || self.role == 'embedding'",
         "voyageai is an embedding-only vendor; set spec.role to 'embedding'"),
        ("self.type != 'cartesia' || self.role == 'tts'",
         "cartesia is a tts-only vendor; set spec.role to 'tts'"),
        ("self.type != 'elevenlabs' || self.role == 'tts'",
         "elevenlabs is a tts-only vendor; set spec.role to 'tts'"),
        ("self.type != 'imagen' || self.role == 'image'",
         "imagen is an image-only vendor; set spec.role to 'image'"),
        ("!has(self.platform) || self.role in ['llm', 'embedding']",
         "spec.platform is only valid when spec.role is 'llm' or 'embedding'"),
        ("!has(self.platform) || (self.type in ['claude', 'openai', 'gemini'])",
         "platform is only valid for provider types claude, openai, or gemini"),
        ("has(self.platform) == has(self.auth)", "spec.platform and spec.auth must be set together"),
        ("!has(self.platform) || self.platform.type != 'bedrock' || self.auth.type in "
         "['workloadIdentity', 'accessKey']",
         "platform.type bedrock requires auth.type of workloadIdentity or accessKey"),
        ("!has(self.platform) || self.platform.type != 'vertex' || self.auth.type in "
         "['workloadIdentity', 'serviceAccount']",
         "platform.type vertex requires auth.type of workloadIdentity or serviceAccount"),
        ("!has(self.platform) || self.platform.type != 'azure' || self.auth.type in "
         "['workloadIdentity', 'servicePrincipal']",
         "platform.type azure requires auth.type of workloadIdentity or servicePrincipal"),
        ("!(has(self.auth) && self.auth.type != 'workloadIdentity') || "
         "has(self.auth.credentialsSecretRef)",
         "credentialsSecretRef is required for non-workloadIdentity auth types"),
        ("!has(self.platform) || self.platform.type != 'vertex' || self.type != 'openai'",
         "openai on vertex is not supported: Vertex AI does not host OpenAI as a partner"),
        ("!has(self.platform) || self.platform.type != 'bedrock' || self.type != 'gemini'",
         "gemini on bedrock is not supported: AWS Bedrock does not host Gemini"),
        ("!has(self.platform) || self.platform.type != 'azure' || self.type != 'gemini'",
         "gemini on azure is not supported: Azure AI Foundry does not host Gemini"),
        ("self.type == 'mock' || (has(self.model) && size(self.model) > 0) || "
         "(self.type == 'local' && has(self.engine) && has(self.engine.model))",
         "spec.model is required for all provider types except mock (type local may set "
         "spec.engine.model instead)"),
        ("self.type != 'local' || self.role in ['llm', 'embedding', 'inference']",
         "type local serves the llm, embedding and inference roles")])

# ------------------------------------------------------------------ PromptPack
PROMPTPACK = Obj({
    "packName": Str(min_len=1),
    "source": Obj({"type": Enum("configmap"), "configMapRef": LOCAL_REF}, ["type"]),
    "version": Str(pattern=SEMVER),
    "skills": Arr(Obj({"source": Str(min_len=1), "include": Arr(Str()),
                       "mountAs": Str(pattern=r"^[a-z0-9]([a-z0-9-]*[a-z0-9])?$")}, ["source"])),
    "skillsConfig": Obj({"maxActive": Int(minimum=1),
                         "selector": Enum("model-driven", "tag", "embedding",
                                          default="model-driven")})},
    ["packName", "source", "version"],
    [("self == oldSelf",
      "a published PromptPack version is immutable; publish a new version instead")])

# ------------------------------------------------------------------ ToolRegistry
def _retry(extra: dict | None = None) -> dict:
    return Obj({"maxAttempts": Int(minimum=1, maximum=10), "initialBackoff": Str("100ms"),
                "backoffMultiplier": Str("2.0", pattern=DECIMAL), "maxBackoff": Str("30s"),
                **(extra or {})}, ["maxAttempts"])


HTTP_CONFIG = Obj({
    "endpoint": Str(), "method": Str("POST"), "headers": Map(),
    "contentType": Str("application/json"), "authType": Enum("bearer", "basic"),
    "authSecretRef": SECRET_KEY_SELECTOR, "queryParams": Arr(Str()), "headerParams": Map(),
    "staticQuery": Map(), "staticBody": JSON_ANY, "bodyMapping": Str(),
    "responseMapping": Str(), "redact": Arr(Str()), "urlTemplate": Str(),
    "retryPolicy": _retry({"retryOn": Arr(Int()), "retryOnNetworkError": Bool(True),
                           "respectRetryAfter": Bool(True)})}, ["endpoint"])
TOOL_DEF = Obj({"name": Str(pattern=r"^[a-z][a-z0-9_]*$", max_len=64),
                "description": Str(), "inputSchema": JSON_ANY, "outputSchema": JSON_ANY},
               ["name", "description", "inputSchema"])
TOOL_AUTH = Obj({
    "type": Enum("none", "bearer", "basic", "serviceAccount", "workloadIdentity",
                 default="none"),
    "secretRef": SECRET_KEY_SELECTOR,
    "serviceAccount": Obj({"audience": Str()}, ["audience"]),
    "workloadIdentity": Obj({"cloud": Enum("azure"), "audience": Str(),
                             "header": Str("Authorization")}, ["audience"])}, ["type"],
    [("self.type != 'bearer' && self.type != 'basic' || has(self.secretRef)",
      "auth.type bearer/basic requires secretRef"),
     ("self.type != 'serviceAccount' || has(self.serviceAccount)",
      "auth.type serviceAccount requires the serviceAccount block"),
     ("self.type != 'workloadIdentity' || has(self.workloadIdentity)",
      "auth.type workloadIdentity requires the workloadIdentity block")])
HANDLER = Obj({
    "name": Str(pattern=DNS_LABEL, max_len=63),
    "type": Enum("http", "openapi", "grpc", "mcp", "client"),
    "tool": TOOL_DEF, "httpConfig": HTTP_CONFIG,
    "openAPIConfig": Obj({"specURL": Str(), "baseURL": Str(), "operationFilter": Arr(Str()),
                          "headers": Map(), "authType": Enum("bearer", "basic"),
                          "authSecretRef": SECRET_KEY_SELECTOR, "retryPolicy": _retry(
                              {"retryOn": Arr(Int()), "retryOnNetworkError": Bool(True),
                               "respectRetryAfter": Bool(True)})}, ["specURL"]),
    "grpcConfig": Obj({"endpoint": Str(), "tls": Bool(), "tlsCertPath": Str(),
                       "tlsKeyPath": Str(), "tlsCAPath": Str(), "tlsInsecureSkipVerify": Bool(),
                       "retryPolicy": _retry({"retryableStatusCodes": Arr(Str())})},
                      ["endpoint"]),
    "mcpConfig": Obj({"transport": Enum("sse", "stdio", "streamable-http"), "endpoint": Str(),
                      "command": Str(), "args": Arr(Str()), "workDir": Str(), "env": Map(),
                      "toolFilter": Obj({"allowlist": Arr(Str()), "blocklist": Arr(Str())}),
                      "retryPolicy": _retry()}, ["transport"]),
    "clientConfig": Obj({"consentMessage": Str(), "categories": Arr(Str())}),
    "auth": TOOL_AUTH, "timeout": Str("30s"),
    "endpoint": Str()},  # MI355X shorthand for httpConfig/grpcConfig.endpoint
    ["name", "type"],
    [("!(has(self.auth) && ((has(self.httpConfig) && (has(self.httpConfig.authType) || "
      "has(self.httpConfig.authSecretRef))) || (has(self.openAPIConfig) && "
      "(has(self.openAPIConfig.authType) || has(self.openAPIConfig.authSecretRef)))))",
      "set either the handler-level auth stanza or the legacy httpConfig/openAPIConfig "
      "authType/authSecretRef, not both")])
TOOLREGISTRY = Obj({"handlers": Arr(HANDLER, min_items=1),
                    "probe": Obj({"enabled": Bool(), "interval": Str("60s"),
                                  "timeout": Str("5s")}, ["enabled"])}, ["handlers"])

# ------------------------------------------------------------------ Workspace
WS_ROLE = Enum("owner", "editor", "viewer")
DATABASE = Obj({"secretRef": LOCAL_REF}, ["secretRef"])
LABEL_SEL = Obj({"matchLabels": Map()})
NET_RULE = Obj({
    "peers": Arr(Obj({"namespaceSelector": LABEL_SEL, "podSelector": LABEL_SEL,
                      "ipBlock": Obj({"cidr": Str(), "except": Arr(Str())}, ["cidr"])})),
    "ports": Arr(Obj({"protocol": Enum("TCP", "UDP", "SCTP", default="TCP"), "port": Int()},
                     ["port"]))})
SERVICE_GROUP = Obj({
    "name": Str(pattern=r"^[a-z0-9]([a-z0-9-]*[a-z0-9])?$", max_len=63),
    "mode": Enum("managed", "external", default="managed"), "redis": REDIS,
    "memory": Obj({"database": DATABASE, "providerRef": LOCAL_REF, "policyRef": LOCAL_REF,
                   "redis": REDIS, "podOverrides": POD_OVERRIDES}, ["database"],
                  [_one_redis("memory")]),
    "session": Obj({"database": DATABASE, "policyRef": LOCAL_REF, "redis": REDIS,
                    "podOverrides": POD_OVERRIDES}, ["database"], [_one_redis("session")]),
    "external": Obj({"sessionURL": Str(pattern=r"^https?://"),
                     "memoryURL": Str(pattern=r"^https?://")}, ["sessionURL", "memoryURL"]),
    "privacyPolicyRef": LOCAL_REF,
    "evalWorker": Obj({"enabled": Bool(), "podOverrides": POD_OVERRIDES}),
    "autoscaling": AUTOSCALING}, ["name"],
    [("self.mode != 'managed' || (has(self.memory) && has(self.session))",
      "managed mode requires both memory and session configuration"),
     ("self.mode != 'external' || has(self.external)", "external mode requires external endpoints"),
     _one_redis("services[]")])
WORKSPACE = Obj({
    "displayName": Str(min_len=1, max_len=256), "description": Str(),
    "environment": Enum("development", "staging", "production", default="development"),
    "defaultTags": Map(),
    "namespace": Obj({"name": Str(min_len=1, max_len=63, pattern=DNS_LABEL), "create": Bool(),
                      "labels": Map(), "annotations": Map()}, ["name"]),
    "runtime": Obj({"serviceAccountName": Str(), "podLabels": Map(), "podAnnotations": Map()}),
    "roleBindings": Arr(Obj({
        "groups": Arr(Str()),
        "serviceAccounts": Arr(Obj({"name": Str(min_len=1), "namespace": Str(min_len=1)},
                                   ["name", "namespace"])),
        "role": WS_ROLE}, ["role"])),
    "directGrants": Arr(Obj({"user": Str(min_len=1), "role": WS_ROLE, "expires": TIME},
                            ["user", "role"])),
    "anonymousAccess": Obj({"enabled": Bool(), "role": WS_ROLE}, ["enabled"]),
    "costControls": Obj({"dailyBudget": Str(), "monthlyBudget": Str(),
                         "budgetExceededAction": Enum("warn", "pauseJobs", "block",
                                                      default="warn"),
                         "alertThresholds": Arr(Obj({"percent": Int(minimum=1, maximum=100),
                                                     "notify": Arr(Str())}, ["percent"]))}),
    "networkPolicy": Obj({"isolate": Bool(), "allowFrom": Arr(NET_RULE),
                          "allowTo": Arr(NET_RULE), "allowExternalAPIs": Bool(),
                          "allowSharedNamespaces": Bool(), "allowPrivateNetworks": Bool()}),
    "storage": Obj({"enabled": Bool(True), "storageClass": Str(), "size": Str("10Gi"),
                    "accessModes": Arr(Str(), default=["ReadWriteMany"]),
                    "retentionPolicy": Enum("Delete", "Retain", default="Delete")}),
    "services": Arr(SERVICE_GROUP, max_items=64),
    "mgmtPlaneMintServiceAccounts": Arr(Str(), max_items=16),
    "privacy": Obj({"database": DATABASE}, ["database"])},
    ["displayName", "namespace"])

# ------------------------------------------------------------------ policies
AGENTPOLICY = Obj({
    "selector": Obj({"agents": Arr(Str())}),
    "toolAccess": Obj({"mode": Enum("allowlist", "denylist"),
                       "rules": Arr(Obj({"registry": Str(min_len=1),
                                         "tools": Arr(Str(), min_items=1)},
                                        ["registry", "tools"]), min_items=1)},
                      ["mode", "rules"]),
    "mode": Enum("enforce", "permissive", default="enforce"),
    "onFailure": Enum("deny", "allow", default="deny")})


def _tier(leaf: bool) -> dict:
    props = {
        "mode": Enum("Manual", "TTL", "Decay", "LRU", "Composite", default="Manual"),
        "softDeleteGraceDays": Int(30, 0, 3650),
        "ttl": Obj({"default": Str(pattern=DAYS_DURATION), "maxAge": Str(pattern=DAYS_DURATION)}),
        "decay": Obj({"enabled": Bool(True), "minScore": Str("0.2", pattern=UNIT_FRACTION),
                      "scoreFormula": Obj({
                          "confidenceWeight": Str("0.5", pattern=UNIT_FRACTION),
                          "accessFrequencyWeight": Str("0.3", pattern=UNIT_FRACTION),
                          "recencyWeight": Str("0.2", pattern=UNIT_FRACTION)}),
                      "halfLifeDays": Int(90, 1, 3650)}),
        "lru": Obj({"enabled": Bool(True), "staleAfter": Str("120d", pattern=DAYS_DURATION)})}
    if not leaf:
        props["perCategory"] = Map(_tier(True))
    return Obj(props)


FUNCTION_REF = Obj({"name": Str(), "namespace": Str()}, ["name"])
MEMORYPOLICY = Obj({
    "tiers": Obj({"institutional": _tier(False), "agent": _tier(False), "user": _tier(False)}),
    "recall": Obj({"halfLife": Obj({"user": Str(pattern=DAYS_DURATION),
                                    "agent": Str(pattern=DAYS_DURATION),
                                    "institutional": Str(pattern=DAYS_DURATION)}),
                   "inlineThresholdBytes": Int(minimum=0, maximum=1048576),
                   "maxRelatedPerMemory": Int(minimum=0, maximum=50)}),
    "dedup": Obj({"requireAboutForKinds": Arr(Str()),
                  "embeddingSimilarity": Obj({
                      "enabled": Bool(True), "autoSupersedeAbove": Str(pattern=UNIT_FRACTION),
                      "surfaceDuplicatesAbove": Str(pattern=UNIT_FRACTION),
                      "candidateLimit": Int(minimum=0, maximum=50)}, (),
                      [("!has(self.autoSupersedeAbove) || !has(self.surfaceDuplicatesAbove) || "
                        "double(self.surfaceDuplicatesAbove) < double(self.autoSupersedeAbove)",
                        "surfaceDuplicatesAbove must be strictly less than autoSupersedeAbove")])}),
    "tierPrecedence": Obj({"multiplicative": Obj({
        "institutional": Str("1.0", pattern=r"^(10(\.0+)?|[0-9](\.[0-9]+)?)$"),
        "agent": Str("1.0", pattern=r"^(10(\.0+)?|[0-9](\.[0-9]+)?)$"),
        "user": Str("1.0", pattern=r"^(10(\.0+)?|[0-9](\.[0-9]+)?)$")})}, (),
        [("has(self.multiplicative)", "spec.tierPrecedence.multiplicative must be set")]),
    "consentRevocation": Obj({"action": Enum("SoftDelete", "HardDelete", "Stop",
                                             default="SoftDelete"),
                              "graceDays": Int(7, 0, 365)}),
    "supersession": Obj({"enabled": Bool(False), "graceDays": Int(14, 0, 365)}),
    "schedule": Str("0 3 * * *"), "batchSize": Int(1000, 1, 100000),
    "consolidation": Obj({
        "schedule": Str("0 2 * * *"),
        "schedules": Obj({"staleObservations": Str(), "crossScopeCandidates": Str(),
                          "entityDuplicateCandidates": Str()}),
        "functionRefs": Obj({"staleObservations": FUNCTION_REF,
                             "crossScopeCandidates": FUNCTION_REF,
                             "entityDuplicateCandidates": FUNCTION_REF}),
        "candidateLimits": Obj({"maxBucketsPerPass": Int(100, 1), "maxPerBucket": Int(50, 1)}),
        "safetyGates": Obj({"minDistinctUserCount": Map(Int()),
                            "maxScopeWidening": Str("workspace"),
                            "requirePIIRedaction": Bool(True)}),
        "timeouts": Obj({"functionCall": DURATION, "passWallClock": DURATION})}),
    "projection": Obj({"enabled": Bool(), "schedule": Str(), "changeThreshold": Int()}),
    "ingestion": Obj({"strategy": Enum("chunk", "summary", "summaryThenChunk", default="chunk"),
                      "summarizer": Enum("extractive", "agent", default="extractive"),
                      "chunk": Obj({"size": Int(200, 1), "overlap": Int(40, 0)}, (),
                                   [("self.overlap < self.size",
                                     "chunk.overlap must be less than chunk.size")])})},
    ["tiers"])
SESSIONRETENTIONPOLICY = Obj({
    "hotCache": Obj({"enabled": Bool(True),
                     "ttlAfterInactive": Str("24h", pattern=r"^([0-9]+h)?([0-9]+m)?([0-9]+s)?$"),
                     "maxSessions": Int(minimum=1), "maxMessagesPerSession": Int(minimum=1)}),
    "warmStore": Obj({"retentionDays": Int(7, 1, 3650),
                      "partitionBy": Enum("week", default="week")}),
    "coldArchive": Obj({"enabled": Bool(False), "retentionDays": Int(minimum=1, maximum=36500),
                        "compactionSchedule": Str("0 2 * * *")}, (),
                       [("!self.enabled || (has(self.retentionDays) && self.retentionDays > 0)",
                         "retentionDays is required when cold archive is enabled")])})
SOURCE_TIMING = {"interval": Str(pattern=GO_DURATION), "timeout": Str("60s"),
                 "suspend": Bool(False)}
SKILLSOURCE = Obj({
    "type": Enum("git", "oci", "configmap"), "git": GIT_SOURCE, "oci": OCI_SOURCE,
    "configMap": CONFIGMAP_SOURCE, **SOURCE_TIMING, "targetPath": Str(),
    "filter": Obj({"include": Arr(Str()), "exclude": Arr(Str()), "names": Arr(Str())}),
    "createVersionOnSync": Bool(True)}, ["type", "interval"],
    [("self.type != 'git' || has(self.git)", "git source requires spec.git"),
     ("self.type != 'oci' || has(self.oci)", "oci source requires spec.oci"),
     ("self.type != 'configmap' || has(self.configMap)", "configmap source requires spec.configMap")])

# ------------------------------------------------------------------ enterprise
LOAD_METRICS = ("latency_avg", "latency_p50", "latency_p90", "latency_p95", "latency_p99",
                "ttft_avg", "ttft_p50", "ttft_p90", "ttft_p95", "ttft_p99", "error_rate",
                "pass_rate", "total_cost", "rate_limit_rate")
ARENAJOB = Obj({
    "sourceRef": NAME_REF, "arenaFile": Str("config.arena.yaml"),
    "type": Enum("evaluation", "loadtest", "datagen", default="evaluation"),
    "trials": Int(minimum=1),
    "scenarios": Obj({"include": Arr(Str()), "exclude": Arr(Str())}),
    "evaluation": Obj({"outputFormats": Arr(Str())}),
    "loadTest": Obj({"concurrency": Int(1, 1), "vusPerWorker": Int(1, 1),
                     "ramp": Obj({"up": Str(), "down": Str()}), "budgetLimit": Str(),
                     "budgetCurrency": Str("USD"),
                     "thresholds": Arr(Obj({"metric": Enum(*LOAD_METRICS),
                                            "operator": Enum("<", ">", "<=", ">="),
                                            "value": Str(min_len=1)},
                                           ["metric", "operator", "value"]))}),
    "dataGen": Obj({"count": Int(100, 1), "format": Str("jsonl")}),
    "workers": Obj({"replicas": Int(1, 1), "minReplicas": Int(minimum=1),
                    "maxReplicas": Int(minimum=1), "podOverrides": POD_OVERRIDES}),
    "cancelled": Bool(),
    "output": Obj({"type": Enum("s3", "pvc"),
                   "s3": Obj({"bucket": Str(min_len=1), "prefix": Str(), "region": Str(),
                              "endpoint": Str(), "secretRef": NAME_REF}, ["bucket"]),
                   "pvc": Obj({"claimName": Str(min_len=1), "subPath": Str()}, ["claimName"])},
                  ["type"]),
    "schedule": Obj({"cron": Str(min_len=9), "timezone": Str("UTC"),
                     "concurrencyPolicy": Enum("Allow", "Forbid", "Replace", default="Forbid")}),
    "ttlSecondsAfterFinished": Int(minimum=0),
    "providers": Map(JSON_ANY),  # polymorphic group: list of entries or name -> entry
    "toolRegistries": Arr(NAME_REF), "verbose": Bool(), "sessionRecording": Bool()},
    ["sourceRef"])
ARENASOURCE = Obj({
    "type": Enum("git", "oci", "configmap", "workspace"), "git": GIT_SOURCE, "oci": OCI_SOURCE,
    "configMap": CONFIGMAP_SOURCE, "workspace": WORKSPACE_SOURCE, **SOURCE_TIMING,
    "targetPath": Str(), "createVersionOnSync": Bool(True)}, ["type", "interval"],
    [("[has(self.git), has(self.oci), has(self.configMap), has(self.workspace)].filter(x, x)"
      ".size() == 1", "exactly one of git, oci, configMap, or workspace must be set"),
     ("(self.type == 'git' && has(self.git)) || (self.type == 'oci' && has(self.oci)) || "
      "(self.type == 'configmap' && has(self.configMap)) || (self.type == 'workspace' && "
      "has(self.workspace))", "the source block must match the chosen type")])
ARENATEMPLATESOURCE = Obj({
    "type": Enum("git", "oci", "configmap"), "git": GIT_SOURCE, "oci": OCI_SOURCE,
    "configMap": CONFIGMAP_SOURCE, "syncInterval": Str("1h", pattern=GO_DURATION),
    "suspend": Bool(False), "timeout": Str("60s"), "templatesPath": Str("templates/")},
    ["type"])
ARENADEVSESSION = Obj({
    "projectId": Str(), "workspace": Str(), "idleTimeout": Str("30m"), "image": Str(),
    "resources": Obj({"requests": Map(), "limits": Map()}), "podOverrides": POD_OVERRIDES},
    ["projectId", "workspace"])
PROMPTPACKSOURCE = Obj({
    "type": Enum("git", "oci"), "git": GIT_SOURCE, "oci": OCI_SOURCE,
    "packName": Str(min_len=1), "interval": Str(pattern=GO_DURATION), "timeout": Str("60s"),
    "suspend": Bool(False), "historyLimit": Int(10, 0)}, ["type", "packName", "interval"],
    [("(self.type == 'git' && has(self.git) && !has(self.oci)) || (self.type == 'oci' && "
      "has(self.oci) && !has(self.git))", "exactly the source block matching type must be set")])
ROLLOUTANALYSIS = Obj({
    "args": Arr(Obj({"name": Str(min_len=1), "value": Str()}, ["name"])),
    "metrics": Arr(Obj({
        "name": Str(min_len=1), "interval": Str(min_len=1), "count": Int(minimum=1),
        "failureLimit": Int(minimum=0), "successCondition": Str(min_len=1),
        "failureCondition": Str(),
        "provider": Obj({
            "prometheus": Obj({"address": Str(min_len=1), "query": Str(min_len=1),
                               "timeout": Int(30)}, ["address", "query"]),
            "arenaEval": Obj({"workspace": Str(min_len=1), "evalDef": Str(min_len=1)},
                             ["workspace", "evalDef"]),
            "web": Obj({"url": Str(min_len=1), "method": Enum("GET", "POST", default="GET"),
                        "headers": Map(), "jsonPath": Str(), "timeout": Int(30)}, ["url"])})},
        ["name", "interval", "successCondition", "provider"]), min_items=1)},
    ["metrics"])
SESSIONPRIVACYPOLICY = Obj({
    "recording": Obj({"enabled": Bool(), "facadeData": Bool(), "runtimeData": Bool(),
                      "pii": Obj({"redact": Bool(), "encrypt": Bool(), "patterns": Arr(Str()),
                                  "strategy": Enum("replace", "hash", "mask")})}, ["enabled"]),
    "retention": Obj({"facade": Obj({"warmDays": Int(minimum=0), "coldDays": Int(minimum=0)}),
                      "richData": Obj({"warmDays": Int(minimum=0),
                                       "coldDays": Int(minimum=0)})}),
    "userOptOut": Obj({"enabled": Bool(), "honorDeleteRequests": Bool(),
                       "deleteWithinDays": Int(minimum=1)}),
    "encryption": Obj({"enabled": Bool(),
                       "kmsProvider": Enum("aws-kms", "azure-keyvault", "gcp-kms", "vault"),
                       "keyID": Str(), "secretRef": NAME_REF,
                       "keyRotation": Obj({"enabled": Bool(), "schedule": Str(),
                                           "reEncryptExisting": Bool(),
                                           "batchSize": Int(minimum=1, maximum=1000)})}, (),
                      [("!self.enabled || has(self.kmsProvider)",
                        "kmsProvider is required when encryption is enabled"),
                       ("!self.enabled || has(self.keyID)",
                        "keyID is required when encryption is enabled")]),
    "auditLog": Obj({"enabled": Bool(), "retentionDays": Int(minimum=1)})}, ["recording"])
TOOLPOLICY = Obj({
    "selector": Obj({"registry": Str(min_len=1), "tools": Arr(Str())}, ["registry"]),
    "rules": Arr(Obj({"name": Str(min_len=1), "description": Str(),
                      "deny": Obj({"cel": Str(min_len=1), "message": Str(min_len=1)},
                                  ["cel", "message"])}, ["name", "deny"]), min_items=1),
    "requiredClaims": Arr(Obj({"claim": Str(min_len=1), "message": Str(min_len=1)},
                              ["claim", "message"])),
    "mode": Enum("enforce", "audit", default="enforce"),
    "onFailure": Enum("deny", "allow", default="deny"),
    "headerInjection": Arr(Obj({"header": Str(min_len=1), "value": Str(), "cel": Str()},
                               ["header"]))}, ["selector", "rules"])

SPECS = {
    "AgentRuntime": AGENTRUNTIME, "Provider": PROVIDER, "PromptPack": PROMPTPACK,
    "ToolRegistry": TOOLREGISTRY, "Workspace": WORKSPACE, "AgentPolicy": AGENTPOLICY,
    "MemoryPolicy": MEMORYPOLICY, "SessionRetentionPolicy": SESSIONRETENTIONPOLICY,
    "SkillSource": SKILLSOURCE, "ArenaJob": ARENAJOB, "ArenaSource": ARENASOURCE,
    "ArenaTemplateSource": ARENATEMPLATESOURCE, "ArenaDevSession": ARENADEVSESSION,
    "PromptPackSource": PROMPTPACKSOURCE, "RolloutAnalysis": ROLLOUTANALYSIS,
    "SessionPrivacyPolicy": SESSIONPRIVACYPOLICY, "ToolPolicy": TOOLPOLICY,
}
