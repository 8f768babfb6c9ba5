"""Omnia CRD surface (group ``omnia.altairalabs.ai``, version ``v1alpha1``).

17 kinds -- the 9 core kinds (AgentRuntime, Provider, PromptPack, ToolRegistry,
Workspace, AgentPolicy, MemoryPolicy, SessionRetentionPolicy, SkillSource) and
the 8 enterprise kinds (ArenaJob, ArenaSource, ArenaTemplateSource,
ArenaDevSession, PromptPackSource, RolloutAnalysis, SessionPrivacyPolicy,
ToolPolicy) -- with the reference's names, short names, scope, required
fields, enums, defaults and printer columns (``api/v1alpha1/*_types.go``,
``ee/api/v1alpha1``).  The full structural ``spec`` schemas -- nested blocks,
bounds, patterns, defaults and the kubebuilder CEL rules as
``x-kubernetes-validations`` evaluated by the in-repo CEL interpreter -- are in
``crd_types.py``; ``schema.py`` is the validator (defaulting, strict unknown
fields, CEL with ``oldSelf`` transition rules).

Additive MI355X extensions (SURVEY §7.1 design choice 3): Provider
``spec.type: local`` + ``spec.engine`` -- the in-node MI355X engine -- and the
few fields listed in ``crd_types.py``'s docstring.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

GROUP = "omnia.altairalabs.ai"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"

S = {"type": "string"}
OBJ = {"type": "object"}
ANY_OBJ = {"type": "object", "additionalProperties": True}


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


# ------------------------------------------------------------------ kinds
# Full structural schemas (nested blocks, enums, bounds, patterns, defaults and
# the kubebuilder CEL rules as x-kubernetes-validations) live in crd_types.py;
# the Python validators below cover only what a schema cannot express.
from . import crd_types as T  # noqa: E402

PROVIDER_TYPES = T.PROVIDER_TYPES
ROLE_TYPES = {
    "llm": {"claude", "openai", "gemini", "ollama", "mock", "vllm", "local"},
    "embedding": {"openai", "gemini", "ollama", "voyageai", "mock", "local"},
    "tts": {"openai", "cartesia", "elevenlabs", "mock"},
    "stt": {"openai", "mock"},
    "image": {"imagen", "mock"},
    "inference": {"huggingface", "local", "mock"},
}
NEEDS_CREDENTIAL = {"claude", "openai", "gemini", "voyageai", "cartesia", "elevenlabs"}


def _unique_names(field: str):
    """``+listType=map`` / ``+listMapKey=name``: list entries are keyed by name."""
    def check(spec: dict) -> list[str]:
        names = [h.get("name") for h in spec.get(field) or []]
        dup = sorted({n for n in names if names.count(n) > 1})
        return [f"spec.{field}: Duplicate value: {d!r}" for d in dup]
    return check


KINDS: dict[str, Kind] = {}


def _reg(k: Kind):
    KINDS[k.kind] = k


_reg(Kind("AgentRuntime", "agentruntimes", ["agent", "ar"], "Namespaced", T.AGENTRUNTIME,
          [("Phase", ".status.phase"), ("Ready", ".status.replicas.ready"),
           ("Version", ".status.activeVersion"), ("Age", ".metadata.creationTimestamp")],
          [_unique_names("providers")]))
_reg(Kind("Provider", "providers", ["prov"], "Namespaced", T.PROVIDER,
          [("Type", ".spec.type"), ("Model", ".spec.model"), ("Phase", ".status.phase"),
           ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("PromptPack", "promptpacks", ["pp"], "Namespaced", T.PROMPTPACK,
          [("Version", ".spec.version"), ("Phase", ".status.phase"),
           ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("ToolRegistry", "toolregistries", ["tr"], "Namespaced", T.TOOLREGISTRY,
          [("Tools", ".status.discoveredToolsCount"), ("Phase", ".status.phase"),
           ("Age", ".metadata.creationTimestamp")], [_unique_names("handlers")]))
_reg(Kind("Workspace", "workspaces", ["ws"], "Cluster", T.WORKSPACE,
          [("Display Name", ".spec.displayName"), ("Environment", ".spec.environment"),
           ("Phase", ".status.phase"), ("Namespace", ".spec.namespace.name"),
           ("Age", ".metadata.creationTimestamp")], [_unique_names("services")]))
_reg(Kind("AgentPolicy", "agentpolicies", ["ap"], "Namespaced", T.AGENTPOLICY,
          [("Mode", ".spec.mode"), ("Phase", ".status.phase"),
           ("Matched", ".status.matchedAgents"), ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("MemoryPolicy", "memorypolicies", ["mp"], "Cluster", T.MEMORYPOLICY,
          [("Phase", ".status.phase"), ("Schedule", ".spec.schedule"),
           ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("SessionRetentionPolicy", "sessionretentionpolicies", ["srp"], "Cluster",
          T.SESSIONRETENTIONPOLICY,
          [("Phase", ".status.phase"), ("Hot Cache TTL", ".spec.hotCache.ttlAfterInactive"),
           ("Warm Days", ".spec.warmStore.retentionDays"),
           ("Cold Archive", ".spec.coldArchive.enabled"), ("Age", ".metadata.creationTimestamp")]))
_reg(Kind("SkillSource", "skillsources", ["skl"], "Namespaced", T.SKILLSOURCE,
          [("Type", ".spec.type"), ("Phase", ".status.phase"), ("Skills", ".status.skillCount"),
           ("Age", ".metadata.creationTimestamp")]))
# ---- enterprise
_reg(Kind("ArenaJob", "arenajobs", ["aj"], "Namespaced", T.ARENAJOB,
          [("Source", ".spec.sourceRef.name"), ("Type", ".spec.type"), ("Phase", ".status.phase"),
           ("Progress", ".status.progress"), ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("ArenaSource", "arenasources", ["as"], "Namespaced", T.ARENASOURCE,
          [("Type", ".spec.type"), ("Phase", ".status.phase"), ("Revision", ".status.revision"),
           ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("ArenaTemplateSource", "arenatemplatesources", ["ats"], "Namespaced",
          T.ARENATEMPLATESOURCE,
          [("Type", ".spec.type"), ("Phase", ".status.phase"),
           ("Templates", ".status.templateCount"), ("Age", ".metadata.creationTimestamp")],
          ee=True))
_reg(Kind("ArenaDevSession", "arenadevsessions", ["ads"], "Namespaced", T.ARENADEVSESSION,
          [("Phase", ".status.phase"), ("Project", ".spec.projectId"),
           ("Endpoint", ".status.endpoint"), ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("PromptPackSource", "promptpacksources", ["pps"], "Namespaced", T.PROMPTPACKSOURCE,
          [("Pack", ".spec.packName"), ("Type", ".spec.type"), ("Phase", ".status.phase"),
           ("Version", ".status.lastSyncedVersion"), ("Age", ".metadata.creationTimestamp")],
          ee=True))
_reg(Kind("RolloutAnalysis", "rolloutanalyses", ["ra"], "Namespaced", T.ROLLOUTANALYSIS,
          [("Metrics", ".status.metricCount"), ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("SessionPrivacyPolicy", "sessionprivacypolicies", ["spp"], "Namespaced",
          T.SESSIONPRIVACYPOLICY,
          [("Recording", ".spec.recording.enabled"), ("PII Redact", ".spec.recording.pii.redact"),
           ("Encryption", ".spec.encryption.enabled"), ("Phase", ".status.phase"),
           ("Age", ".metadata.creationTimestamp")], ee=True))
_reg(Kind("ToolPolicy", "toolpolicies", ["tp"], "Namespaced", T.TOOLPOLICY,
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
    from .schema import apply_defaults as _ad

    return _ad(schema, obj)


def validate_object(obj: dict, old: dict | None = None, field_validation: str = "Strict",
                    warnings: list | None = None) -> list[str]:
    """Admission-time validation: apiVersion/kind, metadata, then the structural
    schema (defaults, strict fields, bounds, CEL rules with ``oldSelf`` on
    updates) and the Python validators."""
    from . import schema as SCH

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
    SCH.apply_defaults(k.spec, spec)
    old_spec = (old or {}).get("spec") if old is not None else None
    errs += SCH.validate(k.spec, spec, "spec", old_spec, field_validation=field_validation,
                         warnings=warnings)
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
