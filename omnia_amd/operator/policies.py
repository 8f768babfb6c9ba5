"""Policy reconcilers: AgentPolicy, MemoryPolicy, SessionRetentionPolicy.

Reference: ``internal/controller/agentpolicy_controller.go:70-520``,
``memorypolicy_controller.go:61-365``, ``sessionretentionpolicy_controller.go:
66-306``.

AgentPolicy
    Validates ``toolAccess`` (every rule names a registry and at least one
    non-empty tool), counts the matched AgentRuntimes, and enforces in two
    places:

    * cluster: Istio ``security.istio.io/v1 AuthorizationPolicy`` objects
      keyed on the ``X-Omnia-Tool-Name`` / ``X-Omnia-Agent-Name`` request
      headers -- allowlist: an ALLOW policy for the listed tools plus a DENY
      policy for every other tool (``notValues``: Istio evaluates DENY first, so
      a bare catch-all would block the allowlist too), or an AUDIT policy in
      permissive mode; denylist: one DENY
      (AUDIT) policy.  Owned by the AgentPolicy, stale ones deleted.  When the
      Istio kind is not served, ``onFailure: deny`` (default) puts the policy in
      Error, ``allow`` keeps it Active with enforcement inactive;
    * in-node: the matched agents' tool ConfigMaps carry the compiled access
      list and the runtime's executor refuses a call before any handler runs
      (:class:`omnia_amd.tools.executor.ToolAccess`), so the policy holds
      without a mesh.

MemoryPolicy
    Validates the tier set (TTL ``default <= maxAge``, extended durations with
    ``d`` days, decay ``minScore`` and score weights in [0, 1], LRU
    ``staleAfter``, per-category leaves), the cron ``schedule`` and the
    multiplicative tier precedence weights in [0, 10]; publishes the spec as
    ConfigMap ``memory-policy-<name>`` for memory-api's retention worker
    (:mod:`omnia_amd.memory.retention`).

SessionRetentionPolicy
    Validates durations / retention days / the compaction cron, resolves the
    tier config and syncs ConfigMap ``retention-policy-<name>`` (YAML, operator
    namespace) that session-api compaction reads; a finalizer deletes the
    ConfigMap with the policy.
"""
from __future__ import annotations

import json
import re

import yaml

from ..api import crds
from ..utils.durations import parse_duration as _parse_duration
from .apistore import APIStore, Conflict, NotFound, owner_ref, set_condition

ISTIO_API = "security.istio.io/v1"
ISTIO_KIND = "AuthorizationPolicy"
HEADER_TOOL = "X-Omnia-Tool-Name"
HEADER_AGENT = "X-Omnia-Agent-Name"
LABEL_MANAGED_BY = "app.kubernetes.io/managed-by"
LABEL_OWNER_POLICY = "omnia.altairalabs.ai/agent-policy"
RETENTION_FINALIZER = "sessionretentionpolicy.omnia.altairalabs.ai/configmap-cleanup"


class PolicyInvalid(ValueError):
    pass


# ------------------------------------------------------------------ parsing helpers
def parse_duration(s: str) -> float:
    """Go ``time.ParseDuration`` plus ``d`` days (``parseExtendedDuration``):
    "720h", "30d", "1d12h", "90m".  Returns seconds."""
    try:
        return _parse_duration(s)
    except ValueError as e:
        raise PolicyInvalid(str(e)) from None


_CRON_FIELD = r"(\*|\d+(,\d+)*|\d+[-/]\d+|\*/\d+)"
_CRON = re.compile(r"^(@(every +\d+(ns|us|µs|ms|s|m|h)|hourly|daily|weekly|monthly|yearly|"
                   r"reboot)|" + _CRON_FIELD + r"( " + _CRON_FIELD + r"){4,5})$")


def validate_cron(s: str):
    if not _CRON.match(s.strip()):
        raise PolicyInvalid(f"invalid cron schedule {s!r}")


def _weight(name: str, raw, lo: float = 0.0, hi: float = 1.0):
    if raw in (None, ""):
        return
    try:
        v = float(raw)
    except (TypeError, ValueError):
        raise PolicyInvalid(f"{name} {raw!r} is not a valid decimal") from None
    if not lo <= v <= hi:
        raise PolicyInvalid(f"{name} {raw!r} must be between {lo:g} and {hi:g}")


# ------------------------------------------------------------------ AgentPolicy
def validate_agent_policy(spec: dict):
    ta = spec.get("toolAccess")
    if ta is None:
        return
    if ta.get("mode") not in ("allowlist", "denylist"):
        raise PolicyInvalid(f"toolAccess.mode must be allowlist or denylist, got "
                            f"{ta.get('mode')!r}")
    if not ta.get("rules"):
        raise PolicyInvalid("toolAccess.rules must not be empty")
    for r in ta["rules"]:
        if not r.get("registry"):
            raise PolicyInvalid("toolAccess rule registry must not be empty")
        if not r.get("tools"):
            raise PolicyInvalid(f"toolAccess rule tools must not be empty for registry "
                                f"{r['registry']!r}")
        if any(not t for t in r["tools"]):
            raise PolicyInvalid(f"tool name must not be empty in registry {r['registry']!r}")


def matched_agents(policy: dict, agents: list[dict]) -> list[str]:
    sel = set(((policy["spec"].get("selector") or {}).get("agents")) or [])
    return sorted(a["metadata"]["name"] for a in agents
                  if not sel or a["metadata"]["name"] in sel)


def _tool_values(rule: dict) -> list[str]:
    return [f"{rule['registry']}/{t}" for t in rule["tools"]]


def desired_authorization_policies(policy: dict) -> list[dict]:
    spec, md = policy["spec"], policy["metadata"]
    ta = spec.get("toolAccess")
    if not ta:
        return []
    sel_agents = (spec.get("selector") or {}).get("agents") or []
    permissive = spec.get("mode") == "permissive"
    action = "AUDIT" if permissive else ("ALLOW" if ta["mode"] == "allowlist" else "DENY")

    def base(name):
        return {"apiVersion": ISTIO_API, "kind": ISTIO_KIND,
                "metadata": {"name": name, "namespace": md["namespace"],
                             "labels": {LABEL_MANAGED_BY: "omnia-operator",
                                        LABEL_OWNER_POLICY: md["name"]},
                             "ownerReferences": [owner_ref(policy)]}}

    def agent_cond():
        return {"key": f"request.headers[{HEADER_AGENT}]", "values": list(sel_agents)}

    rules = []
    for r in ta["rules"]:
        when = [{"key": f"request.headers[{HEADER_TOOL}]", "values": _tool_values(r)}]
        if sel_agents:
            when.append(agent_cond())
        rules.append({"when": when})
    if ta["mode"] == "allowlist":
        out = [dict(base(md["name"] + "-allow"), spec={"action": action, "rules": rules})]
        if action == "ALLOW":
            # enforce: every other tool is denied.  Istio evaluates DENY before
            # ALLOW, so the catch-all must exclude the allowed tools (notValues);
            # a bare catch-all would deny the allowlisted tools too
            allowed = [v for r in ta["rules"] for v in _tool_values(r)]
            catch = {"when": [{"key": f"request.headers[{HEADER_TOOL}]",
                               "notValues": allowed}]}
            if sel_agents:
                catch["when"].append(agent_cond())
            out.append(dict(base(md["name"] + "-deny-all"),
                            spec={"action": "DENY", "rules": [catch]}))
        return out
    return [dict(base(md["name"] + "-deny"), spec={"action": action, "rules": rules})]


def compile_tool_access(policies: list[dict], agent: str) -> list[dict]:
    """The in-node access list of one agent: every Active AgentPolicy selecting it."""
    out = []
    for p in sorted(policies, key=lambda p: p["metadata"]["name"]):
        spec = p["spec"]
        if not spec.get("toolAccess") or (p.get("status") or {}).get("phase") != "Active":
            continue
        sel = set(((spec.get("selector") or {}).get("agents")) or [])
        if sel and agent not in sel:
            continue
        out.append({"policy": p["metadata"]["name"], "mode": spec["toolAccess"]["mode"],
                    "enforce": spec.get("mode", "enforce") != "permissive",
                    "rules": [{"registry": r["registry"], "tools": list(r["tools"])}
                              for r in spec["toolAccess"]["rules"]]})
    return out


class AgentPolicyReconciler:
    kind = "AgentPolicy"

    def __init__(self, istio: bool | None = None):
        self.istio = istio  # None: use the store's own knowledge of served kinds

    def _istio_served(self, store) -> bool:
        if self.istio is not None:
            return self.istio
        served = getattr(store, "serves", None)
        return bool(served and served(ISTIO_API, ISTIO_KIND))

    def reconcile(self, store: APIStore, ns, name: str):
        p = store.try_get("AgentPolicy", name, ns)
        if p is None:
            return None
        st = p.get("status") or {}
        gen = p["metadata"].get("generation", 1)
        spec = p["spec"]
        try:
            validate_agent_policy(spec)
        except PolicyInvalid as e:
            set_condition(st, "Valid", False, "PolicyInvalid", str(e), gen)
            st.update(phase="Error", observedGeneration=gen)
            p["status"] = st
            store.update_status(p)
            return None
        set_condition(st, "Valid", True, "PolicyValid", "Policy configuration is valid", gen)
        matched = matched_agents(p, store.list("AgentRuntime", ns))
        mesh_msg = ""
        if spec.get("toolAccess"):
            if self._istio_served(store):
                desired = desired_authorization_policies(p)
                names = {d["metadata"]["name"] for d in desired}
                for d in desired:
                    store.apply(d)
                for old in store.list(ISTIO_KIND, ns):
                    if (old["metadata"].get("labels") or {}).get(LABEL_OWNER_POLICY) == name \
                            and old["metadata"]["name"] not in names:
                        store.delete(ISTIO_KIND, old["metadata"]["name"], ns)
            elif spec.get("onFailure", "deny") == "deny":
                msg = "istio CRDs not installed — cannot enforce policy (onFailure=deny)"
                set_condition(st, "Applied", False, "PolicyInvalid", msg, gen)
                st.update(phase="Error", matchedAgents=len(matched), observedGeneration=gen)
                p["status"] = st
                store.update_status(p)
                return None
            else:
                mesh_msg = "; mesh enforcement inactive (istio not installed, onFailure=allow)"
        applied = (f"Policy applied in permissive mode to {len(matched)} agent(s) (audit only, "
                   f"not enforcing)" if spec.get("mode") == "permissive"
                   else f"Policy applied to {len(matched)} agent(s)") + mesh_msg
        set_condition(st, "Applied", True, "PolicyApplied", applied, gen)
        st.update(phase="Active", matchedAgents=len(matched), observedGeneration=gen)
        p["status"] = st
        store.update_status(p)
        return None


# ------------------------------------------------------------------ MemoryPolicy
def _validate_ttl(t: dict, where: str):
    d = parse_duration(t["default"]) if t.get("default") else None
    m = parse_duration(t["maxAge"]) if t.get("maxAge") else None
    if d is not None and m is not None and d > m:
        raise PolicyInvalid(f"{where}.ttl: default ({t['default']}) must not exceed maxAge "
                            f"({t['maxAge']})")


def _validate_leaf(c: dict, where: str):
    try:
        if c.get("ttl"):
            _validate_ttl(c["ttl"], where)
        dec = c.get("decay") or {}
        _weight(f"{where}.decay.minScore", dec.get("minScore"))
        for w in ("confidenceWeight", "accessFrequencyWeight", "recencyWeight"):
            _weight(f"{where}.decay.{w}", (dec.get("scoreFormula") or {}).get(w))
        if (c.get("lru") or {}).get("staleAfter"):
            parse_duration(c["lru"]["staleAfter"])
    except PolicyInvalid as e:
        raise PolicyInvalid(f"{where}: {e}" if not str(e).startswith(where) else str(e)) \
            from None


def validate_memory_policy(spec: dict):
    for tier in ("institutional", "agent", "user"):
        c = (spec.get("tiers") or {}).get(tier)
        if c is None:
            continue
        _validate_leaf(c, tier)
        for cat, leaf in (c.get("perCategory") or {}).items():
            _validate_leaf(leaf, f"{tier}.perCategory[{cat}]")
    if spec.get("schedule"):
        validate_cron(spec["schedule"])
    mult = (spec.get("tierPrecedence") or {}).get("multiplicative") or {}
    for tier in ("institutional", "agent", "user"):
        _weight(f"tierPrecedence.multiplicative.{tier}", mult.get(tier), 0.0, 10.0)


def _status_fail(store, obj, st, gen, reason, msg):
    set_condition(st, "PolicyValid", False, reason, msg, gen)
    set_condition(st, "Ready", False, reason, "See PolicyValid condition for details", gen)
    st.update(phase="Error", observedGeneration=gen)
    obj["status"] = st
    store.update_status(obj)


class MemoryPolicyReconciler:
    kind = "MemoryPolicy"

    def __init__(self, namespace: str = "omnia-system"):
        self.namespace = namespace

    def reconcile(self, store: APIStore, ns, name: str):
        p = store.try_get("MemoryPolicy", name, None)
        if p is None:
            return None
        st = p.get("status") or {}
        gen = p["metadata"].get("generation", 1)
        try:
            validate_memory_policy(p["spec"])
        except PolicyInvalid as e:
            _status_fail(store, p, st, gen, "ValidationFailed", str(e))
            return None
        set_condition(st, "PolicyValid", True, "Valid", "Policy spec is valid", gen)
        set_condition(st, "WorkspacesResolved", True, "NotApplicable",
                      "Workspace binding is via Workspace.spec.services[].memory.policyRef", gen)
        store.apply({"apiVersion": "v1", "kind": "ConfigMap",
                     "metadata": {"name": f"memory-policy-{name}", "namespace": self.namespace,
                                  "labels": {LABEL_MANAGED_BY: "omnia-operator",
                                             "omnia.altairalabs.ai/component": "memory-policy"},
                                  "ownerReferences": [owner_ref(p)]},
                     "data": {"policy.json": json.dumps(p["spec"], sort_keys=True)}})
        set_condition(st, "Ready", True, "AllChecksPass", "Policy is valid", gen)
        st.update(phase="Active", observedGeneration=gen)
        p["status"] = st
        store.update_status(p)
        return None


# ------------------------------------------------------------------ SessionRetentionPolicy
def validate_retention_policy(spec: dict):
    hot = spec.get("hotCache") or {}
    if hot.get("ttlAfterInactive"):
        parse_duration(hot["ttlAfterInactive"])
    for k in ("maxSessions", "maxMessagesPerSession"):
        if hot.get(k) is not None and int(hot[k]) < 1:
            raise PolicyInvalid(f"hotCache.{k} must be >= 1")
    warm = spec.get("warmStore") or {}
    if warm.get("retentionDays") is not None and int(warm["retentionDays"]) < 1:
        raise PolicyInvalid("warmStore.retentionDays must be >= 1")
    cold = spec.get("coldArchive") or {}
    if cold.get("retentionDays") is not None and int(cold["retentionDays"]) < 1:
        raise PolicyInvalid("coldArchive.retentionDays must be >= 1")
    if cold.get("compactionSchedule"):
        validate_cron(cold["compactionSchedule"])


def resolved_retention(spec: dict) -> dict:
    out = {}
    for k in ("hotCache", "warmStore", "coldArchive"):
        if spec.get(k) is not None:
            out[k] = spec[k]
    return out


class SessionRetentionPolicyReconciler:
    kind = "SessionRetentionPolicy"

    def __init__(self, namespace: str = "omnia-system"):
        self.namespace = namespace

    def reconcile(self, store: APIStore, ns, name: str):
        p = store.try_get("SessionRetentionPolicy", name, None)
        if p is None:
            return None
        md = p["metadata"]
        cm_name = f"retention-policy-{name}"
        if md.get("deletionTimestamp"):
            if RETENTION_FINALIZER in (md.get("finalizers") or []):
                try:
                    store.delete("ConfigMap", cm_name, self.namespace)
                except NotFound:
                    pass
                md["finalizers"] = [f for f in md["finalizers"] if f != RETENTION_FINALIZER]
                store.update(p)
            return None
        if RETENTION_FINALIZER not in (md.get("finalizers") or []):
            md.setdefault("finalizers", []).append(RETENTION_FINALIZER)
            try:
                p = store.update(p)
            except Conflict:
                return 0.5
        st = p.get("status") or {}
        gen = p["metadata"].get("generation", 1)
        try:
            validate_retention_policy(p["spec"])
        except (PolicyInvalid, ValueError, TypeError) as e:
            _status_fail(store, p, st, gen, "ValidationFailed", str(e))
            return None
        set_condition(st, "PolicyValid", True, "Valid", "Policy spec is valid", gen)
        set_condition(st, "WorkspacesResolved", True, "NotApplicable",
                      "Workspace binding is now via Workspace.spec.services[].session.policyRef",
                      gen)
        store.apply({"apiVersion": "v1", "kind": "ConfigMap",
                     "metadata": {"name": cm_name, "namespace": self.namespace,
                                  "labels": {LABEL_MANAGED_BY: "omnia-operator",
                                             "omnia.altairalabs.ai/component":
                                                 "retention-config",
                                             "omnia.altairalabs.ai/retention-policy": name}},
                     "data": {"retention.yaml": yaml.safe_dump(resolved_retention(p["spec"]),
                                                               sort_keys=True)}})
        set_condition(st, "Ready", True, "AllChecksPass", "Policy is valid and config synced",
                      gen)
        st.update(phase="Active", observedGeneration=gen, workspaceCount=0)
        p["status"] = st
        store.update_status(p)
        return None


def retention_from_config(doc: dict) -> dict:
    """CompactionConfig fields from a ``retention.yaml`` (session-api side)."""
    out = {}
    warm = doc.get("warmStore") or {}
    if warm.get("retentionDays"):
        out["warm_retention_s"] = float(warm["retentionDays"]) * 86400
    cold = doc.get("coldArchive") or {}
    if cold.get("retentionDays"):
        out["cold_retention_s"] = float(cold["retentionDays"]) * 86400
    hot = doc.get("hotCache") or {}
    if hot.get("ttlAfterInactive"):
        out["hot_ttl_s"] = parse_duration(hot["ttlAfterInactive"])
    if hot.get("maxSessions"):
        out["hot_max_sessions"] = int(hot["maxSessions"])
    if hot.get("maxMessagesPerSession"):
        out["hot_max_messages"] = int(hot["maxMessagesPerSession"])
    return out


_ = crds  # kinds are registered in api/crds.py
