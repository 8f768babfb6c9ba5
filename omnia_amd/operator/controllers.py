"""Reconcilers (``internal/controller``).

Each reconciler is ``reconcile(store, ns, name) -> requeue_after | None`` and is
idempotent.  The manager (manager.py) feeds them from watch events, including
cross-kind mappings (a PromptPack/Provider/ToolRegistry change re-queues the
AgentRuntimes that reference it, a Deployment change re-queues its owner).
"""
from __future__ import annotations

import json
import os
import re
import logging
import time

import yaml

from ..api import crds
from ..models.config import REGISTRY as MODEL_REGISTRY
from ..runtime.promptpack import PackError, PromptPack
from . import builders as B
from . import subresources as SR
from .chart import COMPONENTS
from .apistore import APIStore, NotFound, get_condition, owner_ref, set_condition

log = logging.getLogger("omnia.operator")

PENDING, RUNNING, FAILED = "Pending", "Running", "Failed"


def _semver_key(v: str):
    v = v.lstrip("v")
    core, _, pre = v.partition("-")
    nums = [int(x) for x in core.split(".")[:3] if x.isdigit()]
    while len(nums) < 3:
        nums.append(0)
    # a release sorts after its prereleases
    return (nums, 1 if not pre else 0, pre)


def packs_for(store: APIStore, ns: str, pack_name: str) -> list[dict]:
    return [p for p in store.list("PromptPack", ns)
            if p["spec"].get("packName") == pack_name or
            p["metadata"].get("labels", {}).get(B.LABEL_PACK_NAME) == pack_name or
            p["metadata"]["name"] == pack_name]


def resolve_promptpack(store: APIStore, ns: str, ref: dict) -> dict | None:
    """By exact version, else by track (stable = highest non-prerelease, prerelease =
    highest overall) (``internal/controller/promptpack_resolve.go:20-70``)."""
    cands = [p for p in packs_for(store, ns, ref["name"])
             if (p.get("status") or {}).get("phase") in ("Active", "Superseded", None, "")]
    if not cands:
        return None
    if ref.get("version"):
        for p in cands:
            if p["spec"]["version"].lstrip("v") == ref["version"].lstrip("v"):
                return p
        return None
    track = ref.get("track", "stable")
    pool = cands if track == "prerelease" else [p for p in cands if "-" not in
                                                 p["spec"]["version"]]
    if not pool:
        return None
    return max(pool, key=lambda p: _semver_key(p["spec"]["version"]))


# ===================================================================== PromptPack
class PromptPackReconciler:
    kind = "PromptPack"

    def reconcile(self, store: APIStore, ns: str, name: str):
        pp = store.try_get("PromptPack", name, ns)
        if pp is None:
            return None
        st = pp.get("status") or {}
        src = pp["spec"]["source"]
        ref = src.get("configMapRef") or {}
        cm = store.try_get("ConfigMap", ref.get("name", ""), ns)
        ok, msg = True, ""
        if cm is None:
            ok, msg = False, f"ConfigMap {ref.get('name')} not found"
        else:
            raw = (cm.get("data") or {}).get(ref.get("key", "pack.json"))
            if raw is None:
                ok, msg = False, "pack.json key missing from ConfigMap"
            else:
                try:
                    pack = PromptPack(json.loads(raw))
                    st["packId"] = pack.id
                    st["prompts"] = sorted(pack.prompts)
                except (json.JSONDecodeError, PackError) as e:
                    ok, msg = False, str(e)[:300]
                else:
                    # eval types nobody registered (runtime/evals.py ValidateEvalDefs):
                    # surfaced on the pack, not silently skipped at run time
                    from ..runtime.evals import validate_eval_defs

                    defs = list(pack.data.get("evals") or [])
                    for pr in pack.prompts.values():
                        defs.extend(pr.evals or [])
                    missing = validate_eval_defs(defs)
                    set_condition(st, "EvalTypesRegistered", not missing,
                                  "Registered" if not missing else "UnknownEvalType",
                                  ", ".join(missing)[:300], pp["metadata"]["generation"])
        set_condition(st, "PackContentValid", ok, "Valid" if ok else "Invalid", msg,
                      pp["metadata"]["generation"])
        if not ok:
            st["phase"] = "Failed"
        else:
            siblings = [p for p in packs_for(store, ns, pp["spec"]["packName"])
                        if get_condition(p, "PackContentValid") is None or
                        get_condition(p, "PackContentValid")["status"] == "True"
                        or p["metadata"]["name"] == name]
            newest = max(siblings, key=lambda p: _semver_key(p["spec"]["version"]))
            st["phase"] = "Active" if newest["metadata"]["name"] == name else "Superseded"
        st["observedGeneration"] = pp["metadata"]["generation"]
        pp["status"] = st
        store.update_status(pp)
        return None


# ===================================================================== Provider
class ProviderReconciler:
    kind = "Provider"

    def __init__(self, gpu_count: int | None = None, cfg: SR.OperatorConfig | None = None):
        self.gpu_count = gpu_count
        self.cfg = cfg or SR.OperatorConfig.from_env()

    def reconcile(self, store: APIStore, ns: str, name: str):
        pv = store.try_get("Provider", name, ns)
        if pv is None:
            return None
        spec, st = pv["spec"], pv.get("status") or {}
        gen = pv["metadata"]["generation"]
        cred_ok, cred_msg = True, ""
        cred = spec.get("credential") or {}
        if spec["type"] in crds.NEEDS_CREDENTIAL and not cred:
            cred_ok, cred_msg = False, f"type {spec['type']} requires a credential"
        if cred.get("secretRef"):
            sref = cred["secretRef"]
            sec = store.try_get("Secret", sref["name"], ns)
            if sec is None:
                cred_ok, cred_msg = False, f"secret {sref['name']} not found"
            elif sref.get("key") and sref["key"] not in (sec.get("data") or {}) and \
                    sref["key"] not in (sec.get("stringData") or {}):
                cred_ok, cred_msg = False, f"secret {sref['name']} has no key {sref['key']}"
        set_condition(st, "CredentialValid", cred_ok, "Valid" if cred_ok else "Invalid",
                      cred_msg, gen)
        model_ok, model_msg = True, ""
        if spec["type"] == "local":
            eng = spec.get("engine") or {}
            m = eng.get("model") or spec.get("model")
            from ..models.config import ALIASES

            cfg = MODEL_REGISTRY.get(ALIASES.get(m, m))
            if eng.get("checkpoint"):
                # the checkpoint's config.json is the architecture (any name); a
                # directory this process cannot read is checked by the engine at load
                try:
                    from ..models.loader import config_from_hf

                    cfg = config_from_hf(eng["checkpoint"], m)
                except (OSError, ValueError, KeyError):
                    cfg = None
            elif cfg is None:
                model_ok, model_msg = False, f"unknown engine model {m}"
            tp = int(eng.get("tp", 1))
            # GPUs a pod's ranks may share (OMNIA_RANKS_PER_GPU, the launcher's
            # DeviceAllocator): the capacity is GPUs x ranks per GPU
            rpg = max(1, int(os.environ.get("OMNIA_RANKS_PER_GPU", "1") or 1))
            if self.gpu_count is not None and tp > self.gpu_count * rpg:
                model_ok, model_msg = False, f"engine.tp={tp} exceeds {self.gpu_count} GPUs"
            if cfg is not None and cfg.num_heads % tp:
                model_ok, model_msg = False, f"tp={tp} does not divide {cfg.num_heads} heads"
            st["engine"] = {"model": m, "tp": tp, "kvBytesPerToken":
                            cfg.kv_bytes_per_token() // tp if cfg else None}
        set_condition(st, "ModelValid", model_ok, "Valid" if model_ok else "Invalid", model_msg,
                      gen)
        ok = cred_ok and model_ok
        # endpoint liveness (provider_controller.go:135-161): any HTTP response
        # is reachable; a connection failure makes the provider Unavailable
        url = SR.provider_health_url(spec) if cred_ok else ""
        if url:
            err = SR.check_endpoint_health(url, self.cfg)
            if err is not None:
                set_condition(st, "EndpointReachable", False, "EndpointUnreachable",
                              f"health check failed: {err}"[:300], gen)
                st["phase"] = "Unavailable"
                set_condition(st, "Ready", False, "EndpointUnreachable", err[:300], gen)
                st["observedGeneration"] = gen
                pv["status"] = st
                store.update_status(pv)
                return SR.HEALTH_REQUEUE_S
            set_condition(st, "EndpointReachable", True, "EndpointReachable",
                          "health check passed", gen)
        st["phase"] = "Ready" if ok else "Error"
        set_condition(st, "Ready", ok, "Ready" if ok else "NotReady", cred_msg or model_msg, gen)
        st["observedGeneration"] = gen
        pv["status"] = st
        store.update_status(pv)
        return None


# ===================================================================== ToolRegistry
class ToolRegistryReconciler:
    """Validate handlers, resolve endpoints, build ``discoveredTools`` and,
    when ``spec.probe.enabled``, TCP-probe them on an interval
    (``internal/controller/toolregistry_controller.go:55-346``,
    ``toolregistry_probe.go:53-155``).  Phase: Ready (all available) /
    Degraded (some) / Failed (none, or a handler failed validation)."""

    kind = "ToolRegistry"

    def __init__(self, cfg: SR.OperatorConfig | None = None):
        self.cfg = cfg or SR.OperatorConfig.from_env()

    @staticmethod
    def validate_handler(h: dict) -> str | None:
        from ..tools.resilience import RetryPolicy

        t = h.get("type")
        cfgk = {"http": "httpConfig", "grpc": "grpcConfig", "mcp": "mcpConfig",
                "openapi": "openAPIConfig"}.get(t)
        if t not in ("http", "grpc", "mcp", "openapi", "client"):
            return f"unknown handler type: {t}"
        conf = h.get(cfgk) if cfgk else None
        if t in ("http", "grpc") and conf is None and not h.get("endpoint"):
            return f"{cfgk} is required for {t} handlers"
        if t in ("http", "grpc", "client") and not h.get("tool"):
            return f"tool definition is required for {t} handlers"
        if t == "mcp":
            if conf is None and not h.get("endpoint"):
                return "mcpConfig is required for mcp handlers"
            tr = (conf or {}).get("transport", "streamable-http" if h.get("endpoint") else "")
            if tr in ("sse", "streamable-http") and not ((conf or {}).get("endpoint") or
                                                          h.get("endpoint")):
                return f"endpoint is required for mcp handlers with {tr} transport"
            if tr == "stdio" and not (conf or {}).get("command"):
                return "command is required for mcp handlers with stdio transport"
        if t == "openapi" and conf is None:
            return "openAPIConfig is required for openapi handlers"
        auth = h.get("auth") or {}
        if auth.get("type") == "workloadIdentity":
            # resolved by the runtime on network handlers only (auth.go): a type
            # it cannot honor is rejected here, not sent unauthenticated
            w = auth.get("workloadIdentity") or {}
            if (w.get("cloud") or "azure") != "azure":
                return f"workloadIdentity cloud {w.get('cloud')!r} not supported (only 'azure')"
            if t == "client" or (t == "mcp" and (conf or {}).get("transport") == "stdio"):
                return f"workloadIdentity auth is not supported on {t} " \
                       f"{'stdio ' if t == 'mcp' else ''}handlers"
        for rp in [(conf or {}).get("retryPolicy"), h.get("retryPolicy")]:
            if not rp:
                continue
            try:
                p = RetryPolicy.from_cfg(rp)
            except (TypeError, ValueError) as e:
                return f"invalid retryPolicy: {e}"
            if p.max_attempts < 1:
                return "retryPolicy.maxAttempts must be >= 1"
            if p.multiplier < 1:
                return "retryPolicy.backoffMultiplier must be >= 1"
            if p.max_backoff < p.initial_backoff:
                return "retryPolicy.maxBackoff must be >= initialBackoff"
        return None

    @staticmethod
    def resolve_endpoint(h: dict) -> str:
        t = h.get("type")
        conf = h.get({"http": "httpConfig", "grpc": "grpcConfig", "mcp": "mcpConfig",
                      "openapi": "openAPIConfig"}.get(t, ""), None) or {}
        if t in ("http", "grpc"):
            return conf.get("endpoint") or h.get("endpoint", "")
        if t == "mcp":
            if conf.get("endpoint") or h.get("endpoint"):
                return conf.get("endpoint") or h["endpoint"]
            return f"stdio://{conf.get('command', '')}"
        if t == "openapi":
            return conf.get("specURL") or conf.get("baseURL") or h.get("endpoint", "")
        return "client://browser"

    def reconcile(self, store: APIStore, ns: str, name: str):
        tr = store.try_get("ToolRegistry", name, ns)
        if tr is None:
            return None
        st = tr.get("status") or {}
        gen = tr["metadata"]["generation"]
        now = SR._rfc3339(time.time())
        tools, errors = [], []
        for h in tr["spec"].get("handlers", []):
            err = self.validate_handler(h)
            if err:
                errors.append(f"handler {h.get('name')!r}: {err}")
                continue
            ep = self.resolve_endpoint(h)
            t = h.get("tool")
            if t and h["type"] in ("http", "grpc", "client"):
                d = {"name": t["name"], "handlerName": h["name"],
                     "description": t.get("description", ""), "endpoint": ep,
                     "status": "Available", "lastChecked": now}
                if t.get("inputSchema") is not None:
                    d["inputSchema"] = t["inputSchema"]
                if t.get("outputSchema") is not None:
                    d["outputSchema"] = t["outputSchema"]
                tools.append(d)
            else:  # self-describing (mcp / openapi): discovered at runtime
                tools.append({"name": h["name"], "handlerName": h["name"],
                              "description": f"Self-describing {h['type']} handler (tools "
                                             "discovered at runtime)",
                              "endpoint": ep, "status": "Available", "lastChecked": now})
        probe = tr["spec"].get("probe") or {}
        if probe.get("enabled"):
            from ..runtime.context_store import parse_ttl

            SR.probe_tools(tools, float(parse_ttl(probe.get("timeout", "5s")) or
                                        SR.PROBE_TIMEOUT_S), self.cfg.dial)
        st["discoveredTools"] = tools
        st["discoveredToolsCount"] = st["toolCount"] = len(tools)
        st["lastDiscoveryTime"] = now
        avail = sum(1 for t in tools if t["status"] == "Available")
        if errors:
            st["phase"] = "Failed"
            set_condition(st, "HandlersValid", False, "ValidationFailed",
                          f"Handler validation errors: {errors}"[:1000], gen)
        else:
            st["phase"] = "Failed" if not tools or avail == 0 else (
                "Ready" if avail == len(tools) else "Degraded")
            set_condition(st, "HandlersValid", True, "HandlersValid",
                          "All handlers validated successfully", gen)
        set_condition(st, "ToolsDiscovered", True, "ToolsDiscovered",
                      f"Discovered {len(tools)} tool(s) from "
                      f"{len(tr['spec'].get('handlers', []))} handler(s)", gen)
        set_condition(st, "Ready", st["phase"] == "Ready", st["phase"], "", gen)
        st["observedGeneration"] = gen
        tr["status"] = st
        store.update_status(tr)
        if probe.get("enabled"):
            from ..runtime.context_store import parse_ttl

            return float(parse_ttl(probe.get("interval", "60s")) or SR.PROBE_INTERVAL_S)
        return None


# ===================================================================== AgentRuntime
def workspace_service_group(store: APIStore, ns: str, group: str) -> dict | None:
    """The ServiceGroupStatus of the Workspace that owns namespace ``ns``
    (``resolveSessionURLForWorkspace``, ``internal/controller/eval_worker.go:434``)."""
    for ws in store.list("Workspace"):
        if ((ws.get("spec") or {}).get("namespace") or {}).get("name") != ns:
            continue
        for sg in (ws.get("status") or {}).get("services") or []:
            if sg.get("name") == group:
                return {**sg, "_workspace": ws["metadata"]["name"]}
    return None


def resolve_a2a_clients(store, ar: dict) -> tuple[list, list]:
    """``spec.facades[].a2a.clients[]`` -> (resolved ``OMNIA_A2A_CLIENTS`` entries,
    per-client status ``{name, ready, resolvedURL | error}``)
    (``internal/controller/a2a_client_resolver.go``)."""
    from .builders import FACADE_PORT

    md = ar["metadata"]
    out, status = [], []
    for fac in ar["spec"].get("facades") or []:
        for c in ((fac.get("a2a") or {}).get("clients") or []):
            st = {"name": c["name"]}
            url = ""
            ref = c.get("agentRuntimeRef")
            if ref:
                ns = ref.get("namespace") or md["namespace"]
                tgt = store.try_get("AgentRuntime", ref["name"], ns)
                if tgt is None:
                    st.update(ready=False, error=f"AgentRuntime {ns}/{ref['name']} not found")
                    status.append(st)
                    continue
                ep = ((tgt.get("status") or {}).get("a2a") or {}).get("endpoint")
                url = ep or f"http://{ref['name']}.{ns}.svc.cluster.local:{FACADE_PORT}/a2a"
            elif c.get("url"):
                url = c["url"]
            else:
                st.update(ready=False, error="either agentRuntimeRef or url must be specified")
                status.append(st)
                continue
            st.update(ready=True, resolvedURL=url)
            status.append(st)
            rc = {"name": c["name"], "url": url, "exposeAsTools": bool(c.get("exposeAsTools"))}
            if c.get("timeout"):  # one delegated turn (default: the executor's 30 s)
                rc["timeout"] = c["timeout"]
            if (c.get("authentication") or {}).get("secretRef"):
                rc["authTokenEnv"] = "OMNIA_A2A_CLIENT_TOKEN_" + re.sub(
                    r"[^A-Z0-9]", "_", c["name"].upper())
            out.append(rc)
    return out, status


class AgentRuntimeReconciler:
    kind = "AgentRuntime"

    def __init__(self, gpu_count: int | None = None, cfg: SR.OperatorConfig | None = None,
                 rollout_engine=None):
        self.gpu_count = gpu_count
        self.cfg = cfg or SR.OperatorConfig.from_env()
        self.rollout_engine = rollout_engine  # injectable clock / HTTP for tests

    def _fail(self, store, ar, st, cond, reason, msg, phase=PENDING):
        set_condition(st, cond, False, reason, msg, ar["metadata"]["generation"])
        set_condition(st, "Ready", False, reason, msg, ar["metadata"]["generation"])
        st["phase"] = phase
        ar["status"] = st
        store.update_status(ar)
        return 10.0

    def reconcile(self, store: APIStore, ns: str, name: str):
        ar = store.try_get("AgentRuntime", name, ns)
        if ar is None:
            return None
        md = ar["metadata"]
        if md.get("deletionTimestamp"):
            # the departing agent no longer holds its group's eval worker
            SR.reconcile_eval_workers(store, ns, self.cfg)
            md["finalizers"] = [f for f in md.get("finalizers", []) if f != B.FINALIZER]
            store.update(ar)
            return None
        if B.FINALIZER not in md.get("finalizers", []):
            md.setdefault("finalizers", []).append(B.FINALIZER)
            ar = store.update(ar)
        spec = ar["spec"]
        st = ar.get("status") or {}
        st["observedGeneration"] = ar["metadata"]["generation"]
        gen = ar["metadata"]["generation"]
        # ---- references
        pack = resolve_promptpack(store, ns, spec["promptPackRef"])
        if pack is None:
            return self._fail(store, ar, st, "PromptPackReady", "NotFound",
                              f"no PromptPack matches {spec['promptPackRef']}")
        if (pack.get("status") or {}).get("phase") == "Failed":
            return self._fail(store, ar, st, "PromptPackReady", "Invalid",
                              "referenced PromptPack failed validation", FAILED)
        set_condition(st, "PromptPackReady", True, "Resolved", pack["spec"]["version"], gen)
        providers = []
        for pref in spec.get("providers") or []:
            ref = pref.get("providerRef") or {"name": pref.get("name")}
            pns = ref.get("namespace") or ns
            pv = store.try_get("Provider", ref["name"], pns)
            if pv is None:
                return self._fail(store, ar, st, "ProviderReady", "NotFound",
                                  f"Provider {ref['name']} not found")
            if (pv.get("status") or {}).get("phase") != "Ready":
                return self._fail(store, ar, st, "ProviderReady", "NotReady",
                                  f"Provider {ref['name']} is not Ready")
            want_role = pref.get("role")
            if want_role and pv["spec"].get("role", "llm") != want_role:
                return self._fail(store, ar, st, "ProviderReady", "RoleMismatch",
                                  f"Provider {ref['name']} has role "
                                  f"{pv['spec'].get('role', 'llm')}, want {want_role}")
            caps = set(pv["spec"].get("capabilities") or [])
            missing = [c for c in pref.get("requiredCapabilities") or [] if caps and c not in caps]
            if missing:
                return self._fail(store, ar, st, "ProviderReady", "CapabilityMissing",
                                  f"Provider {ref['name']} lacks {missing}")
            providers.append(pv)
        set_condition(st, "ProviderReady", True, "Resolved",
                      ",".join(p["metadata"]["name"] for p in providers) or "mock", gen)
        registry = None
        trr = spec.get("toolRegistryRef")
        if trr:
            if trr.get("namespace") and trr["namespace"] != ns:
                return self._fail(store, ar, st, "ToolRegistryReady", "CrossNamespace",
                                  "cross-namespace ToolRegistry references are not allowed",
                                  FAILED)
            registry = store.try_get("ToolRegistry", trr["name"], ns)
            if registry is None:
                return self._fail(store, ar, st, "ToolRegistryReady", "NotFound",
                                  f"ToolRegistry {trr['name']} not found")
            set_condition(st, "ToolRegistryReady", True, "Resolved", "", gen)
        set_condition(st, "FrameworkReady", True, "Resolved",
                      (spec.get("framework") or {}).get("type", "omnia-mi355x"), gen)
        # ---- capability gate: a local engine needs GPUs on the node
        rc = B.runtime_config(ar, pack, providers, registry)
        # ---- outbound A2A clients (a2a_client_resolver.go): agentRuntimeRef -> the
        # target's service DNS (the node launcher rewrites it to the local endpoint)
        rc.a2a_clients, a2a_status = resolve_a2a_clients(store, ar)
        if a2a_status:
            st["a2a"] = {**(st.get("a2a") or {}), "clients": a2a_status}
        else:
            (st.get("a2a") or {}).pop("clients", None)
        replicas = None
        cap_ok = True
        if rc.provider.get("type") == "local" and self.gpu_count is not None:
            need = int(rc.engine.get("tp", 1))
            if rc.engine.get("ep_mode") == "a2a":  # one rank per GPU of the EP group
                need = max(need, int(rc.engine.get("ep", 1) or 1))
            if need > self.gpu_count and rc.engine.get("device", "cuda") != "cpu":
                cap_ok = False
                replicas = 0
        set_condition(st, "CapabilitiesSatisfied", cap_ok,
                      "CapabilitiesSatisfied" if cap_ok else "CapabilitiesMissing",
                      "" if cap_ok else "insufficient GPUs for the engine's TP/EP group", gen)
        # ---- workspace service group: session-api / memory-api endpoints
        facade_extra = {}
        sg = workspace_service_group(store, ns, spec.get("serviceGroup") or "default")
        if sg is not None:
            if sg.get("sessionURL"):
                rc.session_api_url = sg["sessionURL"]
                facade_extra["OMNIA_SESSION_API_URL"] = sg["sessionURL"]
            if rc.memory_enabled and sg.get("memoryURL"):
                rc.memory_api_url = sg["memoryURL"]
            if not rc.workspace:
                rc.workspace = sg.get("_workspace", "")
        elif spec.get("serviceGroup"):
            set_condition(st, "ServiceGroupReady", False, "NotFound",
                          f"service group {spec['serviceGroup']!r} not found", gen)
        # ---- owned objects
        sa_name = SR.reconcile_facade_rbac(store, ar, self.cfg)
        sidecars = []
        if self.cfg.policy_broker_image:
            sidecars.append(SR.policy_broker_container(ar, self.cfg))
            rc.policy_broker_url = f"http://127.0.0.1:{SR.POLICY_BROKER_PORT}"
        from .policies import compile_tool_access

        store.apply(B.tools_configmap(ar, registry, compile_tool_access(
            store.list("AgentPolicy", ns), name)))
        pack_cm = pack["spec"]["source"].get("configMapRef", {}).get("name", "")
        a = ((spec.get("runtime") or {}).get("autoscaling") or {})
        if a.get("enabled") and replicas is None:
            cur = store.try_get("Deployment", name, ns)
            if cur is not None:
                replicas = cur["spec"].get("replicas")
        dep = B.deployment(ar, rc, pack_cm, "stable", replicas,
                           extra_hash=[pack["spec"]["version"], (registry or {}).get("spec")],
                           facade_extra=facade_extra, sidecars=sidecars, sa_name=sa_name)
        store.apply(dep)
        store.apply(B.service(ar))
        route = SR.reconcile_facade_route(store, ar, self.cfg)
        if route is not None:
            st["externalURL"] = f"https://{route['host']}"
        else:
            st.pop("externalURL", None)
        workers = SR.reconcile_eval_workers(store, ns, self.cfg)
        if (spec.get("evals") or {}).get("enabled"):
            grp = spec.get("serviceGroup") or "default"
            set_condition(st, "EvalWorkerReady", True,
                          "WorkerDeployed" if grp in workers else "InlineEvals",
                          f"arena-eval-worker-{grp}" if grp in workers else
                          "evaluated inline by the runtime", gen)
        jwks_after = SR.reconcile_oidc_jwks(store, ar, st, self.cfg)
        want_r = dep["spec"]["replicas"]
        if want_r and want_r > 1:
            store.apply(B.pdb(ar))
        else:
            store.delete("PodDisruptionBudget", name, ns)
        # autoscaling
        if a.get("enabled"):
            if a.get("type", "hpa") == "keda":
                store.apply(B.scaled_object(ar, a))
                store.delete("HorizontalPodAutoscaler", name, ns)
            else:
                store.apply(B.hpa(ar, a))
                store.delete("ScaledObject", name, ns)
            set_condition(st, "AutoscalingReady", True, "Scaling", a.get("type", "hpa"), gen)
        else:
            store.delete("ScaledObject", name, ns)
            store.delete("HorizontalPodAutoscaler", name, ns)
            set_condition(st, "AutoscalingReady", True, "Disabled", "", gen)
        requeue = self._rollout(store, ar, st, rc, pack_cm, pack)
        # ---- status from the Deployment
        d = store.try_get("Deployment", name, ns) or {}
        ds = d.get("status") or {}
        st["replicas"] = {"desired": d.get("spec", {}).get("replicas", 0),
                          "ready": ds.get("readyReplicas", 0),
                          "available": ds.get("availableReplicas", 0)}
        st["activeVersion"] = pack["spec"]["version"]
        svc = store.try_get("Service", name, ns) or {}
        ep = (svc.get("status") or {}).get("endpoint") or \
            f"{name}.{ns}.svc.cluster.local:{B.FACADE_PORT}"
        st["serviceEndpoint"] = ep
        st["facade"] = {"endpoints": [{"type": f["type"], "url": (
            f"ws://{ep}/ws" if f["type"] == "websocket" else f"http://{ep}")}
            for f in spec.get("facades", [])]}
        me = B.management_endpoints(ar)
        if me:
            st["managementEndpoints"] = me
        else:
            st.pop("managementEndpoints", None)
        dep_ok = st["replicas"]["ready"] > 0
        set_condition(st, "DeploymentReady", dep_ok, "Available" if dep_ok else "Progressing",
                      "", gen)
        set_condition(st, "ServiceReady", bool(svc), "Created", "", gen)
        if not cap_ok:
            st["phase"] = PENDING
        else:
            st["phase"] = RUNNING if dep_ok else PENDING
        set_condition(st, "Ready", dep_ok and cap_ok, "Ready" if dep_ok else "Pending", "", gen)
        ar["status"] = st
        store.update_status(ar)
        if not dep_ok:
            return 2.0
        if jwks_after is not None:
            requeue = min(requeue, jwks_after) if requeue else jwks_after
        return requeue

    # ---------------------------------------------------------------- rollout
    def _rollout(self, store, ar, st, rc, pack_cm, pack):
        """Canary rollout engine (:mod:`.rollout`, ``internal/controller/
        rollout.go:73-851``)."""
        from .rollout import RolloutEngine

        ns = ar["metadata"]["namespace"]
        eng = self.rollout_engine or RolloutEngine()
        return eng.reconcile(store, ar, st, rc, pack,
                             lambda ref: resolve_promptpack(store, ns, ref),
                             lambda pack_name: packs_for(store, ns, pack_name))


# ===================================================================== Workspace
class WorkspaceReconciler:
    """Namespace, service accounts, RBAC, network policy, storage and the
    per-service-group session-api / memory-api (``workspace_services.go``)."""

    kind = "Workspace"

    def reconcile(self, store: APIStore, ns_unused, name: str):
        ws = store.try_get("Workspace", name, None)
        if ws is None:
            return None
        spec, st = ws["spec"], ws.get("status") or {}
        nsname = spec["namespace"]["name"]
        own = [owner_ref(ws)]
        if spec["namespace"].get("create", True):
            store.apply({"apiVersion": "v1", "kind": "Namespace", "metadata": {
                "name": nsname, "labels": {"omnia.altairalabs.ai/workspace": name,
                                           **(spec["namespace"].get("labels") or {})},
                "ownerReferences": own}})
        for role in ("owner", "editor", "viewer"):
            store.apply({"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {
                "name": f"workspace-{name}-{role}-sa", "namespace": nsname,
                "ownerReferences": own}})
        for i, rb in enumerate(spec.get("roleBindings") or []):
            store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                         "metadata": {"name": f"workspace-{name}-{i}", "namespace": nsname,
                                      "ownerReferences": own},
                         "roleRef": {"kind": "ClusterRole",
                                     "name": f"omnia-workspace-{rb.get('role', 'viewer')}"},
                         "subjects": rb.get("groups") or rb.get("subjects") or []})
        np = spec.get("networkPolicy") or {}
        if np.get("isolate"):
            store.apply({"apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
                         "metadata": {"name": f"workspace-{name}-isolation",
                                      "namespace": nsname, "ownerReferences": own},
                         "spec": {"podSelector": {}, "policyTypes": ["Ingress", "Egress"],
                                  "ingress": [{"from": [{"podSelector": {}}] +
                                               (np.get("allowFrom") or [])}],
                                  "egress": [{"to": [{"podSelector": {}}] +
                                              (np.get("allowTo") or [])}]}})
        stor = spec.get("storage") or {}
        if stor.get("enabled"):
            store.apply({"apiVersion": "v1", "kind": "PersistentVolumeClaim",
                         "metadata": {"name": f"workspace-{name}-storage", "namespace": nsname,
                                      "ownerReferences": own},
                         "spec": {"accessModes": stor.get("accessModes", ["ReadWriteMany"]),
                                  "resources": {"requests": {"storage": stor.get("size",
                                                                                 "10Gi")}}}})
        groups = []
        for sg in spec.get("services") or [{"name": "default"}]:
            g = sg.get("name", "default")
            if sg.get("mode") == "external":
                ext = sg.get("external") or {}
                groups.append({"name": g, "sessionURL": ext.get("sessionURL", ""),
                               "memoryURL": ext.get("memoryURL", ""), "ready": True})
                continue
            urls = {}
            ready = True
            for svc in ("session-api", "memory-api"):
                dn = f"{svc}-{name}-{g}"
                cmd, _, _ = COMPONENTS[svc]
                cfg = sg.get("session" if svc == "session-api" else "memory") or {}
                args = list(cmd[3:]) + ["--port", "8080"]
                redis = (cfg.get("redis") or sg.get("redis") or {}).get("url")
                if redis:
                    args += ["--redis-url" if svc == "session-api" else "--redis", redis]
                volumes, mounts = [], []
                pref = (cfg.get("policyRef") or {}).get("name")
                if pref:
                    # the cluster-scoped policy, copied next to the service so the pod
                    # can mount it (the operator's own copy lives in its namespace)
                    pkind = "SessionRetentionPolicy" if svc == "session-api" \
                        else "MemoryPolicy"
                    pol = store.try_get(pkind, pref, None)
                    if pol is not None:
                        if svc == "session-api":
                            from .policies import resolved_retention

                            fname, body = "retention.yaml", yaml.safe_dump(
                                resolved_retention(pol["spec"]), sort_keys=True)
                            args += ["--retention-config", f"/etc/omnia/policy/{fname}"]
                        else:
                            fname, body = "policy.json", json.dumps(pol["spec"],
                                                                    sort_keys=True)
                            args += ["--policy-file", f"/etc/omnia/policy/{fname}"]
                        store.apply({"apiVersion": "v1", "kind": "ConfigMap",
                                     "metadata": {"name": f"{dn}-policy", "namespace": nsname,
                                                  "ownerReferences": own},
                                     "data": {fname: body}})
                        volumes = [{"name": "policy",
                                    "configMap": {"name": f"{dn}-policy"}}]
                        mounts = [{"name": "policy", "mountPath": "/etc/omnia/policy",
                                   "readOnly": True}]
                store.apply({"apiVersion": "apps/v1", "kind": "Deployment",
                             "metadata": {"name": dn, "namespace": nsname,
                                          "labels": {"omnia.altairalabs.ai/component": svc,
                                                     "omnia.altairalabs.ai/service-group": g,
                                                     "omnia.altairalabs.ai/workspace": name},
                                          "ownerReferences": own},
                             "spec": {"replicas": int(cfg.get("replicas", 1)),
                                      "selector": {"matchLabels": {"app": dn}},
                                      "template": {"metadata": {"labels": {"app": dn}},
                                                   "spec": {"containers": [{
                                                       "name": svc, "image": f"omnia-{svc}",
                                                       "command": cmd[:3], "args": args,
                                                       "env": list((cfg.get("podOverrides")
                                                                    or {}).get("extraEnv")
                                                                   or []),
                                                       "ports": [{"name": "http",
                                                                  "containerPort": 8080}],
                                                       "volumeMounts": mounts,
                                                       "readinessProbe": {"httpGet": {
                                                           "path": "/healthz",
                                                           "port": 8080}}}],
                                                       "volumes": volumes}}}})
                store.apply({"apiVersion": "v1", "kind": "Service",
                             "metadata": {"name": dn, "namespace": nsname,
                                          "ownerReferences": own},
                             "spec": {"selector": {"app": dn},
                                      "ports": [{"name": "http", "port": 8080}]}})
                urls[svc] = f"http://{dn}.{nsname}:8080"
                if svc == "session-api":
                    self._compaction_cronjob(store, nsname, name, g, dn, own,
                                             store.try_get("SessionRetentionPolicy", pref, None)
                                             if pref else None)
                dep = store.try_get("Deployment", dn, nsname) or {}
                if not (dep.get("status") or {}).get("readyReplicas"):
                    ready = False
            groups.append({"name": g, "sessionURL": urls["session-api"],
                           "memoryURL": urls["memory-api"], "ready": ready})
        # ServiceGroupStatus list (workspace_types.go:825)
        st["services"] = groups
        st.pop("serviceGroups", None)
        all_ready = all(g["ready"] for g in groups)
        st["namespace"] = nsname
        st["phase"] = "Ready"
        gen = ws["metadata"]["generation"]
        set_condition(st, "Ready", True, "Reconciled", "", gen)
        set_condition(st, "ServicesReady", all_ready,
                      "AllServicesReady" if all_ready else "ServicesPending", "", gen)
        st["observedGeneration"] = gen
        ws["status"] = st
        store.update_status(ws)
        return None if all_ready else 5.0  # re-check service readiness

    @staticmethod
    def _compaction_cronjob(store: APIStore, nsname: str, ws: str, group: str, dn: str, own,
                            policy: dict | None):
        """The service group's session compaction CronJob (the chart's
        ``compaction-cronjob.yaml``, per workspace here): scheduled by the
        SessionRetentionPolicy's ``coldArchive.compactionSchedule`` when its cold
        archive is enabled; each run asks the group's session-api to compact its
        own tiers (``python -m omnia_amd.session.compaction --session-api``)."""
        name = f"compaction-{ws}-{group}"
        cold = ((policy or {}).get("spec") or {}).get("coldArchive") or {}
        if not cold.get("enabled"):
            try:
                store.delete("CronJob", name, nsname)
            except NotFound:
                pass
            return
        labels = {"app.kubernetes.io/component": "compaction",
                  "omnia.altairalabs.ai/workspace": ws,
                  "omnia.altairalabs.ai/service-group": group}
        store.apply({"apiVersion": "batch/v1", "kind": "CronJob",
                     "metadata": {"name": name, "namespace": nsname, "labels": labels,
                                  "ownerReferences": own},
                     "spec": {"schedule": cold.get("compactionSchedule", "0 2 * * *"),
                              "concurrencyPolicy": "Forbid",
                              "successfulJobsHistoryLimit": 3, "failedJobsHistoryLimit": 1,
                              "jobTemplate": {"metadata": {"labels": labels}, "spec": {
                                  "backoffLimit": 2, "template": {"spec": {
                                      "restartPolicy": "Never",
                                      "containers": [{
                                          "name": "compaction", "image": "omnia-compaction",
                                          "command": ["python", "-m",
                                                      "omnia_amd.session.compaction"],
                                          "args": ["--session-api",
                                                   f"http://{dn}.{nsname}:8080"]}]}}}}}})


# ===================================================================== policies
class SimplePolicyReconciler:
    """ToolPolicy (enforced by the policy broker) / SessionPrivacyPolicy /
    RolloutAnalysis / ArenaDevSession: admission already validated; mark Active
    and count.  AgentPolicy / MemoryPolicy / SessionRetentionPolicy have their
    own reconcilers (``operator/policies.py``)."""

    def __init__(self, kind: str):
        self.kind = kind

    def reconcile(self, store: APIStore, ns, name: str):
        ns_eff = ns if crds.KINDS[self.kind].scope == "Namespaced" else None
        o = store.try_get(self.kind, name, ns_eff)
        if o is None:
            return None
        st = o.get("status") or {}
        spec = o["spec"]
        if self.kind == "AgentPolicy":
            agents = set((spec.get("selector") or {}).get("agents") or [])
            ars = store.list("AgentRuntime", ns)
            st["matchedCount"] = sum(1 for a in ars if not agents or
                                     a["metadata"]["name"] in agents)
        if self.kind == "ToolPolicy":
            st["ruleCount"] = len(spec.get("rules") or [])
        if self.kind == "RolloutAnalysis":
            st["metricCount"] = len(spec.get("metrics") or [])
        st["phase"] = "Active"
        set_condition(st, "Ready", True, "Valid", "", o["metadata"]["generation"])
        st["observedGeneration"] = o["metadata"]["generation"]
        o["status"] = st
        store.update_status(o)
        return None


def default_reconcilers(gpu_count: int | None = None,
                        cfg: SR.OperatorConfig | None = None) -> list:
    cfg = cfg or SR.OperatorConfig.from_env()
    rs = [PromptPackReconciler(), ProviderReconciler(gpu_count, cfg),
          ToolRegistryReconciler(cfg), AgentRuntimeReconciler(gpu_count, cfg),
          WorkspaceReconciler()]
    from .policies import (AgentPolicyReconciler, MemoryPolicyReconciler,
                           SessionRetentionPolicyReconciler)

    rs += [AgentPolicyReconciler(cfg.istio), MemoryPolicyReconciler(cfg.namespace),
           SessionRetentionPolicyReconciler(cfg.namespace)]
    from ..ee.controllers import SessionPrivacyPolicyReconciler, ToolPolicyReconciler

    rs += [ToolPolicyReconciler(), SessionPrivacyPolicyReconciler()]
    rs.append(SimplePolicyReconciler("RolloutAnalysis"))
    from ..ee.arena.devsession import ArenaDevSessionReconciler

    rs.append(ArenaDevSessionReconciler())
    from .sourcesync import SourceReconciler

    for k in ("SkillSource", "ArenaSource", "ArenaTemplateSource", "PromptPackSource"):
        rs.append(SourceReconciler(k))
    from ..ee.arena.controller import ArenaJobReconciler

    rs.append(ArenaJobReconciler())
    return rs
