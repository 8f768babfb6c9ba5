"""Canary rollout engine of the AgentRuntime reconciler.

Reference: ``internal/controller/rollout.go:73-851`` (state machine, steps,
auto-rollback on the candidate's progress deadline, rollback / promote),
``rollout_analysis.go:48-345`` (RolloutAnalysis templates, args, metric
providers, ``result[0] <op> <n>`` success conditions), ``rollout_promote.go``
(two-phase promotion), ``rollout_version_trigger.go`` (version-triggered
rollouts), ``rollout_metrics.go`` (Prometheus series), events
``RolloutStep`` / ``RolloutPromoting`` / ``RolloutPromoted`` /
``RolloutRolledBack`` / ``RolloutAnalysisPassed`` / ``RolloutAnalysisFailed`` /
``RolloutTriggered``.

A rollout is active while ``spec.rollout.candidate`` differs from the live
spec (pack name / track / version, provider refs, tool registry).  Each
reconcile:

1. **trigger** -- with ``rollout.trigger.promptPackChannel`` and no rollout in
   flight, the highest version published on that channel (stable excludes
   prereleases) newer than ``status.activeVersion`` -- and newer than the last
   rolled-back version -- becomes the candidate (spec update + event);
2. **candidate Deployment** (track ``candidate``) with the candidate's pack,
   providers and registry;
3. **auto-rollback** (``rollback.mode: automatic``) when the candidate misses
   its progress deadline (the Deployment's ``Progressing=False /
   ProgressDeadlineExceeded`` condition, or not ready within
   ``progressDeadlineSeconds`` of creation where no controller sets it);
4. **steps** from ``status.rollout.currentStep``: ``setWeight`` (route, advance,
   event), ``pause`` (timed: requeue for the remainder; no duration: hold until
   the user edits the spec), ``analysis`` (run the RolloutAnalysis now: pass ->
   advance, fail -> automatic rollback or a manual hold with condition
   ``AnalysisFailed``, provider error -> retry in 30 s);
5. after the last step, **two-phase promotion**: the candidate's refs move into
   the live spec and traffic goes 100 % to the candidate while the stable
   Deployment rolls to the new config (``promoting``), then routing resets,
   the candidate Deployment and ``spec.rollout.candidate`` are removed.

Rollback copies the live refs back into the candidate (so it no longer
differs), records ``omnia.altairalabs.ai/last-rolled-back-version`` and removes
the candidate Deployment.

Analysis metric providers: ``prometheus`` ({address, query}: instant query,
first sample of a vector or a scalar), ``web`` ({url, jsonPath, headers}: a
JSON document's value at a dotted path) and ``arenaEval`` ({workspace,
evalDef}: the eval's pass rate); ``{{args.NAME}}`` is substituted from the
template's ``args`` overridden by the step's.  Each metric takes ``count``
measurements ``interval`` apart (progress kept in the rollout status across
reconciles); a measurement fails when ``failureCondition`` holds or
``successCondition`` does not, and the metric fails past ``failureLimit``.
"""
from __future__ import annotations

import json
import logging
import math
import re
import calendar
import time
import urllib.parse
import urllib.request

from ..observability import metrics as M
from . import builders as B
from . import rollout_routing
from .apistore import Conflict, set_condition

log = logging.getLogger("omnia.operator.rollout")

LAST_ROLLED_BACK = "omnia.altairalabs.ai/last-rolled-back-version"
DEFAULT_PROGRESS_DEADLINE_S = 600
ANALYSIS_RETRY_S = 30.0
PROMOTE_POLL_S = 5.0
_COND = re.compile(r"^result(?:\[0\])?\s*(>=|<=|==|!=|>|<)\s*(-?[\d.]+(?:e-?\d+)?)$")


class AnalysisError(RuntimeError):
    pass


# ------------------------------------------------------------------ versions
def _ver(v: str):
    m = re.match(r"^v?(\d+)\.(\d+)\.(\d+)(?:-([0-9A-Za-z.-]+))?", v or "")
    if not m:
        return None
    pre = m.group(4)
    # a release sorts above its prereleases
    return (int(m.group(1)), int(m.group(2)), int(m.group(3)), pre is None,
            tuple(int(p) if p.isdigit() else p for p in (pre or "").split(".")) if pre else ())


def version_newer(a: str, b: str) -> bool:
    va, vb = _ver(a), _ver(b)
    if va is None or vb is None:
        return False
    try:
        return va > vb
    except TypeError:  # mixed numeric / text prerelease identifiers
        return str(va) > str(vb)


def channel_max(packs: list[dict], channel: str) -> dict | None:
    best = None
    for p in packs:
        v = _ver(p["spec"].get("version", ""))
        if v is None or (channel in ("", "stable") and not v[3]):
            continue
        if best is None or version_newer(p["spec"]["version"], best["spec"]["version"]):
            best = p
    return best


# ------------------------------------------------------------------ candidate
def _track(ref: dict) -> str:
    return ref.get("track") or "stable"


def pack_ref_differs(c: dict, spec: dict) -> bool:
    ref = c.get("promptPackRef")
    if not ref:
        return False
    live = spec["promptPackRef"]
    return (ref.get("name") != live.get("name") or _track(ref) != _track(live) or
            (ref.get("version") or "").lstrip("v") != (live.get("version") or "").lstrip("v"))


def provider_refs_differ(c: dict, spec: dict) -> bool:
    cand = c.get("providerRefs") or []
    if not cand:
        return False
    live = {p.get("name"): (p.get("providerRef") or {}).get("name")
            for p in spec.get("providers") or []}
    return len(cand) != len(live) or any(
        live.get(p.get("name"), object()) != (p.get("providerRef") or {}).get("name")
        for p in cand)


def registry_differs(c: dict, spec: dict) -> bool:
    ref = c.get("toolRegistryRef")
    if not ref:
        return False
    return (spec.get("toolRegistryRef") or {}).get("name") != ref.get("name")


def candidate_differs(spec: dict) -> bool:
    c = (spec.get("rollout") or {}).get("candidate")
    if not c:
        return False
    return pack_ref_differs(c, spec) or provider_refs_differ(c, spec) or \
        registry_differs(c, spec)


def candidate_version(spec: dict) -> str:
    ref = ((spec.get("rollout") or {}).get("candidate") or {}).get("promptPackRef") or {}
    return ref.get("version") or ref.get("track") or ref.get("name") or ""


def apply_candidate(spec: dict) -> dict:
    """The AgentRuntime spec the candidate track runs (and promotion installs)."""
    out = json.loads(json.dumps(spec))
    c = (spec.get("rollout") or {}).get("candidate") or {}
    if c.get("promptPackRef"):
        out["promptPackRef"] = dict(c["promptPackRef"])
    if c.get("providerRefs"):
        out["providers"] = [dict(p) for p in c["providerRefs"]]
    if c.get("toolRegistryRef"):
        out["toolRegistryRef"] = dict(c["toolRegistryRef"])
    return out


# ------------------------------------------------------------------ analysis
def substitute_args(text: str, args: dict) -> str:
    for k, v in args.items():
        text = text.replace("{{args." + k + "}}", str(v))
    return text


def evaluate_condition(cond: str, value: float) -> bool:
    m = _COND.match(cond.strip())
    if not m:
        raise AnalysisError(f'invalid condition format: {cond!r} (expected "result[0] <op> '
                            f'<number>")')
    op, thr = m.group(1), float(m.group(2))
    return {">=": value >= thr, "<=": value <= thr, ">": value > thr, "<": value < thr,
            "==": value == thr, "!=": value != thr}[op]


def _http_json(url: str, headers: dict | None = None, timeout: float = 10.0):
    req = urllib.request.Request(url, headers=headers or {})
    with urllib.request.urlopen(req, timeout=timeout) as r:  # noqa: S310 - template URL
        return json.loads(r.read() or b"null")


def query_prometheus(address: str, query: str, http_json=_http_json) -> float:
    doc = http_json(address.rstrip("/") + "/api/v1/query?" +
                    urllib.parse.urlencode({"query": query}))
    if (doc or {}).get("status") != "success":
        raise AnalysisError(f"prometheus: {(doc or {}).get('error', 'query failed')}")
    data = doc["data"]
    if data["resultType"] == "vector":
        if not data["result"]:
            raise AnalysisError("empty vector result")
        return float(data["result"][0]["value"][1])
    if data["resultType"] == "scalar":
        return float(data["result"][1])
    raise AnalysisError(f"unsupported result type: {data['resultType']}")


def query_web(url: str, json_path: str, headers: dict | None = None,
              http_json=_http_json) -> float:
    cur = http_json(url, headers)
    for part in [p for p in (json_path or "").lstrip("$").split(".") if p]:
        m = re.match(r"^(\w+)?(?:\[(\d+)\])?$", part)
        if not m:
            raise AnalysisError(f"unsupported jsonPath segment {part!r}")
        if m.group(1):
            cur = cur[m.group(1)]
        if m.group(2) is not None:
            cur = cur[int(m.group(2))]
    return float(cur)


def measure(metric: dict, args: dict, http_json=_http_json, eval_lookup=None) -> float:
    """One measurement of a metric's provider."""
    name = metric.get("name") or "?"
    prov = metric.get("provider") or {}
    try:
        if "prometheus" in prov:
            p = prov["prometheus"]
            if not p.get("address") or not p.get("query"):
                raise AnalysisError(f"metric {name!r}: prometheus address and query are "
                                    f"required")
            return query_prometheus(p["address"], substitute_args(p["query"], args), http_json)
        if "web" in prov:
            w = prov["web"]
            return query_web(substitute_args(w["url"], args), w.get("jsonPath", ""),
                             w.get("headers"), http_json)
        if "arenaEval" in prov:
            if eval_lookup is None:
                raise AnalysisError(f"metric {name!r}: no session-api to read eval results "
                                    f"from")
            ae = prov["arenaEval"]
            return float(eval_lookup(ae["workspace"], substitute_args(ae["evalDef"], args)))
    except AnalysisError:
        raise
    except Exception as e:  # noqa: BLE001 - transport / parse failures
        raise AnalysisError(f"metric {name!r}: {e}") from e
    raise AnalysisError(f"metric {name!r}: provider must be prometheus, web or arenaEval")


def measurement_failed(metric: dict, value: float) -> bool:
    cond = metric.get("successCondition")
    if not cond:
        raise AnalysisError(f"metric {metric.get('name')!r} missing successCondition")
    if metric.get("failureCondition") and evaluate_condition(metric["failureCondition"], value):
        return True
    return not evaluate_condition(cond, value)


def run_analysis(template: dict, step: dict, http_json=_http_json, eval_lookup=None,
                 state: dict | None = None, now: float | None = None):
    """Advance an analysis run.  ``state`` (kept in the rollout status between
    reconciles) holds each metric's measurements; a metric takes ``count``
    (default 1) measurements ``interval`` apart, and fails when more than
    ``failureLimit`` of them fail.  Returns ``(verdict, message, wait_s)``:
    verdict True / False once every metric has all its measurements, else None
    with the seconds until the next measurement is due.  Raises AnalysisError
    on a provider / template error."""
    from .policies import PolicyInvalid, parse_duration

    now = time.time() if now is None else now
    state = {} if state is None else state
    spec = template.get("spec") or {}
    args = {a["name"]: a.get("value", "") for a in spec.get("args") or [] if a.get("name")}
    args.update({a["name"]: a.get("value", "") for a in step.get("args") or []})
    metrics = spec.get("metrics") or []
    if not metrics:
        raise AnalysisError("RolloutAnalysis has no metrics")
    wait, failed, done = None, [], True
    for m in metrics:
        name = m.get("name") or "?"
        count = int(m.get("count") or 1)
        try:
            interval = parse_duration(m["interval"]) if m.get("interval") else 0.0
        except PolicyInvalid as e:
            raise AnalysisError(f"metric {name!r}: {e}") from None
        ms = state.setdefault(name, {"values": [], "failures": 0, "last": None})
        if len(ms["values"]) < count and (ms["last"] is None or
                                          now - ms["last"] >= interval):
            v = measure(m, args, http_json, eval_lookup)
            ms["values"].append(v)
            ms["failures"] += int(measurement_failed(m, v))
            ms["last"] = now
        if len(ms["values"]) < count:
            done = False
            due = interval - (now - ms["last"])
            wait = due if wait is None else min(wait, due)
        if ms["failures"] > int(m.get("failureLimit") or 0):
            failed.append(name)
    if failed:  # a metric past its failure limit fails the run at once
        return False, "failed metrics: " + ", ".join(failed), None
    if not done:
        return None, "measuring", max(1.0, wait or 1.0)
    return True, "all metrics passed", None


# ------------------------------------------------------------------ engine
def _event(store, ar: dict, reason: str, message: str, warning: bool = False):
    md = ar["metadata"]
    try:
        store.create({"apiVersion": "v1", "kind": "Event",
                      "metadata": {"generateName": f"{md['name']}.", "namespace":
                                   md["namespace"]},
                      "involvedObject": {"apiVersion": ar.get("apiVersion", ""),
                                         "kind": "AgentRuntime", "name": md["name"],
                                         "namespace": md["namespace"], "uid": md.get("uid", "")},
                      "reason": reason, "message": message,
                      "type": "Warning" if warning else "Normal",
                      "source": {"component": "omnia-operator"},
                      "firstTimestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())})
    except Exception as e:  # noqa: BLE001 - events are best effort
        log.debug("event %s not recorded: %s", reason, e)


def _ts(t: float) -> str:
    """RFC 3339 with microseconds (metav1.MicroTime form): a pause measured from a
    second-truncated start could end up to a second early."""
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + f".{int(t % 1 * 1e6):06d}Z"


def _parse_ts(s: str | None) -> float | None:
    if not s:
        return None
    try:
        base, _, frac = s.rstrip("Z").partition(".")
        return float(calendar.timegm(time.strptime(base, "%Y-%m-%dT%H:%M:%S"))) + \
            (float("0." + frac) if frac else 0.0)
    except (TypeError, ValueError):
        return None


def progress_deadline_exceeded(dep: dict | None, now: float) -> bool:
    if dep is None:
        return False
    for c in (dep.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Progressing" and c.get("status") == "False" and \
                c.get("reason") == "ProgressDeadlineExceeded":
            return True
    st = dep.get("status") or {}
    if st.get("readyReplicas"):
        return False
    created = _parse_ts(dep["metadata"].get("creationTimestamp"))
    limit = dep["spec"].get("progressDeadlineSeconds", DEFAULT_PROGRESS_DEADLINE_S)
    return created is not None and now - created > limit


def deployment_complete(dep: dict | None) -> bool:
    if dep is None:
        return False
    st, spec = dep.get("status") or {}, dep.get("spec") or {}
    want = spec.get("replicas", 1)
    return (st.get("readyReplicas", 0) >= want and st.get("updatedReplicas", want) >= want and
            st.get("observedGeneration", dep["metadata"].get("generation", 0)) >=
            dep["metadata"].get("generation", 0))


class RolloutEngine:
    """Runs inside AgentRuntimeReconciler.reconcile (after the stable objects)."""

    def __init__(self, http_json=_http_json, clock=time.time, mesh=None, eval_lookup=None):
        self.http_json = http_json
        self.clock = clock
        self.mesh = mesh
        # (workspace, evalDef) -> pass rate, for arenaEval metrics (session-api
        # eval aggregates); None: arenaEval metrics are an analysis error
        self.eval_lookup = eval_lookup

    # ------------------------------------------------------------ spec writes
    def _write_spec(self, store, ar: dict, mutate) -> dict:
        """Mutate the live spec (fresh read, retried on conflict); ``ar`` follows."""
        md = ar["metadata"]
        for _ in range(5):
            cur = store.get("AgentRuntime", md["name"], md["namespace"])
            mutate(cur)
            try:
                new = store.update(cur)
            except Conflict:
                continue
            ar["spec"] = new["spec"]
            ar["metadata"] = new["metadata"]
            return new
        raise Conflict("rollout spec update kept conflicting")

    # ------------------------------------------------------------ pieces
    def maybe_trigger(self, store, ar: dict, st: dict, packs_for) -> bool:
        spec = ar["spec"]
        trig = (spec.get("rollout") or {}).get("trigger") or {}
        ro = st.get("rollout") or {}
        if not trig or candidate_differs(spec) or ro.get("promoting"):
            return False
        active = st.get("activeVersion")
        if not active:
            return False  # first deploy: let stable come up, no canary
        latest = channel_max(packs_for(spec["promptPackRef"]["name"]),
                             trig.get("promptPackChannel", "stable"))
        if latest is None or not version_newer(latest["spec"]["version"], active):
            return False
        lrb = (ar["metadata"].get("annotations") or {}).get(LAST_ROLLED_BACK)
        if lrb and not version_newer(latest["spec"]["version"], lrb):
            return False  # just rolled back: wait for a strictly newer version
        ver = latest["spec"]["version"]

        def m(cur):
            cur["spec"]["rollout"]["candidate"] = {"promptPackRef": {
                "name": cur["spec"]["promptPackRef"]["name"], "version": ver}}
        self._write_spec(store, ar, m)
        _event(store, ar, "RolloutTriggered",
               f"version-triggered rollout: candidate {spec['promptPackRef']['name']}@{ver} "
               f"(channel {trig.get('promptPackChannel', 'stable')})")
        return True

    def rollback(self, store, ar: dict, st: dict, reason: str, message: str):
        def m(cur):
            c = cur["spec"]["rollout"].get("candidate") or {}
            ver = (c.get("promptPackRef") or {}).get("version")
            if ver:
                cur["metadata"].setdefault("annotations", {})[LAST_ROLLED_BACK] = ver
            c["promptPackRef"] = dict(cur["spec"]["promptPackRef"])
            c["providerRefs"] = [dict(p) for p in cur["spec"].get("providers") or []] or None
            if c["providerRefs"] is None:
                c.pop("providerRefs")
            if cur["spec"].get("toolRegistryRef"):
                c["toolRegistryRef"] = dict(cur["spec"]["toolRegistryRef"])
            else:
                c.pop("toolRegistryRef", None)
            cur["spec"]["rollout"]["candidate"] = c
        self._write_spec(store, ar, m)
        md = ar["metadata"]
        store.delete("Deployment", md["name"] + "-candidate", md["namespace"])
        st["rollout"] = {"active": False, "message": "auto-rollback: " + message,
                         "traffic": rollout_routing.apply(store, ar, 0, False)}
        M.ROLLOUT_ROLLBACKS.labels(md["namespace"], md["name"], reason).inc()
        M.ROLLOUT_WEIGHT.labels(md["namespace"], md["name"], "canary").set(0)
        M.ROLLOUT_WEIGHT.labels(md["namespace"], md["name"], "stable").set(100)
        _event(store, ar, "RolloutRolledBack", "auto-rollback: " + message, warning=True)
        set_condition(st, "RolloutActive", False, "NoActiveRollout",
                      f"auto-rollback triggered: {reason.replace('_', ' ')}",
                      md.get("generation", 1))

    # ------------------------------------------------------------ main
    def reconcile(self, store, ar: dict, st: dict, rc, pack: dict, resolve_pack,
                  packs_for) -> float | None:
        md, now = ar["metadata"], self.clock()
        ns, name, gen = md["namespace"], md["name"], md.get("generation", 1)
        if self.maybe_trigger(store, ar, st, packs_for):
            gen = ar["metadata"].get("generation", gen)
        spec = ar["spec"]
        ro_spec = spec.get("rollout") or {}
        ro = dict(st.get("rollout") or {})
        if ro.get("promoting"):
            return self._advance_promotion(store, ar, st)
        if not candidate_differs(spec):
            store.delete("Deployment", name + "-candidate", ns)
            M.ROLLOUT_ACTIVE.labels(ns, name).set(0)
            if ro.get("active"):
                ro["active"] = False
            traffic = rollout_routing.apply(store, ar, 0, False) if ro_spec else None
            if ro:
                ro.pop("currentStep", None)
                if traffic:
                    ro["traffic"] = traffic
                st["rollout"] = ro
            set_condition(st, "RolloutActive", False, "NoActiveRollout", ro.get("message", ""),
                          gen)
            return None
        M.ROLLOUT_ACTIVE.labels(ns, name).set(1)
        cand_spec = apply_candidate(spec)
        cand_ar = dict(ar, spec=cand_spec)
        cand_pack = resolve_pack(cand_spec["promptPackRef"]) or pack
        dep = B.deployment(cand_ar, rc, cand_pack["spec"]["source"]["configMapRef"]["name"],
                           "candidate", 1, extra_hash=[cand_pack["spec"]["version"]])
        dep["spec"].setdefault("progressDeadlineSeconds", DEFAULT_PROGRESS_DEADLINE_S)
        store.apply(dep)
        cand_dep = store.try_get("Deployment", name + "-candidate", ns)
        if (ro_spec.get("rollback") or {}).get("mode") == "automatic" and \
                progress_deadline_exceeded(cand_dep, now):
            self.rollback(store, ar, st, "pod_unhealthy", "pod unhealthy (progress deadline "
                                                          "exceeded)")
            return None
        steps = ro_spec.get("steps") or [{"setWeight": 100}]
        i = int(ro.get("currentStep", 0)) if ro.get("active") else 0
        if not ro.get("active"):
            ro = {"active": True, "currentStep": 0, "startedAt": _ts(now),
                  "stepStartedAt": _ts(now), "currentWeight": 0}
            _event(store, ar, "RolloutStep", f"rollout started: candidate "
                                              f"{candidate_version(spec)}")
        ro.update(stableVersion=st.get("activeVersion", ""),
                  candidateVersion=candidate_version(spec))
        requeue = None
        while True:  # consecutive instant steps (setWeight) run in one reconcile
            if i >= len(steps):
                st["rollout"] = ro
                return self._enter_promotion(store, ar, st)
            step = steps[i]
            if "setWeight" in step:
                ro["currentWeight"] = int(step["setWeight"])
                msg = f"step {i}: setWeight {step['setWeight']}"
                _event(store, ar, "RolloutStep", msg)
                M.ROLLOUT_STEPS.labels(ns, name, "setWeight").inc()
                i += 1
                ro.update(currentStep=i, stepStartedAt=_ts(now), message=msg)
                continue
            if "pause" in step:
                dur = (step.get("pause") or {}).get("duration")
                if not dur:
                    ro["message"] = f"step {i}: paused indefinitely"
                    break
                from .policies import PolicyInvalid, parse_duration

                try:
                    d = parse_duration(dur)
                except PolicyInvalid:
                    ro["message"] = f"step {i}: invalid pause duration {dur!r}"
                    break
                started = _parse_ts(ro.get("stepStartedAt")) or now
                if now - started < d:
                    ro["message"] = f"step {i}: pause {dur}"
                    requeue = max(1.0, d - (now - started))
                    break
                msg = f"step {i}: pause {dur} elapsed"
                M.ROLLOUT_STEPS.labels(ns, name, "pause").inc()
                i += 1
                ro.update(currentStep=i, stepStartedAt=_ts(now), message=msg)
                continue
            if "analysis" in step:
                a = step["analysis"] or {}
                tpl = store.try_get("RolloutAnalysis", a.get("templateName", ""), ns)
                run_state = ro.setdefault("analysisRun", {"step": i, "metrics": {}})
                if run_state.get("step") != i:
                    run_state.clear()
                    run_state.update(step=i, metrics={})
                try:
                    if tpl is None:
                        raise AnalysisError(f"RolloutAnalysis {a.get('templateName')!r} not "
                                            f"found")
                    passed, msg, wait = run_analysis(tpl, a, self.http_json, self.eval_lookup,
                                                     run_state["metrics"], now)
                except AnalysisError as e:
                    ro["message"] = f"step {i}: analysis {a.get('templateName')} error: {e}"
                    requeue = ANALYSIS_RETRY_S
                    break
                if passed is None:
                    ro["message"] = f"step {i}: analysis {a.get('templateName')} measuring"
                    requeue = wait
                    break
                ro.pop("analysisRun", None)
                M.ROLLOUT_ANALYSIS.labels(ns, name, a.get("templateName", ""),
                                          "pass" if passed else "fail").inc()
                if passed:
                    _event(store, ar, "RolloutAnalysisPassed",
                           f"analysis {a.get('templateName')} passed")
                    i += 1
                    ro.update(currentStep=i, stepStartedAt=_ts(now),
                              message=f"analysis {a.get('templateName')} passed")
                    continue
                if (ro_spec.get("rollback") or {}).get("mode") == "automatic":
                    self.rollback(store, ar, st, "analysis_failed", "analysis failed: " + msg)
                    return None
                ro["message"] = "analysis failed: " + msg
                _event(store, ar, "RolloutAnalysisFailed",
                       "analysis failed (manual intervention required): " + msg, warning=True)
                set_condition(st, "RolloutActive", True, "AnalysisFailed", ro["message"], gen)
                st["rollout"] = self._route(store, ar, ro)
                return ANALYSIS_RETRY_S
            ro["message"] = f"step {i}: unknown step type"
            break
        st["rollout"] = self._route(store, ar, ro)
        set_condition(st, "RolloutActive", True, "RolloutInProgress", ro.get("message", ""), gen)
        return requeue if requeue is not None else None

    def _route(self, store, ar, ro: dict) -> dict:
        md = ar["metadata"]
        w = int(ro.get("currentWeight", 0))
        traffic = rollout_routing.apply(store, ar, w, True)
        ro["traffic"] = traffic
        ro["trafficRoutingMode"] = traffic["trafficRoutingMode"]
        ro["trafficWeightEnforced"] = not traffic.get("degraded")
        if traffic["trafficRoutingMode"] == "replica-weighted":
            cand = store.try_get("Deployment", md["name"] + "-candidate", md["namespace"])
            if cand is not None and cand["spec"].get("replicas") != traffic["candidateReplicas"]:
                cand["spec"]["replicas"] = max(1, traffic["candidateReplicas"])
                store.apply(cand)
        M.ROLLOUT_WEIGHT.labels(md["namespace"], md["name"], "canary").set(w)
        M.ROLLOUT_WEIGHT.labels(md["namespace"], md["name"], "stable").set(100 - w)
        return ro

    def _enter_promotion(self, store, ar: dict, st: dict) -> float:
        md = ar["metadata"]

        def m(cur):
            cur["spec"].update({k: v for k, v in apply_candidate(cur["spec"]).items()
                                if k in ("promptPackRef", "providers", "toolRegistryRef")})
        self._write_spec(store, ar, m)
        ro = st.get("rollout") or {}
        ro.update(active=True, promoting=True, currentWeight=100,
                  message="promoting: waiting for stable to roll to the new config")
        st["rollout"] = self._route(store, ar, ro)
        M.ROLLOUT_PROMOTIONS.labels(md["namespace"], md["name"]).inc()
        set_condition(st, "RolloutActive", True, "Promoting",
                      "promotion in progress: stable rolling to new config, candidate still "
                      "serving", md.get("generation", 1))
        _event(store, ar, "RolloutPromoting", "promotion started: stable rolling to the new "
                                              "config, candidate still serving 100%")
        return PROMOTE_POLL_S

    def _advance_promotion(self, store, ar: dict, st: dict) -> float | None:
        md = ar["metadata"]
        stable = store.try_get("Deployment", md["name"], md["namespace"])
        if not deployment_complete(stable):
            st["rollout"] = self._route(store, ar, st["rollout"])
            return PROMOTE_POLL_S

        def m(cur):
            cur["spec"]["rollout"].pop("candidate", None)
        self._write_spec(store, ar, m)
        store.delete("Deployment", md["name"] + "-candidate", md["namespace"])
        traffic = rollout_routing.apply(store, ar, 0, False)
        st["rollout"] = {"active": False, "message": "promoted", "traffic": traffic,
                         "promotedVersion": ((ar["spec"].get("promptPackRef") or {})
                                             .get("version") or st.get("activeVersion", ""))}
        M.ROLLOUT_WEIGHT.labels(md["namespace"], md["name"], "canary").set(0)
        M.ROLLOUT_WEIGHT.labels(md["namespace"], md["name"], "stable").set(100)
        set_condition(st, "RolloutActive", False, "NoActiveRollout",
                      "rollout promoted successfully", md.get("generation", 1))
        _event(store, ar, "RolloutPromoted", "promotion complete: stable healthy on the new "
                                             "config, traffic cut over, candidate removed")
        return None


_ = math  # (replica math lives in rollout_routing)
