"""ArenaJob reconciler (``ee/internal/controller/arenajob_controller.go``).

Pending job -> resolve its ArenaSource (inline ``spec.config`` or ConfigMap-like
data), partition scenarios x providers x trials into work items, enqueue, start
``workers.replicas`` worker tasks ("pods" in single-node mode), then aggregate
results, evaluate ``loadTest.thresholds`` and write ``status``
(phase Running -> Succeeded / Failed, progress, per-metric verdicts)."""
from __future__ import annotations

import asyncio
import os
import json
import logging
import time

import yaml

from ...operator.apistore import set_condition
from .profile import LoadProfile
from .queue import WorkItem
from .aggregate import aggregate, to_job_result
from .stats import JobStats, evaluate
from .worker import ArenaWorker

log = logging.getLogger("omnia.arena.controller")


def partition(job_name: str, scenarios: dict, providers: dict, trials: int = 1) -> list:
    return [WorkItem(job_id=job_name, scenario_id=s, provider_id=p, config={"trial": t})
            for t in range(max(1, trials)) for s in scenarios for p in providers]


def load_arena_config(store, job: dict) -> dict:
    spec = job["spec"]
    ns = job["metadata"].get("namespace", "default")
    src = store.get("ArenaSource", spec["sourceRef"]["name"], ns)
    sspec = src.get("spec", {})
    fname = spec.get("arenaFile") or "config.arena.yaml"
    if sspec.get("type") == "configmap":
        cm = store.get("ConfigMap", sspec["configMap"]["name"], ns)
        return yaml.safe_load((cm.get("data") or {}).get(fname, "")) or {}
    # git / oci / workspace sources are materialised on disk by the source syncer
    path = (src.get("status") or {}).get("artifact", {}).get("path")
    if not path:
        raise RuntimeError(f"ArenaSource {ns}/{src['metadata']['name']} has no synced artifact")
    import os

    with open(os.path.join(path, fname)) as f:
        return yaml.safe_load(f) or {}


class JobInvalid(ValueError):
    """The job cannot run as specified (license limits, missing provider groups)."""


def select_scenarios(scenarios: dict, sel: dict | None) -> dict:
    """``spec.scenarios.include`` / ``exclude`` glob patterns over scenario ids."""
    import fnmatch

    sel = sel or {}
    inc, exc = sel.get("include") or ["*"], sel.get("exclude") or []
    return {k: v for k, v in scenarios.items()
            if any(fnmatch.fnmatchcase(k, p) for p in inc)
            and not any(fnmatch.fnmatchcase(k, p) for p in exc)}


def required_provider_groups(cfg: dict) -> list[str]:
    """Provider groups the arena config needs (``arena_config_validation.go``):
    every provider's ``group`` (default "default") plus self-play role providers."""
    groups = {(p.get("group") or "default") for p in cfg.get("providers", [])}
    sp = cfg.get("self_play") or {}
    if sp.get("enabled"):
        groups |= {r["provider"] for r in sp.get("roles") or [] if r.get("provider")}
    return sorted(groups)


def validate_job(spec: dict, cfg: dict, scenarios: dict, lic=None, source_type: str = ""):
    """License gates and provider-group coverage; raises :class:`JobInvalid`."""
    errs = []
    if lic is not None:
        jt = spec.get("type", "evaluation")
        if not lic.can_use_job_type(jt):
            errs.append(f"job type {jt!r} requires an enterprise license")
        reps = int((spec.get("workers") or {}).get("replicas") or 1)
        if not lic.can_use_worker_replicas(reps):
            errs.append(f"{reps} worker replicas exceed the license limit "
                        f"({lic.limits.maxWorkerReplicas})")
        if not lic.can_use_scenario_count(len(scenarios)):
            errs.append(f"{len(scenarios)} scenarios exceed the license limit "
                        f"({lic.limits.maxScenarios})")
        if source_type and not lic.can_use_source_type(source_type) and \
                source_type != "workspace":
            errs.append(f"source type {source_type!r} requires an enterprise license")
        if spec.get("schedule") and not lic.can_use_scheduling():
            errs.append("scheduled jobs require an enterprise license")
    pg = spec.get("providers")
    if pg:
        need = required_provider_groups(cfg)
        missing = [g for g in need if not pg.get(g)]
        if missing:
            errs.append(f"arena config needs provider groups {', '.join(need)}; "
                        f"missing in spec.providers: {', '.join(missing)}")
    if not scenarios:
        errs.append("no scenarios selected")
    if errs:
        raise JobInvalid("; ".join(errs))


def check_budget(limit, currency: str, total_cost: float) -> dict:
    """``budget.go`` ``checkBudget``: result details when the job's total cost
    exceeds ``loadTest.budgetLimit`` (the workers also stop claiming work once
    their share is spent); {} otherwise or when no / an unparsable limit is set."""
    try:
        lim = float(limit) if limit not in (None, "") else None
    except (TypeError, ValueError):
        lim = None
    if lim is None or total_cost <= lim:
        return {}
    return {"budgetBreached": "true", "totalCost": f"{total_cost:.2f}",
            "budgetLimit": f"{lim:.2f}", "budgetCurrency": currency}


def output_location(output: dict | None) -> dict | None:
    """``spec.output`` (``ee/api/v1alpha1/arenajob_types.go:197-257``) -> where a
    job's artefacts go: ``pvc`` = ``<OMNIA_PVC_ROOT>/<claimName>/<subPath>`` (the
    claim's mount point on this node), ``s3`` = bucket + prefix (+ endpoint)."""
    import os

    if not output:
        return None
    if output.get("type") == "pvc":
        pvc = output.get("pvc") or {}
        root = os.environ.get("OMNIA_PVC_ROOT", "/var/lib/omnia/pvc")
        return {"type": "pvc", "path": os.path.join(root, pvc.get("claimName", ""),
                                                     pvc.get("subPath", ""))}
    if output.get("type") == "s3":
        return {"type": "s3", **(output.get("s3") or {})}
    return None


def put_s3_object(loc: dict, key: str, body: bytes, creds: dict) -> str:
    """PUT ``body`` at ``s3://bucket/prefix/key`` with a SigV4-presigned URL
    (``media.sigv4_presign``); a custom ``endpoint`` (MinIO, Ceph) is path-style."""
    import urllib.parse
    import urllib.request

    from ...media import sigv4_presign

    ep = loc.get("endpoint") or ""
    prefix = (loc.get("prefix") or "").strip("/")
    obj = "/".join(p for p in (prefix, key) if p)
    if ep:
        u = urllib.parse.urlsplit(ep if "://" in ep else "https://" + ep)
        host, scheme, path = u.netloc, u.scheme, f"/{loc['bucket']}/{obj}"
    else:
        host = f"{loc['bucket']}.s3.{loc.get('region') or 'us-east-1'}.amazonaws.com"
        scheme, path = "https", f"/{obj}"
    url = sigv4_presign("PUT", host, path, loc.get("region") or "us-east-1", "s3",
                        creds.get("access_key", ""), creds.get("secret_key", ""),
                        scheme=scheme)
    req = urllib.request.Request(url, data=body, method="PUT")
    with urllib.request.urlopen(req, timeout=30) as r:
        if r.status >= 300:
            raise OSError(f"S3 PUT {r.status}")
    return f"s3://{loc['bucket']}/{obj}"


def write_dataset(records: list[dict], fmt: str, output: dict | None, job: str,
                  creds: dict | None = None) -> dict:
    """Serialise datagen records as json / jsonl / csv (``DataGenSettings.format``)
    into ``spec.output`` (a PVC directory or an S3 object); inline when unset."""
    import csv
    import io
    import os

    records = sorted(records, key=lambda r: str(r.get("id")))
    fmt = (fmt or "jsonl").lower()
    if fmt == "json":
        body = json.dumps(records, indent=1)
    elif fmt == "csv":
        buf = io.StringIO()
        w = csv.DictWriter(buf, fieldnames=["id", "scenario", "input", "output", "variables"])
        w.writeheader()
        for r in records:
            w.writerow({**{k: r.get(k) for k in ("id", "scenario", "input", "output")},
                        "variables": json.dumps(r.get("variables") or {})})
        body = buf.getvalue()
    elif fmt == "jsonl":
        body = "".join(json.dumps(r) + "\n" for r in records)
    else:
        raise ValueError(f"unsupported datagen format {fmt!r}")
    out = {"records": len(records), "format": fmt}
    loc = output_location(output)
    if loc is not None and loc["type"] == "pvc":
        os.makedirs(loc["path"], exist_ok=True)
        fn = os.path.join(loc["path"], f"{job}.{fmt}")
        with open(fn, "w") as f:
            f.write(body)
        out["path"] = fn
        out["url"] = "file://" + fn
    elif loc is not None and loc["type"] == "s3":
        out["url"] = put_s3_object(loc, f"{job}.{fmt}", body.encode(), creds or {})
    else:
        out["inline"] = body
    return out


class ArenaJobController:
    def _s3_creds(self, output: dict | None, ns: str) -> dict:
        """Access keys for an s3 output from its secretRef (AWS-style key names)."""
        import base64

        ref = ((output or {}).get("s3") or {}).get("secretRef") or {}
        sec = self.store.try_get("Secret", ref.get("name", ""), ns) if ref else None
        if sec is None:
            return {}
        data = {k: base64.b64decode(v).decode() for k, v in (sec.get("data") or {}).items()}
        data.update(sec.get("stringData") or {})
        return {"access_key": data.get("AWS_ACCESS_KEY_ID") or data.get("access-key", ""),
                "secret_key": data.get("AWS_SECRET_ACCESS_KEY") or data.get("secret-key", "")}

    def __init__(self, store, queue, provider_objects: dict | None = None,
                 worker_mode: str = "inproc", redis_url: str = "", license=None,
                 worker_image: str = "ghcr.io/altairalabs/omnia-arena-worker:latest",
                 poll_s: float = 2.0, session_api_url: str = ""):
        """``worker_mode`` "inproc": worker tasks on this event loop (single
        process); "pods": a batch/v1 Job of worker pods sharing the Redis-Streams
        queue at ``redis_url`` (``arenajob_controller_pod.go``)."""
        self.store = store
        self.q = queue
        self.provider_objects = provider_objects or {}
        self.tasks: dict[str, asyncio.Task] = {}
        self.worker_mode = worker_mode
        self.redis_url = redis_url
        self.session_api_url = session_api_url
        self.license = license  # ee/license.License (or a Validator); None = no gates
        self.worker_image = worker_image
        self.poll_s = poll_s

    async def reconcile(self, ns: str, name: str):
        job = self.store.get("ArenaJob", name, ns)
        phase = (job.get("status") or {}).get("phase", "")
        if phase in ("Succeeded", "Failed", "Cancelled") or name in self.tasks:
            return
        if (job.get("spec") or {}).get("cancelled"):
            self._status(job, "Cancelled")
            return
        self.tasks[name] = asyncio.create_task(self._run(job))

    def _status(self, job, phase, **extra):
        st = dict(job.get("status") or {})
        st.update(phase=phase, **extra)
        set_condition(st, "Complete" if phase in ("Succeeded", "Failed") else "Running",
                      True, phase, extra.get("message", ""))
        job["status"] = st
        try:
            self.store.update_status(job)
        except Exception as e:  # noqa: BLE001
            log.debug("status update failed: %s", e)

    async def _run(self, job):
        try:
            return await self._run_inner(job)
        except JobInvalid as e:
            cur = self.store.try_get("ArenaJob", job["metadata"]["name"],
                                     job["metadata"].get("namespace", "default"))
            if cur is not None:
                self._status(cur, "Failed", message=str(e)[:500], completionTime=time.time(),
                             reason="ValidationFailed")
            return None
        except Exception as e:  # noqa: BLE001 - surfaced in status, not lost in a task
            log.exception("arena job %s failed", job["metadata"]["name"])
            cur = self.store.try_get("ArenaJob", job["metadata"]["name"],
                                     job["metadata"].get("namespace", "default"))
            if cur is not None:
                self._status(cur, "Failed", message=str(e)[:500], completionTime=time.time())
            return None

    async def _run_inner(self, job):
        md, spec = job["metadata"], job["spec"]
        cfg = load_arena_config(self.store, job)
        cfg["scenarios"] = list(select_scenarios(
            {s_["id"]: s_ for s_ in cfg.get("scenarios", [])}, spec.get("scenarios")).values())
        lic = self.license
        if lic is not None and hasattr(lic, "get_or_default"):
            lic = lic.get_or_default()
        src = self.store.try_get("ArenaSource", spec["sourceRef"]["name"],
                                 md.get("namespace", "default")) or {}
        validate_job(spec, cfg, cfg["scenarios"], lic,
                     (src.get("spec") or {}).get("type", ""))
        if self.worker_mode == "pods":
            return await self._run_pods(job, cfg)
        scenarios = {s["id"]: s for s in cfg.get("scenarios", [])}
        providers = {}
        for p in cfg.get("providers", []):
            p = dict(p)
            if p.get("mode") == "direct":
                p["object"] = self.provider_objects[p["id"]]
            if p.get("persona"):
                p["persona_object"] = self.provider_objects[p["persona"]]
            providers[p["id"]] = p
        job_type = spec.get("type", "evaluation")
        trials = int(spec.get("trials") or 1)
        if job_type == "datagen":
            trials = int((spec.get("dataGen") or {}).get("count") or 100)
        items = partition(md["name"], scenarios, providers, trials)
        await self.q.enqueue(items)
        lt = spec.get("loadTest") or {}
        ramp = lt.get("ramp") or {}
        conc = int(lt.get("concurrency") or lt.get("vusPerWorker") or 4)
        replicas = int((spec.get("workers") or {}).get("replicas") or 1)
        self._status(job, "Running", progress={"total": len(items), "done": 0},
                     startTime=time.time())
        t0 = time.perf_counter()
        budget = float(lt["budgetLimit"]) if lt.get("budgetLimit") else None
        recorder = sess = None
        if self.session_api_url:
            from ...session.httpclient import SessionHTTPClient
            from .recording import ArenaSessionRecorder

            sess = SessionHTTPClient(self.session_api_url)
            recorder = ArenaSessionRecorder(sess, md["name"], md.get("namespace", "default"),
                                            spec.get("workspace", ""), job_type)
        workers = [ArenaWorker(self.q, md["name"], scenarios, providers,
                               LoadProfile(max(1, conc // replicas),
                                           float(ramp.get("upSeconds") or 0),
                                           float(ramp.get("downSeconds") or 0)),
                               budget=budget / replicas if budget else None,
                               job_type=job_type, recorder=recorder)
                   for _ in range(replicas)]
        try:
            await asyncio.gather(*(w.run() for w in workers))
        finally:
            if sess is not None:
                await sess.close()
        return await self._finish(job, spec, items, t0)

    async def _finish(self, job, spec, items, t0):
        md = job["metadata"]
        job_type = spec.get("type", "evaluation")
        lt = spec.get("loadTest") or {}
        wall = time.perf_counter() - t0
        results = await self.q.results_of(md["name"])
        turn_results = []
        for r in results:  # per-turn timing drives latency/TTFT percentiles
            for t in r.get("turns") or []:
                turn_results.append({**t, "passed": r.get("passed"), "error": r.get("error")})
        stats = JobStats.from_results(results, wall)
        tstats = JobStats.from_results(turn_results, wall) if turn_results else stats
        stats.latencies_ms, stats.ttfts_ms = tstats.latencies_ms, tstats.ttfts_ms
        verdicts, ok = evaluate(lt.get("thresholds") or [], stats)
        dataset = None
        if job_type == "datagen":
            dataset = write_dataset([r["record"] for r in results if r.get("record")],
                                    (spec.get("dataGen") or {}).get("format", "jsonl"),
                                    spec.get("output"), md["name"],
                                    self._s3_creds(spec.get("output"),
                                                   md.get("namespace", "default")))
        phase = "Succeeded" if ok and stats.errors < max(1, stats.total) else "Failed"
        budget = check_budget(lt.get("budgetLimit"), lt.get("budgetCurrency") or "USD",
                              stats.total_cost)
        job = self.store.get("ArenaJob", md["name"], md.get("namespace", "default"))
        agg = aggregate(results)
        self._status(job, phase, progress={"total": len(items), "done": len(results)},
                     results={**stats.to_json(), **budget},
                     result=to_job_result(agg),
                     thresholds=[str(v) for v in verdicts],
                     completionTime=time.time(), message="thresholds " + (
                         "passed" if ok else "failed") + (
                         "; budget exceeded" if budget else ""),
                     **({"dataset": dataset} if dataset else {}))
        return stats


    # ------------------------------------------------------------ worker pods
    def _worker_objects(self, job, cfg: dict, n_items: int) -> list[dict]:
        """SA / Role / RoleBinding (``arena_worker_rbac.go``), the resolved
        config ConfigMap and the worker Job (``arenajob_controller_pod.go``)."""
        from ...operator.apistore import owner_ref
        from .worker_main import secret_env_name

        md, spec = job["metadata"], job["spec"]
        ns, name = md.get("namespace", "default"), md["name"]
        wn = f"arena-worker-{name}"[:63]
        own = [owner_ref(job)]
        labels = {"app.kubernetes.io/name": "arena-worker",
                  "omnia.altairalabs.ai/component": "arena-worker",
                  "omnia.altairalabs.ai/arena-job": name}
        providers, secret_env = [], []
        for p in cfg.get("providers", []):
            p = dict(p)
            if p.get("mode") == "direct":
                ref = p.get("providerRef") or p["id"]
                pobj = self.store.try_get("Provider", ref if isinstance(ref, str) else
                                          ref.get("name"), ns)
                if pobj is not None:
                    p["spec"] = pobj.get("spec") or {}
                    sref = ((p["spec"].get("credential") or {}).get("secretRef") or
                            p["spec"].get("secretRef") or {})
                    if sref.get("name"):
                        secret_env.append({"name": secret_env_name(p["id"]), "valueFrom": {
                            "secretKeyRef": {"name": sref["name"],
                                             "key": sref.get("key") or "api-key",
                                             "optional": True}}})
                p.pop("object", None)
            providers.append(p)
        lt = spec.get("loadTest") or {}
        ramp = lt.get("ramp") or {}
        replicas = int((spec.get("workers") or {}).get("replicas") or 1)
        conc = int(lt.get("concurrency") or lt.get("vusPerWorker") or 4)
        env = [{"name": "ARENA_JOB_NAME", "value": name},
               {"name": "ARENA_JOB_NAMESPACE", "value": ns},
               {"name": "ARENA_JOB_TYPE", "value": spec.get("type", "evaluation")},
               {"name": "ARENA_SOURCE_NAME", "value": spec["sourceRef"]["name"]},
               {"name": "ARENA_FILE", "value": spec.get("arenaFile") or "config.arena.yaml"},
               {"name": "REDIS_URL", "value": self.redis_url},
               {"name": "ARENA_CONFIG_FILE", "value": "/etc/arena/config.json"},
               {"name": "ARENA_VUS_PER_WORKER", "value": str(max(1, conc // replicas))},
               {"name": "ARENA_CONCURRENCY", "value": str(conc)},
               {"name": "ARENA_RAMP_UP", "value": str(float(ramp.get("upSeconds") or 0))},
               {"name": "ARENA_RAMP_DOWN", "value": str(float(ramp.get("downSeconds") or 0))},
               {"name": "ARENA_TOTAL_ITEMS", "value": str(n_items)},
               {"name": "LOG_LEVEL", "value": "info"}] + secret_env
        sapi = self.session_api_url or os.environ.get("OMNIA_SESSION_API_URL", "")
        if sapi:  # played runs recorded into session-api (recording.py)
            env.append({"name": "SESSION_API_URL", "value": sapi})
        if lt.get("budgetLimit"):
            env.append({"name": "ARENA_BUDGET",
                        "value": str(float(lt["budgetLimit"]) / replicas)})
        ttl = spec.get("ttlSecondsAfterFinished")
        return [
            {"apiVersion": "v1", "kind": "ServiceAccount",
             "metadata": {"name": wn, "namespace": ns, "labels": labels,
                          "ownerReferences": own}},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
             "metadata": {"name": wn, "namespace": ns, "labels": labels, "ownerReferences": own},
             "rules": [{"apiGroups": ["omnia.altairalabs.ai"],
                        "resources": ["arenajobs", "arenasources", "providers"],
                        "verbs": ["get", "list", "watch"]},
                       {"apiGroups": ["omnia.altairalabs.ai"], "resources": ["arenajobs/status"],
                        "verbs": ["get", "patch", "update"]},
                       {"apiGroups": [""], "resources": ["configmaps", "secrets"],
                        "verbs": ["get"]}]},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
             "metadata": {"name": wn, "namespace": ns, "labels": labels, "ownerReferences": own},
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": wn},
             "subjects": [{"kind": "ServiceAccount", "name": wn, "namespace": ns}]},
            {"apiVersion": "v1", "kind": "ConfigMap",
             "metadata": {"name": f"{wn}-config", "namespace": ns, "labels": labels,
                          "ownerReferences": own},
             "data": {"config.json": json.dumps({"scenarios": cfg.get("scenarios", []),
                                                 "providers": providers}, sort_keys=True)}},
            {"apiVersion": "batch/v1", "kind": "Job",
             "metadata": {"name": wn, "namespace": ns, "labels": labels,
                          "ownerReferences": own},
             "spec": {"parallelism": replicas, "completions": replicas,
                      "backoffLimit": int(spec.get("backoffLimit") or 3),
                      "ttlSecondsAfterFinished": int(ttl) if ttl is not None else 3600,
                      "template": {"metadata": {"labels": labels}, "spec": {
                          "serviceAccountName": wn, "restartPolicy": "Never",
                          "containers": [{
                              "name": "worker", "image": self.worker_image,
                              "command": ["python", "-m", "omnia_amd.ee.arena.worker_main"],
                              "env": env,
                              "volumeMounts": [{"name": "config", "mountPath": "/etc/arena",
                                                "readOnly": True}]}],
                          "volumes": [{"name": "config",
                                       "configMap": {"name": f"{wn}-config"}}]}}}},
        ]

    async def _run_pods(self, job, cfg):
        md, spec = job["metadata"], job["spec"]
        ns, name = md.get("namespace", "default"), md["name"]
        scenarios = {s["id"]: s for s in cfg.get("scenarios", [])}
        providers = {p["id"]: p for p in cfg.get("providers", [])}
        trials = int(spec.get("trials") or 1)
        if spec.get("type") == "datagen":
            trials = int((spec.get("dataGen") or {}).get("count") or 100)
        items = partition(name, scenarios, providers, trials)
        await self.q.enqueue(items)
        for obj in self._worker_objects(job, cfg, len(items)):
            self.store.apply(obj)
        self._status(job, "Running", progress={"total": len(items), "done": 0},
                     startTime=time.time(), workerJob=f"arena-worker-{name}"[:63])
        t0 = time.perf_counter()
        wn = f"arena-worker-{name}"[:63]
        while True:
            await asyncio.sleep(self.poll_s)
            kj = self.store.try_get("Job", wn, ns)
            jst = (kj or {}).get("status") or {}
            prog = await self.q.progress(name)
            done = int(prog.get("done", 0))
            cur = self.store.try_get("ArenaJob", name, ns)
            if cur is None:  # deleted: the owned Job goes with it
                return None
            if (cur.get("spec") or {}).get("cancelled"):
                self.store.delete("Job", wn, ns)
                self._status(cur, "Cancelled", completionTime=time.time())
                return None
            st = cur.get("status") or {}
            if (st.get("progress") or {}).get("done") != done or \
                    st.get("activeWorkers") != jst.get("active", 0):
                self._status(cur, "Running", progress={"total": len(items), "done": done},
                             activeWorkers=jst.get("active", 0))
            failed_job = any(c.get("type") == "Failed" and c.get("status") == "True"
                             for c in jst.get("conditions") or [])
            if failed_job:
                self._status(cur, "Failed", message="worker Job failed",
                             completionTime=time.time())
                return None
            complete = int(jst.get("succeeded", 0)) >= int(
                (spec.get("workers") or {}).get("replicas") or 1)
            if complete or done >= len(items):
                return await self._finish(cur, spec, items, t0)


class ArenaJobReconciler:
    """Manager adapter: the operator's reconcile loop is synchronous; jobs run as
    tasks on the manager's event loop (one worker "pod" group per job)."""

    kind = "ArenaJob"

    def __init__(self, queue=None, provider_objects: dict | None = None,
                 worker_mode: str | None = None, redis_url: str | None = None):
        import os

        from .queue import MemoryQueue, StreamQueue

        # OMNIA_ARENA_WORKER_MODE=pods + OMNIA_ARENA_REDIS_URL: worker Jobs on a
        # shared Redis-Streams queue; default: in-process worker tasks
        self.worker_mode = worker_mode or os.environ.get("OMNIA_ARENA_WORKER_MODE", "inproc")
        self.redis_url = redis_url or os.environ.get("OMNIA_ARENA_REDIS_URL", "")
        if queue is None and self.worker_mode == "pods" and self.redis_url:
            from ...utils.resp import RedisClient

            queue = StreamQueue(RedisClient(self.redis_url))
        elif self.worker_mode == "pods" and not self.redis_url:
            self.worker_mode = "inproc"  # worker pods need the shared queue
        self.queue = queue or MemoryQueue()
        self.provider_objects = provider_objects or {}
        self.ctl = None

    def reconcile(self, store, ns, name):
        if self.ctl is None:
            from ...operator import manager as _mgr

            self.ctl = ArenaJobController(store, self.queue, self.provider_objects,
                                          worker_mode=self.worker_mode, redis_url=self.redis_url,
                                          license=getattr(_mgr, "_LICENSE", None))
        try:
            store.get("ArenaJob", name, ns or "default")
        except KeyError:
            return None
        asyncio.get_event_loop().create_task(self.ctl.reconcile(ns or "default", name))
        return None
