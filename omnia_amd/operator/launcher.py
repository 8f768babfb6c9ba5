"""Single-node "kubelet": turns operator-built Deployments into running agent
pods on THIS node, so ``omnia apply -f agentruntime.yaml`` serves end-to-end
on one 8x MI355X box without a cluster.

For every Deployment labelled ``app.kubernetes.io/managed-by=omnia-operator``
and ``omnia.altairalabs.ai/component=agent`` it materialises the pod's mounts
(PromptPack / tools ConfigMaps -> files), builds the runtime from the runtime
container's env (``RuntimeConfig.from_env``) and the facade from the facade
container's env, and starts them on free local ports.  Two pod models:

* ``mode="process"`` (``omnia serve``): every replica is a real pod of OS
  processes (:class:`~omnia_amd.operator.pods.ProcessPod`: ``python -m
  omnia_amd.runtime`` + ``python -m omnia_amd.facade``), ``spec.replicas`` of
  them; local-engine runtimes get their own GPU(s) from a node device
  allocator (``OMNIA_ENGINE_TP`` GPUs each), like the device plugin would.
* ``mode="inproc"``: one in-process runtime + facade per Deployment (tests;
  one shared engine per model).

It writes back ``status.readyReplicas`` and the Service's ``status.endpoint``
(``status.endpoints`` lists every ready replica).  Pod template changes
(config-hash annotation) restart the pods; replicas=0 (scale-to-zero /
capability gate) stops them.

Autoscaling (process mode): KEDA ScaledObjects are evaluated here
(:class:`~omnia_amd.operator.keda.KedaScaler`, metrics scraped from the
replicas' facades), and an agent whose ScaledObject allows zero replicas is
fronted by an :class:`~omnia_amd.operator.keda.Activator` -- the Service's
stable endpoint -- which parks connections while the first replica cold-starts.
Each replica's cold start (process spawn, engine weights + KV allocation, to
readiness) is recorded on the Deployment status (``coldStartSeconds``) and as
``omnia_pod_cold_start_seconds``.
"""
from __future__ import annotations

import asyncio
import threading
import json
import logging
import os
import tempfile
from pathlib import Path

from . import builders as B
from .apistore import APIStore

log = logging.getLogger("omnia.launcher")


def _env(container: dict) -> dict:
    return {e["name"]: e.get("value", "") for e in container.get("env", [])}


class Pod:
    def __init__(self, key, template_hash):
        self.key = key
        self.hash = template_hash
        self.facade = None
        self.runtime_svc = None
        self.grpc = None
        self.port = None
        self.mgmt_port = None
        self.dir = tempfile.mkdtemp(prefix="omnia-pod-")

    async def stop(self):
        if self.facade is not None:
            if getattr(self.facade, "internal", None) is not None:
                await self.facade.internal.stop()
            await self.facade.stop()
        if self.grpc is not None:
            await self.grpc.stop(0)


class DeviceAllocator:
    """GPUs of this node handed to pods (first-fit contiguous ranges, so a TP /
    EP group sits on neighbouring xGMI peers).  ``share`` pods may hold one GPU
    (``OMNIA_PODS_PER_GPU``: a 288 GB MI355X fits e.g. a Mixtral EP shard and an
    8B planner); empty ranges are preferred, so sharing only starts once every
    GPU is taken."""

    def __init__(self, count: int, share: int = 1, ranks_per_gpu: int = 1):
        self.count = count
        self.share = max(1, share)
        # engine ranks one GPU carries (``OMNIA_RANKS_PER_GPU``): > 1 puts a TP / EP
        # pod's ranks on fewer GPUs, which then run the ``ipc`` transport
        # (parallel/state.py) -- a multi-rank pod rehearsed on a one-GPU node
        self.ranks_per_gpu = max(1, ranks_per_gpu)
        self.owner: list[list] = [[] for _ in range(count)]

    def take(self, who, n: int) -> list[int] | None:
        n = -(-n // self.ranks_per_gpu)
        for cap in range(1, self.share + 1):  # least-loaded ranges first
            for start in range(0, self.count - n + 1):
                if all(len(o) < cap for o in self.owner[start:start + n]):
                    for i in range(start, start + n):
                        self.owner[i].append(who)
                    return list(range(start, start + n))
        return None

    def release(self, who):
        self.owner = [[w for w in o if w != who] for o in self.owner]

    def cpus_for(self, devices) -> list[int] | None:
        """Host CPUs for a pod on ``devices``: the union of its GPUs' disjoint
        NUMA-local slices (``utils/affinity.plan`` over every GPU of the node).
        None (unpinned) with < 2 GPUs or ``OMNIA_PIN_CPUS=0``."""
        if not devices or self.count < 2 or os.environ.get("OMNIA_PIN_CPUS", "1") == "0":
            return None
        from ..utils import affinity

        if getattr(self, "_cpu_plan", None) is None:
            self._cpu_plan = affinity.plan(list(range(self.count)))
        if os.environ.get("OMNIA_PIN_CPUS") != "force" and \
                min(len(p) for p in self._cpu_plan) < affinity.MIN_AUTO_PIN_CPUS:
            return None  # oversubscribed host: sharing beats starving slices
        return sorted({c for d in devices for c in self._cpu_plan[d]})

    def load(self, devices) -> int:
        """Pods on the busiest GPU of ``devices`` (sizes the engine's KV slice)."""
        return max((len(self.owner[d]) for d in devices or []), default=1)


class _WaitingForServices(Exception):
    pass


class _ProcReplica:
    """One replica of a Deployment in process mode."""

    def __init__(self, key, index, template_hash, pod, devices):
        self.key = key
        self.index = index
        self.hash = template_hash
        self.pod = pod
        self.devices = devices
        self.port = None
        self.ready = False

    async def stop(self):
        await asyncio.get_running_loop().run_in_executor(None, self.pod.stop)


class LocalLauncher:
    def __init__(self, store: APIStore, engine_factory=None, use_grpc: bool = False,
                 mode: str = "inproc", gpu_count: int = 0):
        self.store = store
        self._starting: set = set()
        self._stopping = False
        self._start_lock = threading.Lock()
        self.pods: dict[tuple, Pod] = {}
        self.replicas: dict[tuple, list] = {}  # process mode: key -> [_ProcReplica]
        self.services: dict[tuple, tuple] = {}  # (ns, name) -> (ServiceProcess, hash)
        self.jobs: dict[tuple, dict] = {}  # (ns, name) -> {"pods": [...], "failed": n, ...}
        self.engine_factory = engine_factory  # fn(engine_cfg) -> AsyncLLMEngine
        self.use_grpc = use_grpc
        self.mode = mode
        self.devices = DeviceAllocator(gpu_count,
                                       int(os.environ.get("OMNIA_PODS_PER_GPU", "1") or 1),
                                       int(os.environ.get("OMNIA_RANKS_PER_GPU", "1") or 1))
        self.task = None
        from .keda import KedaScaler

        self.scaler = KedaScaler(store, self._keda_samples)
        self.activators: dict[tuple, object] = {}  # (ns, name) -> Activator
        self.cold_start_s: dict[tuple, float] = {}
        self._dep_wait: dict[tuple, float] = {}  # key -> first deferral (dependencies)
        self._cron_seen: dict[tuple, float] = {}  # CronJob first seen (schedule origin)

    async def _keda_samples(self, ns: str, name: str) -> list:
        """Metric samples of one scale target: every ready replica's facade
        ``/metrics`` plus the activator's parked connections."""
        import aiohttp

        from .keda import parse_prom_text

        out = []
        reps = [r for r in self.replicas.get((ns, name), []) if r.ready and r.port]
        if reps:
            async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5)) as s:
                for r in reps:
                    async with s.get(f"http://127.0.0.1:{r.port}/metrics") as resp:
                        out.extend(parse_prom_text(await resp.text()))
        act = self.activators.get((ns, name))
        if act is not None:
            out.extend(act.samples())
        return out

    async def _sync_activators(self):
        from .keda import Activator

        want = self.scaler.scale_to_zero_targets()
        for key in [k for k in self.activators if k not in want]:
            await self.activators.pop(key).stop()
        for key in want:
            if key not in self.activators:
                act = Activator(key[1], key[0])
                await act.start()
                self.activators[key] = act

    def _materialise(self, dep: dict, pod: Pod):
        ns = dep["metadata"]["namespace"]
        spec = dep["spec"]["template"]["spec"]
        mounts = {}
        for c in spec["containers"]:
            for vm in c.get("volumeMounts", []):
                mounts[vm["name"]] = vm["mountPath"]
        paths = {}
        for v in spec.get("volumes", []):
            cm = v.get("configMap")
            if not cm:
                continue
            obj = self.store.try_get("ConfigMap", cm["name"], ns)
            d = Path(pod.dir) / v["name"]
            d.mkdir(parents=True, exist_ok=True)
            for fname, content in ((obj or {}).get("data") or {}).items():
                (d / fname).write_text(content)
            paths[mounts.get(v["name"], v["name"])] = str(d)
        return paths

    async def _start_pod(self, dep: dict, pod: Pod):
        from ..facade.runtime_client import GrpcRuntimeClient, InProcessRuntimeClient
        from ..runtime.app import build_runtime
        from ..runtime.config import RuntimeConfig
        from ..runtime.server import serve_grpc

        paths = self._materialise(dep, pod)
        cs = {c["name"]: c for c in dep["spec"]["template"]["spec"]["containers"]}
        renv = _env(cs["runtime"])
        renv["OMNIA_PROMPTPACK_PATH"] = paths.get("/etc/omnia/pack", renv.get(
            "OMNIA_PROMPTPACK_PATH", ""))
        renv["OMNIA_TOOLS_CONFIG_PATH"] = paths.get("/etc/omnia/tools", "")
        rc = RuntimeConfig.from_env(renv)
        engine = None
        if rc.provider.get("type") == "local" and self.engine_factory is not None:
            engine = self.engine_factory(rc.engine)
        svc = await build_runtime(rc, engine=engine)
        pod.runtime_svc = svc
        if self.use_grpc:
            pod.grpc, gport = await serve_grpc(svc, 0, "127.0.0.1")
            client = GrpcRuntimeClient(f"127.0.0.1:{gport}")
        else:
            client = InProcessRuntimeClient(svc)
        from ..facade.app import build_facade

        fac = build_facade(_env(cs["facade"]), client)
        pod.port = await fac.start("127.0.0.1", 0)
        if fac.internal is not None:  # management-plane twin (dashboard / doctor)
            pod.mgmt_port = await fac.internal.start("127.0.0.1", 0)
        pod.facade = fac

    # ------------------------------------------------------------ CronJobs
    def _sync_cronjobs(self, now: float | None = None) -> list[str]:
        """batch/v1 CronJobs (the chart's session compaction, scheduled
        maintenance): at each schedule time a Job is created from
        ``jobTemplate`` (owned by the CronJob, named ``<cron>-<minute>``), which
        ``_sync_jobs`` then runs.  ``concurrencyPolicy: Forbid`` skips a run while
        the previous Job is active, ``Replace`` deletes it first; ``suspend``
        stops scheduling; missed runs are not back-filled (one run per sync at
        most, as with ``startingDeadlineSeconds`` unset after a long outage);
        the ``successfulJobsHistoryLimit`` newest finished Jobs are kept.
        ``status.lastScheduleTime`` / ``active`` are written back."""
        import time

        from ..utils.cron import next_fire
        from .apistore import owner_ref

        now = time.time() if now is None else now
        made = []
        for cj in self.store.list("CronJob"):
            spec, md = cj.get("spec") or {}, cj["metadata"]
            ns, name = md["namespace"], md["name"]
            st = dict(cj.get("status") or {})
            owned = [j for j in self.store.list("Job", ns)
                     if any(o.get("uid") == md.get("uid") for o in
                            j["metadata"].get("ownerReferences") or [])]
            active = [j for j in owned if not any(
                c.get("type") in ("Complete", "Failed") and c.get("status") == "True"
                for c in (j.get("status") or {}).get("conditions") or [])]
            last = float(st.get("lastScheduleTime") or md.get("creationTimestampUnix") or 0) \
                or self._cron_seen.setdefault((ns, name), now)
            try:
                due = next_fire(spec.get("schedule", ""), last)
            except ValueError:
                continue
            if not spec.get("suspend") and due <= now:
                policy = spec.get("concurrencyPolicy", "Allow")
                if active and policy == "Forbid":
                    st["lastScheduleTime"] = now  # this run is skipped, not queued
                else:
                    if active and policy == "Replace":
                        for j in active:
                            self.store.delete("Job", j["metadata"]["name"], ns)
                    jname = f"{name}-{int(due // 60)}"
                    tmpl = spec.get("jobTemplate") or {}
                    if self.store.try_get("Job", jname, ns) is None:
                        self.store.apply({
                            "apiVersion": "batch/v1", "kind": "Job",
                            "metadata": {"name": jname, "namespace": ns,
                                         "labels": dict((tmpl.get("metadata") or {}).get(
                                             "labels") or {}),
                                         "ownerReferences": [owner_ref(cj)]},
                            "spec": dict(tmpl.get("spec") or {})})
                        made.append(jname)
                    st["lastScheduleTime"] = now
            owned = [j for j in self.store.list("Job", ns)
                     if any(o.get("uid") == md.get("uid") for o in
                            j["metadata"].get("ownerReferences") or [])]
            active = [j for j in owned if not any(
                c.get("type") in ("Complete", "Failed") and c.get("status") == "True"
                for c in (j.get("status") or {}).get("conditions") or [])]
            keep = int(spec.get("successfulJobsHistoryLimit", 3))
            done = sorted((j for j in owned if j not in active),
                          key=lambda j: j["metadata"]["name"])
            for j in done[:max(0, len(done) - keep)]:
                self.store.delete("Job", j["metadata"]["name"], ns)
            st["active"] = [{"name": j["metadata"]["name"]} for j in active]
            if st != (cj.get("status") or {}):
                cj["status"] = st
                cj["metadata"].pop("resourceVersion", None)
                self.store.update_status(cj)
        return made

    # ------------------------------------------------------------ batch Jobs
    async def _sync_jobs(self):
        """batch/v1 Jobs (arena workers) as run-to-completion processes:
        ``parallelism`` pods at a time until ``completions`` succeeded; a failed
        pod is retried until ``backoffLimit`` failures, then the Job is Failed.
        Job ``status`` (active / succeeded / failed / conditions) is written back."""
        from .pods import JobPodProcess

        loop = asyncio.get_running_loop()
        live = set()
        for j in self.store.list("Job"):
            ns, name = j["metadata"]["namespace"], j["metadata"]["name"]
            key = (ns, name)
            live.add(key)
            spec = j["spec"]
            st = self.jobs.setdefault(key, {"pods": [], "succeeded": 0, "failed": 0, "n": 0,
                                            "done": False})
            if st["done"]:
                continue
            want = int(spec.get("completions") or 1)
            par = int(spec.get("parallelism") or 1)
            backoff = int(spec.get("backoffLimit") if spec.get("backoffLimit") is not None else 6)
            for p in list(st["pods"]):
                rc = p.poll()
                if rc is None:
                    continue
                st["pods"].remove(p)
                await loop.run_in_executor(None, p.stop)
                if rc == 0:
                    st["succeeded"] += 1
                else:
                    st["failed"] += 1
            conds = []
            if st["succeeded"] >= want:
                conds = [{"type": "Complete", "status": "True"}]
            elif st["failed"] > backoff:
                conds = [{"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded"}]
            if conds:
                for p in st["pods"]:
                    await loop.run_in_executor(None, p.stop)
                st["pods"], st["done"] = [], True
            else:
                tmpl = spec["template"]["spec"]
                while len(st["pods"]) < min(par, want - st["succeeded"]):
                    wd = tempfile.mkdtemp(prefix=f"omnia-job-{name}-")
                    mounts = self._job_mounts(ns, tmpl, wd)
                    st["n"] += 1
                    pod = JobPodProcess(f"{name}-{st['n']}",
                                        self._resolve_env(ns, tmpl["containers"][0]), wd, mounts)
                    try:
                        await loop.run_in_executor(None, pod.start)
                    except Exception:  # noqa: BLE001
                        log.exception("job pod %s failed to start", pod.name)
                        st["failed"] += 1
                        break
                    st["pods"].append(pod)
            new = {"active": len(st["pods"]), "succeeded": st["succeeded"],
                   "failed": st["failed"], **({"conditions": conds} if conds else {})}
            if (j.get("status") or {}) != new:
                j["status"] = new
                j["metadata"].pop("resourceVersion", None)
                self.store.update_status(j)
        for key in [k for k in self.jobs if k not in live]:  # Job deleted: kill its pods
            for p in self.jobs.pop(key)["pods"]:
                await loop.run_in_executor(None, p.stop)

    def _resolve_env(self, ns: str, container: dict) -> dict:
        """Container copy whose ``secretKeyRef`` / ``configMapKeyRef`` env entries
        carry their values (what the kubelet injects); missing optional keys are
        dropped, a missing required key fails the pod start."""
        import base64
        import copy

        c = copy.deepcopy(container)
        env = []
        for e in c.get("env", []):
            vf = e.get("valueFrom") or {}
            ref = vf.get("secretKeyRef") or vf.get("configMapKeyRef")
            if not ref:
                env.append(e)
                continue
            kind = "Secret" if "secretKeyRef" in vf else "ConfigMap"
            obj = self.store.try_get(kind, ref.get("name", ""), ns) or {}
            val = (obj.get("stringData") or {}).get(ref.get("key"))
            if val is None and ref.get("key") in (obj.get("data") or {}):
                raw = obj["data"][ref["key"]]
                val = base64.b64decode(raw).decode() if kind == "Secret" else raw
            if val is None:
                if ref.get("optional"):
                    continue
                raise KeyError(f"{kind} {ref.get('name')}/{ref.get('key')} not found")
            env.append({"name": e["name"], "value": val})
        # cluster DNS on one node: in-cluster Service URLs in env values and args
        # point at the Services' local endpoints (a compaction Job dials its
        # workspace's session-api by Service URL)
        from .pods import resolve_service_urls

        vals = resolve_service_urls({i: e["value"] for i, e in enumerate(env) if "value" in e},
                                    self._service_endpoint)
        for i, v in vals.items():
            env[i] = dict(env[i], value=v)
        c["env"] = env
        if c.get("args"):
            c["args"] = list(resolve_service_urls(dict(enumerate(c["args"])),
                                                  self._service_endpoint).values())
        return c

    def _job_mounts(self, ns: str, tmpl: dict, workdir: str) -> dict[str, str]:
        mounts = {}
        vols = {v["name"]: v for v in tmpl.get("volumes", [])}
        for vm in tmpl["containers"][0].get("volumeMounts", []):
            v = vols.get(vm["name"]) or {}
            local = os.path.join(workdir, vm["name"])
            os.makedirs(local, exist_ok=True)
            cm = v.get("configMap")
            if cm:
                obj = self.store.try_get("ConfigMap", cm["name"], ns)
                for fname, content in ((obj or {}).get("data") or {}).items():
                    with open(os.path.join(local, fname), "w") as f:
                        f.write(content)
            mounts[vm["mountPath"]] = local
        return mounts

    # ------------------------------------------------------------ service pods
    SERVICE_COMPONENTS = ("session-api", "memory-api", "arena-dev-console")

    async def _sync_services(self):
        """Workspace session-api / memory-api Deployments as service processes."""
        loop = asyncio.get_running_loop()
        want = {}
        for d in self.store.list("Deployment"):
            comp = d["metadata"].get("labels", {}).get(B.LABEL_COMPONENT)
            if comp in self.SERVICE_COMPONENTS and (d["spec"].get("replicas", 1) or 0) > 0:
                want[(d["metadata"]["namespace"], d["metadata"]["name"])] = d
        for key in list(self.services):
            sp, h = self.services[key]
            d = want.get(key)
            if d is None or not sp.alive() or h != B.config_hash(d["spec"]["template"]):
                self.services.pop(key)
                await loop.run_in_executor(None, sp.stop)
        for key, d in want.items():
            if key not in self.services:
                from .pods import ServiceProcess

                c = d["spec"]["template"]["spec"]["containers"][0]
                if not c.get("command"):
                    continue
                wd = tempfile.mkdtemp(prefix=f"omnia-{key[1]}-")
                sp = ServiceProcess(key[1], c, wd, mounts=self._job_mounts(
                    key[0], d["spec"]["template"]["spec"], wd))
                try:
                    await loop.run_in_executor(None, sp.start)
                except Exception:  # noqa: BLE001
                    log.exception("service %s/%s failed to start", *key)
                    continue
                self.services[key] = (sp, B.config_hash(d["spec"]["template"]))
            sp = self.services[key][0]
            st = d.get("status") or {}
            if st.get("readyReplicas") != 1 or \
                    st.get("observedGeneration") != d["metadata"]["generation"]:
                d["status"] = {**st, "replicas": 1, "readyReplicas": 1, "availableReplicas": 1,
                               "observedGeneration": d["metadata"]["generation"]}
                d["metadata"].pop("resourceVersion", None)
                self.store.update_status(d)
            svc = self.store.try_get("Service", key[1], key[0])
            if svc is not None and (svc.get("status") or {}).get("endpoint") != sp.endpoint:
                svc["status"] = {**(svc.get("status") or {}), "endpoint": sp.endpoint}
                svc["metadata"].pop("resourceVersion", None)
                self.store.update_status(svc)

    # ------------------------------------------------------------ process mode
    def _pod_envs(self, dep: dict, workdir: str) -> tuple[dict, dict]:
        import types

        paths = self._materialise(dep, types.SimpleNamespace(dir=workdir))
        cs = {c["name"]: c for c in dep["spec"]["template"]["spec"]["containers"]}
        renv = _env(cs["runtime"])
        renv["OMNIA_PROMPTPACK_PATH"] = paths.get("/etc/omnia/pack", renv.get(
            "OMNIA_PROMPTPACK_PATH", ""))
        renv["OMNIA_TOOLS_CONFIG_PATH"] = paths.get("/etc/omnia/tools", "")
        from .pods import resolve_service_urls

        return (resolve_service_urls(renv, self._service_endpoint),
                resolve_service_urls(_env(cs["facade"]), self._service_endpoint))

    def _service_endpoint(self, name: str, ns: str) -> str | None:
        svc = self.store.try_get("Service", name, ns)
        return ((svc or {}).get("status") or {}).get("endpoint")

    def _pending_services(self, key, dep: dict) -> list[str]:
        """In-cluster Services the pod's env points at that exist but have no
        endpoint yet (e.g. an A2A peer still cold-starting).  Cluster DNS would
        resolve them later; a process pod's URLs are rewritten once at start, so
        the start waits for them -- up to ``OMNIA_POD_DEPENDENCY_WAIT_S`` (600 s),
        after which it starts anyway (mutual references cannot deadlock)."""
        from .pods import service_refs

        env = {}
        for c in dep["spec"]["template"]["spec"]["containers"]:
            env.update(_env(c))
        pending = [f"{ns}/{svc}" for svc, ns in sorted(service_refs(env))
                   if (s := self.store.try_get("Service", svc, ns)) is not None
                   and not (s.get("status") or {}).get("endpoint")
                   and (svc, ns) != (key[1], key[0])]
        if not pending:
            self._dep_wait.pop(key, None)
            return []
        import time

        t0 = self._dep_wait.setdefault(key, time.monotonic())
        if time.monotonic() - t0 > float(os.environ.get("OMNIA_POD_DEPENDENCY_WAIT_S", "600")):
            return []
        return pending

    def _start_replica(self, dep: dict, key, index: int, thash) -> _ProcReplica:
        from .pods import ProcessPod

        pending = self._pending_services(key, dep)
        if pending:
            raise _WaitingForServices(", ".join(pending))
        workdir = tempfile.mkdtemp(prefix=f"omnia-{key[1]}-{index}-")
        renv, fenv = self._pod_envs(dep, workdir)
        rc_provider = (json.loads(renv.get("OMNIA_PROVIDER_JSON", "{}") or "{}").get("type")
                       or renv.get("OMNIA_PROVIDER_TYPE", "mock"))
        devices = None
        who = (key, index)
        tp = int(renv.get("OMNIA_ENGINE_TP", "1") or 1)
        world = tp  # engine ranks of one pod: TP group, or the EP (a2a) group
        if renv.get("OMNIA_ENGINE_EP_MODE") == "a2a":
            world = max(tp, int(renv.get("OMNIA_ENGINE_EP", "1") or 1))
        if rc_provider in ("local", "engine", "omnia", "rocm") and self.devices.count and \
                renv.get("OMNIA_ENGINE_DEVICE", "cuda") != "cpu":
            devices = self.devices.take(who, world)
            if devices is None:
                raise RuntimeError(f"no {world} free GPU(s) for {key[0]}/{key[1]} replica "
                                   f"{index}")
        if devices is not None and self.devices.share > 1:
            renv["OMNIA_GPU_SHARE"] = str(self.devices.share)  # KV slice per pod
        for k in ("OMNIA_GRPC_PORT", "OMNIA_HEALTH_PORT"):
            renv.pop(k, None)
        fenv.pop("OMNIA_FACADE_PORT", None)
        pod = ProcessPod(f"{key[1]}-{index}", renv, fenv, device_index=devices,
                         log_dir=os.path.join(workdir, "logs"), tp=world,
                         cpus=self.devices.cpus_for(devices))
        import time

        t0 = time.perf_counter()
        # pods being started are tracked so stop() can kill one mid-start (an
        # executor thread keeps starting it after the sync task is cancelled)
        with self._start_lock:
            if self._stopping:
                self.devices.release(who)
                raise RuntimeError("launcher stopping")
            self._starting.add(pod)
        try:
            pod.start(timeout_s=float(os.environ.get("OMNIA_POD_START_TIMEOUT", "900")))
        except Exception:
            self.devices.release(who)
            raise
        finally:
            with self._start_lock:
                self._starting.discard(pod)
        if self._stopping:
            pod.stop()
            self.devices.release(who)
            raise RuntimeError("launcher stopping")
        cold = time.perf_counter() - t0
        self.cold_start_s[key] = cold
        from ..observability import metrics as M

        M.POD_COLD_START.labels(key[1], key[0]).observe(cold)
        log.info("pod %s/%s replica %d ready in %.2fs (cold start)", key[0], key[1], index, cold)
        r = _ProcReplica(key, index, thash, pod, devices)
        r.port = pod.facade_port
        r.ready = True
        return r

    async def _sync_process(self, d: dict, key, replicas: int, thash) -> int:
        loop = asyncio.get_running_loop()
        cur = self.replicas.setdefault(key, [])
        # template change: replace every replica
        stale = [r for r in cur if r.hash != thash or not r.pod.alive()]
        for r in stale:
            cur.remove(r)
            await r.stop()
            self.devices.release((key, r.index))
        while len(cur) > replicas:
            r = cur.pop()
            await r.stop()
            self.devices.release((key, r.index))
        used = {r.index for r in cur}
        for i in range(replicas):
            if len(cur) >= replicas:
                break
            if i in used:
                continue
            try:
                r = await loop.run_in_executor(None, self._start_replica, d, key, i, thash)
            except _WaitingForServices as e:
                log.info("pod %s/%s replica %d waits for service endpoints: %s", key[0],
                         key[1], i, e)
                break
            except Exception:  # noqa: BLE001
                log.exception("pod %s/%s replica %d failed to start", key[0], key[1], i)
                continue
            cur.append(r)
        cur.sort(key=lambda r: r.index)
        return sum(1 for r in cur if r.ready)

    async def sync(self):
        """One pass: converge running pods to the Deployments."""
        deps = [d for d in self.store.list("Deployment")
                if d["metadata"].get("labels", {}).get(B.LABEL_MANAGED_BY) == "omnia-operator"
                and d["metadata"].get("labels", {}).get(B.LABEL_COMPONENT) == "agent"]
        live = set()
        if self.mode == "process":
            await self._sync_services()
            self._sync_cronjobs()
            await self._sync_jobs()
            await self._sync_activators()
        for d in deps:
            ns, name = d["metadata"]["namespace"], d["metadata"]["name"]
            replicas = d["spec"].get("replicas", 1)
            thash = d["spec"]["template"]["metadata"].get("annotations", {}).get(
                B.ANN_CONFIG_HASH)
            key = (ns, name)
            if self.mode == "process":
                want_n = int(replicas or 0)
                if want_n > 0:
                    live.add(key)
                ready = await self._sync_process(d, key, want_n, thash)
                self._write_status(d, ready, name, ns, key)
                continue
            pod = self.pods.get(key)
            if replicas and replicas > 0:
                live.add(key)
                if pod is not None and pod.hash != thash:
                    await pod.stop()
                    pod = None
                if pod is None:
                    pod = Pod(key, thash)
                    try:
                        await self._start_pod(d, pod)
                    except Exception:  # noqa: BLE001
                        log.exception("pod %s/%s failed to start", ns, name)
                        continue
                    self.pods[key] = pod
                ready = 1
            else:
                ready = 0
            st = d.get("status") or {}
            want = {"replicas": ready, "readyReplicas": ready, "availableReplicas": ready,
                    "observedGeneration": d["metadata"]["generation"]}
            if any(st.get(k) != v for k, v in want.items()):
                d["status"] = {**st, **want}
                d["metadata"].pop("resourceVersion", None)
                self.store.update_status(d)
            track = d["metadata"].get("labels", {}).get(B.LABEL_TRACK, "stable")
            svc = self.store.try_get("Service", name, ns) if track == "stable" else None
            if svc is not None and self.pods.get(key) is not None:
                ep = f"127.0.0.1:{self.pods[key].port}"
                if (svc.get("status") or {}).get("endpoint") != ep:
                    svc["status"] = {**(svc.get("status") or {}), "endpoint": ep}
                    svc["metadata"].pop("resourceVersion", None)
                    self.store.update_status(svc)
        for key in list(self.pods):
            if key not in live:
                await self.pods.pop(key).stop()
        for key in list(self.replicas):
            if key not in live:
                for r in self.replicas.pop(key):
                    await r.stop()
                    self.devices.release((key, r.index))
        if self.mode == "process":
            await self.scaler.tick()

    def _write_status(self, d: dict, ready: int, name: str, ns: str, key):
        st = d.get("status") or {}
        want = {"replicas": ready, "readyReplicas": ready, "availableReplicas": ready,
                "observedGeneration": d["metadata"]["generation"]}
        if key in self.cold_start_s:
            want["coldStartSeconds"] = round(self.cold_start_s[key], 3)
        if any(st.get(k) != v for k, v in want.items()):
            d["status"] = {**st, **want}
            d["metadata"].pop("resourceVersion", None)
            self.store.update_status(d)
        track = d["metadata"].get("labels", {}).get(B.LABEL_TRACK, "stable")
        svc = self.store.try_get("Service", name, ns) if track == "stable" else None
        reps = [r for r in self.replicas.get(key, []) if r.ready]
        eps = [f"127.0.0.1:{r.port}" for r in reps]
        act = self.activators.get(key)
        if act is not None:
            act.set_backends(eps)  # the stable front parks traffic while eps == []
        if svc is not None and (reps or act is not None):
            front = act.endpoint if act is not None else eps[0]
            cur = svc.get("status") or {}
            if cur.get("endpoint") != front or cur.get("endpoints") != eps:
                svc["status"] = {**cur, "endpoint": front, "endpoints": eps}
                svc["metadata"].pop("resourceVersion", None)
                self.store.update_status(svc)

    async def run(self, interval: float = 0.2):
        q = self.store.watch("Deployment")
        try:
            while True:
                try:
                    await self.sync()
                except Exception:  # noqa: BLE001
                    log.exception("launcher sync failed")
                try:
                    await asyncio.wait_for(q.get(), interval)
                    while not q.empty():
                        q.get_nowait()
                except asyncio.TimeoutError:
                    pass
        finally:
            self.store.unwatch(q)

    def start(self):
        self.task = asyncio.ensure_future(self.run())

    async def stop(self):
        with self._start_lock:
            self._stopping = True
            starting = list(self._starting)
        if self.task is not None:
            self.task.cancel()
            await asyncio.gather(self.task, return_exceptions=True)
        loop = asyncio.get_running_loop()
        await asyncio.gather(*(loop.run_in_executor(None, p.stop) for p in starting),
                             return_exceptions=True)
        for _ in range(300):  # start threads notice the stop and clean up their pods
            with self._start_lock:
                if not self._starting:
                    break
            await asyncio.sleep(0.1)
        for p in list(self.pods.values()):
            await p.stop()
        self.pods.clear()
        for act in list(self.activators.values()):
            await act.stop()
        self.activators.clear()
        # replicas stop concurrently: each pod drains its facade for up to 15 s
        reps = [(key, r) for key, rs in list(self.replicas.items()) for r in rs]
        await asyncio.gather(*(r.stop() for _, r in reps), return_exceptions=True)
        for key, r in reps:
            self.devices.release((key, r.index))
        self.replicas.clear()
        for sp, _ in self.services.values():
            sp.stop()
        self.services.clear()
        for st in self.jobs.values():
            for p in st["pods"]:
                p.stop()
        self.jobs.clear()
