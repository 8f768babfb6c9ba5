"""Single-node "kubelet": turns operator-built Deployments into running agent
pods on THIS node, so ``omnia apply -f agentruntime.yaml`` serves end-to-end
on one 8x MI355X box without a cluster.

For every Deployment labelled ``app.kubernetes.io/managed-by=omnia-operator``
and ``omnia.altairalabs.ai/component=agent`` it materialises the pod's mounts
(PromptPack / tools ConfigMaps -> files), builds the runtime from the runtime
container's env (``RuntimeConfig.from_env``) and the facade from the facade
container's env, starts them in-process (one shared GPU engine per model) on
free local ports, and writes back ``status.readyReplicas`` and the Service's
``status.endpoint``.  Pod template changes (config-hash annotation) restart the
pod; replicas=0 (scale-to-zero / capability gate) stops it.
"""
from __future__ import annotations

import asyncio
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
        self.dir = tempfile.mkdtemp(prefix="omnia-pod-")

    async def stop(self):
        if self.facade is not None:
            await self.facade.stop()
        if self.grpc is not None:
            await self.grpc.stop(0)


class LocalLauncher:
    def __init__(self, store: APIStore, engine_factory=None, use_grpc: bool = False):
        self.store = store
        self.pods: dict[tuple, Pod] = {}
        self.engine_factory = engine_factory  # fn(engine_cfg) -> AsyncLLMEngine
        self.use_grpc = use_grpc
        self.task = None

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
        pod.facade = fac

    async def sync(self):
        """One pass: converge running pods to the Deployments."""
        deps = [d for d in self.store.list("Deployment")
                if d["metadata"].get("labels", {}).get(B.LABEL_MANAGED_BY) == "omnia-operator"
                and d["metadata"].get("labels", {}).get(B.LABEL_COMPONENT) == "agent"]
        live = set()
        for d in deps:
            ns, name = d["metadata"]["namespace"], d["metadata"]["name"]
            replicas = d["spec"].get("replicas", 1)
            thash = d["spec"]["template"]["metadata"].get("annotations", {}).get(
                B.ANN_CONFIG_HASH)
            key = (ns, name)
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
        if self.task is not None:
            self.task.cancel()
            await asyncio.gather(self.task, return_exceptions=True)
        for p in list(self.pods.values()):
            await p.stop()
        self.pods.clear()
