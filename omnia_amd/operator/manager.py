"""Controller manager (``cmd/main.go:400-660``): watch -> rate-limited work
queue -> reconcile, with cross-kind enqueue mappings
(``internal/controller/agentruntime_watches.go:36-60``), requeue-after, leader
election on a Lease object, and the admission webhooks
(``internal/webhook/*``: AgentRuntime input/output schemas must compile,
Provider/Workspace sanity).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import socket
import time

from ..api import crds
from ..utils import jsonschema
from .apistore import APIStore, Conflict
from .controllers import default_reconcilers

log = logging.getLogger("omnia.operator.manager")


# ------------------------------------------------------------------ webhooks
_LICENSE = None  # ee.license.Validator when the manager runs with --enterprise


def set_license_validator(v) -> None:
    global _LICENSE
    _LICENSE = v


def license_validator_for(store: APIStore, public_key_pem: str | None):
    """Validator reading Secret ``omnia-license`` (key ``license``) from ``store``."""
    import base64

    from ..ee import license as lic

    def read():
        for ns in (os.environ.get("OMNIA_NAMESPACE", "omnia-system"), "default"):
            try:
                sec = store.get("Secret", lic.SECRET_NAME, ns)
            except Exception:  # noqa: BLE001
                continue
            data = (sec.get("data") or {}).get(lic.SECRET_KEY)
            if data:
                return base64.b64decode(data).decode()
            sd = (sec.get("stringData") or {}).get(lic.SECRET_KEY)
            if sd:
                return sd
        return os.environ.get("OMNIA_LICENSE")

    return lic.Validator(public_key_pem, secret_reader=read)


def agentruntime_webhook(obj, old):
    errs = []
    if _LICENSE is not None:
        from ..ee import license as lic

        errs += lic.gate_agentruntime(obj["spec"], _LICENSE.get_or_default())
    for f in ("inputSchema", "outputSchema"):
        sch = obj["spec"].get(f)
        if sch is not None:
            try:
                jsonschema.check_schema(sch)
            except Exception as e:  # noqa: BLE001
                errs.append(f"spec.{f} does not compile: {e}")
    return errs


def workspace_webhook(obj, old):
    if old is not None and old["spec"]["namespace"]["name"] != obj["spec"]["namespace"]["name"]:
        return ["spec.namespace.name is immutable"]
    return []


def promptpack_webhook(obj, old):
    if old is not None and old["spec"].get("version") != obj["spec"].get("version"):
        return ["PromptPack spec.version is immutable; create a new PromptPack"]
    return []


WEBHOOKS = {"AgentRuntime": agentruntime_webhook, "Workspace": workspace_webhook,
            "PromptPack": promptpack_webhook}


def new_store() -> APIStore:
    return APIStore(webhooks=dict(WEBHOOKS))


# ------------------------------------------------------------------ manager
class Manager:
    def __init__(self, store: APIStore, reconcilers=None, gpu_count: int | None = None,
                 identity: str | None = None, leader_elect: bool = False,
                 namespace: str = "omnia-system"):
        self.store = store
        self.reconcilers = {r.kind: r for r in (reconcilers or default_reconcilers(gpu_count))}
        if reconcilers is None and os.environ.get("OMNIA_LICENSE_SERVER"):
            # EE: activate the license against the license server, heartbeat daily
            from ..ee import license as lic
            from ..ee.license_activation import ActivationClient, LicenseActivationReconciler

            self.reconcilers["Secret"] = LicenseActivationReconciler(
                license_validator_for(store, os.environ.get("OMNIA_LICENSE_PUBLIC_KEY")),
                ActivationClient(os.environ["OMNIA_LICENSE_SERVER"]),
                cluster_name=os.environ.get("OMNIA_CLUSTER_NAME", ""),
                secret_name=lic.SECRET_NAME)
        self.queue: asyncio.Queue | None = None
        self.pending: set = set()
        self.delayed: dict = {}
        self.conflicts: dict = {}  # key -> consecutive write conflicts
        self.identity = identity or f"{socket.gethostname()}-{os.getpid()}"
        self.leader_elect = leader_elect
        self.lease_ns = namespace
        self.tasks: list = []
        self.stats = {"reconciles": 0, "errors": 0}
        self._idle = None
        self._gens: dict = {}
        self.lease = None
        self.lease_duration_s = 15
        self.processing: set = set()
        self.dirty: set = set()
        # a remote apiserver client blocks on HTTP: reconcile off the event loop
        self.threaded = not isinstance(store, APIStore)
        self.is_leader = False

    def enqueue(self, kind: str, ns: str | None, name: str, after: float = 0.0):
        key = (kind, ns or "", name)
        if after > 0:
            self.delayed[key] = time.monotonic() + after
            return
        if key not in self.pending:
            self.pending.add(key)
            self.queue.put_nowait(key)

    def _map(self, etype: str, obj: dict):
        kind = obj["kind"]
        md = obj["metadata"]
        ns = md.get("namespace", "")
        if kind in self.reconcilers:
            # GenerationChangedPredicate: status-only writes of the primary kind
            # do not re-trigger its own reconcile
            gk = (kind, ns, md["name"])
            gen = md.get("generation")
            if etype != "MODIFIED" or self._gens.get(gk) != gen or \
                    md.get("deletionTimestamp"):
                self.enqueue(kind, ns, md["name"])
            self._gens[gk] = gen
        # owner -> re-queue
        for ref in md.get("ownerReferences", []) or []:
            if ref.get("kind") in self.reconcilers:
                self.enqueue(ref["kind"], ns, ref["name"])
        # reference mappings
        if kind in ("PromptPack", "Provider", "ToolRegistry", "ConfigMap", "Secret",
                    "RolloutAnalysis"):
            for ar in self.store.list("AgentRuntime", ns):
                spec = ar["spec"]
                hit = False
                if kind == "PromptPack":
                    hit = spec["promptPackRef"]["name"] in (obj["spec"].get("packName"),
                                                            md["name"])
                elif kind == "Provider":
                    hit = any((p.get("providerRef") or {}).get("name", p.get("name")) ==
                              md["name"] for p in spec.get("providers") or [])
                elif kind == "ToolRegistry":
                    hit = (spec.get("toolRegistryRef") or {}).get("name") == md["name"]
                else:
                    hit = True
                if hit:
                    self.enqueue("AgentRuntime", ns, ar["metadata"]["name"])
        if kind == "AgentPolicy":  # the matched agents' tool config carries the policy
            sel = set(((obj.get("spec") or {}).get("selector") or {}).get("agents") or [])
            for ar in self.store.list("AgentRuntime", ns):
                if not sel or ar["metadata"]["name"] in sel:
                    self.enqueue("AgentRuntime", ns, ar["metadata"]["name"])
        if kind == "ConfigMap":
            for pp in self.store.list("PromptPack", ns):
                if (pp["spec"]["source"].get("configMapRef") or {}).get("name") == md["name"]:
                    self.enqueue("PromptPack", ns, pp["metadata"]["name"])
        if kind == "Secret":
            for pv in self.store.list("Provider", ns):
                if ((pv["spec"].get("credential") or {}).get("secretRef") or {}).get(
                        "name") == md["name"]:
                    self.enqueue("Provider", ns, pv["metadata"]["name"])
        if kind == "PromptPack":
            for pp in self.store.list("PromptPack", ns):
                if pp["spec"].get("packName") == obj["spec"].get("packName") and \
                        pp["metadata"]["name"] != md["name"]:
                    self.enqueue("PromptPack", ns, pp["metadata"]["name"])

    async def _acquire_lease(self) -> bool:
        if not self.leader_elect:
            return True
        if self.lease is None:
            from .kube import LeaseLock

            self.lease = LeaseLock(self.store, "omnia-operator-leader", self.lease_ns,
                                   self.identity, lease_duration_s=self.lease_duration_s,
                                   renew_deadline_s=self.lease_duration_s * 2 / 3,
                                   retry_period_s=self.lease_duration_s / 7.5)
        return await asyncio.to_thread(self.lease.try_acquire_or_renew)

    async def _renew_loop(self):
        """Renew every retry period; a leader that cannot renew within the
        renew deadline stops reconciling (client-go ``OnStoppedLeading``)."""
        while True:
            await asyncio.sleep(self.lease.retry_period_s)
            ok = False
            try:
                ok = await asyncio.to_thread(self.lease.try_acquire_or_renew)
            except Exception:  # noqa: BLE001 - apiserver blip: deadline decides
                log.warning("lease renewal failed", exc_info=True)
            if not ok and not self.lease.holds():
                log.error("lost leader lease %s; stopping", self.identity)
                self.is_leader = False
                for t in self.tasks:
                    if t is not asyncio.current_task():
                        t.cancel()
                return

    async def _watch_loop(self, q):
        try:
            while True:
                etype, obj = await q.get()
                if self.threaded:
                    await asyncio.to_thread(self._map, etype, obj)
                else:
                    self._map(etype, obj)
        finally:
            self.store.unwatch(q)

    async def _timer_loop(self):
        while True:
            await asyncio.sleep(0.05)
            now = time.monotonic()
            for key, t in list(self.delayed.items()):
                if t <= now:
                    self.delayed.pop(key, None)
                    self.enqueue(*key)

    async def _worker(self):
        while True:
            key = await self.queue.get()
            self.pending.discard(key)
            kind, ns, name = key
            r = self.reconcilers.get(kind)
            if r is None:
                continue
            if key in self.processing:
                self.dirty.add(key)  # never reconcile one key concurrently
                continue
            self.processing.add(key)
            try:
                if self.threaded:
                    after = await asyncio.to_thread(r.reconcile, self.store, ns or None, name)
                else:
                    after = r.reconcile(self.store, ns or None, name)
                self.stats["reconciles"] += 1
                self.conflicts.pop(key, None)
                if after:
                    self.enqueue(kind, ns, name, after)
            except Conflict:
                # a write raced another writer's (stale resourceVersion): re-read
                # and retry soon with per-key exponential backoff, as
                # controller-runtime's rate-limited requeue does -- not an error
                n = self.conflicts.get(key, 0) + 1
                self.conflicts[key] = n
                self.stats["conflicts"] = self.stats.get("conflicts", 0) + 1
                log.debug("reconcile %s %s/%s: conflict #%d, requeued", kind, ns, name, n)
                self.enqueue(kind, ns, name, min(5.0, 0.02 * (2 ** min(n, 8))))
            except Exception:  # noqa: BLE001
                self.stats["errors"] += 1
                log.exception("reconcile %s %s/%s failed", kind, ns, name)
                self.enqueue(kind, ns, name, 1.0)
            finally:
                self.processing.discard(key)
                if key in self.dirty:
                    self.dirty.discard(key)
                    self.enqueue(kind, ns, name)

    async def start(self, workers: int = 4):
        self.queue = asyncio.Queue()
        while not await self._acquire_lease():
            await asyncio.sleep(self.lease.retry_period_s if self.lease else 2)
        self.is_leader = True
        q = self.store.watch(None)  # register before listing: no missed events
        if isinstance(self.store, APIStore):
            # in-memory store: its watch has no initial LIST; a KubeClient
            # reflector delivers the initial LIST as ADDED events itself
            for o in [o for kind in self.reconcilers for o in self.store.list(kind)]:
                self._map("ADDED", o)
        self.tasks = [asyncio.ensure_future(self._watch_loop(q)),
                      asyncio.ensure_future(self._timer_loop())]
        if self.lease is not None:
            self.tasks.append(asyncio.ensure_future(self._renew_loop()))
        self.tasks += [asyncio.ensure_future(self._worker()) for _ in range(workers)]

    async def settle(self, timeout: float = 10.0, quiet: float = 0.2) -> None:
        """Wait until the queue drains and stays empty for `quiet` seconds."""
        t0 = time.monotonic()
        calm = None
        while time.monotonic() - t0 < timeout:
            busy = not self.queue.empty() or bool(self.pending) or bool(
                self.processing) or any(
                t <= time.monotonic() + quiet for t in self.delayed.values())
            if busy:
                calm = None
            else:
                calm = calm or time.monotonic()
                if time.monotonic() - calm >= quiet:
                    return
            await asyncio.sleep(0.02)

    async def stop(self):
        for t in self.tasks:
            t.cancel()
        await asyncio.gather(*self.tasks, return_exceptions=True)
        if self.lease is not None and self.is_leader:
            await asyncio.to_thread(self.lease.release)  # ReleaseOnCancel
        self.is_leader = False
