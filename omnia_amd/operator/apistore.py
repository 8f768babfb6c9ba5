"""In-memory Kubernetes-style API server (objects + watch + admission + GC).

Stand-in for the kube-apiserver/etcd pair the reference's envtest suites use
(``internal/controller/suite_test.go:81-135``): resourceVersion / generation
bookkeeping (generation bumps only on spec changes), a status subresource,
finalizers + deletionTimestamp, ownerReference garbage collection, label
selectors, and watch streams (ADDED / MODIFIED / DELETED) that drive the
controllers.  Omnia kinds go through admission (defaults + schema + CEL +
webhooks) on create/update.  Core kinds (ConfigMap, Secret, Deployment,
Service, HPA, ScaledObject, PDB, HTTPRoute, RBAC, NetworkPolicy, PVC,
Namespace, Lease...) are stored as-is.
"""
from __future__ import annotations

import asyncio
import collections
import copy
import datetime as _dt
import itertools
import threading
import uuid

from ..api import crds


class NotFound(KeyError):
    pass


class Conflict(Exception):
    pass


class Gone(Exception):
    """The requested resourceVersion is older than the retained watch history."""


class Invalid(ValueError):
    def __init__(self, errors: list[str]):
        self.errors = errors
        super().__init__("; ".join(errors))


CLUSTER_SCOPED = {"Namespace", "ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition"}


def is_namespaced(kind: str) -> bool:
    k = crds.KINDS.get(kind)
    if k is not None:
        return k.scope == "Namespaced"
    return kind not in CLUSTER_SCOPED


def now_ts() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def match_labels(labels: dict, selector: dict | None) -> bool:
    if not selector:
        return True
    ml = selector.get("matchLabels", selector if "matchExpressions" not in selector else {})
    for k, v in (ml or {}).items():
        if (labels or {}).get(k) != v:
            return False
    for ex in selector.get("matchExpressions", []) or []:
        val = (labels or {}).get(ex["key"])
        op = ex["operator"]
        if op == "In" and val not in ex.get("values", []):
            return False
        if op == "NotIn" and val in ex.get("values", []):
            return False
        if op == "Exists" and val is None:
            return False
        if op == "DoesNotExist" and val is not None:
            return False
    return True


class APIStore:
    def __init__(self, webhooks: dict | None = None, history: int = 10000,
                 field_validation: str = "Strict"):
        self.objs: dict[tuple, dict] = {}
        self.rv = itertools.count(1)
        self.last_rv = 0
        self.lock = threading.RLock()
        self.watchers: list[tuple] = []  # (kind or None, loop, queue)
        self.webhooks = webhooks or {}  # kind -> fn(obj, old) -> list[str] errors
        # bounded event history (etcd's compaction window): a watch may resume
        # from any resourceVersion still inside it, older ones get 410 Gone
        self.history: collections.deque = collections.deque(maxlen=history)
        # default fieldValidation for writes that do not pass one (kubectl: Strict)
        self.field_validation = field_validation
        self.warnings: list[str] = []  # last write's warnings (Warn mode pruning)
        self.compacted_rv = 0
        # third-party API kinds this "cluster" serves, e.g. Istio's
        # ("security.istio.io/v1", "AuthorizationPolicy") -- discovery stand-in
        self.served: set[tuple[str, str]] = set()

    # ------------------------------------------------------------ helpers
    @staticmethod
    def key(kind: str, ns: str | None, name: str) -> tuple:
        return (kind, ns if is_namespaced(kind) else "", name)

    def _next_rv(self) -> str:
        self.last_rv = next(self.rv)
        return str(self.last_rv)

    def serves(self, api_version: str, kind: str) -> bool:
        return kind in crds.KINDS or (api_version, kind) in self.served

    def current_rv(self) -> str:
        return str(self.last_rv)

    def _notify(self, etype: str, obj: dict):
        ev = (etype, copy.deepcopy(obj))
        with self.lock:
            if len(self.history) == self.history.maxlen:
                self.compacted_rv = self.history[0][0]
            self.history.append((int(obj["metadata"].get("resourceVersion") or 0), ev))
        for kind, loop, q in list(self.watchers):
            if kind is None or kind == obj["kind"]:
                try:
                    loop.call_soon_threadsafe(q.put_nowait, ev)
                except RuntimeError:
                    self.watchers.remove((kind, loop, q))

    def watch(self, kind: str | None = None) -> asyncio.Queue:
        q: asyncio.Queue = asyncio.Queue()
        self.watchers.append((kind, asyncio.get_running_loop(), q))
        return q

    def events_since(self, rv: int, kind: str | None = None) -> list[tuple]:
        """Events with resourceVersion > rv, or Gone if rv was compacted away."""
        with self.lock:
            if rv < self.compacted_rv:
                raise Gone(f"too old resource version: {rv} ({self.compacted_rv})")
            return sorted(((r, copy.deepcopy(ev)) for r, ev in self.history
                           if r > rv and (kind is None or ev[1]["kind"] == kind)),
                          key=lambda x: x[0])

    def unwatch(self, q):
        self.watchers = [w for w in self.watchers if w[2] is not q]

    def _admit(self, obj: dict, old: dict | None, field_validation: str | None = None):
        kind = obj.get("kind")
        self.warnings = []
        if kind in crds.KINDS:
            errs = crds.validate_object(obj, old, field_validation or self.field_validation,
                                        self.warnings)
            hook = self.webhooks.get(kind)
            if hook is not None and not errs:
                errs += hook(obj, old) or []
            if errs:
                raise Invalid(errs)

    # ------------------------------------------------------------ CRUD
    def create(self, obj: dict, field_validation: str | None = None) -> dict:
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if not md.get("name") and md.get("generateName"):
            md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
        kind = obj["kind"]
        if is_namespaced(kind):
            md.setdefault("namespace", "default")
        else:
            md.pop("namespace", None)
        self._admit(obj, None, field_validation)
        with self.lock:
            k = self.key(kind, md.get("namespace"), md["name"])
            if k in self.objs:
                raise Conflict(f"{kind} {md['name']} already exists")
            md["uid"] = str(uuid.uuid4())
            md["resourceVersion"] = self._next_rv()
            md["generation"] = 1
            md["creationTimestamp"] = now_ts()
            obj.setdefault("status", {})
            self.objs[k] = obj
            out = copy.deepcopy(obj)
        self._notify("ADDED", obj)
        return out

    def get(self, kind: str, name: str, ns: str | None = "default") -> dict:
        with self.lock:
            o = self.objs.get(self.key(kind, ns, name))
            if o is None:
                raise NotFound(f"{kind} {ns}/{name} not found")
            return copy.deepcopy(o)

    def try_get(self, kind, name, ns="default"):
        try:
            return self.get(kind, name, ns)
        except NotFound:
            return None

    def list(self, kind: str, ns: str | None = None, selector: dict | None = None) -> list[dict]:
        with self.lock:
            out = [copy.deepcopy(o) for (k, n, _), o in self.objs.items()
                   if k == kind and (ns is None or n == (ns if is_namespaced(kind) else ""))
                   and match_labels(o["metadata"].get("labels", {}), selector)]
        return sorted(out, key=lambda o: (o["metadata"].get("namespace", ""),
                                          o["metadata"]["name"]))

    def update(self, obj: dict, subresource: str | None = None,
               field_validation: str | None = None) -> dict:
        obj = copy.deepcopy(obj)
        kind, md = obj["kind"], obj["metadata"]
        with self.lock:
            k = self.key(kind, md.get("namespace"), md["name"])
            cur = self.objs.get(k)
            if cur is None:
                raise NotFound(f"{kind} {md['name']} not found")
            rv = md.get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{kind} {md['name']}: resourceVersion conflict")
            if subresource == "status":
                new = copy.deepcopy(cur)
                new["status"] = obj.get("status", {})
            else:
                new = obj
                new["status"] = cur.get("status", {})
                for f in ("uid", "creationTimestamp", "generation", "deletionTimestamp"):
                    if f in cur["metadata"]:
                        new["metadata"][f] = cur["metadata"][f]
                if new.get("spec") != cur.get("spec") or {k2: v for k2, v in new.items()
                                                          if k2 not in ("metadata", "status",
                                                                        "spec")} != \
                        {k2: v for k2, v in cur.items() if k2 not in ("metadata", "status",
                                                                      "spec")}:
                    self._admit(new, cur, field_validation)
                    if new.get("spec") != cur.get("spec"):
                        new["metadata"]["generation"] = cur["metadata"]["generation"] + 1
            if _same(new, cur):
                return copy.deepcopy(cur)  # no-op write: no new resourceVersion, no event
            new["metadata"]["resourceVersion"] = self._next_rv()
            if new["metadata"].get("deletionTimestamp") and not new["metadata"].get(
                    "finalizers"):
                self.objs.pop(k, None)
                gone = True
            else:
                self.objs[k] = new
                gone = False
            out = copy.deepcopy(new)
        if gone:
            self._notify("DELETED", out)
            self._gc(out)
        else:
            self._notify("MODIFIED", out)
        return out

    def update_status(self, obj: dict) -> dict:
        return self.update(obj, subresource="status")

    def apply(self, obj: dict, field_validation: str | None = None) -> dict:
        """Create-or-update (server-side-apply-lite): spec/labels/annotations/data win."""
        md = obj.get("metadata", {})
        cur = self.try_get(obj["kind"], md.get("name"), md.get("namespace", "default"))
        if cur is None:
            return self.create(obj, field_validation)
        new = copy.deepcopy(cur)
        for k, v in obj.items():
            if k in ("metadata", "status"):
                continue
            new[k] = copy.deepcopy(v)
        for f in ("labels", "annotations", "ownerReferences"):
            if f in md:
                new["metadata"][f] = copy.deepcopy(md[f])
        new["metadata"].pop("resourceVersion", None)
        if new == cur:
            return cur
        return self.update(new, field_validation=field_validation)

    def delete(self, kind: str, name: str, ns: str | None = "default") -> bool:
        with self.lock:
            k = self.key(kind, ns, name)
            cur = self.objs.get(k)
            if cur is None:
                return False
            if cur["metadata"].get("finalizers"):
                if not cur["metadata"].get("deletionTimestamp"):
                    cur["metadata"]["deletionTimestamp"] = now_ts()
                    cur["metadata"]["resourceVersion"] = self._next_rv()
                    out = copy.deepcopy(cur)
                else:
                    return True
                gone = False
            else:
                self.objs.pop(k)
                out = copy.deepcopy(cur)
                out["metadata"]["resourceVersion"] = self._next_rv()
                gone = True
        self._notify("DELETED" if gone else "MODIFIED", out)
        if gone:
            self._gc(out)
        return True

    def _gc(self, owner: dict):
        uid = owner["metadata"].get("uid")
        with self.lock:
            children = [o for o in self.objs.values()
                        if any(r.get("uid") == uid for r in
                               o["metadata"].get("ownerReferences", []) or [])]
        for c in children:
            self.delete(c["kind"], c["metadata"]["name"], c["metadata"].get("namespace"))


def _same(a: dict, b: dict) -> bool:
    def strip(o):
        o = dict(o)
        o["metadata"] = {k: v for k, v in o["metadata"].items() if k != "resourceVersion"}
        return o

    return strip(a) == strip(b)


def owner_ref(owner: dict, controller: bool = True) -> dict:
    return {"apiVersion": owner.get("apiVersion", crds.API_VERSION), "kind": owner["kind"],
            "name": owner["metadata"]["name"], "uid": owner["metadata"]["uid"],
            "controller": controller, "blockOwnerDeletion": True}


def set_condition(status: dict, ctype: str, ok: bool, reason: str, message: str = "",
                  generation: int | None = None) -> None:
    conds = status.setdefault("conditions", [])
    st = "True" if ok else "False"
    for c in conds:
        if c["type"] == ctype:
            if c["status"] != st:
                c["lastTransitionTime"] = now_ts()
            c.update(status=st, reason=reason, message=message)
            if generation is not None:
                c["observedGeneration"] = generation
            return
    conds.append({"type": ctype, "status": st, "reason": reason, "message": message,
                  "lastTransitionTime": now_ts(),
                  **({"observedGeneration": generation} if generation is not None else {})})


def get_condition(obj: dict, ctype: str) -> dict | None:
    for c in (obj.get("status") or {}).get("conditions", []):
        if c["type"] == ctype:
            return c
    return None
