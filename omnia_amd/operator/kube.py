"""Real-cluster mode: a Kubernetes API client with the same surface as the
in-memory :class:`~omnia_amd.operator.apistore.APIStore`.

The reconcilers (``controllers.py``) and the manager only call ``get`` /
``try_get`` / ``list`` / ``create`` / ``update`` / ``update_status`` / ``apply`` /
``delete`` / ``watch`` / ``unwatch``.  :class:`KubeClient` implements those over
the kube-apiserver REST API, so ``omnia operator --kube`` runs the same
controllers against a real cluster the way the reference's controller-runtime
manager does (``cmd/main.go:400-537``):

* credentials: in-cluster service-account token + CA
  (``/var/run/secrets/kubernetes.io/serviceaccount``, re-read on every request
  so projected/bound tokens rotate), or a kubeconfig (token / basic / client
  certificate, ``insecure-skip-tls-verify``);
* CRUD with the REST path rules (core ``/api/v1``, groups
  ``/apis/{group}/{version}``, namespaced vs cluster scope), the ``/status``
  subresource, optimistic concurrency on ``metadata.resourceVersion``;
* ``apply`` is server-side apply (``PATCH`` ``application/apply-patch+yaml``,
  ``fieldManager=omnia-operator``, ``force=true``) like controller-runtime's
  ``client.Apply``; merge-patch / JSON-patch are available via :meth:`patch`;
* ``watch`` runs a reflector per kind: LIST (records the list
  ``resourceVersion``) then WATCH from it with ``allowWatchBookmarks``;
  BOOKMARKs advance the resourceVersion, a dropped stream resumes from the last
  one, and ``410 Gone`` (compacted history) triggers a re-list whose diff
  against the reflector cache is replayed as ADDED / MODIFIED / DELETED so the
  consumer never misses a transition (client-go ``reflector.go`` semantics);
* :class:`LeaseLock` is ``coordination.k8s.io/v1`` Lease leader election
  (holderIdentity / acquireTime / renewTime as MicroTime / leaseDurationSeconds /
  leaseTransitions, compare-and-swap on resourceVersion), usable with either
  backend.

Errors map onto the APIStore exceptions (404 NotFound, 409 Conflict,
422 Invalid) so controller code is backend-agnostic.
"""
from __future__ import annotations

import asyncio
import base64
import copy
import datetime as _dt
import json
import logging
import os
import ssl
import tempfile
import threading
import time
import urllib.error
import urllib.parse
import urllib.request

import yaml

from ..api import crds
from .apistore import Conflict, Invalid, NotFound

log = logging.getLogger("omnia.operator.kube")

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
FIELD_MANAGER = "omnia-operator"


class KubeError(RuntimeError):
    def __init__(self, code: int, message: str, reason: str = ""):
        self.code, self.reason = code, reason
        super().__init__(f"{code} {reason}: {message}")


class Gone(KubeError):
    """410: the requested resourceVersion has been compacted away."""


# (group/version, plural, namespaced) of the built-in kinds the operator touches
BUILTIN: dict[str, tuple[str, str, bool]] = {
    "ConfigMap": ("v1", "configmaps", True), "Secret": ("v1", "secrets", True),
    "Service": ("v1", "services", True), "ServiceAccount": ("v1", "serviceaccounts", True),
    "Namespace": ("v1", "namespaces", False), "Pod": ("v1", "pods", True),
    "Event": ("v1", "events", True),
    "PersistentVolumeClaim": ("v1", "persistentvolumeclaims", True),
    "Deployment": ("apps/v1", "deployments", True),
    "StatefulSet": ("apps/v1", "statefulsets", True),
    "Job": ("batch/v1", "jobs", True), "CronJob": ("batch/v1", "cronjobs", True),
    "HorizontalPodAutoscaler": ("autoscaling/v2", "horizontalpodautoscalers", True),
    "PodDisruptionBudget": ("policy/v1", "poddisruptionbudgets", True),
    "Role": ("rbac.authorization.k8s.io/v1", "roles", True),
    "RoleBinding": ("rbac.authorization.k8s.io/v1", "rolebindings", True),
    "ClusterRole": ("rbac.authorization.k8s.io/v1", "clusterroles", False),
    "ClusterRoleBinding": ("rbac.authorization.k8s.io/v1", "clusterrolebindings", False),
    "NetworkPolicy": ("networking.k8s.io/v1", "networkpolicies", True),
    "Lease": ("coordination.k8s.io/v1", "leases", True),
    "HTTPRoute": ("gateway.networking.k8s.io/v1", "httproutes", True),
    "ScaledObject": ("keda.sh/v1alpha1", "scaledobjects", True),
    "VirtualService": ("networking.istio.io/v1beta1", "virtualservices", True),
    "DestinationRule": ("networking.istio.io/v1beta1", "destinationrules", True),
    "CustomResourceDefinition": ("apiextensions.k8s.io/v1", "customresourcedefinitions",
                                 False),
}


def resource_of(kind: str) -> tuple[str, str, bool]:
    k = crds.KINDS.get(kind)
    if k is not None:
        return crds.API_VERSION, k.plural, k.scope == "Namespaced"
    if kind in BUILTIN:
        return BUILTIN[kind]
    raise KeyError(f"unknown kind {kind}")


def resource_path(kind: str, ns: str | None = None, name: str | None = None,
                  sub: str | None = None) -> str:
    gv, plural, namespaced = resource_of(kind)
    base = "/api/v1" if gv == "v1" else f"/apis/{gv}"
    p = base
    if namespaced and ns:
        p += f"/namespaces/{urllib.parse.quote(ns)}"
    p += f"/{plural}"
    if name:
        p += f"/{urllib.parse.quote(name)}"
        if sub:
            p += f"/{sub}"
    return p


def selector_string(selector: dict | None) -> str:
    """LabelSelector -> the ``labelSelector`` query syntax."""
    if not selector:
        return ""
    ml = selector.get("matchLabels", selector if "matchExpressions" not in selector else {})
    parts = [f"{k}={v}" for k, v in sorted((ml or {}).items())]
    for ex in selector.get("matchExpressions", []) or []:
        op, key, vals = ex["operator"], ex["key"], ex.get("values") or []
        if op == "In":
            parts.append(f"{key} in ({','.join(vals)})")
        elif op == "NotIn":
            parts.append(f"{key} notin ({','.join(vals)})")
        elif op == "Exists":
            parts.append(key)
        elif op == "DoesNotExist":
            parts.append(f"!{key}")
    return ",".join(parts)


def micro_time(t: float | None = None) -> str:
    """metav1.MicroTime wire format."""
    d = _dt.datetime.fromtimestamp(time.time() if t is None else t, _dt.timezone.utc)
    return d.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_time(s: str) -> float:
    s = s.rstrip("Z")
    fmt = "%Y-%m-%dT%H:%M:%S.%f" if "." in s else "%Y-%m-%dT%H:%M:%S"
    return _dt.datetime.strptime(s, fmt).replace(tzinfo=_dt.timezone.utc).timestamp()


# ============================================================== configuration
class KubeConfig:
    def __init__(self, server: str, token: str | None = None, token_file: str | None = None,
                 ca_file: str | None = None, insecure: bool = False,
                 cert_file: str | None = None, key_file: str | None = None,
                 username: str | None = None, password: str | None = None,
                 namespace: str = "default"):
        self.server = server.rstrip("/")
        self.token, self.token_file = token, token_file
        self.ca_file, self.insecure = ca_file, insecure
        self.cert_file, self.key_file = cert_file, key_file
        self.username, self.password = username, password
        self.namespace = namespace

    @classmethod
    def in_cluster(cls, sa_dir: str = SA_DIR) -> "KubeConfig":
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        ns = "default"
        nsf = os.path.join(sa_dir, "namespace")
        if os.path.exists(nsf):
            with open(nsf) as f:
                ns = f.read().strip() or ns
        return cls(f"https://{host}:{port}", token_file=os.path.join(sa_dir, "token"),
                   ca_file=os.path.join(sa_dir, "ca.crt"), namespace=ns)

    @classmethod
    def from_kubeconfig(cls, path: str | None = None, context: str | None = None) -> "KubeConfig":
        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        with open(path) as f:
            kc = yaml.safe_load(f)
        ctx_name = context or kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cl = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in kc.get("users", []) if u["name"] == ctx.get("user")), {})
        tmp = []

        def materialise(data_key, file_key, src):
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="omnia-kube-")
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(src[data_key]))
                tmp.append(p)
                return p
            return None

        return cls(cl["server"], token=user.get("token"), token_file=user.get("tokenFile"),
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cl),
                   insecure=bool(cl.get("insecure-skip-tls-verify")),
                   cert_file=materialise("client-certificate-data", "client-certificate", user),
                   key_file=materialise("client-key-data", "client-key", user),
                   username=user.get("username"), password=user.get("password"),
                   namespace=ctx.get("namespace", "default"))

    @classmethod
    def auto(cls) -> "KubeConfig":
        if os.environ.get("KUBERNETES_SERVICE_HOST") and os.path.exists(
                os.path.join(SA_DIR, "token")):
            return cls.in_cluster()
        return cls.from_kubeconfig()

    def bearer(self) -> str | None:
        if self.token_file and os.path.exists(self.token_file):
            with open(self.token_file) as f:  # re-read: bound tokens rotate
                return f.read().strip()
        return self.token

    def ssl_context(self) -> ssl.SSLContext | None:
        if not self.server.startswith("https"):
            return None
        ctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else \
            ssl.create_default_context()
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        if self.cert_file:
            ctx.load_cert_chain(self.cert_file, self.key_file)
        return ctx


# ============================================================== client
class KubeClient:
    """APIStore-compatible client of a real kube-apiserver."""

    def __init__(self, cfg: KubeConfig, field_manager: str = FIELD_MANAGER,
                 timeout: float = 30.0, watch_timeout_s: int = 300,
                 field_validation: str = "Strict"):
        self.cfg = cfg
        self.field_validation = field_validation  # what kubectl sends
        self.field_manager = field_manager
        self.timeout = timeout
        self.watch_timeout_s = watch_timeout_s
        self._ssl = cfg.ssl_context()
        self._reflectors: list[_Reflector] = []

    # ---------------------------------------------------------------- transport
    def _request(self, method: str, path: str, body=None, query: dict | None = None,
                 content_type: str = "application/json", stream: bool = False,
                 timeout: float | None = None):
        url = self.cfg.server + path
        q = {k: v for k, v in (query or {}).items() if v not in (None, "")}
        if q:
            url += "?" + urllib.parse.urlencode(q)
        data = None
        if body is not None:
            data = body if isinstance(body, bytes) else json.dumps(body).encode()
        req = urllib.request.Request(url, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        tok = self.cfg.bearer()
        if tok:
            req.add_header("Authorization", f"Bearer {tok}")
        elif self.cfg.username:
            cred = base64.b64encode(f"{self.cfg.username}:{self.cfg.password or ''}".encode())
            req.add_header("Authorization", "Basic " + cred.decode())
        try:
            resp = urllib.request.urlopen(req, timeout=timeout or self.timeout,
                                          context=self._ssl)
        except urllib.error.HTTPError as e:
            raw = e.read()
            try:
                st = json.loads(raw)
            except ValueError:
                st = {"message": raw.decode(errors="replace")}
            raise _error(e.code, st) from None
        if stream:
            return resp
        with resp:
            raw = resp.read()
        return json.loads(raw) if raw else {}

    # ---------------------------------------------------------------- CRUD
    @staticmethod
    def _with_type(kind: str, obj: dict) -> dict:
        gv, _, _ = resource_of(kind)
        obj.setdefault("kind", kind)
        obj.setdefault("apiVersion", gv)
        return obj

    def serves(self, api_version: str, kind: str) -> bool:
        """API discovery: is ``kind`` served under ``api_version`` (cached)?"""
        cache = self.__dict__.setdefault("_served", {})
        key = (api_version, kind)
        if key not in cache:
            path = ("/api/" if "/" not in api_version else "/apis/") + api_version
            try:
                doc = self._request("GET", path)
                cache[key] = any(r.get("kind") == kind for r in doc.get("resources", []))
            except Exception:  # noqa: BLE001 - 404: group/version not installed
                cache[key] = False
        return cache[key]

    def get(self, kind: str, name: str, ns: str | None = "default") -> dict:
        return self._with_type(kind, self._request("GET", resource_path(kind, ns, name)))

    def try_get(self, kind, name, ns="default"):
        try:
            return self.get(kind, name, ns)
        except NotFound:
            return None

    def list_with_rv(self, kind: str, ns: str | None = None,
                     selector: dict | None = None) -> tuple[list[dict], str]:
        out = self._request("GET", resource_path(kind, ns),
                            query={"labelSelector": selector_string(selector)})
        items = [self._with_type(kind, o) for o in out.get("items") or []]
        return items, (out.get("metadata") or {}).get("resourceVersion", "")

    def list(self, kind: str, ns: str | None = None, selector: dict | None = None) -> list[dict]:
        items, _ = self.list_with_rv(kind, ns, selector)
        return sorted(items, key=lambda o: (o["metadata"].get("namespace", ""),
                                            o["metadata"]["name"]))

    def create(self, obj: dict) -> dict:
        obj = copy.deepcopy(obj)
        kind = obj["kind"]
        self._with_type(kind, obj)
        md = obj.setdefault("metadata", {})
        ns = md.get("namespace") or ("default" if resource_of(kind)[2] else None)
        if resource_of(kind)[2]:
            md["namespace"] = ns
        return self._with_type(kind, self._request(
            "POST", resource_path(kind, ns), obj,
            query={"fieldValidation": self.field_validation}))

    def update(self, obj: dict, subresource: str | None = None) -> dict:
        kind, md = obj["kind"], obj["metadata"]
        obj = self._with_type(kind, copy.deepcopy(obj))
        return self._with_type(kind, self._request(
            "PUT", resource_path(kind, md.get("namespace"), md["name"], subresource), obj,
            query={"fieldValidation": self.field_validation}))

    def update_status(self, obj: dict) -> dict:
        return self.update(obj, subresource="status")

    def patch(self, kind: str, name: str, ns: str | None, body,
              patch_type: str = "merge", subresource: str | None = None,
              force: bool = False) -> dict:
        ctype = {"merge": "application/merge-patch+json",
                 "json": "application/json-patch+json",
                 "strategic": "application/strategic-merge-patch+json",
                 "apply": "application/apply-patch+yaml"}[patch_type]
        query = {"fieldManager": self.field_manager, "fieldValidation": self.field_validation}
        if patch_type == "apply" and force:
            query["force"] = "true"
        return self._with_type(kind, self._request(
            "PATCH", resource_path(kind, ns, name, subresource), body, query=query,
            content_type=ctype))

    def apply(self, obj: dict) -> dict:
        """Server-side apply with this manager's field ownership (force=true)."""
        obj = copy.deepcopy(obj)
        kind, md = obj["kind"], obj.setdefault("metadata", {})
        self._with_type(kind, obj)
        ns = md.get("namespace") or ("default" if resource_of(kind)[2] else None)
        if resource_of(kind)[2]:
            md["namespace"] = ns
        md.pop("resourceVersion", None)
        obj.pop("status", None)
        return self.patch(kind, md["name"], ns, obj, "apply", force=True)

    def delete(self, kind: str, name: str, ns: str | None = "default",
               propagation: str = "Background") -> bool:
        try:
            self._request("DELETE", resource_path(kind, ns, name),
                          {"kind": "DeleteOptions", "apiVersion": "v1",
                           "propagationPolicy": propagation})
            return True
        except NotFound:
            return False

    # ---------------------------------------------------------------- watch
    def watch_stream(self, kind: str, ns: str | None, resource_version: str,
                     timeout_s: int | None = None):
        """Yield (type, object) from one WATCH request (ends at its timeout)."""
        resp = self._request("GET", resource_path(kind, ns), query={
            "watch": "1", "resourceVersion": resource_version, "allowWatchBookmarks": "true",
            "timeoutSeconds": str(timeout_s or self.watch_timeout_s)}, stream=True,
            timeout=(timeout_s or self.watch_timeout_s) + 30)
        with resp:
            for line in resp:
                line = line.strip()
                if not line:
                    continue
                ev = json.loads(line)
                if ev.get("type") == "ERROR":
                    st = ev.get("object") or {}
                    raise _error(int(st.get("code", 500)), st)
                yield ev["type"], ev["object"]

    def watch(self, kind: str | None = None, ns: str | None = None) -> asyncio.Queue:
        """Queue of (event type, object) fed by reflector threads (one per kind;
        ``kind=None`` watches every kind the operator reconciles or owns)."""
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        kinds = [kind] if kind else list(crds.KINDS) + [
            "ConfigMap", "Secret", "Deployment", "Service"]
        for k in kinds:
            r = _Reflector(self, k, ns, loop, q)
            self._reflectors.append(r)
            r.start()
        return q

    def unwatch(self, q):
        for r in [r for r in self._reflectors if r.q is q]:
            r.stop()
            self._reflectors.remove(r)

    def close(self):
        for r in self._reflectors:
            r.stop()
        self._reflectors.clear()


def _error(code: int, status: dict) -> Exception:
    msg = status.get("message", "")
    reason = status.get("reason", "")
    if code == 404:
        return NotFound(msg)
    if code == 409:
        return Conflict(msg)
    if code == 422:
        causes = [c.get("message", "") for c in (status.get("details") or {}).get(
            "causes", [])] or [msg]
        return Invalid(causes)
    if code == 410:
        return Gone(code, msg, reason or "Expired")
    return KubeError(code, msg, reason)


class _Reflector:
    """LIST + WATCH loop for one kind with bookmark / resume / 410 re-list."""

    def __init__(self, client: KubeClient, kind: str, ns: str | None, loop, q,
                 backoff: float = 0.5):
        self.client, self.kind, self.ns = client, kind, ns
        self.loop, self.q = loop, q
        self.backoff = backoff
        self.rv = ""
        self.cache: dict[tuple, dict] = {}
        self.stats = {"lists": 0, "watches": 0, "bookmarks": 0, "gone": 0, "events": 0}
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True,
                                   name=f"reflector-{kind}")

    def start(self):
        self._t.start()

    def stop(self):
        self._stop.set()

    def _emit(self, etype, obj):
        if self._stop.is_set():
            return
        self.stats["events"] += 1
        try:
            self.loop.call_soon_threadsafe(self.q.put_nowait, (etype, obj))
        except RuntimeError:
            self._stop.set()

    @staticmethod
    def _key(o):
        md = o["metadata"]
        return (md.get("namespace", ""), md["name"])

    def _relist(self):
        items, rv = self.client.list_with_rv(self.kind, self.ns)
        self.stats["lists"] += 1
        fresh = {self._key(o): o for o in items}
        for k, o in fresh.items():
            old = self.cache.get(k)
            if old is None:
                self._emit("ADDED", o)
            elif old["metadata"].get("resourceVersion") != o["metadata"].get("resourceVersion"):
                self._emit("MODIFIED", o)
        for k, o in self.cache.items():
            if k not in fresh:
                self._emit("DELETED", o)
        self.cache = fresh
        self.rv = rv

    def _run(self):
        need_list = True
        while not self._stop.is_set():
            try:
                if need_list:
                    self._relist()
                    need_list = False
                self.stats["watches"] += 1
                for etype, obj in self.client.watch_stream(self.kind, self.ns, self.rv):
                    if self._stop.is_set():
                        return
                    if etype == "BOOKMARK":
                        self.stats["bookmarks"] += 1
                        self.rv = obj["metadata"]["resourceVersion"]
                        continue
                    obj = KubeClient._with_type(self.kind, obj)
                    self.rv = obj["metadata"].get("resourceVersion", self.rv)
                    k = self._key(obj)
                    if etype == "DELETED":
                        self.cache.pop(k, None)
                    else:
                        self.cache[k] = obj
                    self._emit(etype, obj)
            except Gone:
                self.stats["gone"] += 1
                need_list = True
            except (KubeError, OSError, ValueError) as e:
                if self._stop.is_set():
                    return
                log.debug("reflector %s: %s; retrying", self.kind, e)
                time.sleep(self.backoff)
            except NotFound:
                # kind not served (e.g. Gateway API CRDs absent): back off
                time.sleep(max(self.backoff, 5.0))


# ============================================================== leader election
class LeaseLock:
    """Lease-based leader election (client-go ``leaderelection`` semantics).

    Works against any store with the APIStore surface: a renewal is a
    compare-and-swap on ``metadata.resourceVersion``, so two candidates racing
    for an expired lease cannot both win.
    """

    def __init__(self, store, name: str, namespace: str, identity: str,
                 lease_duration_s: int = 15, renew_deadline_s: float = 10.0,
                 retry_period_s: float = 2.0, clock=time.time):
        self.store, self.name, self.ns = store, name, namespace
        self.identity = identity
        self.lease_duration_s = lease_duration_s
        self.renew_deadline_s = renew_deadline_s
        self.retry_period_s = retry_period_s
        self.clock = clock
        self.last_renew = 0.0

    def _spec(self, transitions: int, acquire: str | None = None) -> dict:
        now = micro_time(self.clock())
        return {"holderIdentity": self.identity, "leaseDurationSeconds": self.lease_duration_s,
                "acquireTime": acquire or now, "renewTime": now,
                "leaseTransitions": transitions}

    def try_acquire_or_renew(self) -> bool:
        lease = self.store.try_get("Lease", self.name, self.ns)
        now = self.clock()
        if lease is None:
            try:
                self.store.create({"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                                   "metadata": {"name": self.name, "namespace": self.ns},
                                   "spec": self._spec(0)})
            except Conflict:
                return False
            self.last_renew = now
            return True
        sp = lease.get("spec") or {}
        holder = sp.get("holderIdentity") or ""
        renew = sp.get("renewTime")
        try:
            renewed_at = parse_time(renew) if isinstance(renew, str) else float(renew or 0)
        except ValueError:
            renewed_at = 0.0
        expired = now > renewed_at + float(sp.get("leaseDurationSeconds") or
                                           self.lease_duration_s)
        if holder and holder != self.identity and not expired:
            return False
        transitions = int(sp.get("leaseTransitions") or 0)
        if holder == self.identity:
            lease["spec"] = self._spec(transitions, sp.get("acquireTime"))
        else:
            lease["spec"] = self._spec(transitions + 1)
        try:
            self.store.update(lease)  # carries resourceVersion: CAS
        except Conflict:
            return False
        self.last_renew = now
        return True

    def release(self) -> None:
        # a renew already in flight on a worker thread when the renew task was
        # cancelled can land between our read and write: re-read and retry on
        # the resulting Conflict instead of leaving the lease held
        for _ in range(5):
            lease = self.store.try_get("Lease", self.name, self.ns)
            if lease is None or (lease.get("spec") or {}).get("holderIdentity") != self.identity:
                return
            lease["spec"]["holderIdentity"] = ""
            lease["spec"]["leaseDurationSeconds"] = 1
            try:
                self.store.update(lease)
                return
            except NotFound:
                return
            except Conflict:
                time.sleep(0.02)

    def holds(self) -> bool:
        return self.clock() - self.last_renew < self.renew_deadline_s
