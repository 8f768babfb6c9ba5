"""License activation + heartbeat (``ee/internal/controller/license_activation_controller.go``,
``ee/pkg/license/activation.go``, ``fingerprint.go``).

Enterprise licenses are activated once per cluster against the license server
and then heartbeat every 24 h:

* the reconciler watches only the license Secret ``omnia-system/arena-license``;
  open-core (or missing / invalid) licenses are skipped;
* the cluster fingerprint is ``sha256("<kube-system uid>:<omnia-system uid>")``,
  first 16 bytes as hex (raw UIDs never leave the cluster);
* no activation state yet -> ``POST {server}/v1/licenses/activate``
  (``license_id, cluster_fingerprint, cluster_name, version``); a successful
  activation is stored as JSON under ``data.state`` of the ConfigMap
  ``omnia-system/arena-license-activation`` and the next reconcile is the
  heartbeat interval away; a rejection (activation limit reached) is an Event,
  not a retry loop;
* transport / server failures back off exponentially per license id (1 min,
  doubling, capped at 1 h) and after 24 h of failing drop to one retry every
  6 h; the first failure of a streak records a Warning event;
* with state present, ``POST {server}/v1/licenses/{id}/heartbeat`` runs when the
  last one is 24 h old; failures count ``heartbeat_failures`` (the 7-day grace
  period starts at the last good heartbeat) and retry hourly;
* :meth:`LicenseActivationReconciler.deactivate` releases the activation
  (``DELETE .../activations/{fingerprint}``) and deletes the state ConfigMap.
"""
from __future__ import annotations

import calendar
import hashlib
import json
import logging
import threading
import time
import urllib.error
import urllib.request

from .license import TIER_OPEN_CORE, LicenseError

log = logging.getLogger("omnia.ee.license")

LICENSE_SECRET_NAME = "arena-license"
LICENSE_NAMESPACE = "omnia-system"
ACTIVATION_CONFIGMAP = "arena-license-activation"
DEFAULT_SERVER = "https://license.altairalabs.ai"
HEARTBEAT_INTERVAL_S = 24 * 3600.0
GRACE_PERIOD_S = 7 * 24 * 3600.0
BACKOFF_BASE_S = 60.0
BACKOFF_CAP_S = 3600.0
GIVE_UP_AFTER_S = 24 * 3600.0
SLOW_INTERVAL_S = 6 * 3600.0
MAX_SHIFT = 6
VERSION = "dev"


def _iso(t: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def _parse_iso(v) -> float:
    if not v:
        return 0.0
    return float(calendar.timegm(time.strptime(str(v)[:19], "%Y-%m-%dT%H:%M:%S")))


def cluster_fingerprint(store) -> str:
    ks = store.get("Namespace", "kube-system", None)
    om = store.get("Namespace", LICENSE_NAMESPACE, None)
    raw = f"{ks['metadata']['uid']}:{om['metadata']['uid']}"
    return hashlib.sha256(raw.encode()).hexdigest()[:32]


class ActivationError(Exception):
    pass


class ActivationClient:
    """JSON client for the license server."""

    def __init__(self, server_url: str = DEFAULT_SERVER, timeout_s: float = 30.0):
        self.url = server_url.rstrip("/")
        self.timeout = timeout_s

    def _do(self, method: str, path: str, body: dict | None = None) -> dict:
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(self.url + path, data=data, method=method,
                                     headers={"Content-Type": "application/json",
                                              "User-Agent": f"omnia-operator/{VERSION}"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                raw = r.read()
        except urllib.error.HTTPError as e:
            raise ActivationError(f"license server returned {e.code}: "
                                  f"{e.read()[:200].decode(errors='replace')}") from e
        except (urllib.error.URLError, OSError) as e:
            raise ActivationError(f"license server unreachable: {e}") from e
        return json.loads(raw or b"{}")

    def activate(self, license_id: str, fingerprint: str, cluster_name: str = "") -> dict:
        return self._do("POST", "/v1/licenses/activate", {
            "license_id": license_id, "cluster_fingerprint": fingerprint,
            "cluster_name": cluster_name, "version": VERSION})

    def heartbeat(self, license_id: str, fingerprint: str, active_jobs: int = 0,
                  worker_count: int = 0) -> dict:
        return self._do("POST", f"/v1/licenses/{license_id}/heartbeat", {
            "cluster_fingerprint": fingerprint, "version": VERSION,
            "active_jobs": active_jobs, "worker_count": worker_count})

    def deactivate(self, license_id: str, fingerprint: str) -> dict:
        return self._do("DELETE", f"/v1/licenses/{license_id}/activations/{fingerprint}")

    def activations(self, license_id: str) -> list:
        return self._do("GET", f"/v1/licenses/{license_id}/activations").get("activations", [])


class LicenseActivationReconciler:
    kind = "Secret"

    def __init__(self, validator, client: ActivationClient | None = None,
                 cluster_name: str = "", now=time.time, secret_name: str = LICENSE_SECRET_NAME):
        self.validator = validator
        self.secret_name = secret_name
        self.client = client or ActivationClient()
        self.cluster_name = cluster_name
        self.now = now
        self._lock = threading.Lock()
        self._failures: dict[str, dict] = {}

    # ------------------------------------------------------------------ state
    def _state(self, store) -> dict | None:
        cm = store.try_get("ConfigMap", ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE)
        if cm is None:
            return None
        raw = (cm.get("data") or {}).get("state")
        if not raw:
            raise ValueError("activation state not found in ConfigMap")
        return json.loads(raw)

    def _save(self, store, state: dict):
        store.apply({"apiVersion": "v1", "kind": "ConfigMap",
                     "metadata": {"name": ACTIVATION_CONFIGMAP, "namespace": LICENSE_NAMESPACE,
                                  "labels": {"app.kubernetes.io/managed-by": "omnia-operator"}},
                     "data": {"state": json.dumps(state, sort_keys=True)}})

    def _event(self, store, type_: str, reason: str, message: str):
        try:
            store.create({"apiVersion": "v1", "kind": "Event",
                          "metadata": {"generateName": f"{LICENSE_SECRET_NAME}.",
                                       "namespace": LICENSE_NAMESPACE},
                          "involvedObject": {"apiVersion": "v1", "kind": "Secret",
                                             "name": LICENSE_SECRET_NAME,
                                             "namespace": LICENSE_NAMESPACE},
                          "reason": reason, "message": message, "type": type_,
                          "source": {"component": "omnia-license-activation"},
                          "firstTimestamp": _iso(time.time())})
        except Exception as e:  # noqa: BLE001
            log.debug("event %s not recorded: %s", reason, e)

    @staticmethod
    def in_grace_period(state: dict, now: float) -> bool:
        if not state.get("heartbeat_failures"):
            return True
        return now - _parse_iso(state.get("last_heartbeat")) < GRACE_PERIOD_S

    # ------------------------------------------------------------------ backoff
    def _record_failure(self, lid: str) -> tuple[float, bool, bool]:
        with self._lock:
            st = self._failures.setdefault(lid, {"first": self.now(), "attempts": 0,
                                                 "slow": False})
            st["attempts"] += 1
            first = st["attempts"] == 1
            if self.now() - st["first"] >= GIVE_UP_AFTER_S:
                gave_up = not st["slow"]
                st["slow"] = True
                return SLOW_INTERVAL_S, first, gave_up
            shift = min(st["attempts"] - 1, MAX_SHIFT)
            return min(BACKOFF_BASE_S * (1 << shift), BACKOFF_CAP_S), first, False

    def _failure(self, store, lid: str, reason: str, msg: str) -> float:
        delay, first, gave_up = self._record_failure(lid)
        if first:
            self._event(store, "Warning", reason, msg)
        elif gave_up:
            log.info("license activation still failing; retrying every %.0fs", delay)
        return delay

    # ------------------------------------------------------------------ reconcile
    def reconcile(self, store, ns, name):
        if name != self.secret_name or (ns or "") != LICENSE_NAMESPACE:
            return None
        try:
            self.validator.invalidate()
            lic = self.validator.get()
        except LicenseError as e:
            log.debug("license not found or invalid, skipping activation: %s", e)
            return None
        if lic.tier == TIER_OPEN_CORE:
            return None
        try:
            state = self._state(store)
        except ValueError as e:
            log.warning("%s", e)
            state = None
        if state is not None:
            return self._heartbeat(store, lic, state)
        return self._activate(store, lic)

    def _activate(self, store, lic) -> float | None:
        try:
            fp = cluster_fingerprint(store)
        except Exception as e:  # noqa: BLE001 - namespaces missing
            return self._failure(store, lic.id, "FingerprintFailed",
                                 f"Failed to generate cluster fingerprint: {e}")
        try:
            resp = self.client.activate(lic.id, fp, self.cluster_name)
        except ActivationError as e:
            return self._failure(store, lic.id, "ActivationFailed",
                                 f"License activation failed: {e}")
        if not resp.get("activated"):
            msg = f"License activation rejected: {resp.get('message', '')}"
            if resp.get("active_clusters"):
                msg += (f" (Active clusters: {len(resp['active_clusters'])}/"
                        f"{resp.get('max_activations', 0)})")
            self._event(store, "Warning", "ActivationRejected", msg)
            return None
        now = self.now()
        self._save(store, {"activation_id": resp.get("activation_id", ""),
                           "cluster_fingerprint": fp, "license_id": lic.id,
                           "activated_at": _iso(now), "last_heartbeat": _iso(now)})
        with self._lock:
            self._failures.pop(lic.id, None)
        self._event(store, "Normal", "Activated",
                    f"License activated successfully (ID: {resp.get('activation_id', '')})")
        return HEARTBEAT_INTERVAL_S

    def _heartbeat(self, store, lic, state: dict) -> float:
        now = self.now()
        due = _parse_iso(state.get("last_heartbeat")) + HEARTBEAT_INTERVAL_S
        if now < due:
            return max(60.0, due - now)
        try:
            self.client.heartbeat(lic.id, state.get("cluster_fingerprint", ""))
        except ActivationError as e:
            log.warning("license heartbeat failed: %s", e)
            state["heartbeat_failures"] = int(state.get("heartbeat_failures", 0)) + 1
            if not self.in_grace_period(state, now):
                self._event(store, "Warning", "HeartbeatGracePeriodExpired",
                            "License heartbeat grace period expired. Enterprise features may "
                            "be disabled.")
            self._save(store, state)
            return 3600.0
        state["last_heartbeat"] = _iso(now)
        state["heartbeat_failures"] = 0
        self._save(store, state)
        return HEARTBEAT_INTERVAL_S

    def deactivate(self, store) -> None:
        state = self._state(store)
        if state is None:
            return
        self.client.deactivate(state["license_id"], state["cluster_fingerprint"])
        store.delete("ConfigMap", ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE)
