"""License activation controller (``license_activation_controller_test.go``,
``license_activation_backoff_test.go``, ``pkg/license/activation_test.go``)
against an in-process license server: fingerprint, activation state in the
ConfigMap, rejection events, exponential backoff with the slow-retry switch,
heartbeats and the grace period, deactivation."""
import hashlib
import json
import random
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest

from omnia_amd.ee import license as L
from omnia_amd.ee.license_activation import (ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE,
                                             LICENSE_SECRET_NAME, ActivationClient,
                                             LicenseActivationReconciler, cluster_fingerprint)
from omnia_amd.operator.apistore import APIStore


def _prime(bits, rng):
    while True:
        c = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if all(pow(a, c - 1, c) == 1 for a in (2, 3, 5, 7, 11, 13, 17, 19, 23)):
            return c


@pytest.fixture(scope="module")
def rsa():
    rng = random.Random(9)
    e = 65537
    while True:
        p, q = _prime(512, rng), _prime(512, rng)
        phi = (p - 1) * (q - 1)
        if p != q and phi % e:
            return p * q, e, pow(e, -1, phi)


class _Server:
    def __init__(self):
        self.calls = []
        self.mode = {"activate": "ok", "heartbeat": "ok"}
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _reply(self, code, body):
                raw = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n) or b"{}")
                outer.calls.append(("POST", self.path, body))
                if self.path == "/v1/licenses/activate":
                    m = outer.mode["activate"]
                    if m == "fail":
                        return self._reply(503, {"error": "down"})
                    if m == "reject":
                        return self._reply(200, {"activated": False, "message": "limit",
                                                 "active_clusters": ["a", "b"],
                                                 "max_activations": 2})
                    return self._reply(200, {"activated": True, "activation_id": "act-1"})
                if self.path.endswith("/heartbeat"):
                    if outer.mode["heartbeat"] == "fail":
                        return self._reply(500, {})
                    return self._reply(200, {"valid": True})
                self._reply(404, {})

            def do_DELETE(self):
                outer.calls.append(("DELETE", self.path, None))
                self._reply(200, {"deactivated": True})

        self.httpd = HTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"

    def close(self):
        self.httpd.shutdown()


@pytest.fixture()
def server():
    s = _Server()
    yield s
    s.close()


def _store():
    st = APIStore()
    for name, uid in (("kube-system", "uid-ks"), (LICENSE_NAMESPACE, "uid-om")):
        o = st.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name}})
        st.objs[st.key("Namespace", None, name)]["metadata"]["uid"] = uid
    return st


def _validator(rsa, tier="enterprise"):
    n, e, d = rsa
    tok = L.make_token({"lid": "lic-9", "tier": tier, "customer": "ACME",
                        "iat": time.time(), "exp": time.time() + 86400}, n, d)
    return L.Validator(L.public_pem(n, e), secret_reader=lambda: tok)


def _events(store, reason):
    return [o for (k, _, _), o in store.objs.items() if k == "Event" and o["reason"] == reason]


def test_fingerprint_hashes_namespace_uids():
    fp = cluster_fingerprint(_store())
    assert fp == hashlib.sha256(b"uid-ks:uid-om").hexdigest()[:32] and len(fp) == 32


def test_activation_then_heartbeat(rsa, server):
    store = _store()
    now = [1_800_000_000.0]
    r = LicenseActivationReconciler(_validator(rsa), ActivationClient(server.url),
                                    cluster_name="node-a", now=lambda: now[0])
    assert r.reconcile(store, "default", LICENSE_SECRET_NAME) is None  # other Secret
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) == 24 * 3600
    post = server.calls[0]
    assert post[1] == "/v1/licenses/activate" and post[2]["license_id"] == "lic-9"
    assert post[2]["cluster_fingerprint"] == cluster_fingerprint(store)
    assert post[2]["cluster_name"] == "node-a"
    state = json.loads(store.get("ConfigMap", ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE)[
        "data"]["state"])
    assert state["activation_id"] == "act-1" and _events(store, "Activated")
    # heartbeat not yet due
    now[0] += 3600
    assert abs(r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) - 23 * 3600) < 1
    assert len(server.calls) == 1
    now[0] += 23 * 3600
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) == 24 * 3600
    assert server.calls[-1][1] == "/v1/licenses/lic-9/heartbeat"
    # failing heartbeats count; past the 7-day grace period an event is raised
    server.mode["heartbeat"] = "fail"
    now[0] += 24 * 3600
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) == 3600.0
    st = json.loads(store.get("ConfigMap", ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE)[
        "data"]["state"])
    assert st["heartbeat_failures"] == 1 and not _events(store, "HeartbeatGracePeriodExpired")
    now[0] += 8 * 24 * 3600
    r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME)
    assert _events(store, "HeartbeatGracePeriodExpired")
    # deactivation releases the seat and the state
    r.deactivate(store)
    assert server.calls[-1][0] == "DELETE" and server.calls[-1][1].startswith(
        "/v1/licenses/lic-9/activations/")
    assert store.try_get("ConfigMap", ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE) is None


def test_open_core_and_missing_license_skip(rsa, server):
    store = _store()
    r = LicenseActivationReconciler(_validator(rsa, tier="open-core"),
                                    ActivationClient(server.url))
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) is None
    r2 = LicenseActivationReconciler(L.Validator(None, secret_reader=lambda: None),
                                     ActivationClient(server.url))
    assert r2.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) is None
    assert server.calls == []


def test_rejection_is_an_event_not_a_retry(rsa, server):
    store = _store()
    server.mode["activate"] = "reject"
    r = LicenseActivationReconciler(_validator(rsa), ActivationClient(server.url))
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) is None
    ev = _events(store, "ActivationRejected")
    assert ev and "Active clusters: 2/2" in ev[0]["message"]
    assert store.try_get("ConfigMap", ACTIVATION_CONFIGMAP, LICENSE_NAMESPACE) is None


def test_backoff_doubles_caps_then_goes_slow(rsa, server):
    store = _store()
    server.mode["activate"] = "fail"
    now = [1_000_000.0]
    r = LicenseActivationReconciler(_validator(rsa), ActivationClient(server.url),
                                    now=lambda: now[0])
    delays = [r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) for _ in range(8)]
    assert delays == [60.0, 120.0, 240.0, 480.0, 960.0, 1920.0, 3600.0, 3600.0]
    assert len(_events(store, "ActivationFailed")) == 1  # only the first of the streak
    now[0] += 24 * 3600
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) == 6 * 3600
    # recovery resets the streak
    server.mode["activate"] = "ok"
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) == 24 * 3600
    assert not r._failures


def test_missing_namespaces_back_off(rsa, server):
    r = LicenseActivationReconciler(_validator(rsa), ActivationClient(server.url))
    store = APIStore()
    assert r.reconcile(store, LICENSE_NAMESPACE, LICENSE_SECRET_NAME) == 60.0
    assert _events(store, "FingerprintFailed") and server.calls == []
