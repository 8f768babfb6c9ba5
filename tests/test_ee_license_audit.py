"""EE licensing (RS256 JWT, tiers, gates, activation, nag), audit log (buffered
writer, query/paging, retention, forwarder, HTTP route) and compliance presets."""
import asyncio
import random
import time

import pytest

from omnia_amd.ee import audit, compliance, license as L
from omnia_amd.ee.redaction import Redactor


def _prime(bits, rng):
    while True:
        c = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if all(pow(a, c - 1, c) == 1 for a in (2, 3, 5, 7, 11, 13, 17, 19, 23)):
            return c


@pytest.fixture(scope="module")
def rsa():
    rng = random.Random(5)
    e = 65537
    while True:
        p, q = _prime(512, rng), _prime(512, rng)
        phi = (p - 1) * (q - 1)
        if p != q and phi % e:
            return p * q, e, pow(e, -1, phi)


def _claims(**kw):
    c = {"lid": "lic-1", "tier": "enterprise", "customer": "ACME",
         "features": {"customFacade": True, "loadTesting": True, "ociSource": True},
         "limits": {"maxScenarios": 100, "maxWorkerReplicas": 4},
         "iat": time.time(), "exp": time.time() + 86400 * 90}
    c.update(kw)
    return c


def test_rs256_roundtrip_and_pem(rsa):
    n, e, d = rsa
    assert L.parse_rsa_public_key(L.public_pem(n, e)) == (n, e)
    tok = L.make_token(_claims(), n, d)
    v = L.Validator(L.public_pem(n, e), secret_reader=lambda: tok)
    lic = v.get()
    assert lic.is_valid_enterprise() and lic.customer == "ACME"
    assert lic.can_use_custom_facade() and lic.can_use_job_type("loadtest")
    assert not lic.can_use_job_type("datagen") and lic.can_use_worker_replicas(4)
    assert not lic.can_use_worker_replicas(5) and lic.can_use_source_type("oci")


def test_tampered_expired_and_default(rsa):
    n, e, d = rsa
    tok = L.make_token(_claims(), n, d)
    h, b, s = tok.split(".")
    forged = L._b64e(L._b64d(b).replace(b"ACME", b"EVIL"))
    v = L.Validator(L.public_pem(n, e), secret_reader=lambda: f"{h}.{forged}.{s}")
    with pytest.raises(L.InvalidSignature):
        v.get()
    assert v.get_or_default().tier == L.TIER_OPEN_CORE
    old = L.make_token(_claims(exp=time.time() - 10), n, d)
    v2 = L.Validator(L.public_pem(n, e), secret_reader=lambda: old)
    with pytest.raises(L.LicenseExpired):
        v2.get()
    oc = v2.get_or_default()
    assert oc.features.gitSource and not oc.can_use_custom_facade()
    assert oc.can_use_scenario_count(10) and not oc.can_use_scenario_count(11)
    assert L.Validator(dev_mode=True).get().is_valid_enterprise()
    with pytest.raises(L.LicenseNotFound):
        L.Validator(L.public_pem(n, e), secret_reader=lambda: None).get()


def test_gates_activation_nag(rsa):
    spec = {"facades": [{"type": "custom", "image": "x"}]}
    assert L.gate_agentruntime(spec, L.open_core_license())
    assert not L.gate_agentruntime(spec, L.dev_license())
    st = L.ActivationState(last_heartbeat=time.time() - 3600)
    assert st.needs_heartbeat(600) and st.in_grace_period()
    assert L.nag_message(L.open_core_license(), ["loadTesting"])
    assert L.nag_message(L.open_core_license(), []) is None
    fp1 = L.cluster_fingerprint("uid", ["b", "a"])
    assert fp1 == L.cluster_fingerprint("uid", ["a", "b"]) and len(fp1) == 32


def test_audit_logger_query_retention():
    lg = audit.AuditLogger(batch_size=3, flush_interval_s=0.05, retention_days=30)
    now = time.time()
    try:
        for i in range(10):
            lg.log_event(audit.Entry("session_accessed", timestamp=now - i, sessionId="s1",
                                     userId="u1" if i % 2 else "u2", metadata={"i": str(i)}))
        lg.log_event(audit.Entry("session_deleted", timestamp=now - 40 * 86400, sessionId="s2"))
        lg.flush()
        r = lg.query(session_id="s1", limit=4)
        assert r["total"] == 10 and len(r["entries"]) == 4 and r["hasMore"]
        assert r["entries"][0]["metadata"] == {"i": "0"}
        assert lg.query(user_id="u1")["total"] == 5
        assert lg.query(event_types=["session_deleted"])["total"] == 1
        assert lg.query(start=now - 3.5)["total"] == 4
        assert lg.delete_expired() == 1
    finally:
        lg.close()


def test_audit_buffer_full_drops():
    lg = audit.AuditLogger(buffer_size=1, batch_size=1000, flush_interval_s=10)
    try:
        oks = [lg.log_event(audit.Entry("pii_redacted")) for _ in range(50)]
        assert not all(oks) and lg.dropped > 0
    finally:
        lg.close()


def test_forwarder_marks_only_after_success():
    lg = audit.AuditLogger(flush_interval_s=0.02)
    sent = []
    status = {"code": 503}

    async def post(url, body, headers):
        sent.append((url, len(body["events"]), headers))
        return status["code"]

    try:
        for i in range(5):
            lg.log_event(audit.Entry("memory_accessed", userId=f"u{i}"))
        lg.flush()
        fw = audit.Forwarder(lg, "http://privacy:8085", batch_size=2, token="t", post=post)
        assert asyncio.run(fw.drain_once()) == 0 and fw.failures == 1
        assert len(lg.unforwarded(100)) == 5
        status["code"] = 202
        assert asyncio.run(fw.drain_once()) == 5
        assert lg.unforwarded(100) == []
        assert sent[-1][0].endswith("/api/v1/privacy/audit-events")
        assert sent[-1][2]["Authorization"] == "Bearer t"
    finally:
        lg.close()


def test_audit_http_route():
    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    lg = audit.AuditLogger(flush_interval_s=0.02)

    async def run():
        app = web.Application()
        audit.mount_routes(app, lg)
        c = TestClient(TestServer(app))
        await c.start_server()
        try:
            lg.log_event(audit.Entry("session_searched", sessionId="x", query="hello"))
            lg.flush()
            r = await c.get("/api/v1/audit/sessions?sessionId=x")
            body = await r.json()
            assert body["total"] == 1 and body["entries"][0]["query"] == "hello"
            assert (await c.get("/api/v1/audit/sessions?limit=abc")).status == 400
        finally:
            await c.close()

    try:
        asyncio.run(run())
    finally:
        lg.close()


@pytest.mark.parametrize("name", compliance.list_presets())
def test_presets_use_known_patterns(name):
    spec = compliance.get_preset(name)
    Redactor(spec["recording"]["pii"]["patterns"])  # raises on unknown patterns
    assert spec["auditLog"]["enabled"] and spec["userOptOut"]["honorDeleteRequests"]
    if name == "hipaa":
        assert spec["encryption"]["enabled"] and spec["auditLog"]["retentionDays"] == 2555


def test_preset_merge_and_unknown():
    pol = {"kind": "SessionPrivacyPolicy",
           "spec": {"preset": "gdpr", "auditLog": {"retentionDays": 10}}}
    out = compliance.apply_preset(pol)["spec"]
    assert out["auditLog"] == {"enabled": True, "retentionDays": 10}
    assert out["retention"]["facade"]["coldDays"] == 90
    with pytest.raises(ValueError):
        compliance.get_preset("sox")


def test_operator_webhook_license_gate(rsa):
    import base64

    from omnia_amd.api import crds
    from omnia_amd.operator import manager
    from omnia_amd.operator.apistore import Invalid

    n, e, d = rsa
    store = manager.new_store()
    manager.set_license_validator(manager.license_validator_for(store, L.public_pem(n, e)))
    ar = {"apiVersion": crds.API_VERSION, "kind": "AgentRuntime",
          "metadata": {"name": "c", "namespace": "default"},
          "spec": {"facades": [{"type": "custom", "image": "img"}],
                   "promptPackRef": {"name": "p"}}}
    try:
        with pytest.raises(Invalid):
            store.apply(ar)  # open-core: custom facades need a license
        tok = L.make_token(_claims(), n, d)
        store.apply({"apiVersion": "v1", "kind": "Secret",
                     "metadata": {"name": "omnia-license", "namespace": "default"},
                     "data": {"license": base64.b64encode(tok.encode()).decode()}})
        store.apply(ar)
    finally:
        manager.set_license_validator(None)


def test_session_api_emits_audit_events():
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.session.api import build_app
    from omnia_amd.session.store import TieredSessionService

    lg = audit.AuditLogger(flush_interval_s=0.02)

    async def run():
        c = TestClient(TestServer(build_app(TieredSessionService(), audit_logger=lg)))
        await c.start_server()
        try:
            r = await c.post("/api/v1/sessions", json={"id": "aud-1", "agent_name": "a"})
            assert r.status == 201
            await c.get("/api/v1/sessions/aud-1")
            await c.get("/api/v1/sessions/search?q=x")
            await c.delete("/api/v1/sessions/aud-1")
            lg.flush()
            body = await (await c.get("/api/v1/audit/sessions?sessionId=aud-1")).json()
            return sorted(e["eventType"] for e in body["entries"])
        finally:
            await c.close()

    try:
        assert asyncio.run(run()) == ["session_accessed", "session_created", "session_deleted"]
        assert lg.query(event_types=["session_searched"])["total"] == 1
    finally:
        lg.close()
