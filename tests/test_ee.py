"""Enterprise components: native AES-256-GCM (NIST vectors), envelope encryption
+ rotation, policy broker decisions (claims / CEL rules / audit / fail-closed /
header injection) end-to-end through the runtime's broker client."""
import asyncio
import base64

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.ee.encryption import (Encryptor, LocalKMS, ProviderUnavailable, ReEncryptor,
                                     build_provider)
from omnia_amd.ee.policy_broker import Evaluator, PolicyWatcher, build_app
from omnia_amd.native import native
from omnia_amd.tools.executor import CallContext, PolicyBrokerClient, ToolDef

H = bytes.fromhex


def test_aes_gcm_nist_vectors():
    n = native()
    # GCM spec test cases 13, 14, 16 (AES-256)
    assert n.aes_gcm_encrypt(bytes(32), bytes(12), b"").hex() == "530f8afbc74536b9a963b4f1c4cb738b"
    assert n.aes_gcm_encrypt(bytes(32), bytes(12), bytes(16)).hex() == (
        "cea7403d4d606b6e074ec5d3baf39d18d0d1c8a799996bf0265b98b5d48ab919")
    K = H("feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308")
    P = H("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf"
          "0e2449a6b525b16aedf5aa0de657ba637b39")
    A = H("feedfacedeadbeeffeedfacedeadbeefabaddad2")
    IV = H("cafebabefacedbaddecaf888")
    ct = n.aes_gcm_encrypt(K, IV, P, A)
    assert ct.hex().endswith("76fc6ece0f4e1768cddf8853bb2d551b")
    assert ct.hex().startswith("522dc1f099567d07f47f37a32a84427d")
    assert n.aes_gcm_decrypt(K, IV, ct, A) == P
    bad = bytearray(ct)
    bad[5] ^= 1
    with pytest.raises(ValueError):
        n.aes_gcm_decrypt(K, IV, bytes(bad), A)
    with pytest.raises(ValueError):
        n.aes_gcm_decrypt(K, IV, ct, b"other aad")


def test_envelope_message_roundtrip_and_rotation(tmp_path):
    kms = LocalKMS(path=str(tmp_path / "keys.json"))
    enc = Encryptor(kms)
    m, ev = enc.encrypt_message({"role": "user", "content": "my ssn is 123-45-6789",
                                 "metadata": {"channel": "web"}})
    assert "123-45" not in m["content"] and {e.field for e in ev} == {"content",
                                                                      "metadata.channel"}
    assert enc.decrypt_message(m)["content"] == "my ssn is 123-45-6789"
    old = m["content"]
    prev, new = kms.rotate()
    assert new != prev
    # persisted key ring reloads and still opens old-version envelopes
    kms2 = LocalKMS(path=str(tmp_path / "keys.json"))
    assert kms2.decrypt(base64.b64decode(old)) == b"my ssn is 123-45-6789"
    rr = ReEncryptor(kms2)
    nb = rr.rewrap_b64(old)
    assert rr.stats["rewrapped"] == 1 and rr.rewrap_b64(nb) == nb  # already current
    tc = enc.encrypt_tool_call({"name": "t", "arguments": {"q": "x"}, "result": {"ok": 1}})
    assert enc.is_envelope(tc["arguments"])
    assert enc.decrypt_tool_call(tc)["result"] == {"ok": 1}
    with pytest.raises((KeyError, ValueError)):
        build_provider({"type": "aws-kms"})  # keyID is required (REST provider, tests/test_kms.py)


POLICY = {
    "apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "ToolPolicy",
    "metadata": {"name": "refunds", "namespace": "default", "generation": 1},
    "spec": {
        "selector": {"registry": "billing", "tools": ["refund"]},
        "requiredClaims": [{"claim": "team", "message": "team claim required"}],
        "rules": [
            {"name": "max-amount", "deny": {"cel": "body.amount > 100",
                                            "message": "refunds over 100 need approval"}},
            {"name": "weekday", "deny": {"cel": "headers['x-omnia-claim-team'] == 'interns'",
                                         "message": "interns cannot refund"}}],
        "headerInjection": [{"header": "x-approved-by", "value": "policy-broker"},
                            {"header": "x-tenant", "cel": "identity.workspace"}],
    },
}


def _hdr(team=None):
    h = {"x-omnia-tool-name": "refund", "x-omnia-tool-registry": "billing"}
    if team:
        h["X-Omnia-Claim-Team"] = team
    return h


def test_evaluator_semantics():
    ev = Evaluator()
    ev.set_policy(POLICY)
    d = ev.evaluate(_hdr(), {"amount": 5}, None)
    assert not d.allowed and d.denied_by == "required-claim:team"
    d = ev.evaluate(_hdr("support"), {"amount": 500}, None)
    assert not d.allowed and d.denied_by == "max-amount"
    d = ev.evaluate(_hdr("interns"), {"amount": 5}, None)
    assert not d.allowed and d.denied_by == "weekday"
    d = ev.evaluate(_hdr("support"), {"amount": 5}, {"workspace": "acme"})
    assert d.allowed and not d.denied_by
    assert ev.inject(_hdr("support"), {}, {"workspace": "acme"}) == {
        "x-approved-by": "policy-broker", "x-tenant": "acme"}
    # a tool outside the selector is unaffected
    assert ev.evaluate({"x-omnia-tool-name": "other", "x-omnia-tool-registry": "billing"},
                       {}, None).allowed
    # missing body field -> CEL error -> fail closed by default
    d = ev.evaluate(_hdr("support"), {}, None)
    assert not d.allowed and d.error
    # audit mode: would deny, allowed
    audit = dict(POLICY, spec=dict(POLICY["spec"], mode="audit"))
    ev.set_policy(audit)
    d = ev.evaluate(_hdr("support"), {"amount": 500}, None)
    assert d.allowed and d.would_deny and d.denied_by == "max-amount"
    # onFailure allow
    lax = dict(POLICY, spec=dict(POLICY["spec"], onFailure="allow"))
    ev.set_policy(lax)
    assert ev.evaluate(_hdr("support"), {}, None).allowed


def test_broker_http_with_runtime_client_and_watcher():
    from omnia_amd.operator.apistore import APIStore

    async def go():
        store = APIStore()
        store.create(POLICY)
        ev = Evaluator()
        w = PolicyWatcher(ev, store)
        await w.sync_once()
        assert "default/refunds" in ev.policies
        runner = web.AppRunner(build_app(ev))
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
        try:
            cli = PolicyBrokerClient(url)
            tool = ToolDef(name="refund", handler="billing")
            ctx = CallContext(workspace="acme", headers={"x-omnia-claim-team": "support"})
            ok = await cli.decide(tool, {"amount": 10}, ctx)
            assert ok["allow"] and ok["injectedHeaders"]["x-tenant"] == "acme"
            no = await cli.decide(tool, {"amount": 1000}, ctx)
            assert not no["allow"] and no["deniedBy"] == "max-amount"
            async with aiohttp.ClientSession() as s:
                r = await s.post(url + "/v1/decision", data=b"not json")
                assert r.status == 400
            # broker down -> fail closed
            dead = PolicyBrokerClient("http://127.0.0.1:9")
            d = await dead.decide(tool, {}, ctx)
            assert not d["allow"] and d["deniedBy"] == "broker-unavailable"
            # policy deleted -> watcher drops it -> allowed
            store.delete("ToolPolicy", "refunds", "default")
            await w.sync_once()
            assert (await cli.decide(tool, {"amount": 1000}, ctx))["allow"]
        finally:
            await runner.cleanup()

    asyncio.run(go())


def test_privacy_api_consent_optout_and_dsar_fanout():
    from omnia_amd.ee.privacy import FanoutEraser, PrivacyStore, build_app as privacy_app
    from omnia_amd.memory.api import build_app as memory_app
    from omnia_amd.memory.model import Memory
    from omnia_amd.memory.service import MemoryService
    from omnia_amd.memory.store import MemoryStore
    from omnia_amd.session.api import build_app as session_app
    from omnia_amd.session.model import Session
    from omnia_amd.session.store import TieredSessionService

    async def serve(app):
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"

    async def go():
        ss = TieredSessionService()
        for i in range(3):
            ss.create(Session(id=f"s{i}", namespace="ns",
                              virtual_user_id="alice" if i < 2 else "bob"))
        ms = MemoryService(MemoryStore())
        await ms.save(Memory(content="alice likes tea", scope={"workspace_id": "w",
                                                               "virtual_user_id": "alice"}))
        r1, s_url = await serve(session_app(ss))
        r2, m_url = await serve(memory_app(ms, enterprise=True))
        st = PrivacyStore()
        r3, p_url = await serve(privacy_app(st, FanoutEraser(st, s_url, m_url, ["w"]), m_url))
        try:
            async with aiohttp.ClientSession() as s:
                c = await (await s.get(f"{p_url}/api/v1/privacy/preferences/alice/consent")).json()
                assert "memory:health" in c["denied"] and "memory:context" in c["defaults"]
                r = await s.put(f"{p_url}/api/v1/privacy/preferences/alice/consent",
                                json={"grants": ["memory:health"], "revocations": []})
                assert "memory:health" in (await r.json())["grants"]
                r = await s.put(f"{p_url}/api/v1/privacy/preferences/alice/consent",
                                json={"grants": ["bogus"]})
                assert r.status == 400
                await s.post(f"{p_url}/api/v1/privacy/opt-out", json={"userId": "alice"})
                p = await (await s.get(f"{p_url}/api/v1/privacy/preferences/alice")).json()
                assert p["optedOut"]
                r = await s.post(f"{p_url}/api/v1/privacy/deletion-request",
                                 json={"virtualUserId": "alice", "reason": "gdpr"})
                rid = (await r.json())["id"]
                for _ in range(100):
                    d = await (await s.get(
                        f"{p_url}/api/v1/privacy/deletion-request/{rid}")).json()
                    if d["status"] in ("completed", "failed"):
                        break
                    await asyncio.sleep(0.05)
                assert d["status"] == "completed", d
                assert d["sessionsDeleted"] == 2
        finally:
            for r in (r1, r2, r3):
                await r.cleanup()
        return ss, ms, st

    ss, ms, st = asyncio.run(go())
    assert ss.get("s2") is not None and ss.get("s0") is None
    assert ms.store.list({"workspace_id": "w", "virtual_user_id": "alice"}) == []
    assert any(e["type"] == "dsar.erasure" for e in st.audit())
