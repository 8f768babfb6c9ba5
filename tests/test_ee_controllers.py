"""EE policy controllers (``ee/internal/controller/toolpolicy_controller_test.go``,
``sessionprivacypolicy_controller_test.go``, ``keyrotation_controller_test.go``):
ToolPolicy compile / status / canonical-header lint / evaluator sync;
SessionPrivacyPolicy activation, KMS key rotation on the annotation and on the
cron schedule, batched re-encryption of stored session messages; the cron
parser; the session store's encryption at rest."""
import asyncio
import json
import sqlite3
import time

import pytest

from omnia_amd.ee.controllers import (ROTATE_KEY_ANNOTATION, SessionPrivacyPolicyReconciler,
                                      ToolPolicyReconciler, canonical_header,
                                      non_canonical_header_refs)
from omnia_amd.ee.encryption import META_KEY, Encryptor, LocalKMS
from omnia_amd.operator.apistore import APIStore, get_condition
from omnia_amd.session.model import Message, Session
from omnia_amd.session.store import TieredSessionService, WarmStore
from omnia_amd.utils import cron

API = "omnia.altairalabs.ai/v1alpha1"


def _put(store, obj):
    obj.setdefault("metadata", {}).setdefault("namespace", "default")
    obj["metadata"].setdefault("generation", 1)
    obj["metadata"].setdefault("resourceVersion", "1")
    store.objs[(obj["kind"], "default", obj["metadata"]["name"])] = obj
    return obj


def _events(store, reason=None):
    return [o for (k, _, _), o in store.objs.items() if k == "Event" and
            (reason is None or o["reason"] == reason)]


# ------------------------------------------------------------------ cron
def _t(s):
    import calendar

    return calendar.timegm(time.strptime(s, "%Y-%m-%d %H:%M"))


def test_cron_next_fire():
    assert cron.next_fire("0 * * * *", _t("2026-03-01 10:30")) == _t("2026-03-01 11:00")
    assert cron.next_fire("*/15 * * * *", _t("2026-03-01 10:30")) == _t("2026-03-01 10:45")
    assert cron.next_fire("0 0 1 1 *", _t("2026-03-01 10:30")) == _t("2027-01-01 00:00")
    assert cron.next_fire("@daily", _t("2026-02-28 23:59")) == _t("2026-03-01 00:00")
    # 2026-03-02 is a Monday; dom and dow both restricted -> either matches
    assert cron.next_fire("0 9 15 * 1", _t("2026-03-01 10:00")) == _t("2026-03-02 09:00")
    assert cron.next_fire("0 9 * * 1-5", _t("2026-03-06 10:00")) == _t("2026-03-09 09:00")
    assert cron.next_fire("@every 90s", 1000.0) == 1090.0
    assert cron.next_fire("30 2 29 2 *", _t("2026-03-01 00:00")) == _t("2028-02-29 02:30")
    for bad in ("61 * * * *", "* * *", "@every x", "0 0 32 * *", "a b c d e"):
        with pytest.raises(cron.CronError):
            cron.parse(bad)


# ------------------------------------------------------------------ ToolPolicy
def _tp(name="tp", rules=None, inj=None):
    spec = {"selector": {"registry": "reg", "tools": ["search"]},
            "rules": rules if rules is not None else [
                {"name": "no-prod", "deny": {"cel": 'body.env == "prod"', "message": "no"}}],
            "mode": "enforce", "onFailure": "deny"}
    if inj is not None:
        spec["headerInjection"] = inj
    return {"apiVersion": API, "kind": "ToolPolicy",
            "metadata": {"name": name, "uid": "u-" + name}, "spec": spec}


def test_canonical_header_keys():
    assert canonical_header("x-user-id") == "X-User-Id"
    assert canonical_header("X-User-Id") == "X-User-Id"
    assert canonical_header("bad key") == "bad key"
    refs = non_canonical_header_refs('headers["x-tenant"] == "a" && headers[\'X-Ok\'] != ""'
                                     ' || headers["x-tenant"] == "b"')
    assert refs == [("x-tenant", "X-Tenant")]


def test_tool_policy_compiles_into_evaluator():
    store = APIStore()
    r = ToolPolicyReconciler()
    _put(store, _tp(inj=[{"header": "X-Tenant", "cel": "identity.workspace"},
                         {"header": "X-Static", "value": "1"}]))
    r.reconcile(store, "default", "tp")
    o = store.get("ToolPolicy", "tp", "default")
    st = o["status"]
    assert st["phase"] == "Active" and st["ruleCount"] == 1 and st["observedGeneration"] == 1
    for c in ("Compiled", "Ready", "HeaderRefsCanonical"):
        assert get_condition({"status": st}, c)["status"] == "True", c
    assert list(r.evaluator.policies) == ["default/tp"]
    assert _events(store, "PolicyCompiled")
    # deletion removes it from the evaluator
    store.objs.pop(("ToolPolicy", "default", "tp"))
    r.reconcile(store, "default", "tp")
    assert not r.evaluator.policies


def test_tool_policy_warns_on_non_canonical_header_refs():
    store = APIStore()
    r = ToolPolicyReconciler()
    _put(store, _tp(rules=[{"name": "tenant", "deny": {
        "cel": 'headers["x-tenant"] != "acme"', "message": "tenant"}}]))
    r.reconcile(store, "default", "tp")
    st = store.get("ToolPolicy", "tp", "default")["status"]
    c = get_condition({"status": st}, "HeaderRefsCanonical")
    assert st["phase"] == "Active" and c["status"] == "False"
    assert "X-Tenant" in c["message"] and _events(store, "NonCanonicalHeaderRef")[0][
        "type"] == "Warning"


@pytest.mark.parametrize("rules,inj,needle", [
    ([{"name": "broken", "deny": {"cel": "body.x ==", "message": "m"}}], None, "broken"),
    (None, [{"header": "X-A", "value": "v", "cel": "true"}], "mutually exclusive"),
    (None, [{"header": "X-A"}], "one of value or cel"),
])
def test_tool_policy_compile_errors(rules, inj, needle):
    store = APIStore()
    r = ToolPolicyReconciler()
    _put(store, _tp(rules=rules, inj=inj))
    r.reconcile(store, "default", "tp")
    st = store.get("ToolPolicy", "tp", "default")["status"]
    assert st["phase"] == "Error" and st["ruleCount"] == 0
    assert get_condition({"status": st}, "Ready")["status"] == "False"
    assert needle in get_condition({"status": st}, "Compiled")["message"]
    assert _events(store, "CompileError")


# ------------------------------------------------------------------ encryption at rest
def _svc(tmp_path, kms):
    warm = WarmStore(str(tmp_path / "warm.db"))
    svc = TieredSessionService(warm=warm)
    svc.encryptor = Encryptor(kms)
    return svc, warm


def _fill(svc, n=5, sid="s1"):
    svc.create(Session(id=sid, agent_name="a", namespace="default"))
    for i in range(n):
        asyncio.run(svc.append_message(sid, Message(content=f"secret {i}",
                                                    metadata={"k": f"v{i}"})))


def test_session_store_encrypts_at_rest(tmp_path):
    kms = LocalKMS(path=str(tmp_path / "keys.json"))
    svc, warm = _svc(tmp_path, kms)
    _fill(svc, 3)
    raw = sqlite3.connect(str(tmp_path / "warm.db")).execute(
        "SELECT content, doc FROM messages").fetchall()
    assert raw and all("secret" not in c and "secret" not in d for c, d in raw)
    svc.hot.invalidate("s1")
    s, msgs = svc.get("s1")
    assert [m.content for m in msgs] == ["secret 0", "secret 1", "secret 2"]
    assert msgs[1].metadata == {"k": "v1"} and s.last_message_preview == ""


# ------------------------------------------------------------------ key rotation
def _spp(rotation, name="privacy", annotations=None):
    md = {"name": name, "uid": "u1", "creationTimestamp": "2026-03-01T00:00:00Z"}
    if annotations:
        md["annotations"] = annotations
    return {"apiVersion": API, "kind": "SessionPrivacyPolicy", "metadata": md,
            "spec": {"level": "workspace", "encryption": {
                "enabled": True, "kmsProvider": "vault", "keyID": "local",
                "keyRotation": rotation}}}


def _versions(warm):
    out = []
    for _, _, doc in warm.scan_messages("", 1000):
        out.append(json.loads(doc["metadata"][META_KEY])["keyVersion"])
    return out


def test_annotation_rotation_and_batched_reencryption(tmp_path):
    keyfile = str(tmp_path / "keys.json")
    svc, warm = _svc(tmp_path, LocalKMS(path=keyfile))
    _fill(svc, 5)
    assert set(_versions(warm)) == {"1"}
    store = APIStore()
    rec = SessionPrivacyPolicyReconciler(provider_factory=lambda cfg: LocalKMS(path=keyfile),
                                         store_factory=lambda: svc)
    _put(store, _spp({"enabled": True, "reEncryptExisting": True, "batchSize": 2},
                     annotations={ROTATE_KEY_ANNOTATION: "now"}))
    rq = rec.reconcile(store, "default", "privacy")
    pol = store.get("SessionPrivacyPolicy", "privacy", "default")
    krs = pol["status"]["keyRotation"]
    assert pol["status"]["phase"] == "Active"
    assert krs["currentKeyVersion"] == "2" and krs["previousKeyVersion"] == "1"
    assert ROTATE_KEY_ANNOTATION not in (pol["metadata"].get("annotations") or {})
    assert krs["reEncryptionProgress"]["status"] == "InProgress" and rq == 1.0
    assert get_condition({"status": pol["status"]}, "KeyRotationReady")["status"] == "True"
    steps = 0
    while rq is not None and steps < 10:
        rq = rec.reconcile(store, "default", "privacy")
        steps += 1
    pol = store.get("SessionPrivacyPolicy", "privacy", "default")
    prog = pol["status"]["keyRotation"]["reEncryptionProgress"]
    assert prog["status"] == "Completed" and prog["messagesProcessed"] == 5
    assert steps >= 3  # 5 messages in batches of 2
    assert set(_versions(warm)) == {"2"}
    svc.hot.invalidate("s1")
    assert [m.content for m in svc.get("s1")[1]] == [f"secret {i}" for i in range(5)]
    # the running session-api (its own LocalKMS instance) picks the new key up
    svc2, _ = _svc(tmp_path, LocalKMS(path=keyfile))
    asyncio.run(svc.append_message("s1", Message(content="after")))
    assert _versions(warm)[-1] == "2" or "2" in _versions(warm)
    assert {e["reason"] for e in _events(store)} >= {"KeyRotated", "ReEncryptionStarted",
                                                      "ReEncryptionBatch"}


def test_scheduled_rotation_waits_for_the_cron_time(tmp_path):
    keyfile = str(tmp_path / "keys.json")
    LocalKMS(path=keyfile)
    now = [_t("2026-03-01 00:30")]
    store = APIStore()
    rec = SessionPrivacyPolicyReconciler(provider_factory=lambda cfg: LocalKMS(path=keyfile),
                                         now=lambda: now[0])
    _put(store, _spp({"enabled": True, "schedule": "0 * * * *"}))
    rq = rec.reconcile(store, "default", "privacy")
    krs = store.get("SessionPrivacyPolicy", "privacy", "default")["status"]["keyRotation"]
    assert "currentKeyVersion" not in krs and abs(rq - 1800) < 1
    assert krs["nextRotationAt"] == "2026-03-01T01:00:00Z"
    now[0] = _t("2026-03-01 01:00") + 5
    rq = rec.reconcile(store, "default", "privacy")
    krs = store.get("SessionPrivacyPolicy", "privacy", "default")["status"]["keyRotation"]
    assert krs["currentKeyVersion"] == "2" and krs["nextRotationAt"] == "2026-03-01T02:00:00Z"
    assert 3500 < rq <= 3600
    # not due again within the hour
    now[0] += 60
    rec.reconcile(store, "default", "privacy")
    assert store.get("SessionPrivacyPolicy", "privacy", "default")["status"]["keyRotation"][
        "currentKeyVersion"] == "2"


def test_rotation_failures_surface_in_status(tmp_path):
    def boom(cfg):
        raise ConnectionError("vault unreachable")

    store = APIStore()
    rec = SessionPrivacyPolicyReconciler(provider_factory=boom)
    _put(store, _spp({"enabled": True}, annotations={ROTATE_KEY_ANNOTATION: "x"}))
    rq = rec.reconcile(store, "default", "privacy")
    st = store.get("SessionPrivacyPolicy", "privacy", "default")["status"]
    c = get_condition({"status": st}, "KeyRotationReady")
    assert c["status"] == "False" and "vault unreachable" in c["message"] and rq == 300.0
    # re-encryption without a store factory fails loudly, not silently
    keyfile = str(tmp_path / "k.json")
    rec2 = SessionPrivacyPolicyReconciler(provider_factory=lambda cfg: LocalKMS(path=keyfile))
    _put(store, _spp({"enabled": True, "reEncryptExisting": True}, name="p2",
                     annotations={ROTATE_KEY_ANNOTATION: "x"}))
    rec2.reconcile(store, "default", "p2")
    rec2.reconcile(store, "default", "p2")
    st = store.get("SessionPrivacyPolicy", "p2", "default")["status"]
    assert st["keyRotation"]["reEncryptionProgress"]["status"] == "Failed"
    assert "store factory not configured" in get_condition({"status": st}, "KeyRotationReady")["message"]


def test_policy_without_rotation_is_just_active():
    store = APIStore()
    rec = SessionPrivacyPolicyReconciler()
    _put(store, {"apiVersion": API, "kind": "SessionPrivacyPolicy",
                 "metadata": {"name": "p", "uid": "u"}, "spec": {"level": "global"}})
    assert rec.reconcile(store, "default", "p") is None
    st = store.get("SessionPrivacyPolicy", "p", "default")["status"]
    assert st["phase"] == "Active" and get_condition({"status": st}, "Ready")["reason"] == "PolicyValidated"


def test_rotate_request_is_served_once_even_if_annotation_sticks(tmp_path):
    """If clearing the annotation fails, the same request must not rotate again."""
    keyfile = str(tmp_path / "keys.json")
    store = APIStore()
    rec = SessionPrivacyPolicyReconciler(provider_factory=lambda cfg: LocalKMS(path=keyfile))
    _put(store, _spp({"enabled": True}, annotations={ROTATE_KEY_ANNOTATION: "r1"}))
    orig = store.update

    def no_meta_updates(obj, subresource=None, **kw):
        if subresource is None:
            raise RuntimeError("conflict")
        return orig(obj, subresource=subresource, **kw)

    store.update = no_meta_updates
    rec.reconcile(store, "default", "privacy")
    rec.reconcile(store, "default", "privacy")
    krs = store.get("SessionPrivacyPolicy", "privacy", "default")["status"]["keyRotation"]
    assert krs["currentKeyVersion"] == "2"  # not 3
