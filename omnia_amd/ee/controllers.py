"""Enterprise policy controllers: ToolPolicy and SessionPrivacyPolicy (with KMS
key rotation and background re-encryption of stored messages).

* :class:`ToolPolicyReconciler` (``ee/internal/controller/toolpolicy_controller.go``):
  compiles every deny rule's CEL and every header-injection rule (value XOR
  cel) into the in-process policy evaluator (``ee/policy_broker.py``), sets
  ``Compiled`` / ``Ready`` / ``HeaderRefsCanonical`` conditions, ``ruleCount``
  and phase ``Active`` / ``Error``, warns about CEL that indexes ``headers``
  with a non-canonical key (``headers["x-user-id"]`` never matches: header
  maps are keyed ``X-User-Id``; ``ee/pkg/policy/cel_lint.go``), and removes a
  deleted policy from the evaluator.
* :class:`SessionPrivacyPolicyReconciler`
  (``sessionprivacypolicy_controller.go`` + ``keyrotation_controller.go``):
  marks the policy Active, then -- when ``spec.encryption.keyRotation`` is
  enabled -- rotates the KMS key on the ``omnia.altairalabs.ai/rotate-key``
  annotation (removed afterwards) or when the cron ``schedule`` comes due
  (next fire after ``status.keyRotation.lastRotatedAt``), records
  ``currentKeyVersion`` / ``KeyRotationReady``, and with ``reEncryptExisting``
  walks the session store in ``batchSize`` batches (cursor in
  ``status.keyRotation.reEncryptionProgress``) re-sealing every message still
  under an older key version, one batch per reconcile, requeued until done.
"""
from __future__ import annotations

import base64
import logging
import re
import time

from ..operator.apistore import set_condition
from ..utils import cron

log = logging.getLogger("omnia.ee.controllers")

ROTATE_KEY_ANNOTATION = "omnia.altairalabs.ai/rotate-key"
_HEADER_REF = re.compile(r"""headers\s*\[\s*(?:"([^"]*)"|'([^']*)')\s*\]""")


def canonical_header(key: str) -> str:
    """Go ``textproto.CanonicalMIMEHeaderKey``: dash-separated words with an
    upper-case first letter, the rest lower case (keys with spaces or other
    invalid token bytes are returned unchanged)."""
    if not key or any(c in key for c in " \t\r\n:") or not key.isascii():
        return key
    return "-".join(w[:1].upper() + w[1:].lower() for w in key.split("-"))


def non_canonical_header_refs(expr: str) -> list[tuple[str, str]]:
    out, seen = [], set()
    for m in _HEADER_REF.finditer(expr or ""):
        key = m.group(1) or m.group(2)
        if not key or key in seen:
            continue
        canon = canonical_header(key)
        if canon != key:
            seen.add(key)
            out.append((key, canon))
    return out


def _event(store, obj: dict, kind: str, reason: str, message: str, warning: bool = False):
    md = obj["metadata"]
    try:
        store.create({"apiVersion": "v1", "kind": "Event",
                      "metadata": {"generateName": f"{md['name']}.",
                                   "namespace": md.get("namespace") or "default"},
                      "involvedObject": {"apiVersion": obj.get("apiVersion", ""), "kind": kind,
                                         "name": md["name"], "namespace": md.get("namespace"),
                                         "uid": md.get("uid", "")},
                      "reason": reason, "message": message[:1024],
                      "type": "Warning" if warning else "Normal",
                      "source": {"component": "omnia-ee-controller"},
                      "firstTimestamp": _ts(time.time())})
    except Exception as e:  # noqa: BLE001 - events are best effort
        log.debug("event %s not recorded: %s", reason, e)


def _ts(t: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def _parse_ts(v) -> float | None:
    if v in (None, ""):
        return None
    if isinstance(v, (int, float)):
        return float(v)
    import calendar

    return float(calendar.timegm(time.strptime(str(v)[:19], "%Y-%m-%dT%H:%M:%S")))


# ===================================================================== ToolPolicy
class ToolPolicyReconciler:
    kind = "ToolPolicy"

    def __init__(self, evaluator=None):
        from .policy_broker import Evaluator

        self.evaluator = evaluator if evaluator is not None else Evaluator()

    def reconcile(self, store, ns, name):
        from .policy_broker import compile_policy

        ns = ns or "default"
        tp = store.try_get(self.kind, name, ns)
        if tp is None:
            self.evaluator.remove_policy(ns, name)
            return None
        gen = tp["metadata"].get("generation", 1)
        st = dict(tp.get("status") or {})
        st["observedGeneration"] = gen
        spec = tp.get("spec") or {}
        try:
            for h in spec.get("headerInjection") or []:
                if not h.get("header"):
                    raise ValueError("header injection: header name is required")
                if h.get("value") and h.get("cel"):
                    raise ValueError(f"header {h['header']!r}: value and cel are mutually "
                                     "exclusive")
                if not h.get("value") and not h.get("cel"):
                    raise ValueError(f"header {h['header']!r}: one of value or cel must be set")
            compiled = compile_policy(tp)
        except Exception as e:  # noqa: BLE001 - CEL syntax / type errors
            msg = str(e)
            rule = next((r.get("name") for r in spec.get("rules") or []
                         if _bad_cel((r.get("deny") or {}).get("cel", "false"))), None)
            if rule:
                msg = f"rule {rule!r}: {msg}"
            set_condition(st, "Compiled", False, "CompileError", msg, gen)
            set_condition(st, "Ready", False, "CompileError", "policy has CEL compilation errors",
                          gen)
            st.update(phase="Error", ruleCount=0)
            self.evaluator.remove_policy(ns, name)
            _event(store, tp, self.kind, "CompileError", msg, warning=True)
            tp["status"] = st
            store.update_status(tp)
            return None
        self.evaluator.set_policy(tp)
        warnings = []
        for r in spec.get("rules") or []:
            for raw, canon in non_canonical_header_refs((r.get("deny") or {}).get("cel", "")):
                warnings.append(f"rule {r.get('name')!r} references non-canonical header "
                                f"{raw!r} (use {canon!r})")
        for h in spec.get("headerInjection") or []:
            for raw, canon in non_canonical_header_refs(h.get("cel", "")):
                warnings.append(f"headerInjection {h.get('header')!r} references non-canonical "
                                f"header {raw!r} (use {canon!r})")
        if warnings:
            msg = ("CEL references to non-canonical header keys will silently miss: " +
                   "; ".join(warnings))
            set_condition(st, "HeaderRefsCanonical", False, "NonCanonicalHeaderRef", msg, gen)
            _event(store, tp, self.kind, "NonCanonicalHeaderRef", msg, warning=True)
        else:
            set_condition(st, "HeaderRefsCanonical", True, "HeaderRefsCanonical",
                          "all header references are canonical", gen)
        set_condition(st, "Compiled", True, "PolicyCompiled",
                      f"{len(compiled.rules)} rule(s) compiled", gen)
        set_condition(st, "Ready", True, "PolicyValidated", "policy is active", gen)
        st.update(phase="Active", ruleCount=len(compiled.rules))
        if (tp.get("status") or {}).get("phase") != "Active":
            _event(store, tp, self.kind, "PolicyCompiled",
                   f"compiled {len(compiled.rules)} rule(s)")
        tp["status"] = st
        store.update_status(tp)
        return None


def _bad_cel(src: str) -> bool:
    from ..utils import cel

    try:
        cel.compile(src)
        return False
    except Exception:  # noqa: BLE001
        return True


# ========================================================== SessionPrivacyPolicy
class SessionPrivacyPolicyReconciler:
    """Active status + KMS key rotation + batched re-encryption (module doc)."""

    kind = "SessionPrivacyPolicy"
    DEFAULT_BATCH = 100
    BATCH_REQUEUE_S = 1.0
    FAILED_ROTATION_REQUEUE_S = 300.0

    def __init__(self, provider_factory=None, store_factory=None, now=time.time):
        self.provider_factory = provider_factory or self._default_provider
        self.store_factory = store_factory
        self.now = now

    # -------------------------------------------------------------- factories
    @staticmethod
    def _default_provider(cfg: dict):
        from .encryption import build_provider

        return build_provider(cfg)

    def _provider_cfg(self, store, pol: dict) -> dict:
        enc = (pol.get("spec") or {}).get("encryption") or {}
        cfg = {"type": enc.get("kmsProvider", ""), "keyID": enc.get("keyID", "")}
        ref = (enc.get("secretRef") or {}).get("name")
        if ref:
            sec = store.try_get("Secret", ref, pol["metadata"].get("namespace") or "default")
            if sec is not None:
                for k, v in (sec.get("data") or {}).items():
                    cfg[k] = base64.b64decode(v).decode()
                cfg.update(sec.get("stringData") or {})
        return cfg

    # -------------------------------------------------------------- reconcile
    def reconcile(self, store, ns, name):
        pol = store.try_get(self.kind, name, ns)
        if pol is None:
            return None
        gen = pol["metadata"].get("generation", 1)
        st = dict(pol.get("status") or {})
        st["observedGeneration"] = gen
        was_active = st.get("phase") == "Active"
        set_condition(st, "Ready", True, "PolicyValidated", "policy is valid and active", gen)
        st["phase"] = "Active"
        if not was_active:
            _event(store, pol, self.kind, "PolicyValidated", "Policy validated and active")
        pol["status"] = st
        requeue = None
        kr = ((pol.get("spec") or {}).get("encryption") or {})
        if kr.get("enabled") and (kr.get("keyRotation") or {}).get("enabled"):
            requeue = self._rotation(store, pol)
        store.update_status(pol)
        return requeue

    # -------------------------------------------------------------- rotation
    def _rotation(self, store, pol: dict) -> float | None:
        st = pol["status"]
        krs = st.setdefault("keyRotation", {})
        prog = krs.get("reEncryptionProgress") or {}
        if prog.get("status") == "InProgress":
            return self._reencrypt_batch(store, pol)
        ann = pol["metadata"].get("annotations") or {}
        if ROTATE_KEY_ANNOTATION in ann and krs.get("handledRotateRequest") == \
                f"{ann[ROTATE_KEY_ANNOTATION]}@{pol['metadata'].get('uid', '')}":
            ann = {}  # this request was already served (its removal failed): no re-rotation
        if ROTATE_KEY_ANNOTATION in ann:
            ok = self._rotate(store, pol, "annotation")
            if ok:
                krs["handledRotateRequest"] = \
                    f"{ann[ROTATE_KEY_ANNOTATION]}@{pol['metadata'].get('uid', '')}"
            # clear the trigger (metadata update; status is written by the caller)
            cur = store.try_get(self.kind, pol["metadata"]["name"], pol["metadata"].get(
                "namespace"))
            if cur is not None:
                cur["metadata"].setdefault("annotations", {}).pop(ROTATE_KEY_ANNOTATION, None)
                cur.pop("status", None)
                try:
                    new = store.update(cur)
                    pol["metadata"]["resourceVersion"] = new["metadata"]["resourceVersion"]
                    pol["metadata"]["annotations"] = new["metadata"].get("annotations") or {}
                except Exception as e:  # noqa: BLE001
                    log.debug("could not clear rotate annotation: %s", e)
            if ok and (krs.get("reEncryptionProgress") or {}).get("status") == "InProgress":
                return self.BATCH_REQUEUE_S
            return None if ok else self.FAILED_ROTATION_REQUEUE_S
        return self._scheduled(store, pol)

    def _scheduled(self, store, pol: dict) -> float | None:
        krc = pol["spec"]["encryption"]["keyRotation"]
        sched = krc.get("schedule")
        if not sched:
            return None
        try:
            base = _parse_ts(pol["status"]["keyRotation"].get("lastRotatedAt")) or _parse_ts(
                pol["metadata"].get("creationTimestamp")) or self.now()
            nxt = cron.next_fire(sched, base)
        except (cron.CronError, ValueError) as e:
            self._fail(store, pol, f"invalid key rotation schedule: {e}")
            return None
        now = self.now()
        pol["status"]["keyRotation"]["nextRotationAt"] = _ts(nxt)
        if now < nxt:
            return max(1.0, nxt - now)
        ok = self._rotate(store, pol, "schedule")
        if not ok:
            return self.FAILED_ROTATION_REQUEUE_S
        if (pol["status"]["keyRotation"].get("reEncryptionProgress") or {}).get(
                "status") == "InProgress":
            return self.BATCH_REQUEUE_S
        nxt = cron.next_fire(sched, self.now())
        pol["status"]["keyRotation"]["nextRotationAt"] = _ts(nxt)
        return max(1.0, nxt - self.now())

    def _rotate(self, store, pol: dict, trigger: str) -> bool:
        try:
            prov = self.provider_factory(self._provider_cfg(store, pol))
            try:
                prev, new = prov.rotate()
            finally:
                close = getattr(prov, "close", None)
                if close:
                    close()
        except Exception as e:  # noqa: BLE001 - provider / network failures
            self._fail(store, pol, f"key rotation failed: {e}")
            return False
        krs = pol["status"]["keyRotation"]
        krs.update(lastRotatedAt=_ts(self.now()), currentKeyVersion=new,
                   previousKeyVersion=prev)
        gen = pol["metadata"].get("generation", 1)
        set_condition(pol["status"], "KeyRotationReady", True, "KeyRotated",
                      f"rotated key to version {new} ({trigger})", gen)
        _event(store, pol, self.kind, "KeyRotated",
               f"key rotated from version {prev} to {new} ({trigger})")
        if pol["spec"]["encryption"]["keyRotation"].get("reEncryptExisting"):
            krs["reEncryptionProgress"] = {"status": "InProgress", "startedAt": _ts(self.now()),
                                           "messagesProcessed": 0, "errors": 0,
                                           "lastProcessedID": ""}
            _event(store, pol, self.kind, "ReEncryptionStarted",
                   f"re-encrypting existing messages under key version {new}")
        return True

    def _reencrypt_batch(self, store, pol: dict) -> float | None:
        krs = pol["status"]["keyRotation"]
        prog = krs["reEncryptionProgress"]
        if self.store_factory is None:
            return self._fail_reencrypt(store, pol, "store factory not configured")
        try:
            sstore = self.store_factory()
            batch = int(pol["spec"]["encryption"]["keyRotation"].get("batchSize")
                        or self.DEFAULT_BATCH)
            last, more, done, errors = sstore.reencrypt_batch(
                krs.get("currentKeyVersion", ""), prog.get("lastProcessedID", ""), batch)
        except Exception as e:  # noqa: BLE001
            return self._fail_reencrypt(store, pol, f"re-encryption batch failed: {e}")
        prog["messagesProcessed"] = int(prog.get("messagesProcessed", 0)) + done
        prog["errors"] = int(prog.get("errors", 0)) + errors
        prog["lastProcessedID"] = last
        if done:
            _event(store, pol, self.kind, "ReEncryptionBatch",
                   f"re-encrypted {done} message(s), {prog['messagesProcessed']} so far")
        if more:
            return self.BATCH_REQUEUE_S
        prog["status"] = "Completed"
        prog["completedAt"] = _ts(self.now())
        return None

    def _fail_reencrypt(self, store, pol, msg: str):
        prog = pol["status"]["keyRotation"].get("reEncryptionProgress") or {}
        prog["status"] = "Failed"
        pol["status"]["keyRotation"]["reEncryptionProgress"] = prog
        self._fail(store, pol, msg)
        return None

    def _fail(self, store, pol, msg: str):
        set_condition(pol["status"], "KeyRotationReady", False, "KeyRotationFailed", msg,
                      pol["metadata"].get("generation", 1))
        _event(store, pol, self.kind, "KeyRotationFailed", msg, warning=True)
