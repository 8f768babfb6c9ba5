"""Compliance presets -> SessionPrivacyPolicy specs (SURVEY §2.2 E6;
reference ``ee/pkg/compliance/presets.go``).

``get_preset("gdpr" | "hipaa" | "ccpa")`` returns a complete
``SessionPrivacyPolicy.spec`` dict (recording + PII redaction/encryption,
retention tiers, user opt-out / delete-within, audit-log retention) that the
privacy reconciler and the session/memory write paths consume like any
hand-written policy.  Pattern names are the redaction engine's
(:mod:`omnia_amd.ee.redaction`), so a preset can never reference a pattern the
redactor cannot apply (checked in the tests)."""
from __future__ import annotations

import copy

PRESETS = ("gdpr", "hipaa", "ccpa")

_BASE = {
    "recording": {"enabled": True, "facadeData": True, "runtimeData": True,
                  "pii": {"redact": True, "encrypt": True, "strategy": "replace",
                          "patterns": []}},
    "userOptOut": {"enabled": True, "honorDeleteRequests": True, "deleteWithinDays": 30},
    "auditLog": {"enabled": True, "retentionDays": 365},
}

_SPECS = {
    # GDPR Art. 5(1)(e) storage limitation; Art. 17 erasure within one month
    "gdpr": {"patterns": ["email", "phone_number", "ip_address", "credit_card"],
             "retention": {"facade": {"warmDays": 30, "coldDays": 90}},
             "audit_days": 365, "encryption": False},
    # HIPAA: 6-year documentation retention (~2555 days used by the reference)
    "hipaa": {"patterns": ["ssn", "email", "phone_number", "ip_address", "credit_card"],
              "retention": {"facade": {"warmDays": 30, "coldDays": 2555}},
              "audit_days": 2555, "encryption": True},
    # CCPA: 45-day response window for deletion requests
    "ccpa": {"patterns": ["email", "phone_number", "ip_address", "ssn"],
             "retention": {"facade": {"warmDays": 30, "coldDays": 365}},
             "audit_days": 730, "encryption": False, "delete_within": 45},
}


def list_presets() -> list[str]:
    return list(PRESETS)


def get_preset(name: str) -> dict:
    key = (name or "").lower()
    if key not in _SPECS:
        raise ValueError(f"unknown compliance preset: {name!r}")
    p = _SPECS[key]
    spec = copy.deepcopy(_BASE)
    spec["recording"]["pii"]["patterns"] = list(p["patterns"])
    spec["retention"] = copy.deepcopy(p["retention"])
    spec["auditLog"]["retentionDays"] = p["audit_days"]
    if p.get("delete_within"):
        spec["userOptOut"]["deleteWithinDays"] = p["delete_within"]
    if p["encryption"]:
        spec["encryption"] = {"enabled": True}
    return spec


def apply_preset(policy: dict) -> dict:
    """Expand ``spec.preset`` of a SessionPrivacyPolicy object; explicit fields in
    the object's spec win over the preset's."""
    spec = policy.get("spec") or {}
    name = spec.get("preset")
    if not name:
        return policy

    def merge(base, over):
        out = copy.deepcopy(base)
        for k, v in over.items():
            out[k] = merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) \
                else v
        return out

    merged = merge(get_preset(name), {k: v for k, v in spec.items() if k != "preset"})
    return {**policy, "spec": merged}
