"""PII detection, redaction and consent classification.

* built-in patterns + ``custom:<regex>`` (``ee/pkg/redaction/patterns.go``);
  structural patterns survive the explicit-trust filter;
* strategies replace / hash (``[HASH_<LABEL>:<12 hex>]``) / mask (keep last 4)
  (``ee/pkg/redaction/strategy.go:20-55``);
* rule classifier health > location > identity
  (``ee/pkg/privacy/classify/rules.go``).
"""
from __future__ import annotations

import hashlib
import re
from dataclasses import dataclass

# name -> (regex, token, structural)
BUILTIN = {
    "ssn": (r"\b\d{3}-\d{2}-\d{4}\b", "[REDACTED_SSN]", True),
    "credit_card": (r"\b\d{4}[- ]?\d{4}[- ]?\d{4}[- ]?\d{4}\b", "[REDACTED_CC]", True),
    "phone_number": (r"\b\d{3}[-.)\s]?\d{3}[-.)\s]?\d{4}\b", "[REDACTED_PHONE]", False),
    "email": (r"(?i)\b[A-Za-z0-9._%+\-]+@[A-Za-z0-9.\-]+\.[A-Za-z]{2,}\b", "[REDACTED_EMAIL]",
              False),
    "ip_address": (r"\b\d{1,3}\.\d{1,3}\.\d{1,3}\.\d{1,3}\b", "[REDACTED_IP]", True),
}
_COMPILED = {k: (re.compile(v[0]), v[1], v[2]) for k, v in BUILTIN.items()}

TRUST_INFERRED = "inferred"
TRUST_EXPLICIT = "explicit"


@dataclass
class Pattern:
    name: str
    regex: re.Pattern
    token: str
    structural: bool


def resolve_patterns(names: list[str] | None) -> list[Pattern]:
    names = list(names or BUILTIN)
    out = []
    for n in names:
        if n.startswith("custom:"):
            try:
                out.append(Pattern(n, re.compile(n[len("custom:"):]), "[REDACTED_CUSTOM]", True))
            except re.error as e:
                raise ValueError(f"invalid custom pattern {n!r}: {e}") from e
            continue
        if n not in _COMPILED:
            raise ValueError(f"unknown PII pattern: {n!r}")
        rx, tok, st = _COMPILED[n]
        out.append(Pattern(n, rx, tok, st))
    return out


def find_pii(text: str, patterns: list[str] | None = None) -> set[str]:
    return {p.name for p in resolve_patterns(patterns) if p.regex.search(text or "")}


def _hash(token: str, value: str) -> str:
    label = token.removeprefix("[REDACTED_").removesuffix("]")
    return f"[HASH_{label}:{hashlib.sha256(value.encode()).hexdigest()[:12]}]"


def _mask(value: str) -> str:
    return "*" * len(value) if len(value) <= 4 else "*" * (len(value) - 4) + value[-4:]


def apply_strategy(strategy: str, token: str, matched: str) -> str:
    if strategy == "hash":
        return _hash(token, matched)
    if strategy == "mask":
        return _mask(matched)
    return token


class Redactor:
    """``PIIConfig`` {redact, patterns, strategy} -> callable text redactor."""

    def __init__(self, patterns: list[str] | None = None, strategy: str = "replace"):
        if strategy not in ("", "replace", "hash", "mask"):
            raise ValueError(f"unknown redaction strategy {strategy!r}")
        self.patterns = resolve_patterns(patterns)
        self.strategy = strategy or "replace"

    @classmethod
    def from_config(cls, cfg: dict | None):
        if not cfg or not cfg.get("redact"):
            return None
        return cls(cfg.get("patterns"), cfg.get("strategy") or "replace")

    def redact(self, text: str, trust: str = TRUST_INFERRED) -> tuple[str, dict]:
        counts: dict[str, int] = {}
        pats = self.patterns if trust != TRUST_EXPLICIT else [p for p in self.patterns
                                                               if p.structural]
        for p in pats:
            def sub(m, p=p):
                counts[p.name] = counts.get(p.name, 0) + 1
                return apply_strategy(self.strategy, p.token, m.group(0))

            text = p.regex.sub(sub, text)
        return text, counts

    def __call__(self, text: str) -> str:
        return self.redact(text)[0]


def redact_json(obj, redactor: Redactor):
    """Deep-redact every string in a JSON-like value (``privacy/redact_body.go``)."""
    if isinstance(obj, str):
        return redactor(obj)
    if isinstance(obj, list):
        return [redact_json(x, redactor) for x in obj]
    if isinstance(obj, dict):
        return {k: redact_json(v, redactor) for k, v in obj.items()}
    return obj


HEALTH_KEYWORDS = ("allergy", "allergic", "diagnosis", "diagnosed", "medication", "prescription",
                   "disability", "blood type", "medical", "symptom")
_HEALTH = [re.compile(r"(?i)\b" + re.escape(k) + r"\b") for k in HEALTH_KEYWORDS]
_LOCATION = [re.compile(BUILTIN["ip_address"][0]),
             re.compile(r"(?i)\b(?:lives?\s+in|located\s+in|based\s+in|address\s+is)\b")]
_IDENTITY = [_COMPILED[k][0] for k in ("ssn", "credit_card", "email", "phone_number")]


def classify(content: str) -> str:
    """Most sensitive matching category ('' when none)."""
    if not content:
        return ""
    if any(r.search(content) for r in _HEALTH):
        return "memory:health"
    if any(r.search(content) for r in _LOCATION):
        return "memory:location"
    if any(r.search(content) for r in _IDENTITY):
        return "memory:identity"
    return ""


def classify_categories(content: str) -> list[str]:
    c = classify(content)
    return [c] if c else []
