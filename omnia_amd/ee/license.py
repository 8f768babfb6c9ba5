"""Enterprise licensing (reference ``ee/pkg/license/``).

Behaviour kept from the reference:
* tiers ``open-core`` / ``enterprise``; feature flags and limits as in
  ``ee/pkg/license/types.go`` (open-core: git sources only, 10 scenarios,
  1 worker replica; dev mode: everything, unlimited);
* the license is an RS256-signed JWT in Secret ``omnia-license`` (key
  ``license``), verified against a PEM public key (ConfigMap / env), with a
  cache TTL; an expired or badly signed token falls back to open-core
  (``GetLicenseOrDefault``), never to enterprise;
* activation state with heartbeat interval + offline grace period, a cluster
  fingerprint, and the "nag" message for unlicensed enterprise usage.

No JWT/crypto library ships in this image, so RS256 verification is done here
in pure Python (SubjectPublicKeyInfo DER parse + PKCS#1 v1.5 / SHA-256); the
tests sign tokens with a freshly generated key.
"""
from __future__ import annotations

import base64
import dataclasses
import hashlib
import json
import os
import time
from dataclasses import dataclass, field

TIER_OPEN_CORE = "open-core"
TIER_ENTERPRISE = "enterprise"
SECRET_NAME = "omnia-license"
SECRET_KEY = "license"


class LicenseError(Exception):
    pass


class LicenseExpired(LicenseError):
    pass


class InvalidSignature(LicenseError):
    pass


class LicenseNotFound(LicenseError):
    pass


@dataclass
class Features:
    gitSource: bool = False
    ociSource: bool = False
    s3Source: bool = False
    loadTesting: bool = False
    dataGeneration: bool = False
    scheduling: bool = False
    distributedWorkers: bool = False
    whiteLabel: bool = False
    memoryEnterprise: bool = False
    privacyEnterprise: bool = False
    policyProxy: bool = False
    customFacade: bool = False


@dataclass
class Limits:
    maxScenarios: int = 0  # 0 = unlimited
    maxWorkerReplicas: int = 0
    maxActivations: int = 0


@dataclass
class License:
    id: str
    tier: str
    customer: str
    features: Features = field(default_factory=Features)
    limits: Limits = field(default_factory=Limits)
    issued_at: float = field(default_factory=time.time)
    expires_at: float = field(default_factory=lambda: time.time() + 100 * 365 * 86400)

    def is_expired(self, now: float | None = None) -> bool:
        return (now or time.time()) > self.expires_at

    def is_enterprise(self) -> bool:
        return self.tier == TIER_ENTERPRISE

    def is_valid_enterprise(self) -> bool:
        return self.is_enterprise() and not self.is_expired()

    def can_use_source_type(self, t: str) -> bool:
        return {"git": self.features.gitSource, "oci": self.features.ociSource,
                "s3": self.features.s3Source, "configmap": True}.get(t.lower(), False)

    def can_use_job_type(self, t: str) -> bool:
        return {"evaluation": True, "loadtest": self.features.loadTesting,
                "datagen": self.features.dataGeneration}.get(t.lower(), False)

    def can_use_scheduling(self) -> bool:
        return self.features.scheduling

    def can_use_custom_facade(self) -> bool:
        return self.features.customFacade

    def can_use_tool_policy(self) -> bool:
        return self.features.policyProxy

    def can_use_memory_enterprise(self) -> bool:
        return self.features.memoryEnterprise

    def can_use_privacy_enterprise(self) -> bool:
        return self.features.privacyEnterprise

    def can_use_worker_replicas(self, n: int) -> bool:
        m = self.limits.maxWorkerReplicas
        return m == 0 or n <= m

    def can_use_scenario_count(self, n: int) -> bool:
        return self.limits.maxScenarios == 0 or n <= self.limits.maxScenarios

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def open_core_license() -> License:
    return License(id="open-core", tier=TIER_OPEN_CORE, customer="Open Core User",
                   features=Features(gitSource=True), limits=Limits(maxScenarios=10,
                                                                    maxWorkerReplicas=1))


def dev_license() -> License:
    return License(id="dev-mode", tier=TIER_ENTERPRISE, customer="Development Mode",
                   features=Features(**{f.name: True for f in dataclasses.fields(Features)}),
                   limits=Limits())


# ------------------------------------------------------------------ RS256 (pure Python)
def _b64d(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def _b64e(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _der(buf: bytes, i: int):
    tag = buf[i]
    ln = buf[i + 1]
    i += 2
    if ln & 0x80:
        n = ln & 0x7F
        ln = int.from_bytes(buf[i:i + n], "big")
        i += n
    return tag, buf[i:i + ln], i + ln


def parse_rsa_public_key(pem: str) -> tuple[int, int]:
    """(n, e) from a PEM ``PUBLIC KEY`` (SPKI) or ``RSA PUBLIC KEY`` (PKCS#1)."""
    lines = [ln for ln in pem.strip().splitlines() if not ln.startswith("-----")]
    der = base64.b64decode("".join(lines))
    tag, body, _ = _der(der, 0)
    if tag != 0x30:
        raise LicenseError("bad public key")
    t1, v1, nxt = _der(body, 0)
    if t1 == 0x30:  # SPKI: AlgorithmIdentifier, BIT STRING(RSAPublicKey)
        t2, bits, _ = _der(body, nxt)
        if t2 != 0x03:
            raise LicenseError("bad SPKI")
        _, rsa, _ = _der(bits[1:], 0)
        _, nb, j = _der(rsa, 0)
        _, eb, _ = _der(rsa, j)
    else:  # PKCS#1 RSAPublicKey
        nb = v1
        _, eb, _ = _der(body, nxt)
    return int.from_bytes(nb, "big"), int.from_bytes(eb, "big")


_SHA256_PREFIX = bytes.fromhex("3031300d060960864801650304020105000420")


def _emsa(digest: bytes, k: int) -> bytes:
    t = _SHA256_PREFIX + digest
    return b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t


def rs256_verify(signing_input: bytes, sig: bytes, n: int, e: int) -> bool:
    k = (n.bit_length() + 7) // 8
    if len(sig) != k:
        return False
    m = pow(int.from_bytes(sig, "big"), e, n).to_bytes(k, "big")
    return m == _emsa(hashlib.sha256(signing_input).digest(), k)


def rs256_sign(signing_input: bytes, n: int, d: int) -> bytes:
    k = (n.bit_length() + 7) // 8
    m = int.from_bytes(_emsa(hashlib.sha256(signing_input).digest(), k), "big")
    return pow(m, d, n).to_bytes(k, "big")


def make_token(claims: dict, n: int, d: int) -> str:
    """Sign a license JWT (issuer-side tooling and tests)."""
    head = _b64e(json.dumps({"alg": "RS256", "typ": "JWT"}).encode())
    body = _b64e(json.dumps(claims).encode())
    sig = rs256_sign(f"{head}.{body}".encode(), n, d)
    return f"{head}.{body}.{_b64e(sig)}"


def public_pem(n: int, e: int) -> str:
    """PKCS#1 ``RSA PUBLIC KEY`` PEM for (n, e)."""
    def enc_len(ln):
        if ln < 0x80:
            return bytes([ln])
        b = ln.to_bytes((ln.bit_length() + 7) // 8, "big")
        return bytes([0x80 | len(b)]) + b

    def integer(v):
        b = v.to_bytes((v.bit_length() + 8) // 8, "big")
        return b"\x02" + enc_len(len(b)) + b

    body = integer(n) + integer(e)
    der = b"\x30" + enc_len(len(body)) + body
    b64 = base64.b64encode(der).decode()
    return "-----BEGIN RSA PUBLIC KEY-----\n" + "\n".join(
        b64[i:i + 64] for i in range(0, len(b64), 64)) + "\n-----END RSA PUBLIC KEY-----\n"


# ------------------------------------------------------------------ validator
class Validator:
    """License lookup with caching; never raises from :meth:`get_or_default`."""

    def __init__(self, public_key_pem: str | None = None, secret_reader=None,
                 cache_ttl_s: float = 300.0, dev_mode: bool | None = None):
        self.key = parse_rsa_public_key(public_key_pem) if public_key_pem else None
        self.read_secret = secret_reader  # () -> token str | None
        self.ttl = cache_ttl_s
        self.dev = dev_mode if dev_mode is not None else \
            os.environ.get("OMNIA_LICENSE_DEV_MODE", "") in ("1", "true")
        self._cache: tuple[float, License] | None = None

    def invalidate(self) -> None:
        self._cache = None

    def validate_token(self, token: str, now: float | None = None) -> License:
        if self.key is None:
            raise InvalidSignature("no license public key configured")
        try:
            h, b, s = token.strip().split(".")
            head = json.loads(_b64d(h))
        except Exception as e:  # noqa: BLE001
            raise LicenseError(f"malformed license token: {e}") from e
        if not isinstance(head, dict):
            raise LicenseError("malformed license token: header is not a JSON object")
        if head.get("alg") != "RS256":
            raise InvalidSignature(f"unexpected signing method {head.get('alg')!r}")
        if not rs256_verify(f"{h}.{b}".encode(), _b64d(s), *self.key):
            raise InvalidSignature("license signature invalid")
        now = now or time.time()
        try:
            return self._claims(json.loads(_b64d(b)), now)
        except LicenseError:
            raise
        except (ValueError, TypeError, AttributeError) as e:  # signed but ill-typed claims
            raise LicenseError(f"malformed license claims: {e}") from e

    @staticmethod
    def _claims(c: dict, now: float) -> License:
        if "exp" in c and now > float(c["exp"]):
            raise LicenseExpired("license expired")
        for f in ("lid", "tier", "customer"):
            if not isinstance(c.get(f, ""), str):
                raise TypeError(f"license claim {f} is not a string")
        feats = {f.name: bool((c.get("features") or {}).get(f.name, False))
                 for f in dataclasses.fields(Features)}
        lim = c.get("limits") or {}
        return License(id=c.get("lid", ""), tier=c.get("tier", TIER_OPEN_CORE),
                       customer=c.get("customer", ""), features=Features(**feats),
                       limits=Limits(int(lim.get("maxScenarios", 0)),
                                     int(lim.get("maxWorkerReplicas", 0)),
                                     int(lim.get("maxActivations", 0))),
                       issued_at=float(c.get("iat", now)),
                       expires_at=float(c.get("exp", now + 365 * 86400)))

    def get(self) -> License:
        if self.dev:
            return dev_license()
        now = time.time()
        if self._cache and now - self._cache[0] < self.ttl:
            return self._cache[1]
        token = self.read_secret() if self.read_secret else os.environ.get("OMNIA_LICENSE")
        if not token:
            raise LicenseNotFound("no license secret")
        lic = self.validate_token(token, now)
        self._cache = (now, lic)
        return lic

    def get_or_default(self) -> License:
        try:
            return self.get()
        except LicenseError:
            return open_core_license()


# ------------------------------------------------------------------ activation / nag
def cluster_fingerprint(cluster_uid: str, node_names: list[str] | None = None) -> str:
    """Stable installation id (kube-system namespace UID + sorted node names)."""
    h = hashlib.sha256(cluster_uid.encode())
    for n in sorted(node_names or []):
        h.update(b"\x00" + n.encode())
    return h.hexdigest()[:32]


@dataclass
class ActivationState:
    activation_id: str = ""
    fingerprint: str = ""
    activated_at: float = 0.0
    last_heartbeat: float = 0.0
    grace_period_s: float = 7 * 86400

    def needs_heartbeat(self, interval_s: float, now: float | None = None) -> bool:
        return (now or time.time()) - self.last_heartbeat >= interval_s

    def in_grace_period(self, now: float | None = None) -> bool:
        return (now or time.time()) - self.last_heartbeat <= self.grace_period_s


def nag_message(lic: License, used_features: list[str]) -> str | None:
    """Warning for enterprise features used without an enterprise license
    (reference ``nag.go``); None when nothing to say."""
    if lic.is_valid_enterprise():
        days = (lic.expires_at - time.time()) / 86400
        return (f"Omnia Enterprise license {lic.id} expires in {int(days)} days"
                if days < 30 else None)
    if not used_features:
        return None
    return ("Enterprise features in use without a valid license: "
            + ", ".join(sorted(used_features))
            + ". Open-core limits apply; see the license Secret 'omnia-license'.")


def gate_agentruntime(spec: dict, lic: License) -> list[str]:
    """Admission checks that depend on the license (custom facade, tool policy)."""
    errs = []
    if any((f or {}).get("type") == "custom" for f in spec.get("facades") or []) and \
            not lic.can_use_custom_facade():
        errs.append("spec.facades: custom facades require an enterprise license "
                    "(feature customFacade)")
    return errs
