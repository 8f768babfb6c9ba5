"""Facade authentication chain (``pkg/facade/auth/chain.go:45-59`` and siblings).

Validators are tried in order; each returns an :class:`Identity`, ``None``
("not mine, try the next one") or raises :class:`AuthError` (credential present
but invalid -> 401).  Provided: shared token, client API keys (sha-256 at rest),
OIDC/JWT (RS256 via JWKS or static PEM-free JWK, HS256), edge-trust headers
from a trusted proxy, and management-plane JWTs (dashboard twin ports).
``cryptography`` is not installed, so RS256 verification is a small pure-Python
PKCS#1 v1.5 check.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time
from dataclasses import dataclass, field


class AuthError(Exception):
    pass


@dataclass
class Identity:
    origin: str  # shared-token | client-key | oidc | edge | mgmt-plane | anonymous
    subject: str = ""
    end_user: str = ""
    workspace: str = ""
    agent: str = ""
    claims: dict = field(default_factory=dict)
    role: str = ""

    def to_metadata(self) -> dict:
        """Flat x-omnia-* propagation (pkg/policy/context.go:80-147); never the bearer."""
        md = {"x-omnia-origin": self.origin}
        if self.end_user or self.subject:
            md["x-omnia-user-id"] = self.end_user or self.subject
        if self.workspace:
            md["x-omnia-workspace"] = self.workspace
        if self.claims.get("email"):
            md["x-omnia-user-email"] = str(self.claims["email"])
        for k, v in self.claims.items():
            if isinstance(v, (str, int, float, bool)) and k not in ("exp", "iat", "nbf"):
                md[f"x-omnia-claim-{k}"] = str(v)
        return md


def _b64url_dec(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def _b64url_enc(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


_SHA256_DI = bytes.fromhex("3031300d060960864801650304020105000420")


def rsa_verify_pkcs1_sha256(n: int, e: int, msg: bytes, sig: bytes) -> bool:
    k = (n.bit_length() + 7) // 8
    if len(sig) != k:
        return False
    m = pow(int.from_bytes(sig, "big"), e, n).to_bytes(k, "big")
    digest = hashlib.sha256(msg).digest()
    t = _SHA256_DI + digest
    expected = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return hmac.compare_digest(m, expected)


def jwt_encode_hs256(claims: dict, key: bytes, kid: str | None = None) -> str:
    hdr = {"alg": "HS256", "typ": "JWT", **({"kid": kid} if kid else {})}
    h = _b64url_enc(json.dumps(hdr, separators=(",", ":")).encode())
    p = _b64url_enc(json.dumps(claims, separators=(",", ":")).encode())
    sig = hmac.new(key, f"{h}.{p}".encode(), hashlib.sha256).digest()
    return f"{h}.{p}.{_b64url_enc(sig)}"


def jwt_decode(token: str, hs_key: bytes | None = None, jwks: dict | None = None,
               issuer: str | None = None, audience: str | None = None, leeway: int = 30) -> dict:
    try:
        h64, p64, s64 = token.split(".")
        hdr = json.loads(_b64url_dec(h64))
        claims = json.loads(_b64url_dec(p64))
        sig = _b64url_dec(s64)
    except Exception as e:  # noqa: BLE001
        raise AuthError("malformed token") from e
    alg = hdr.get("alg")
    signed = f"{h64}.{p64}".encode()
    if alg == "HS256":
        if not hs_key or not hmac.compare_digest(
                hmac.new(hs_key, signed, hashlib.sha256).digest(), sig):
            raise AuthError("bad signature")
    elif alg == "RS256":
        keys = (jwks or {}).get("keys", [])
        cand = [k for k in keys if k.get("kty") == "RSA" and
                (hdr.get("kid") is None or k.get("kid") == hdr.get("kid"))]
        ok = False
        for k in cand:
            n = int.from_bytes(_b64url_dec(k["n"]), "big")
            e = int.from_bytes(_b64url_dec(k["e"]), "big")
            if rsa_verify_pkcs1_sha256(n, e, signed, sig):
                ok = True
                break
        if not ok:
            raise AuthError("bad signature")
    else:
        raise AuthError(f"unsupported alg {alg}")
    now = time.time()
    if "exp" in claims and now > claims["exp"] + leeway:
        raise AuthError("token expired")
    if "nbf" in claims and now + leeway < claims["nbf"]:
        raise AuthError("token not yet valid")
    if issuer and claims.get("iss") != issuer:
        raise AuthError("bad issuer")
    if audience:
        aud = claims.get("aud")
        auds = aud if isinstance(aud, list) else [aud]
        if audience not in auds:
            raise AuthError("bad audience")
    return claims


def bearer(headers) -> str | None:
    h = headers.get("Authorization") or headers.get("authorization") or ""
    if h.lower().startswith("bearer "):
        return h[7:].strip()
    return None


class SharedTokenValidator:
    def __init__(self, token: str):
        self.token = token

    def validate(self, headers, query, peer) -> Identity | None:
        tok = bearer(headers) or query.get("token")
        if tok is None:
            return None
        if hmac.compare_digest(tok.encode(), self.token.encode()):
            return Identity("shared-token", subject="shared")
        return None


class ClientKeyValidator:
    """API keys: {sha256_hex: {"name":..., "workspace":..., "user":...}} (client_key.go)."""

    def __init__(self, keys: dict):
        self.keys = keys

    @staticmethod
    def hash_key(k: str) -> str:
        return hashlib.sha256(k.encode()).hexdigest()

    def validate(self, headers, query, peer):
        k = headers.get("X-API-Key") or headers.get("x-api-key")
        if not k:
            tok = bearer(headers)
            if tok and tok.startswith("omk_"):
                k = tok
        if not k:
            return None
        rec = self.keys.get(self.hash_key(k))
        if rec is None:
            raise AuthError("invalid API key")
        if rec.get("expires") and time.time() > rec["expires"]:
            raise AuthError("API key expired")
        return Identity("client-key", subject=rec.get("name", ""), end_user=rec.get("user", ""),
                        workspace=rec.get("workspace", ""))


class OIDCValidator:
    def __init__(self, issuer: str | None = None, audience: str | None = None,
                 jwks: dict | None = None, hs_key: bytes | None = None,
                 claim_map: dict | None = None, jwks_loader=None):
        self.issuer = issuer
        self.audience = audience
        self.jwks = jwks
        self.hs_key = hs_key
        self.claim_map = claim_map or {"subject": "sub", "end_user": "sub"}
        self.jwks_loader = jwks_loader

    def validate(self, headers, query, peer):
        tok = bearer(headers) or query.get("access_token")
        if not tok or tok.count(".") != 2:
            return None
        jwks = self.jwks
        if jwks is None and self.jwks_loader is not None:
            jwks = self.jwks = self.jwks_loader()
        claims = jwt_decode(tok, self.hs_key, jwks, self.issuer, self.audience)
        return Identity("oidc", subject=str(claims.get(self.claim_map["subject"], "")),
                        end_user=str(claims.get(self.claim_map["end_user"], "")),
                        workspace=str(claims.get("workspace", "")), claims=claims)


class EdgeTrustValidator:
    """Trust claim headers injected by an authenticating edge, e.g. Istio
    RequestAuthentication with outputClaimToHeaders (``edge_trust.go``):
    subject / end user default to ``x-user-id``, email ``x-user-email``, role
    ``x-user-roles`` (default role viewer); ``claims_from_headers`` maps extra
    inbound headers to claim names.  The reference relies on the pod's network
    policy to keep the headers honest; here the peer must also be in
    ``trusted_peers`` (the sidecar / edge on loopback by default)."""

    def __init__(self, subject_header: str = "x-user-id", end_user_header: str = "x-user-id",
                 email_header: str = "x-user-email", role_header: str = "x-user-roles",
                 claims_from_headers: dict | None = None, default_role: str = "viewer",
                 trusted_peers=("127.0.0.1", "::1")):
        self.subject_header = subject_header or "x-user-id"
        self.end_user_header = end_user_header or "x-user-id"
        self.email_header = email_header or "x-user-email"
        self.role_header = role_header
        self.extra = {k.lower(): v for k, v in (claims_from_headers or {}).items() if k and v}
        self.default_role = default_role
        self.trusted = set(trusted_peers) if trusted_peers else None

    @staticmethod
    def _get(headers, name):
        v = headers.get(name)
        if v is None:
            low = name.lower()
            v = next((hv for hk, hv in headers.items() if hk.lower() == low), None)
        return v or ""

    def validate(self, headers, query, peer):
        subject = self._get(headers, self.subject_header)
        if not subject:
            return None
        if self.trusted is not None and peer not in self.trusted:
            raise AuthError("untrusted edge")
        claims = {"role": self._get(headers, self.role_header) or self.default_role}
        email = self._get(headers, self.email_header)
        if email:
            claims["email"] = email
        for h, name in self.extra.items():
            v = self._get(headers, h)
            if v:
                claims[name] = v
        return Identity("edge", subject=subject,
                        end_user=self._get(headers, self.end_user_header) or subject,
                        claims=claims, role=claims["role"])


class MgmtPlaneValidator:
    """Dashboard-minted HS256 JWTs on the management twin ports (mgmt_plane.go)."""

    def __init__(self, key: bytes, audience: str = "omnia-facade"):
        self.key = key
        self.audience = audience

    def validate(self, headers, query, peer):
        tok = bearer(headers) or query.get("mgmt_token")
        if not tok or tok.count(".") != 2:
            return None
        try:
            claims = jwt_decode(tok, self.key, None, None, self.audience)
        except AuthError:
            return None  # let other validators try (it may be an OIDC token)
        return Identity("mgmt-plane", subject=str(claims.get("sub", "")),
                        workspace=str(claims.get("workspace", "")), claims=claims,
                        role=str(claims.get("role", "")))


class AuthChain:
    def __init__(self, validators: list | None = None, allow_anonymous: bool = True):
        self.validators = validators or []
        self.allow_anonymous = allow_anonymous

    def authenticate(self, headers, query=None, peer: str = "") -> Identity:
        query = query or {}
        for v in self.validators:
            ident = v.validate(headers, query, peer)
            if ident is not None:
                return ident
        if self.allow_anonymous or not self.validators:
            return Identity("anonymous")
        raise AuthError("unauthenticated")
