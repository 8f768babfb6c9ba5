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
import math
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
    if not isinstance(hdr, dict) or not isinstance(claims, dict):
        raise AuthError("malformed token: header and claims must be JSON objects")
    for c in ("exp", "nbf"):  # RFC 7519 NumericDate
        v = claims.get(c)
        if v is not None and (isinstance(v, bool) or not isinstance(v, (int, float))
                              or not math.isfinite(v)):
            raise AuthError(f"malformed token: {c} is not a number")
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
    if claims.get("exp") is not None and now > claims["exp"] + leeway:
        raise AuthError("token expired")
    if claims.get("nbf") is not None and now + leeway < claims["nbf"]:
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


MGMT_ISSUER = "omnia-dashboard"  # pkg/facade/auth/mgmt_plane.go DefaultMgmtPlaneIssuer
MGMT_AUDIENCE = "omnia-facade"
ORIGIN_MGMT = "management-plane"  # pkg/policy/identity.go OriginManagementPlane


class JWKSResolver:
    """Signing keys of the management plane by ``kid`` (``auth.JWKSResolver``).

    Keys come from ``url`` (the dashboard's ``/api/auth/jwks``), fetched lazily
    and re-fetched on an unknown ``kid`` at most every ``min_refresh_s`` (key
    rotation without hammering the dashboard), or from a static ``jwks`` dict.
    A fetch failure resolves to no key, i.e. an invalid credential."""

    def __init__(self, url: str | None = None, jwks: dict | None = None,
                 min_refresh_s: float = 2.0, timeout_s: float = 3.0, fetch=None):
        if not url and jwks is None:
            raise ValueError("mgmt-plane: JWKS URL required")
        self.url = url
        self.min_refresh_s = min_refresh_s
        self.timeout_s = timeout_s
        self._fetch = fetch or self._http_fetch
        self._keys: dict = {}
        self._last = float("-inf")
        if jwks is not None:
            self._load(jwks)

    def _load(self, jwks: dict) -> None:
        self._keys = {k.get("kid", ""): k for k in (jwks or {}).get("keys", [])
                      if k.get("kty") == "RSA"}

    def _http_fetch(self) -> dict:
        import urllib.request

        with urllib.request.urlopen(self.url, timeout=self.timeout_s) as r:
            return json.loads(r.read())

    def resolve(self, kid: str) -> dict | None:
        k = self._keys.get(kid)
        if k is not None or not self.url:
            return k
        now = time.monotonic()
        if now - self._last < self.min_refresh_s:
            return None
        self._last = now
        try:
            self._load(self._fetch())
        except Exception:  # noqa: BLE001 - dashboard down / DNS: invalid credential
            return None
        return self._keys.get(kid)

    def refresh(self, kid: str) -> dict | None:
        """Re-fetch (rate-limited like an unknown kid) after a signature failed
        against the cached key of ``kid``: the issuer may have rotated its key
        without changing the kid.  Returns the (possibly new) key."""
        if not self.url:
            return None
        now = time.monotonic()
        if now - self._last < self.min_refresh_s:
            return None
        self._last = now
        try:
            self._load(self._fetch())
        except Exception:  # noqa: BLE001
            return None
        return self._keys.get(kid)


class MgmtPlaneValidator:
    """Dashboard-minted RS256 JWTs on the management-plane twin listeners only
    (``pkg/facade/auth/mgmt_plane.go``): issuer ``omnia-dashboard``, audience
    ``omnia-facade``, ``exp`` required, ``kid`` resolved through the JWKS,
    claim ``origin == "management-plane"``, and when the facade knows its agent
    / workspace a token naming another one is refused."""

    def __init__(self, resolver: JWKSResolver, issuer: str = MGMT_ISSUER,
                 audience: str = MGMT_AUDIENCE, expected_agent: str = "",
                 expected_workspace: str = ""):
        self.resolver = resolver
        self.blocking = bool(resolver.url)
        self.issuer, self.audience = issuer, audience
        self.expected_agent, self.expected_workspace = expected_agent, expected_workspace

    def validate(self, headers, query, peer):
        tok = bearer(headers)
        if tok is None:
            return None
        if not tok or tok.count(".") != 2:
            raise AuthError("invalid credential: malformed bearer")
        try:
            hdr = json.loads(_b64url_dec(tok.split(".")[0]))
        except Exception as e:  # noqa: BLE001
            raise AuthError("invalid credential: malformed header") from e
        if not isinstance(hdr, dict):
            raise AuthError("invalid credential: malformed header")
        if hdr.get("alg") != "RS256":
            raise AuthError(f"unexpected signing method {hdr.get('alg')!r}")
        kid = hdr.get("kid") or ""
        if not isinstance(kid, str) or not kid:
            raise AuthError("mgmt-plane JWT missing kid header")
        key = self.resolver.resolve(kid)
        if key is None:
            raise AuthError("invalid credential: unknown signing key")
        try:
            claims = jwt_decode(tok, None, {"keys": [key]}, self.issuer, self.audience)
        except AuthError:
            # the cached key under this kid may be stale (issuer restarted with a
            # new key but the same kid): one rate-limited re-fetch, then retry
            fresh = self.resolver.refresh(kid)
            if fresh is None or fresh == key:
                raise
            claims = jwt_decode(tok, None, {"keys": [fresh]}, self.issuer, self.audience)
        if "exp" not in claims:
            raise AuthError("invalid credential: exp required")
        if claims.get("origin") != ORIGIN_MGMT:
            raise AuthError(f"origin {claims.get('origin')!r} is not management-plane")
        agent, ws = str(claims.get("agent") or ""), str(claims.get("workspace") or "")
        if self.expected_agent and agent and agent != self.expected_agent:
            raise AuthError(f"token agent {agent!r} does not match {self.expected_agent!r}")
        if self.expected_workspace and ws and ws != self.expected_workspace:
            raise AuthError(f"token workspace {ws!r} does not match {self.expected_workspace!r}")
        sub = str(claims.get("sub", ""))
        return Identity(ORIGIN_MGMT, subject=sub, end_user=sub, workspace=ws, agent=agent,
                        claims=claims, role=str(claims.get("role", "")))


def jwk_thumbprint(key) -> str:
    """RFC 7638 SHA-256 thumbprint of an RSA key's public part (base64url): the
    default ``kid`` of a signing key, so a new key always gets a new kid and
    every JWKS cache keyed by kid misses on it (re-fetch) instead of verifying
    against the old key."""
    import hashlib

    n = key.n.to_bytes((key.n.bit_length() + 7) // 8, "big")
    e = key.e.to_bytes((key.e.bit_length() + 7) // 8, "big")
    canon = json.dumps({"e": _b64url_enc(e), "kty": "RSA", "n": _b64url_enc(n)},
                       separators=(",", ":"), sort_keys=True).encode()
    return _b64url_enc(hashlib.sha256(canon).digest())


def jwk_from_private(key, kid: str) -> dict:
    """Public JWK of an :class:`omnia_amd.utils.rsa.PrivateKey` (JWKS endpoint)."""
    n = key.n.to_bytes((key.n.bit_length() + 7) // 8, "big")
    e = key.e.to_bytes((key.e.bit_length() + 7) // 8, "big")
    return {"kty": "RSA", "kid": kid, "alg": "RS256", "use": "sig",
            "n": _b64url_enc(n), "e": _b64url_enc(e)}


def mint_mgmt_token(key, kid: str, subject: str, agent: str = "", workspace: str = "",
                    ttl_s: int = 300, issuer: str = MGMT_ISSUER,
                    audience: str = MGMT_AUDIENCE, **extra) -> str:
    """RS256 management-plane JWT as the dashboard mints it for its WS proxy and
    the doctor (origin ``management-plane``)."""
    from ..utils.rsa import sign_pkcs1_sha256

    now = int(time.time())
    claims = {"iss": issuer, "aud": audience, "sub": subject, "iat": now, "exp": now + ttl_s,
              "origin": ORIGIN_MGMT, **extra}
    if agent:
        claims["agent"] = agent
    if workspace:
        claims["workspace"] = workspace
    hdr = {"alg": "RS256", "typ": "JWT", "kid": kid}
    h = _b64url_enc(json.dumps(hdr, separators=(",", ":")).encode())
    p = _b64url_enc(json.dumps(claims, separators=(",", ":")).encode())
    sig = sign_pkcs1_sha256(key, f"{h}.{p}".encode())
    return f"{h}.{p}.{_b64url_enc(sig)}"


class AuthChain:
    """``strict`` chains (the management-plane twin) never admit an anonymous
    caller, even when empty (no JWKS configured): the twin exists only for
    dashboard-minted tokens."""

    def __init__(self, validators: list | None = None, allow_anonymous: bool = True,
                 strict: bool = False):
        self.validators = validators or []
        self.allow_anonymous = allow_anonymous and not strict
        self.strict = strict

    @property
    def blocking(self) -> bool:
        """True when a validator may do network I/O (a JWKS fetch)."""
        return any(getattr(v, "blocking", False) for v in self.validators)

    def authenticate(self, headers, query=None, peer: str = "") -> Identity:
        query = query or {}
        for v in self.validators:
            ident = v.validate(headers, query, peer)
            if ident is not None:
                return ident
        if self.allow_anonymous or (not self.validators and not self.strict):
            return Identity("anonymous")
        raise AuthError("unauthenticated")
