"""Workspace authorization, pseudonymous identities, service discovery and
service-account auth (SURVEY §2.1 C18 authz, C42, C43).

* Workspace roles (reference ``pkg/workspaceauth``): ``viewer < editor <
  owner``; a principal's role is the highest of its IdP-group role bindings and
  its (unexpired, case-insensitive) direct grant; identity-less / anonymous
  principals get ``anonymousAccess.role`` (default viewer) only when enabled.
  GET/HEAD need viewer, every other verb editor.
* :class:`IdentityVerifier` -- dashboard-minted RS256 JWTs (JWKS), issuer /
  audience / exp checked; claims ``identity``, ``groups``, ``workspace``,
  ``anonymous``.
* :func:`authz_middleware` -- guards operator REST routes that carry a
  ``{ws}`` path variable (workspace content API): 401 without/invalid token,
  403 on workspace mismatch or insufficient role, 404 unknown workspace.
* :func:`pseudonymize_id` (reference ``pkg/identity``): 16-hex SHA-256 (or
  HMAC-SHA-256 under ``OMNIA_PSEUDONYM_HMAC_KEY``) so facade ingestion and
  dashboard queries agree on user pseudonyms.
* :class:`ServiceResolver` (reference ``pkg/servicediscovery``): session /
  memory / privacy API URLs of a workspace's service group from
  ``Workspace.status.services`` (URLs returned as soon as the session URL is
  populated, even before the group is Ready).
* :class:`ServiceAccountAuth` (reference ``internal/serviceauth``): bearer
  tokens reviewed by a TokenReview callable, subject
  ``system:serviceaccount:<ns>:<name>`` checked against allowed subjects /
  namespaces, with exempt paths (health probes).
"""
from __future__ import annotations

import hashlib
import hmac
import os
import time
from dataclasses import dataclass, field
from datetime import datetime

ROLE_VIEWER, ROLE_EDITOR, ROLE_OWNER = "viewer", "editor", "owner"
_RANK = {"": 0, ROLE_VIEWER: 1, ROLE_EDITOR: 2, ROLE_OWNER: 3}


def max_role(a: str, b: str) -> str:
    return a if _RANK.get(a or "", 0) >= _RANK.get(b or "", 0) else b


def meets_required(granted: str, required: str) -> bool:
    if not required:
        return True
    return _RANK.get(granted or "", 0) >= _RANK[required]


def required_role_for_method(method: str) -> str:
    return ROLE_VIEWER if method.upper() in ("GET", "HEAD") else ROLE_EDITOR


def _expired(expires: str, now: float) -> bool:
    if not expires:
        return False
    try:
        ts = datetime.fromisoformat(expires.replace("Z", "+00:00")).timestamp()
    except ValueError:
        return False  # unparseable expiry: treated as no expiry (reference behaviour)
    return now > ts


def compute_role(role_bindings: list, direct_grants: list, anonymous_access: dict | None,
                 user_groups: list, user_identity: str, anonymous: bool,
                 now: float | None = None) -> str:
    now = time.time() if now is None else now
    if anonymous or not user_identity:
        if anonymous_access and anonymous_access.get("enabled"):
            return anonymous_access.get("role") or ROLE_VIEWER
        return ""
    groups = set(user_groups or [])
    role = ""
    for b in role_bindings or []:
        if any(g in groups for g in b.get("groups") or []):
            role = max_role(role, b.get("role", ""))
    ident = user_identity.lower()
    for g in direct_grants or []:
        if (g.get("user") or "").lower() != ident:
            continue
        if _expired(g.get("expires", ""), now):
            continue
        role = max_role(role, g.get("role", ""))
        break
    return role


def workspace_inputs(ws: dict) -> dict:
    spec = ws.get("spec") or {}
    return {"role_bindings": spec.get("roleBindings") or [],
            "direct_grants": spec.get("directGrants") or [],
            "anonymous_access": spec.get("anonymousAccess")}


# ------------------------------------------------------------------ identity tokens
@dataclass
class VerifiedIdentity:
    subject: str = ""
    identity: str = ""
    groups: list = field(default_factory=list)
    workspace: str = ""
    anonymous: bool = False


class IdentityVerifier:
    def __init__(self, jwks: dict | None = None, issuer: str = "", audience: str = "",
                 hs_key: bytes | None = None, leeway_s: float = 30.0):
        self.jwks, self.issuer, self.audience = jwks, issuer, audience
        self.hs_key = hs_key  # tests / dev only; production tokens are RS256 via JWKS
        self.leeway = leeway_s

    def verify(self, token: str, now: float | None = None) -> VerifiedIdentity:
        from ..facade.auth import AuthError, jwt_decode

        try:
            claims = jwt_decode(token, hs_key=self.hs_key, jwks=self.jwks)
        except AuthError as e:
            raise PermissionError(f"invalid token: {e}") from e
        now = time.time() if now is None else now
        if "exp" not in claims or now > float(claims["exp"]) + self.leeway:
            raise PermissionError("token expired or missing exp")
        if self.issuer and claims.get("iss") != self.issuer:
            raise PermissionError("issuer mismatch")
        aud = claims.get("aud")
        if self.audience and self.audience not in (aud if isinstance(aud, list) else [aud]):
            raise PermissionError("audience mismatch")
        return VerifiedIdentity(subject=claims.get("sub", ""),
                                identity=claims.get("identity") or claims.get("email", ""),
                                groups=list(claims.get("groups") or []),
                                workspace=claims.get("workspace", ""),
                                anonymous=bool(claims.get("anonymous", False)))


def authz_middleware(verifier: IdentityVerifier, store, path_var: str = "ws"):
    """aiohttp middleware: enforce workspace roles on routes with ``{ws}``."""
    from aiohttp import web

    @web.middleware
    async def mw(request, handler):
        ws_name = request.match_info.get(path_var)
        if ws_name is None:
            return await handler(request)
        h = request.headers.get("Authorization", "")
        if not h.lower().startswith("bearer "):
            return web.json_response({"error": "missing bearer token"}, status=401)
        try:
            vid = verifier.verify(h[7:].strip())
        except PermissionError:
            return web.json_response({"error": "invalid token"}, status=401)
        if vid.workspace != ws_name:
            return web.json_response({"error": "token workspace mismatch"}, status=403)
        ws = store.try_get("Workspace", ws_name, None)
        if ws is None:
            return web.json_response({"error": "workspace not found"}, status=404)
        role = compute_role(user_groups=vid.groups, user_identity=vid.identity,
                            anonymous=vid.anonymous, **workspace_inputs(ws))
        if not meets_required(role, required_role_for_method(request.method)):
            return web.json_response({"error": "insufficient role"}, status=403)
        request["omnia_identity"] = vid
        request["omnia_role"] = role
        return await handler(request)

    return mw


# ------------------------------------------------------------------ pseudonyms
PSEUDONYM_LEN = 16


def pseudonymize_id(raw: str) -> str:
    if not raw:
        return ""
    key = os.environ.get("OMNIA_PSEUDONYM_HMAC_KEY", "")
    if key:
        return hmac.new(key.encode(), raw.encode(), hashlib.sha256).hexdigest()[:PSEUDONYM_LEN]
    return hashlib.sha256(raw.encode()).hexdigest()[:PSEUDONYM_LEN]


# ------------------------------------------------------------------ service discovery
@dataclass
class ServiceURLs:
    session_url: str
    memory_url: str = ""
    privacy_url: str = ""


class ServiceResolver:
    def __init__(self, store):
        self.store = store

    def workspace(self, name: str) -> dict:
        ws = self.store.try_get("Workspace", name, None)
        if ws is None:
            raise LookupError(f"workspace {name!r} not found")
        return ws

    def resolve(self, workspace: str, service_group: str = "default") -> ServiceURLs:
        ws = self.workspace(workspace)
        st = ws.get("status") or {}
        for svc in st.get("services") or []:
            if svc.get("name") != service_group:
                continue
            if not svc.get("sessionURL"):
                raise LookupError(f"service group {service_group!r} is not ready")
            return ServiceURLs(svc["sessionURL"], svc.get("memoryURL", ""),
                               st.get("privacyURL", ""))
        raise LookupError(f"service group {service_group!r} not found in workspace "
                          f"{workspace!r}")

    def session_url(self, workspace: str, group: str = "default") -> str:
        return self.resolve(workspace, group).session_url

    def memory_url(self, workspace: str, group: str = "default") -> str:
        return self.resolve(workspace, group).memory_url


def detect_namespace(path: str = "/var/run/secrets/kubernetes.io/serviceaccount/namespace"
                     ) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return os.environ.get("OMNIA_NAMESPACE", "omnia-system")


# ------------------------------------------------------------------ service-account auth
def parse_service_account(subject: str) -> tuple[str, str] | None:
    parts = (subject or "").split(":")
    if len(parts) == 4 and parts[0] == "system" and parts[1] == "serviceaccount" and \
            parts[2] and parts[3]:
        return parts[2], parts[3]
    return None


class ServiceAccountAuth:
    """``review(token) -> (authenticated, subject)`` is the TokenReview call."""

    def __init__(self, review, allowed_subjects=(), allowed_namespaces=(),
                 exempt=("/healthz", "/readyz", "/metrics")):
        self.review = review
        self.subjects = set(allowed_subjects)
        self.namespaces = set(allowed_namespaces)
        self.exempt = set(exempt)

    def allowed(self, subject: str) -> bool:
        if subject in self.subjects:
            return True
        sa = parse_service_account(subject)
        return sa is not None and sa[0] in self.namespaces

    def check(self, token: str | None) -> tuple[int, str]:
        if not token:
            return 401, "missing bearer token"
        ok, subject = self.review(token)
        if not ok:
            return 401, "token review failed"
        if not self.allowed(subject):
            return 403, f"subject {subject} not allowed"
        return 200, subject

    def middleware(self):
        from aiohttp import web

        @web.middleware
        async def mw(request, handler):
            if request.path in self.exempt:
                return await handler(request)
            h = request.headers.get("Authorization", "")
            tok = h[7:].strip() if h.lower().startswith("bearer ") else None
            status, detail = self.check(tok)
            if status != 200:
                return web.json_response({"error": detail}, status=status)
            request["omnia_subject"] = detail
            return await handler(request)

        return mw


class ProjectedTokenSource:
    """Reads the projected SA token from disk with a refresh TTL (reference
    ``tokensource.go``) and authorises outgoing requests with it."""

    def __init__(self, path: str = "/var/run/secrets/omnia/token", ttl_s: float = 300.0):
        self.path, self.ttl = path, ttl_s
        self._tok, self._at = "", 0.0

    def token(self) -> str:
        now = time.monotonic()
        if not self._tok or now - self._at > self.ttl:
            with open(self.path) as f:
                self._tok = f.read().strip()
            self._at = now
        return self._tok

    def headers(self) -> dict:
        return {"Authorization": f"Bearer {self.token()}"}
