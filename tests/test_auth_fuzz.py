"""Fuzz test of the facade JWT paths (facade/auth.py): any bearer token --
garbage, a non-object header or claims, ``exp`` / ``nbf`` of the wrong JSON
type, a non-string ``kid`` -- either authenticates or raises ``AuthError``
(401); nothing else may escape into the connection handler.  Mirrors the
reference's typed claim parsing (``pkg/facade/auth/mgmt_plane.go``).

It found that a token whose header or claims decode to a non-object (``null``,
an array) raised ``AttributeError`` instead of a 401; a correctly signed
``"exp": "soon"`` raised ``TypeError``, and a non-string ``kid`` on the
management-plane listener raised ``TypeError``."""
import base64
import functools
import json

from hypothesis import given, settings
from hypothesis import strategies as st

from omnia_amd.facade.auth import (AuthError, JWKSResolver, MgmtPlaneValidator, OIDCValidator,
                                   jwk_from_private, jwt_decode)
from omnia_amd.utils.rsa import generate_private_key, sign_pkcs1_sha256

KEY = b"k" * 32
JSON = st.recursive(st.none() | st.booleans() | st.integers() | st.text(max_size=6)
                    | st.floats(),
                    lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=5), c,
                                                                         max_size=3),
                    max_leaves=8)
CLAIMS = st.one_of(JSON, st.fixed_dictionaries(
    {}, optional={"exp": JSON, "nbf": JSON, "iss": JSON, "aud": JSON, "sub": JSON,
                  "origin": st.sampled_from(["management-plane", "x"]), "agent": JSON,
                  "workspace": JSON, "role": JSON}))
HDR = st.one_of(JSON, st.fixed_dictionaries(
    {"alg": st.sampled_from(["HS256", "RS256", "none", 5])}, optional={"kid": JSON}))


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


@functools.lru_cache(maxsize=None)
def _rsa():
    return generate_private_key(1024)


def _token(hdr, claims, rs: bool) -> str:
    h = _b64(json.dumps(hdr).encode())
    p = _b64(json.dumps(claims).encode())
    msg = f"{h}.{p}".encode()
    if rs:
        sig = sign_pkcs1_sha256(_rsa(), msg)
    else:
        import hashlib
        import hmac
        sig = hmac.new(KEY, msg, hashlib.sha256).digest()
    return f"{h}.{p}.{_b64(sig)}"


def _ok_or_auth_error(fn):
    try:
        out = fn()
    except AuthError:
        return None
    return out


@given(HDR, CLAIMS, st.booleans(), st.sampled_from([None, "iss"]), st.sampled_from([None, "aud"]))
@settings(max_examples=300, deadline=None)
def test_signed_tokens_with_arbitrary_claims(hdr, claims, rs, iss, aud):
    tok = _token(hdr, claims, rs)
    jwks = {"keys": [jwk_from_private(_rsa(), "kid1")]}
    out = _ok_or_auth_error(lambda: jwt_decode(tok, KEY, jwks, iss, aud))
    assert out is None or isinstance(out, dict)
    _ok_or_auth_error(lambda: OIDCValidator(hs_key=KEY, jwks=jwks).validate(
        {"Authorization": "Bearer " + tok}, {}, "127.0.0.1"))
    mg = MgmtPlaneValidator(JWKSResolver(jwks=jwks), expected_agent="a", expected_workspace="w")
    _ok_or_auth_error(lambda: mg.validate({"Authorization": "Bearer " + tok}, {}, "127.0.0.1"))


@given(st.one_of(st.text(max_size=40), st.lists(st.text(max_size=12), min_size=3, max_size=3)
                 .map(".".join)))
@settings(max_examples=300, deadline=None)
def test_garbage_tokens(tok):
    _ok_or_auth_error(lambda: jwt_decode(tok, KEY))
    mg = MgmtPlaneValidator(JWKSResolver(jwks={"keys": []}))
    _ok_or_auth_error(lambda: mg.validate({"Authorization": "Bearer " + tok}, {}, "127.0.0.1"))


@given(st.one_of(JSON, st.fixed_dictionaries(
    {}, optional={"exp": JSON, "iat": JSON, "lid": JSON, "tier": JSON, "features": JSON,
                  "limits": st.one_of(JSON, st.dictionaries(
                      st.sampled_from(["maxScenarios", "maxWorkerReplicas"]), JSON))})),
       st.sampled_from([{"alg": "RS256"}, None, [], "RS256"]))
@settings(max_examples=200, deadline=None)
def test_license_tokens_never_escape_get_or_default(claims, hdr):
    """A license token signed with the right key but ill-typed claims (or a
    non-object header) is a LicenseError, so ``get_or_default`` falls back to
    open-core instead of raising (``ee/license.py`` promises it never raises)."""
    from omnia_amd.ee import license as L

    k = _rsa()
    h = _b64(json.dumps(hdr).encode())
    b = _b64(json.dumps(claims).encode())
    tok = f"{h}.{b}.{_b64(L.rs256_sign(f'{h}.{b}'.encode(), k.n, k.d))}"
    v = L.Validator(L.public_pem(k.n, k.e), secret_reader=lambda: tok)
    lic = v.get_or_default()
    assert isinstance(lic, L.License)
    assert isinstance(lic.tier, str) and isinstance(lic.id, str)
