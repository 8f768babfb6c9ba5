"""Workspace roles (+ the reference's own parity fixture), dashboard identity
tokens and the REST authz middleware, pseudonymous user ids, service discovery
from Workspace status, service-account token review."""
import asyncio
import hashlib
import json
import os
import time

import pytest

from omnia_amd.facade.auth import jwt_encode_hs256
from omnia_amd.operator import authz as A

REF_CASES = "/root/reference/pkg/workspaceauth/testdata/parity_cases.json"


def test_roles_basic():
    rb = [{"groups": ["eng"], "role": "viewer"}, {"groups": ["admins"], "role": "owner"}]
    assert A.compute_role(rb, [], None, ["eng", "admins"], "u@x.io", False) == "owner"
    assert A.compute_role(rb, [], None, ["x"], "u@x.io", False) == ""
    dg = [{"user": "U@X.io", "role": "editor", "expires": "2000-01-01T00:00:00Z"}]
    assert A.compute_role([], dg, None, [], "u@x.io", False) == ""  # expired
    dg[0]["expires"] = "2999-01-01T00:00:00Z"
    assert A.compute_role([], dg, None, [], "u@x.io", False) == "editor"
    assert A.compute_role([], [], {"enabled": True}, [], "", True) == "viewer"
    assert A.compute_role([], [], {"enabled": True, "role": "editor"}, [], "", True) == "editor"
    assert A.meets_required("owner", "editor") and not A.meets_required("viewer", "editor")
    assert A.required_role_for_method("GET") == "viewer"
    assert A.required_role_for_method("DELETE") == "editor"


@pytest.mark.skipif(not os.path.exists(REF_CASES), reason="reference fixture not mounted")
def test_reference_parity_cases():
    with open(REF_CASES) as f:
        cases = json.load(f)
    for c in cases:
        got = A.compute_role(c.get("roleBindings") or [], c.get("directGrants") or [],
                             c.get("anonymousAccess"), c.get("userGroups") or [],
                             c.get("userIdentity", ""), c.get("anonymous", False))
        assert got == c["expectedRole"], c["name"]


def test_pseudonyms(monkeypatch):
    monkeypatch.delenv("OMNIA_PSEUDONYM_HMAC_KEY", raising=False)
    assert A.pseudonymize_id("") == ""
    assert A.pseudonymize_id("alice") == hashlib.sha256(b"alice").hexdigest()[:16]
    monkeypatch.setenv("OMNIA_PSEUDONYM_HMAC_KEY", "k")
    p = A.pseudonymize_id("alice")
    assert len(p) == 16 and p != hashlib.sha256(b"alice").hexdigest()[:16]


def _store():
    from omnia_amd.api import crds
    from omnia_amd.operator.apistore import APIStore

    st = APIStore()
    st.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace",
              "metadata": {"name": "team-a"},
              "spec": {"displayName": "A", "namespace": {"name": "team-a"},
                       "roleBindings": [{"groups": ["eng"], "role": "editor"}],
                       "directGrants": [{"user": "boss@x.io", "role": "owner"}]}})
    return st


def test_service_discovery():
    st = _store()
    ws = st.get("Workspace", "team-a", None)
    ws["status"] = {"privacyURL": "http://privacy:8085", "services": [
        {"name": "default", "sessionURL": "http://sess:8300", "memoryURL": "http://mem:8400"},
        {"name": "pending", "sessionURL": ""}]}
    st.update_status(ws) if hasattr(st, "update_status") else st.apply(ws)
    r = A.ServiceResolver(st)
    urls = r.resolve("team-a")
    assert (urls.session_url, urls.memory_url, urls.privacy_url) == \
        ("http://sess:8300", "http://mem:8400", "http://privacy:8085")
    with pytest.raises(LookupError):
        r.resolve("team-a", "pending")
    with pytest.raises(LookupError):
        r.resolve("team-a", "nope")
    with pytest.raises(LookupError):
        r.resolve("missing")


def test_identity_verifier_and_middleware():
    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    st = _store()
    key = b"dash-secret"
    ver = A.IdentityVerifier(hs_key=key, issuer="omnia-dashboard", audience="omnia-api")

    def tok(**kw):
        c = {"iss": "omnia-dashboard", "aud": "omnia-api", "exp": time.time() + 60,
             "sub": "u1", "identity": "dev@x.io", "groups": ["eng"], "workspace": "team-a"}
        c.update(kw)
        return jwt_encode_hs256(c, key)

    with pytest.raises(PermissionError):
        ver.verify(tok(exp=time.time() - 3600))
    with pytest.raises(PermissionError):
        ver.verify(tok(aud="other"))

    async def handler(request):
        return web.json_response({"role": request["omnia_role"]})

    async def run():
        app = web.Application(middlewares=[A.authz_middleware(ver, st)])
        app.router.add_route("*", "/api/v1/workspaces/{ws}/content/{path:.*}", handler)
        c = TestClient(TestServer(app))
        await c.start_server()
        try:
            u = "/api/v1/workspaces/team-a/content/x"
            assert (await c.get(u)).status == 401
            h = {"Authorization": f"Bearer {tok()}"}
            r = await c.get(u, headers=h)
            assert r.status == 200 and (await r.json())["role"] == "editor"
            assert (await c.put(u, headers=h)).status == 200
            viewer = {"Authorization": f"Bearer {tok(groups=['x'], identity='v@x.io')}"}
            assert (await c.get(u, headers=viewer)).status == 403  # no role at all
            other = {"Authorization": f"Bearer {tok(workspace='team-b')}"}
            assert (await c.get(u, headers=other)).status == 403
            nows = {"Authorization": f"Bearer {tok(workspace='ghost')}"}
            assert (await c.get("/api/v1/workspaces/ghost/content/x",
                                headers=nows)).status == 404
        finally:
            await c.close()

    asyncio.run(run())


def test_service_account_auth():
    reviews = {"good": (True, "system:serviceaccount:omnia-system:facade"),
               "stranger": (True, "system:serviceaccount:other:x"),
               "listed": (True, "system:serviceaccount:other:eval")}
    sa = A.ServiceAccountAuth(lambda t: reviews.get(t, (False, "")),
                              allowed_subjects=["system:serviceaccount:other:eval"],
                              allowed_namespaces=["omnia-system"])
    assert sa.check("good") == (200, "system:serviceaccount:omnia-system:facade")
    assert sa.check("listed")[0] == 200
    assert sa.check("stranger")[0] == 403
    assert sa.check("bogus")[0] == 401 and sa.check(None)[0] == 401
    assert A.parse_service_account("system:serviceaccount:ns:n") == ("ns", "n")
    assert A.parse_service_account("user:bob") is None
