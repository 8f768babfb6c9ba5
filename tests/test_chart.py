"""Helm chart / kustomize bases (C48) and the dashboard backend (C47).

* deploy/ is exactly what omnia_amd.operator.chart generates (no drift);
* every ``.Values.x.y`` a template references exists in values.yaml;
* all CRD kinds are shipped, static YAML parses, and every python entrypoint a
  template runs is importable;
* the dashboard proxies the operator REST API."""
import asyncio
import glob
import importlib
import json
import os
import re

import yaml

from omnia_amd.api import crds
from omnia_amd.operator import chart

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")


def test_no_drift():
    files = chart.chart_files()
    for rel, body in files.items():
        with open(os.path.join(DEPLOY, rel)) as f:
            assert f.read() == body, f"deploy/{rel} is stale: run `omnia chart --out deploy`"
    on_disk = {os.path.relpath(p, DEPLOY) for p in glob.glob(DEPLOY + "/**/*", recursive=True)
               if os.path.isfile(p)}
    assert on_disk == set(files), on_disk ^ set(files)


def test_values_references_resolve():
    paths = chart.values_paths(chart.VALUES)
    for rel, body in chart.chart_files().items():
        for m in re.finditer(r"\.Values\.([A-Za-z0-9_.]+)", body):
            assert m.group(1).rstrip(".") in paths, (rel, m.group(1))


def test_crds_and_static_yaml():
    files = chart.chart_files()
    for k in crds.KINDS.values():
        doc = yaml.safe_load(files[f"charts/omnia/crds/{crds.GROUP}_{k.plural}.yaml"])
        assert doc["kind"] == "CustomResourceDefinition"
        assert doc["spec"]["names"]["kind"] == k.kind
    for rel, body in files.items():
        if rel.startswith("config/") or "/crds/" in rel or rel.endswith(("values.yaml",
                                                                         "Chart.yaml")):
            assert list(yaml.safe_load_all(body))


def test_entrypoints_importable():
    mods = set()
    for body in chart.chart_files().values():
        mods |= set(re.findall(r'"-m", "([a-z_.]+)"', body))
    assert "omnia_amd.session.api" in mods and "omnia_amd.cli" in mods
    for m in mods:
        mod = importlib.import_module(m)
        assert hasattr(mod, "main"), m


def test_dashboard_proxies_operator_api():
    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.operator.apiserver import build_app as api_app
    from omnia_amd.operator.apistore import APIStore
    from omnia_amd.operator.dashboard import build_app

    async def run():
        store = APIStore()
        store.apply({"apiVersion": crds.API_VERSION, "kind": "Provider",
                     "metadata": {"name": "mock", "namespace": "default"},
                     "spec": {"type": "mock"}})
        api = TestServer(api_app(store))
        await api.start_server()
        dash = TestClient(TestServer(build_app(str(api.make_url("")).rstrip("/"))))
        await dash.start_server()
        try:
            r = await dash.get("/")
            assert r.status == 200 and "Omnia" in await r.text()
            r = await dash.get("/api/resources/providers")
            body = await r.json()
            assert [i["metadata"]["name"] for i in body["items"]] == ["mock"]
            r = await dash.get("/api/overview")
            assert (await r.json())["agents"] == []
            assert (await dash.get("/api/resources/nope")).status == 404
        finally:
            await dash.close()
            await api.close()

    asyncio.run(run())


def _rsa_jwk(seed=7):
    import base64
    import random

    rng = random.Random(seed)

    def prime(bits):
        while True:
            c = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
            if all(pow(a, c - 1, c) == 1 for a in (2, 3, 5, 7, 11, 13, 17, 19, 23)):
                return c
    e = 65537
    while True:
        p, q = prime(512), prime(512)
        phi = (p - 1) * (q - 1)
        if p != q and phi % e:
            break
    n, d = p * q, pow(e, -1, (p - 1) * (q - 1))

    def b64(i):
        return base64.urlsafe_b64encode(i.to_bytes((i.bit_length() + 7) // 8, "big")
                                        ).rstrip(b"=").decode()
    return {"kty": "RSA", "kid": "idp", "n": b64(n), "e": b64(e)}, n, d


def _rs256(claims, n, d, kid="idp"):
    import base64

    from omnia_amd.ee.license import rs256_sign

    def enc(b):
        return base64.urlsafe_b64encode(b).rstrip(b"=").decode()
    h = enc(json.dumps({"alg": "RS256", "kid": kid}).encode())
    p = enc(json.dumps(claims).encode())
    return f"{h}.{p}.{enc(rs256_sign(f'{h}.{p}'.encode(), n, d))}"


def test_dashboard_views_and_oidc_gate():
    import time

    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.operator.apiserver import build_app as api_app
    from omnia_amd.operator.apistore import APIStore
    from omnia_amd.operator.dashboard import build_app

    pub, n, d = _rsa_jwk()

    async def run():
        store = APIStore()
        store.apply({"apiVersion": crds.API_VERSION, "kind": "ArenaJob",
                     "metadata": {"name": "lt", "namespace": "default"},
                     "spec": {"type": "loadtest", "sourceRef": {"name": "s"}}})
        api = TestServer(api_app(store))
        await api.start_server()
        side = web.Application()
        side.router.add_get("/api/v1/sessions/{id}/messages", lambda r: web.json_response(
            {"messages": [{"role": "user", "content": "hi " + r.match_info["id"]}]}))
        side.router.add_get("/api/v1/privacy/preferences/{u}/consent", lambda r: web.json_response(
            {"userId": r.match_info["u"], "grants": ["analytics"]}))
        sides = TestServer(side)
        await sides.start_server()
        sbase = str(sides.make_url("")).rstrip("/")
        dash = TestClient(TestServer(build_app(
            str(api.make_url("")).rstrip("/"), session_api=sbase, privacy_api=sbase,
            oidc={"jwks": {"keys": [pub]}, "issuer": "https://idp", "audience": "dash"})))
        await dash.start_server()
        try:
            assert (await dash.get("/")).status == 200  # the page itself is public
            assert (await dash.get("/api/arena/jobs")).status == 401
            bad = _rs256({"iss": "https://other", "aud": "dash", "exp": time.time() + 60}, n, d)
            r = await dash.get("/api/arena/jobs", headers={"Authorization": f"Bearer {bad}"})
            assert r.status == 401
            tok = _rs256({"iss": "https://idp", "aud": "dash", "sub": "u1",
                          "exp": time.time() + 60}, n, d)
            h = {"Authorization": f"Bearer {tok}"}
            jobs = (await (await dash.get("/api/arena/jobs", headers=h)).json())["jobs"]
            assert [(j["name"], j["type"]) for j in jobs] == [("lt", "loadtest")]
            m = await (await dash.get("/api/sessions/s%201/messages", headers=h)).json()
            assert m["messages"][0]["content"] == "hi s 1"
            c = await (await dash.get("/api/consent/alice", headers=h)).json()
            assert c == {"userId": "alice", "grants": ["analytics"]}
        finally:
            await dash.close()
            await api.close()
            await sides.close()

    asyncio.run(run())


def test_dashboard_management_writes():
    """--allow-writes: create from YAML (admission applies), scale an agent,
    cancel an arena job, delete; read-only by default."""
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.operator.apiserver import build_app as api_app
    from omnia_amd.operator.apistore import APIStore
    from omnia_amd.operator.dashboard import build_app

    prov = ("apiVersion: %s\nkind: Provider\nmetadata: {name: p1, namespace: default}\n"
            "spec: {type: mock}\n" % crds.API_VERSION)

    async def run():
        store = APIStore()
        store.objs[store.key("AgentRuntime", "default", "a1")] = {
            "apiVersion": crds.API_VERSION, "kind": "AgentRuntime",
            "metadata": {"name": "a1", "namespace": "default", "generation": 1,
                         "resourceVersion": "1", "uid": "u1"},
            "spec": {"promptPackRef": {"name": "pack"}, "facades": [{"type": "websocket"}],
                     "runtime": {"replicas": 1}}}
        api = TestServer(api_app(store))
        await api.start_server()
        url = str(api.make_url("")).rstrip("/")
        ro = TestClient(TestServer(build_app(url)))
        rw = TestClient(TestServer(build_app(url, allow_writes=True, insecure_dev_writes=True)))
        await ro.start_server()
        await rw.start_server()
        Y = {"Content-Type": "application/yaml"}
        try:
            assert (await ro.post("/api/resources/providers", data=prov, headers=Y)).status == 403
            # CSRF guards: a text/plain (form-simple) body and a foreign Origin are refused
            assert (await rw.post("/api/resources/providers", data=prov)).status == 415
            r = await rw.post("/api/resources/providers", data=prov,
                              headers={**Y, "Origin": "https://evil.example"})
            assert r.status == 403 and store.try_get("Provider", "p1", "default") is None
            r = await rw.post("/api/resources/providers", data=prov, headers=Y)
            assert r.status in (200, 201), await r.text()
            assert store.try_get("Provider", "p1", "default") is not None
            bad = prov.replace("type: mock", "type: nosuchtype")
            r = await rw.post("/api/resources/providers", data=bad.replace("p1", "p2"), headers=Y)
            assert r.status >= 400  # the API server's admission rejected it
            assert (await rw.post("/api/resources/providers", data="- a\n- b",
                                  headers=Y)).status == 400
            r = await rw.post("/api/agents/default/a1/scale", json={"replicas": 3})
            assert r.status == 200, await r.text()
            assert store.get("AgentRuntime", "a1", "default")["spec"]["runtime"]["replicas"] == 3
            assert (await rw.post("/api/agents/default/a1/scale", json={"replicas": -1})
                    ).status == 400
            r = await rw.delete("/api/resources/providers/default/p1")
            assert r.status == 200 and store.try_get("Provider", "p1", "default") is None
        finally:
            await ro.close()
            await rw.close()
            await api.close()

    asyncio.run(run())


def test_dashboard_writes_need_oidc_and_a_write_group():
    import time

    import pytest
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.operator.apiserver import build_app as api_app
    from omnia_amd.operator.apistore import APIStore
    from omnia_amd.operator.dashboard import build_app

    with pytest.raises(ValueError, match="OIDC"):
        build_app("http://127.0.0.1:1", allow_writes=True)
    pub, n, d = _rsa_jwk()
    prov = ("apiVersion: %s\nkind: Provider\nmetadata: {name: p9, namespace: default}\n"
            "spec: {type: mock}\n" % crds.API_VERSION)

    async def run():
        store = APIStore()
        api = TestServer(api_app(store))
        await api.start_server()
        dash = TestClient(TestServer(build_app(
            str(api.make_url("")).rstrip("/"), allow_writes=True,
            oidc={"jwks": {"keys": [pub]}, "issuer": "https://idp", "audience": "dash",
                  "write_groups": ["ops"]})))
        await dash.start_server()
        try:
            base = {"iss": "https://idp", "aud": "dash", "sub": "u1", "exp": time.time() + 60}
            reader = _rs256(base, n, d)
            writer = _rs256({**base, "groups": ["dev", "ops"]}, n, d)
            Y = {"Content-Type": "application/yaml"}
            r = await dash.post("/api/resources/providers", data=prov,
                                headers={**Y, "Authorization": f"Bearer {reader}"})
            assert r.status == 403 and "write group" in (await r.json())["error"]
            assert store.try_get("Provider", "p9", "default") is None
            r = await dash.post("/api/resources/providers", data=prov,
                                headers={**Y, "Authorization": f"Bearer {writer}"})
            assert r.status in (200, 201), await r.text()
            assert store.try_get("Provider", "p9", "default") is not None
        finally:
            await dash.close()
            await api.close()

    asyncio.run(run())
