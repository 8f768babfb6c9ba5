"""Helm chart / kustomize bases (C48) and the dashboard backend (C47).

* deploy/ is exactly what omnia_amd.operator.chart generates (no drift);
* every ``.Values.x.y`` a template references exists in values.yaml;
* all CRD kinds are shipped, static YAML parses, and every python entrypoint a
  template runs is importable;
* the dashboard proxies the operator REST API."""
import asyncio
import glob
import importlib
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
