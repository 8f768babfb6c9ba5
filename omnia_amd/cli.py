"""``omnia`` command line.

  omnia serve [--port 8090] [-f manifests.yaml ...]   single-node operator: API server +
                                                      controllers + local launcher
  omnia apply -f FILE [--server URL]                  create/update objects
  omnia get KIND [NAME] [-n NS] [-o yaml|json|wide]   list/get with printer columns
  omnia delete KIND NAME [-n NS]
  omnia crds                                          emit CustomResourceDefinitions
  omnia conformance --target HOST:PORT                runtime conformance suite
  omnia doctor [--facade ws://...]                    diagnostics
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

import yaml


def load_manifests(paths: list[str]) -> list[dict]:
    docs = []
    for p in paths:
        text = sys.stdin.read() if p == "-" else open(p).read()
        for d in yaml.safe_load_all(text):
            if not d:
                continue
            if d.get("kind", "").endswith("List") and "items" in d:
                docs.extend(d["items"])
            else:
                docs.append(d)
    return docs


def _jsonpath(obj, path: str):
    cur = obj
    for part in path.strip(".").split("."):
        if isinstance(cur, dict):
            cur = cur.get(part)
        else:
            return None
    return cur


def _http(method, url, body=None):
    import urllib.request

    data = json.dumps(body).encode() if body is not None else None
    req = urllib.request.Request(url, data=data, method=method,
                                 headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            return r.status, json.loads(r.read() or b"null")
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read() or b"null")


def _path(kind: str, ns: str | None, name: str | None = None) -> str:
    from .api import crds
    from .operator.apiserver import CORE

    if kind in crds.KINDS:
        k = crds.KINDS[kind]
        base = f"/apis/{crds.GROUP}/{crds.VERSION}"
        p = f"{base}/namespaces/{ns or 'default'}/{k.plural}" if k.scope == "Namespaced" \
            else f"{base}/{k.plural}"
    else:
        plural = next(pl for pl, kk in CORE.items() if kk == kind)
        p = f"/api/v1/namespaces/{ns or 'default'}/{plural}"
    return p + (f"/{name}" if name else "")


def cmd_apply(a):
    for d in load_manifests(a.filename):
        kind = d["kind"]
        ns = d.get("metadata", {}).get("namespace") or a.namespace
        st, out = _http("PATCH", a.server + _path(kind, ns, d["metadata"]["name"]), d)
        if st == 404:
            st, out = _http("POST", a.server + _path(kind, ns), d)
        verb = "configured" if st == 200 else "created" if st == 201 else f"error {st}"
        print(f"{kind.lower()}/{d['metadata']['name']} {verb}"
              + ("" if st < 300 else f": {out.get('message')}"))


def cmd_get(a):
    from .api import crds

    kind = crds.resolve_kind(a.kind) if a.kind.lower() not in ("deployment", "deployments",
                                                                "service", "services",
                                                                "configmap", "configmaps") \
        else {"deployment": "Deployment", "deployments": "Deployment", "service": "Service",
              "services": "Service", "configmap": "ConfigMap",
              "configmaps": "ConfigMap"}[a.kind.lower()]
    st, out = _http("GET", a.server + _path(kind, a.namespace, a.name))
    if st >= 300:
        print(out.get("message"), file=sys.stderr)
        sys.exit(1)
    items = [out] if a.name else out["items"]
    if a.output in ("yaml", "json"):
        print(yaml.safe_dump(items if not a.name else out) if a.output == "yaml"
              else json.dumps(items if not a.name else out, indent=2))
        return
    cols = [("NAME", ".metadata.name")]
    if kind in crds.KINDS:
        cols += [(n.upper(), p) for n, p in crds.KINDS[kind].printer]
    rows = [[str(_jsonpath(o, p) if _jsonpath(o, p) is not None else "") for _, p in cols]
            for o in items]
    widths = [max([len(c[0])] + [len(r[i]) for r in rows]) for i, c in enumerate(cols)]
    print("   ".join(c[0].ljust(w) for c, w in zip(cols, widths)))
    for r in rows:
        print("   ".join(v.ljust(w) for v, w in zip(r, widths)))


def cmd_delete(a):
    from .api import crds

    kind = crds.resolve_kind(a.kind)
    st, out = _http("DELETE", a.server + _path(kind, a.namespace, a.name))
    ok = bool(out) and (out.get("deleted") or out.get("status") == "Success")
    print(f"{kind.lower()}/{a.name} {'deleted' if ok else 'not found'}")


def cmd_crds(a):
    from .api import crds

    print(yaml.safe_dump_all([crds.crd_manifest(k) for k in crds.KINDS.values()],
                             sort_keys=False))


async def serve(port: int, manifests: list[str], engine: bool, host: str = "127.0.0.1",
                enterprise: bool = False, leader_elect: bool = True):
    from aiohttp import web

    from .operator.apiserver import build_app
    from .operator.launcher import LocalLauncher
    from .operator.manager import Manager, new_store

    store = new_store()
    if enterprise:
        from .operator.manager import license_validator_for, set_license_validator

        set_license_validator(license_validator_for(
            store, os.environ.get("OMNIA_LICENSE_PUBLIC_KEY") or None))
    gpus = None
    try:
        import torch

        gpus = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        pass
    mgr = Manager(store, gpu_count=gpus, leader_elect=leader_elect)
    await mgr.start()
    factory = None
    if engine:
        from .runtime.app import shared_engine

        factory = shared_engine
    # every replica is a pod of OS processes with its own GPU(s)
    launcher = LocalLauncher(store, engine_factory=factory, mode="process",
                             gpu_count=gpus or 0)
    launcher.start()
    for d in load_manifests(manifests):
        try:
            store.apply(d)
        except Exception as e:  # noqa: BLE001
            print(f"apply {d.get('kind')}/{d.get('metadata', {}).get('name')}: {e}",
                  file=sys.stderr)
    runner = web.AppRunner(build_app(store))
    await runner.setup()
    await web.TCPSite(runner, host, port).start()
    print(f"omnia single-node operator on http://{host}:{port} (gpus={gpus})", flush=True)
    # SIGTERM / SIGINT: stop every pod before exiting -- pods run in their own
    # sessions, so an abrupt exit would orphan them (engines holding GPU memory)
    import signal

    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    await stop.wait()
    print("omnia serve: stopping pods", flush=True)
    try:
        await launcher.stop()
    finally:
        await mgr.stop()
        await runner.cleanup()


async def run_operator(kubeconfig: str | None, in_cluster: bool, leader_elect: bool,
                       namespace: str, enterprise: bool, gpus: int | None) -> None:
    """Real-cluster mode: the same reconcilers against a kube-apiserver
    (``cmd/main.go:400-660``); pods are run by the kubelet, not a launcher."""
    from .operator.kube import KubeClient, KubeConfig
    from .operator.manager import Manager, license_validator_for, set_license_validator

    cfg = KubeConfig.in_cluster() if in_cluster else (
        KubeConfig.from_kubeconfig(kubeconfig) if kubeconfig else KubeConfig.auto())
    client = KubeClient(cfg)
    if enterprise:
        set_license_validator(license_validator_for(
            client, os.environ.get("OMNIA_LICENSE_PUBLIC_KEY") or None))
    mgr = Manager(client, gpu_count=gpus, leader_elect=leader_elect, namespace=namespace)
    await mgr.start()
    print(f"omnia operator reconciling against {cfg.server} (leader={mgr.is_leader})",
          flush=True)
    try:
        await asyncio.gather(*mgr.tasks)
    finally:
        await mgr.stop()
        client.close()


def main(argv=None):
    args = list(sys.argv[1:] if argv is None else argv)
    if args[:1] == ["doctor"]:  # its own parser (omnia_amd/doctor)
        from .doctor import main as dmain

        return dmain(args[1:])
    ap = argparse.ArgumentParser("omnia")
    ap.add_argument("--server", default=os.environ.get("OMNIA_SERVER", "http://127.0.0.1:8090"))
    sp = ap.add_subparsers(dest="cmd", required=True)
    p = sp.add_parser("serve")
    p.add_argument("--port", type=int, default=8090)
    p.add_argument("-f", "--filename", action="append", default=[])
    p.add_argument("--no-engine", action="store_true")
    p.add_argument("--leader-elect", action="store_true",
                   help="cluster mode: run reconcilers only while holding the Lease")
    p.add_argument("--enterprise", action="store_true", help="also run the EE controllers")
    p = sp.add_parser("operator", help="run the controllers against a real kube-apiserver")
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--in-cluster", action="store_true")
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--namespace", default=os.environ.get("OMNIA_NAMESPACE", "omnia-system"))
    p.add_argument("--enterprise", action="store_true")
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs per node for the capability gate (default: unchecked)")
    p = sp.add_parser("chart", help="write the Helm chart + kustomize bases (deploy/)")
    p.add_argument("--out", default="deploy")
    p = sp.add_parser("apply")
    p.add_argument("-f", "--filename", action="append", required=True)
    p.add_argument("-n", "--namespace", default="default")
    p = sp.add_parser("get")
    p.add_argument("kind")
    p.add_argument("name", nargs="?")
    p.add_argument("-n", "--namespace", default="default")
    p.add_argument("-o", "--output", default="table")
    p = sp.add_parser("delete")
    p.add_argument("kind")
    p.add_argument("name")
    p.add_argument("-n", "--namespace", default="default")
    sp.add_parser("crds")
    p = sp.add_parser("conformance")
    p.add_argument("--target", default="127.0.0.1:9000")
    sp.add_parser("doctor", help="diagnostics: omnia doctor --run-once --facade ... | "
                                 "serve the doctor UI (see omnia doctor -h)")
    a = ap.parse_args(argv)
    if a.cmd == "serve":
        asyncio.run(serve(a.port, a.filename, not a.no_engine, enterprise=a.enterprise,
                          leader_elect=True))
    elif a.cmd == "operator":
        asyncio.run(run_operator(a.kubeconfig, a.in_cluster, a.leader_elect, a.namespace,
                                 a.enterprise, a.gpus))
    elif a.cmd == "apply":
        cmd_apply(a)
    elif a.cmd == "get":
        cmd_get(a)
    elif a.cmd == "delete":
        cmd_delete(a)
    elif a.cmd == "crds":
        cmd_crds(a)
    elif a.cmd == "chart":
        from .operator import chart

        for rel in chart.write(a.out):
            print(f"{a.out}/{rel}")
    elif a.cmd == "conformance":
        from .runtime import conformance

        conformance.main(["--target", a.target])


if __name__ == "__main__":
    main()
