"""omnia doctor: end-to-end diagnostics of a deployment (``cmd/doctor``,
``internal/doctor``).

Two modes, like the reference binary:

* ``--run-once`` runs every check, prints the run as JSON (or a table with
  ``--table``) and, with ``--exit-code``, exits 1 when a check failed;
* otherwise it serves the doctor UI + API on ``--addr`` (``server.py``: SSE
  stream of a run, trigger, latest result, healthz).

Checks live in ``checks.py``; ``runner.py`` runs categories concurrently and the
categories that share state (workspace -> agent -> sessions -> memory ->
privacy) in one sequential group.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

from .checks import (AgentChecker, CRDChecker, MemoryChecker, PrivacyChecker, SessionChecker,
                     State, WorkspaceChecker, gpu_check, metrics_check, probe_check,
                     redis_check)
from .result import FAIL, PASS, SKIP, RunResult, TestResult
from .runner import Check, Runner


def build_runner(a) -> Runner:
    """A fresh runner (and shared state) for one run from parsed options."""
    st = State()
    st.session_url = (a.session_api_url or "").rstrip("/")
    st.memory_url = (a.memory_api_url or "").rstrip("/")
    st.workspace = a.workspace or ""
    r = Runner()
    r.register(*CRDChecker(a.operator_url, a.namespace).checks())
    r.register(*WorkspaceChecker(a.operator_url, a.namespace, st, a.service_group).checks())
    # infrastructure probes run after the workspace resolved the service URLs
    r.register(probe_check("SessionAPI", lambda: st.session_url, suffix="Healthy"),
               probe_check("MemoryAPI", lambda: st.memory_url, suffix="Healthy"),
               probe_check("PrivacyAPI", a.privacy_api_url), probe_check("OperatorAPI",
                                                                          a.operator_url))
    r.register(redis_check(a.redis_url), gpu_check())
    headers = dict(h.split(":", 1) for h in a.header) if a.header else {}
    if a.mgmt_signing_key:
        # the reference doctor dials the agent's management-plane twin (18080)
        # with a dashboard-minted JWT: mint one from the dashboard's signing key
        from ..facade.auth import jwk_thumbprint, mint_mgmt_token
        from ..utils.rsa import load_private_key

        with open(a.mgmt_signing_key) as f:
            key = load_private_key(f.read())
        headers["Authorization"] = "Bearer " + mint_mgmt_token(
            key, a.mgmt_kid or jwk_thumbprint(key), "omnia-doctor", agent=a.agent, workspace=a.workspace or "")
    r.register(*AgentChecker(a.facade, st, a.token, {k.strip(): v.strip()
                                                     for k, v in headers.items()}).checks())
    r.register(*SessionChecker(st, a.namespace).checks())
    r.register(*MemoryChecker(st, a.workspace).checks())
    r.register(*PrivacyChecker(a.privacy_api_url or "", st, a.workspace).checks())
    for spec in a.metrics or []:
        name, _, url = spec.partition("=")
        prefix = None
        if "@" in name:
            name, prefix = name.split("@", 1)
        r.register(metrics_check(name, url, prefix))
    # metrics are read last, after the probes generated traffic
    r.sequential_group("flow", "Workspace", "Infrastructure", "Agent", "Sessions", "Memory",
                       "Privacy", "Observability")
    return r


def parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="omnia doctor")
    env = os.environ.get
    ap.add_argument("--addr", default="127.0.0.1:8080", help="serve the doctor UI/API here")
    ap.add_argument("--port", type=int, default=0, help="serve on 0.0.0.0:PORT (chart)")
    ap.add_argument("--run-once", action="store_true", help="run once, print, exit")
    ap.add_argument("--exit-code", action="store_true", help="with --run-once: exit 1 on fail")
    ap.add_argument("--table", action="store_true", help="with --run-once: a table, not JSON")
    ap.add_argument("--facade", default=env("OMNIA_DOCTOR_FACADE", ""), help="agent WebSocket URL (ws://host:port/ws)")
    ap.add_argument("--token", default="")
    ap.add_argument("--mgmt-signing-key", default=env("OMNIA_DOCTOR_MGMT_KEY", ""),
                    help="dashboard PEM key: mint a management-plane JWT and dial the "
                         "agent's twin listener (--facade ws://agent:18080/ws)")
    ap.add_argument("--mgmt-kid", default="",
                    help="kid of the signing key (default: its RFC 7638 thumbprint, as the "
                         "dashboard publishes it)")
    ap.add_argument("--agent", default="", help="agent name claimed in the mgmt-plane token")
    ap.add_argument("--header", action="append", default=[],
                    help="extra WebSocket header 'Name: value' (e.g. x-user-id behind an edge)")
    ap.add_argument("--namespace", default="default", help="agent namespace")
    ap.add_argument("--workspace", default="")
    ap.add_argument("--service-group", default="default")
    ap.add_argument("--session-api-url", "--session-api", default=env("OMNIA_SESSION_API_URL", ""))
    ap.add_argument("--memory-api-url", "--memory-api", default=env("OMNIA_MEMORY_API_URL", ""))
    ap.add_argument("--privacy-api-url", "--privacy-api", default=env("OMNIA_PRIVACY_API_URL", ""))
    ap.add_argument("--operator-url", default=env("OMNIA_OPERATOR_URL", ""), help="operator API server (omnia serve)")
    ap.add_argument("--redis-url", "--redis", default=env("REDIS_URL", ""))
    ap.add_argument("--metrics", action="append", default=[],
                    help="NAME[@prefix]=URL of a /metrics endpoint (repeatable)")
    return ap


def print_table(run: RunResult) -> None:
    for c in run.categories:
        for t in c.tests:
            extra = t.detail or t.error
            print(f"[{t.status.upper():4}] {c.name:<14} {t.name:<28} {extra} "
                  f"({t.duration_ms:.0f} ms)")
    s = run.summary
    print(f"{s['passed']} passed, {s['failed']} failed, {s['skipped']} skipped")


def main(argv=None):
    a = parser().parse_args(argv)
    if a.run_once:
        run = asyncio.run(build_runner(a).run())
        if a.table:
            print_table(run)
        else:
            print(json.dumps(run.to_json(), indent=1))
        if a.exit_code and run.status == FAIL:
            sys.exit(1)
        return run
    from aiohttp import web

    from .server import build_app

    host, _, port = a.addr.rpartition(":")
    if a.port:
        host, port = "0.0.0.0", a.port
    web.run_app(build_app(lambda: build_runner(a)), host=host or "0.0.0.0", port=int(port))


__all__ = ["Runner", "Check", "RunResult", "TestResult", "build_runner", "main", "PASS",
           "FAIL", "SKIP"]
