"""omnia doctor: end-to-end diagnostics (``cmd/doctor``, ``internal/doctor/checks``).

Each check returns a :class:`Result` (pass / fail / skip + detail + duration):

* agent       -- WebSocket round trip through a facade (connected -> message -> done)
* sessions    -- session-api create / append / read back / delete
* memory      -- memory-api save + retrieve ("smoke-42" marker, like the reference's
                 ``memory__remember`` probe) + delete
* crds        -- every CRD kind renders a valid CustomResourceDefinition
* redis       -- PING over RESP
* gpu         -- the gfx950 kernel extension loads and a device is visible; the
                 in-node engine replaces the reference's Ollama probe
* privacy     -- privacy-api health + consent read
* observability -- /metrics of a service exposes omnia_* series

``python -m omnia_amd.doctor --facade ws://host:8080/ws --session-api http://...``
(exit status 1 when any check fails; ``--json`` for machine output).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time
import uuid
from dataclasses import asdict, dataclass

PASS, FAIL, SKIP = "pass", "fail", "skip"


@dataclass
class Result:
    name: str
    status: str
    detail: str = ""
    duration_ms: float = 0.0


async def _timed(name, coro):
    t0 = time.perf_counter()
    try:
        status, detail = await coro
    except Exception as e:  # noqa: BLE001
        status, detail = FAIL, f"{type(e).__name__}: {e}"
    return Result(name, status, detail, (time.perf_counter() - t0) * 1e3)


async def check_agent(url: str, token: str = ""):
    import aiohttp

    if not url:
        return SKIP, "no facade URL"
    u = url.replace("ws://", "http://").replace("wss://", "https://")
    if token:
        u += ("&" if "?" in u else "?") + f"token={token}"
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(u, timeout=10) as ws:
            hello = await ws.receive_json(timeout=10)
            if hello.get("type") != "connected":
                return FAIL, f"unexpected handshake {hello.get('type')}"
            await ws.send_json({"type": "message", "content": "doctor ping"})
            while True:
                m = await ws.receive_json(timeout=60)
                if m.get("type") == "done":
                    return PASS, f"turn ok ({len(m.get('content', ''))} chars)"
                if m.get("type") == "error":
                    return FAIL, json.dumps(m.get("error"))


async def check_sessions(base: str):
    import aiohttp

    if not base:
        return SKIP, "no session-api URL"
    sid = "doctor-" + uuid.uuid4().hex[:8]
    async with aiohttp.ClientSession() as s:
        r = await s.post(f"{base}/api/v1/sessions", json={"id": sid, "namespace": "doctor"})
        if r.status >= 300:
            return FAIL, f"create HTTP {r.status}"
        await s.post(f"{base}/api/v1/sessions/{sid}/messages",
                     json={"role": "user", "content": "doctor"})
        msgs = await (await s.get(f"{base}/api/v1/sessions/{sid}/messages")).json()
        n = len(msgs.get("messages", []))
        await s.delete(f"{base}/api/v1/sessions/{sid}")
        return (PASS, "create/append/read/delete ok") if n == 1 else (FAIL, f"{n} messages")


async def check_memory(base: str, workspace: str = "doctor"):
    import aiohttp

    if not base:
        return SKIP, "no memory-api URL"
    user = "doctor-" + uuid.uuid4().hex[:6]
    scope = {"workspace_id": workspace, "virtual_user_id": user}
    async with aiohttp.ClientSession() as s:
        r = await s.post(f"{base}/api/v1/memories", json={"content": "smoke-42 marker",
                                                          "scope": scope})
        if r.status >= 300:
            return FAIL, f"save HTTP {r.status}"
        got = await (await s.post(f"{base}/api/v1/memories/retrieve", json={
            "workspace_id": workspace, "virtual_user_id": user, "query": "smoke-42"})).json()
        await s.delete(f"{base}/api/v1/memories", params={"workspace": workspace,
                                                          "virtual_user_id": user})
        ok = any("smoke-42" in m.get("content", "") for m in got.get("memories", []))
        return (PASS, "smoke-42 persisted and recalled") if ok else (FAIL, "not recalled")


async def check_crds():
    from ..api import crds

    bad = []
    for k in crds.KINDS.values():
        m = crds.crd_manifest(k)
        if m.get("kind") != "CustomResourceDefinition":
            bad.append(k.kind)
    return (PASS, f"{len(crds.KINDS)} kinds") if not bad else (FAIL, f"invalid: {bad}")


async def check_redis(url: str):
    if not url:
        return SKIP, "no redis URL"
    from ..utils.resp import RedisClient

    r = RedisClient(url)
    try:
        pong = await r.ping()
    finally:
        r.close()
    return (PASS, "PONG") if pong in (b"PONG", "PONG", True) else (FAIL, repr(pong))


async def check_gpu():
    import torch

    if not torch.cuda.is_available():
        return SKIP, "no GPU visible"
    from .. import ops

    k = ops.kernels()
    name = torch.cuda.get_device_name(0)
    free, total = torch.cuda.mem_get_info()
    return PASS, f"{name}, kernels arch {k.arch}, {free / 2**30:.0f}/{total / 2**30:.0f} GiB free"


async def check_privacy(base: str):
    import aiohttp

    if not base:
        return SKIP, "no privacy-api URL"
    async with aiohttp.ClientSession() as s:
        if (await s.get(f"{base}/healthz")).status != 200:
            return FAIL, "unhealthy"
        c = await (await s.get(f"{base}/api/v1/privacy/preferences/doctor/consent")).json()
        return PASS, f"{len(c.get('denied', []))} categories need explicit grant"


async def check_metrics(url: str):
    import aiohttp

    if not url:
        return SKIP, "no metrics URL"
    async with aiohttp.ClientSession() as s:
        body = await (await s.get(url)).text()
    n = sum(1 for line in body.splitlines() if line.startswith("omnia_"))
    return (PASS, f"{n} omnia_* samples") if n else (FAIL, "no omnia_* series")


async def run_checks(a) -> list[Result]:
    checks = [("crds", check_crds()), ("gpu", check_gpu()),
              ("agent", check_agent(a.facade, a.token)),
              ("sessions", check_sessions(a.session_api)),
              ("memory", check_memory(a.memory_api)), ("redis", check_redis(a.redis)),
              ("privacy", check_privacy(a.privacy_api)),
              ("observability", check_metrics(a.metrics))]
    return [await _timed(n, c) for n, c in checks]


def main(argv=None):
    ap = argparse.ArgumentParser(prog="omnia doctor")
    ap.add_argument("--facade", default="")
    ap.add_argument("--token", default="")
    ap.add_argument("--session-api", default="")
    ap.add_argument("--memory-api", default="")
    ap.add_argument("--privacy-api", default="")
    ap.add_argument("--redis", default="")
    ap.add_argument("--metrics", default="")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    res = asyncio.run(run_checks(a))
    if a.json:
        print(json.dumps([asdict(r) for r in res], indent=1))
    else:
        for r in res:
            print(f"[{r.status.upper():4}] {r.name:<14} {r.detail} ({r.duration_ms:.0f} ms)")
    if any(r.status == FAIL for r in res):
        sys.exit(1)
    return res
