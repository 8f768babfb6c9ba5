"""Process-level e2e (config 1): ``python -m omnia_amd.runtime`` (mock provider)
and ``python -m omnia_amd.facade`` as separate OS processes talking gRPC, a
WebSocket client behind a shared-token auth chain, then SIGTERM drain."""
import asyncio
import os
import signal
import socket
import subprocess
import sys
import time

import aiohttp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait_port(port, timeout=60):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            socket.create_connection(("127.0.0.1", port), 0.5).close()
            return True
        except OSError:
            time.sleep(0.2)
    return False


def test_runtime_and_facade_processes():
    gport, hport, fport = _port(), _port(), _port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMNIA_AGENT_NAME="bin-agent",
               OMNIA_NAMESPACE="e2e", OMNIA_GRPC_PORT=str(gport), OMNIA_HEALTH_PORT=str(hport),
               OMNIA_PROVIDER_TYPE="mock", OMNIA_PROMPTPACK_PATH="/nonexistent",
               OMNIA_RUNTIME_ADDRESS=f"127.0.0.1:{gport}", OMNIA_FACADE_PORT=str(fport),
               OMNIA_AUTH_SHARED_TOKEN="s3cret", LOG_LEVEL="WARNING")
    rt = subprocess.Popen([sys.executable, "-m", "omnia_amd.runtime"], env=env, cwd=ROOT)
    fa = subprocess.Popen([sys.executable, "-m", "omnia_amd.facade"], env=env, cwd=ROOT)
    try:
        assert _wait_port(fport), "facade did not start"

        async def go():
            async with aiohttp.ClientSession() as s:
                r = await s.get(f"http://127.0.0.1:{fport}/ws")
                assert r.status in (401, 403)
                async with s.ws_connect(f"http://127.0.0.1:{fport}/ws?token=s3cret") as ws:
                    hello = await ws.receive_json(timeout=30)
                    assert hello["type"] == "connected"
                    await ws.send_json({"type": "message", "content": "hello"})
                    while True:
                        m = await ws.receive_json(timeout=30)
                        if m["type"] in ("done", "error"):
                            return m

        done = asyncio.run(go())
        assert done["type"] == "done" and done["content"]
    finally:
        for p in (fa, rt):
            p.send_signal(signal.SIGTERM)
        for p in (fa, rt):
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    assert fa.returncode == 0 and rt.returncode == 0


def test_doctor_against_live_services():
    """Doctor probes a live facade + session-api + memory-api + metrics."""
    from aiohttp import web

    from omnia_amd.doctor import FAIL, PASS, SKIP, run_checks
    from omnia_amd.memory.api import build_app as memory_app
    from omnia_amd.memory.service import MemoryService
    from omnia_amd.session.api import build_app as session_app
    from omnia_amd.session.store import TieredSessionService

    async def serve(app):
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"

    class A:
        token = ""
        redis = ""
        privacy_api = ""

    async def go():
        from omnia_amd.facade.runtime_client import InProcessRuntimeClient
        from omnia_amd.facade.server import FacadeConfig, FacadeServer
        from omnia_amd.runtime.app import build_runtime
        from omnia_amd.runtime.config import RuntimeConfig

        svc = await build_runtime(RuntimeConfig(provider={"type": "mock"}))
        fac = FacadeServer(FacadeConfig(), runtime_client=InProcessRuntimeClient(svc))
        port = await fac.start("127.0.0.1", 0)
        r1, s_url = await serve(session_app(TieredSessionService()))
        r2, m_url = await serve(memory_app(MemoryService()))
        a = A()
        a.facade, a.session_api, a.memory_api = f"ws://127.0.0.1:{port}/ws", s_url, m_url
        a.metrics = f"http://127.0.0.1:{port}/metrics"
        try:
            return {r.name: r for r in await run_checks(a)}
        finally:
            await fac.stop()
            await r1.cleanup()
            await r2.cleanup()

    res = asyncio.run(go())
    for n in ("crds", "agent", "sessions", "memory", "observability"):
        assert res[n].status == PASS, res[n]
    assert res["redis"].status == SKIP and res["gpu"].status in (SKIP, PASS)
    assert all(r.status != FAIL for r in res.values())
