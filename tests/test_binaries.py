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
