"""End to end on the GPU: ``omnia serve -f examples/llama3-8b-agent/manifests.yaml``
(the real CLI as its own process tree: operator + apiserver + launcher, the
agent pod as facade + runtime + engine-core processes on cuda:0) reconciles the
manifests, the AgentRuntime reaches Running, and a WebSocket turn streams
tokens from Llama-3-8B (random init) -- the reference's ``kubectl apply`` ->
running agent -> WS turn path (SURVEY §3.1 + §3.2) on one MI355X."""
import asyncio
import os
import signal
import socket
import subprocess
import sys
import time

import aiohttp
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AGENT = os.path.join(ROOT, "examples", "llama3-8b-agent", "manifests.yaml")
API = "/apis/omnia.altairalabs.ai/v1alpha1/namespaces/default"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_omnia_serve_llama3_8b_streams_a_websocket_turn(tmp_path):
    from omnia_amd.ee.arena.fleet import FleetSession

    port = _free_port()
    log = open(tmp_path / "serve.log", "w")
    env = {**os.environ, "PYTHONPATH": ROOT}
    proc = subprocess.Popen([sys.executable, "-m", "omnia_amd.cli", "serve", "--port", str(port),
                             "-f", AGENT], cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                            start_new_session=True)
    base = f"http://127.0.0.1:{port}"

    async def go():
        async with aiohttp.ClientSession() as s:
            ar, ep = {}, None
            deadline = time.time() + 240
            while time.time() < deadline:
                assert proc.poll() is None, open(tmp_path / "serve.log").read()[-3000:]
                try:
                    r = await s.get(base + API + "/agentruntimes/assistant")
                    if r.status == 200:
                        ar = await r.json()
                        r2 = await s.get(base + "/api/v1/namespaces/default/services/assistant")
                        if r2.status == 200:
                            ep = ((await r2.json()).get("status") or {}).get("endpoint")
                        if (ar.get("status") or {}).get("phase") == "Running" and ep:
                            break
                except aiohttp.ClientError:
                    pass
                await asyncio.sleep(1.0)
            st = ar.get("status") or {}
            assert st.get("phase") == "Running" and ep, (st, open(tmp_path / "serve.log").read()
                                                          [-3000:])
            conds = {c["type"]: c["status"] for c in st.get("conditions", [])}
            assert conds.get("PromptPackReady") == "True" and conds.get("ProviderReady") == "True"
            async with FleetSession(f"ws://{ep}/ws", timeout_s=120) as fs:
                t1 = await fs.turn("Hello! What can you do?")
                t2 = await fs.turn("And the weather in Lisbon?")
            return st, t1, t2

    import psutil

    pods = []
    try:
        st, t1, t2 = asyncio.run(go())
        pods = psutil.Process(proc.pid).children(recursive=True)  # pod process trees
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(10)
        log.close()
    # SIGTERM stopped every pod (they run in their own sessions: an abrupt exit of
    # the operator would orphan engine-cores holding most of the GPU's memory)
    gone, alive = psutil.wait_procs(pods, timeout=20)
    assert not alive, [p.cmdline()[:4] for p in alive]
    for t in (t1, t2):
        assert t["usage"].get("output_tokens", 0) > 0 and t["usage"].get("input_tokens", 0) > 0
        assert len(t["chunk_times_s"]) >= 1
    # the second turn re-used the session's resident KV (multi-turn on one engine)
    assert t2["usage"]["input_tokens"] > t1["usage"]["input_tokens"]
    print("serve e2e:", {"ttft_ms": [round(t1["ttft_ms"]), round(t2["ttft_ms"])],
                         "out": [t1["usage"]["output_tokens"], t2["usage"]["output_tokens"]],
                         "phase": st["phase"]})
