"""``omnia serve`` (the CLI as its own process tree) on the CPU: the echo agent's
pod processes come up, and SIGTERM to the operator stops every pod before it
exits (pods run in their own sessions; an abrupt exit would orphan them)."""
import os
import signal
import socket
import subprocess
import sys
import time

import psutil
import requests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "examples", "echo-function", "manifests.yaml")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sigterm_stops_every_pod(tmp_path):
    port = _free_port()
    log = open(tmp_path / "serve.log", "w")
    env = {**os.environ, "PYTHONPATH": ROOT, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}
    proc = subprocess.Popen([sys.executable, "-m", "omnia_amd.cli", "serve", "--port", str(port),
                             "--no-engine", "-f", ECHO], cwd=ROOT, env=env, stdout=log,
                            stderr=subprocess.STDOUT, start_new_session=True)
    pods = []
    try:
        deadline = time.time() + 120
        while time.time() < deadline:
            assert proc.poll() is None, open(tmp_path / "serve.log").read()[-3000:]
            kids = psutil.Process(proc.pid).children(recursive=True)
            if any("omnia_amd.facade" in " ".join(k.cmdline()) for k in kids):
                pods = kids
                break
            time.sleep(0.5)
        assert pods, open(tmp_path / "serve.log").read()[-3000:]
        r = requests.get(f"http://127.0.0.1:{port}/healthz", timeout=5)
        assert r.status_code == 200
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(60)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(10)
        log.close()
    gone, alive = psutil.wait_procs(pods, timeout=20)
    assert not alive, [p.cmdline()[:4] for p in alive]
    assert "stopping pods" in open(tmp_path / "serve.log").read()
