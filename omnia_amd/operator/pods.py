"""Agent pods as OS processes on this node (the single-node kubelet's pod model).

An AgentRuntime pod is two containers (``internal/controller/deployment_builder.go``):
the runtime (``python -m omnia_amd.runtime``: gRPC :9000, health :9001, which in
turn starts its engine-core child on the pod's GPU) and the facade
(``python -m omnia_amd.facade``: WebSocket/REST on :8080, dialing the runtime
over gRPC).  :class:`ProcessPod` runs exactly those two entrypoints as child
processes with the container env the operator built, on free local ports:

* the pod's GPU is pinned with ``HIP_VISIBLE_DEVICES`` (the kubelet's device
  plugin equivalent), so the runtime's engine sees it as ``cuda:0``;
* with ``cpus`` every process of the pod is pinned to that CPU set (a slice
  of its GPU's NUMA node, ``utils/affinity.py``), so co-located replicas do
  not migrate across sockets or steal each other's cores;
* each container gets its own process group; stopping the pod sends SIGTERM to
  the group (graceful drain in both entrypoints) and SIGKILL after a grace
  period, so the engine-core grandchild never outlives its runtime;
* readiness = runtime ``/readyz`` (engine loaded and healthy), then facade
  ``/readyz``; the facade is started only once the runtime is ready (the
  reference's facade retries its dial instead, ``cmd/agent/runtime_dial.go``).

Nothing here touches the GPU itself, so a parent that will later fork GPU
workers (the bench, the operator) stays safe.
"""
from __future__ import annotations

import json
import logging
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time
import urllib.error
import urllib.request

log = logging.getLogger("omnia.pods")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_next_port: dict = {}


def free_port() -> int:
    """A port for a pod process to listen on.

    bind(0) draws from the kernel's ephemeral range, so processes choosing at
    the same moment can draw the same port -- with 8 bench replicas starting
    ~5 servers each, a birthday collision is a few-percent event that kills a
    replica.  With ``OMNIA_PORT_BASE`` set (bench.py gives every local rank its
    own window below the ephemeral range) ports are handed out sequentially
    from that window, skipping any that are taken; ``OMNIA_PORT_SPAN`` bounds
    the window (default 200)."""
    base = os.environ.get("OMNIA_PORT_BASE", "")
    if base.isdigit():
        lo = int(base)
        span = int(os.environ.get("OMNIA_PORT_SPAN", "200"))
        for _ in range(span):
            port = _next_port.get(lo, lo)
            _next_port[lo] = lo + (port + 1 - lo) % span
            with socket.socket() as s:
                try:
                    s.bind(("127.0.0.1", port))
                except OSError:
                    continue
            return port
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(url: str, timeout: float = 2.0) -> tuple[int, dict]:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, json.loads(r.read() or b"{}")
    except urllib.error.HTTPError as e:
        return e.code, {}
    except (OSError, ValueError):
        return 0, {}


class PodFailed(RuntimeError):
    pass


class ProcessPod:
    def __init__(self, name: str, runtime_env: dict, facade_env: dict,
                 device_index: int | list | None = None, log_dir: str | None = None,
                 python: str = sys.executable, tp: int = 1, cpus: list | None = None):
        self.name = name
        # host CPUs this pod's processes are pinned to (utils/affinity.py: a slice on
        # its GPU's NUMA node, disjoint from the other pods'); None = unpinned
        self.cpus = list(cpus) if cpus else None
        self.runtime_env = dict(runtime_env)
        self.facade_env = dict(facade_env)
        if isinstance(device_index, int):
            device_index = [device_index]
        self.devices = list(device_index) if device_index is not None else None
        self.tp = tp
        self.log_dir = log_dir or tempfile.mkdtemp(prefix=f"omnia-pod-{name}-")
        os.makedirs(self.log_dir, exist_ok=True)
        self.python = python
        self.grpc_port = self.health_port = self.facade_port = None
        self.runtime: subprocess.Popen | None = None
        self.facade: subprocess.Popen | None = None
        self._logs = []

    # ------------------------------------------------------------ lifecycle
    def _spawn(self, module: str, env: dict, tag: str, launcher: list | None = None
               ) -> subprocess.Popen:
        full = dict(os.environ)
        full.update({k: str(v) for k, v in env.items()})
        full["PYTHONPATH"] = ROOT + os.pathsep + full.get("PYTHONPATH", "")
        full.setdefault("PYTHONUNBUFFERED", "1")
        if self.devices is not None:
            # indices are relative to what this process sees: map them through an
            # inherited visibility list (a launcher may have restricted it)
            vis = next((os.environ[k] for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
                        if os.environ.get(k)), None)
            phys = [x.strip() for x in vis.split(",")] if vis else None
            devs = [phys[d] if phys is not None and d < len(phys) else str(d)
                    for d in self.devices]
            full["HIP_VISIBLE_DEVICES"] = ",".join(devs)
            full.pop("CUDA_VISIBLE_DEVICES", None)
        # a pod is never a torchrun rank itself
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                  "TORCHELASTIC_RUN_ID"):
            if k not in env:
                full.pop(k, None)
        path = os.path.join(self.log_dir, f"{tag}.log")
        f = open(path, "wb")
        self._logs.append(f)
        p = subprocess.Popen([self.python] + (launcher or []) + ["-m", module], env=full,
                             stdout=f, stderr=subprocess.STDOUT, cwd=ROOT,
                             start_new_session=True)
        if self.cpus:
            # right after the fork, before the child starts its threads and the
            # engine-core grandchild: everything it spawns inherits the set
            from ..utils import affinity

            affinity.pin(self.cpus, p.pid)
        return p

    def start_runtime(self):
        self.grpc_port = int(self.runtime_env.get("OMNIA_GRPC_PORT") or free_port())
        self.health_port = int(self.runtime_env.get("OMNIA_HEALTH_PORT") or free_port())
        env = {**self.runtime_env, "OMNIA_GRPC_PORT": self.grpc_port,
               "OMNIA_HEALTH_PORT": self.health_port}
        launcher = None
        if self.tp > 1:
            # one runtime process per GPU of the pod; rank 0 serves gRPC
            # (``omnia_amd/runtime/__main__.py``); torchrun's agent itself never
            # touches a GPU, it only starts the ranks.  ``tp`` is the pod's engine
            # world: the TP group, or the EP group under ep_mode a2a
            if env.get("OMNIA_ENGINE_EP_MODE") != "a2a":
                env["OMNIA_ENGINE_TP"] = self.tp
            launcher = ["-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={self.tp}", "--master-addr=127.0.0.1",
                        f"--master-port={free_port()}"]
        self.runtime = self._spawn("omnia_amd.runtime", env, "runtime", launcher)

    def start_facade(self):
        self.facade_port = int(self.facade_env.get("OMNIA_FACADE_PORT") or free_port())
        env = {**self.facade_env, "OMNIA_FACADE_PORT": self.facade_port,
               "OMNIA_RUNTIME_ADDRESS": f"127.0.0.1:{self.grpc_port}"}
        # the twin / dual-protocol ports are per-pod on a shared node: remap each
        # allocated one to a free port (pods.mgmt_ports keeps the mapping)
        self.mgmt_ports = {}
        for k in ("OMNIA_INTERNAL_FACADE_PORT", "OMNIA_INTERNAL_A2A_PORT",
                  "OMNIA_INTERNAL_MCP_PORT", "OMNIA_A2A_PORT", "OMNIA_MCP_PORT"):
            if str(env.get(k, "") or "0") not in ("", "0"):
                env[k] = self.mgmt_ports[k] = free_port()
        self.facade = self._spawn("omnia_amd.facade", env, "facade")

    def log_tail(self, tag: str, n: int = 4000) -> str:
        try:
            with open(os.path.join(self.log_dir, f"{tag}.log"), "rb") as f:
                f.seek(0, 2)
                f.seek(max(0, f.tell() - n))
                return f.read().decode(errors="replace")
        except OSError:
            return ""

    def _wait(self, proc, url: str, tag: str, deadline: float):
        while time.monotonic() < deadline:
            if proc.poll() is not None:
                raise PodFailed(f"pod {self.name}: {tag} exited with {proc.returncode}:\n"
                                + self.log_tail(tag))
            st, body = _get(url)
            if st == 200:
                return
            time.sleep(0.25)
        raise PodFailed(f"pod {self.name}: {tag} not ready after timeout:\n" + self.log_tail(tag))

    def start(self, timeout_s: float = 600.0) -> "ProcessPod":
        deadline = time.monotonic() + timeout_s
        self.start_runtime()
        try:
            # both containers start at once, as in a Kubernetes pod: the facade's
            # own start-up (imports, listeners) overlaps the engine load, and its
            # /readyz reports ready only once the runtime answers
            self.start_facade()
            self._wait(self.runtime, f"http://127.0.0.1:{self.health_port}/readyz", "runtime",
                       deadline)
            self._wait(self.facade, f"http://127.0.0.1:{self.facade_port}/readyz", "facade",
                       deadline)
        except BaseException:
            self.stop()
            raise
        log.info("pod %s ready: ws://127.0.0.1:%d/ws (runtime gRPC :%d)", self.name,
                 self.facade_port, self.grpc_port)
        return self

    @property
    def ws_url(self) -> str:
        return f"ws://127.0.0.1:{self.facade_port}/ws"

    @property
    def endpoint(self) -> str:
        return f"127.0.0.1:{self.facade_port}"

    def alive(self) -> bool:
        return all(p is not None and p.poll() is None for p in (self.runtime, self.facade))

    def stop(self, grace_s: float = 15.0):
        procs = [p for p in (self.facade, self.runtime) if p is not None]
        for p in procs:  # facade first: it drains in-flight turns against the runtime
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
            try:
                p.wait(timeout=grace_s)
            except subprocess.TimeoutExpired:
                pass
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)  # stragglers incl. the engine-core child
            except ProcessLookupError:
                pass
            try:
                p.wait(timeout=5)
            except subprocess.TimeoutExpired:
                pass
        for f in self._logs:
            f.close()
        self._logs.clear()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


class ServiceProcess:
    """A single-container service pod (workspace session-api / memory-api,
    ``internal/controller/workspace_services.go``) as one OS process: the
    container's ``command`` + ``args`` with its port rebound to a free local port,
    ``/data`` mapped into a per-pod directory and ConfigMap volume ``mounts``
    (mountPath -> materialised local dir) rewritten in args and env values."""

    def __init__(self, name: str, container: dict, workdir: str,
                 python: str = sys.executable, mounts: dict[str, str] | None = None):
        self.name = name
        self.container = container
        self.workdir = workdir
        self.mounts = mounts or {}
        self.python = python
        self.port = None
        self.proc: subprocess.Popen | None = None
        self._log = None

    def argv(self) -> list[str]:
        cmd = list(self.container.get("command") or []) + list(self.container.get("args") or [])
        if cmd and cmd[0] in ("python", "python3"):
            cmd[0] = self.python
        out, i = [], 0
        data = os.path.join(self.workdir, "data")
        os.makedirs(data, exist_ok=True)
        while i < len(cmd):
            a = cmd[i]
            if a == "--port" and i + 1 < len(cmd):
                out += ["--port", str(self.port)]
                i += 2
                continue
            out.append(a.replace("/data/", data + "/") if a.startswith("/data/")
                       else self._map(a))
            i += 1
        if "--port" not in out:
            out += ["--port", str(self.port)]
        return out

    def _map(self, v: str) -> str:
        for mp, local in self.mounts.items():
            if v == mp or v.startswith(mp.rstrip("/") + "/"):
                return local + v[len(mp.rstrip("/")):]
        return v

    def start(self, timeout_s: float = 60.0) -> "ServiceProcess":
        self.port = free_port()
        env = dict(os.environ)
        env.update({e["name"]: self._map(str(e.get("value", "")))
                    for e in self.container.get("env", [])})
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        os.makedirs(self.workdir, exist_ok=True)
        self._log = open(os.path.join(self.workdir, "service.log"), "wb")
        self.proc = subprocess.Popen(self.argv(), env=env, stdout=self._log,
                                     stderr=subprocess.STDOUT, cwd=ROOT, start_new_session=True)
        path = ((self.container.get("readinessProbe") or {}).get("httpGet") or {}).get(
            "path", "/healthz")
        deadline = time.monotonic() + timeout_s
        while time.monotonic() < deadline:
            if self.proc.poll() is not None:
                raise PodFailed(f"service {self.name} exited with {self.proc.returncode}")
            if _get(f"http://127.0.0.1:{self.port}{path}")[0] == 200:
                return self
            time.sleep(0.2)
        self.stop()
        raise PodFailed(f"service {self.name} not ready")

    @property
    def endpoint(self) -> str:
        return f"127.0.0.1:{self.port}"

    def alive(self) -> bool:
        return self.proc is not None and self.proc.poll() is None

    def stop(self, grace_s: float = 10.0):
        if self.proc is not None and self.proc.poll() is None:
            try:
                os.killpg(self.proc.pid, signal.SIGTERM)
                self.proc.wait(timeout=grace_s)
            except (ProcessLookupError, subprocess.TimeoutExpired):
                try:
                    os.killpg(self.proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        if self._log is not None:
            self._log.close()
            self._log = None


_SVC_URL = None


def service_refs(env: dict) -> set[tuple[str, str]]:
    """(service, namespace) of every in-cluster URL in ``env``'s values."""
    resolve_service_urls({}, lambda *_: None)  # compiles the pattern
    out = set()
    for v in env.values():
        if isinstance(v, str):
            out.update((m.group(2), m.group(3)) for m in _SVC_URL.finditer(v))
    return out


def resolve_service_urls(env: dict, lookup) -> dict:
    """Cluster DNS for a single node: rewrite ``http://<svc>.<ns>[.svc...]:<port>``
    in env values to the local endpoint ``lookup(svc, ns)`` returns (or leave it)."""
    import re

    global _SVC_URL
    if _SVC_URL is None:
        _SVC_URL = re.compile(r"(https?://)([a-z0-9-]+)\.([a-z0-9-]+)(?:\.svc[.a-z0-9-]*)?:\d+")

    def sub(m):
        ep = lookup(m.group(2), m.group(3))
        return f"{m.group(1)}{ep}" if ep else m.group(0)

    return {k: _SVC_URL.sub(sub, v) if isinstance(v, str) else v for k, v in env.items()}


class JobPodProcess:
    """One pod of a batch/v1 Job (arena workers) as a run-to-completion OS
    process: the container's command + args + env, its ConfigMap volumes
    materialised under a per-pod directory (``mountPath`` prefixes in env values
    and args are rewritten to it)."""

    def __init__(self, name: str, container: dict, workdir: str, mounts: dict[str, str],
                 python: str = sys.executable):
        self.name = name
        self.container = container
        self.workdir = workdir
        self.mounts = mounts  # mountPath -> local dir
        self.python = python
        self.proc: subprocess.Popen | None = None
        self._log = None

    def _map(self, v: str) -> str:
        for mp, local in self.mounts.items():
            if v == mp or v.startswith(mp.rstrip("/") + "/"):
                return local + v[len(mp.rstrip("/")):]
        return v

    def start(self) -> "JobPodProcess":
        cmd = list(self.container.get("command") or []) + list(self.container.get("args") or [])
        if cmd and cmd[0] in ("python", "python3"):
            cmd[0] = self.python
        cmd = [self._map(a) for a in cmd]
        env = dict(os.environ)
        for e in self.container.get("env", []):
            if "value" in e:
                env[e["name"]] = self._map(str(e["value"]))
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        env["HOSTNAME"] = self.name
        os.makedirs(self.workdir, exist_ok=True)
        self._log = open(os.path.join(self.workdir, "pod.log"), "wb")
        self.proc = subprocess.Popen(cmd, env=env, stdout=self._log, stderr=subprocess.STDOUT,
                                     cwd=ROOT, start_new_session=True)
        return self

    def poll(self) -> int | None:
        return None if self.proc is None else self.proc.poll()

    def stop(self):
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
        if self._log:
            self._log.close()
            self._log = None
