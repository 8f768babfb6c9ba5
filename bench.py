#!/usr/bin/env python3
"""Headline benchmark: streamed tokens/sec + p50 turn latency of an AgentRuntime
serving Llama-3-8B (BASELINE.json metric) on 1/2/4/8 MI355X GPUs.

One rank process per GPU (DP = N replicas, weak scaling: per-GPU concurrency is
fixed as N grows).  ``--gpus N`` without a torchrun environment spawns the N
rank processes itself (the parent never touches a GPU); under
``torch.distributed.run`` the world size must equal ``--gpus``.

A "step" is one wave of C concurrent agent turns per GPU.  Every turn sends a
fresh synthetic message whose rendered prompt (PromptPack system prompt + Llama-3
chat template + user text) is exactly ``--prompt-len`` tokens and streams
``--gen-len`` tokens with ignore_eos.  Timing follows the reference's arena load
tester (``ee/pkg/arena/fleet/client.go:124-157``): TTFT = first streamed frame,
turn latency = ``done``, tokens = ``done.usage.output_tokens``.  Weights are
random-init bf16 of the exact Llama-3-8B architecture; data is synthetic.

Paths (``--path``):
  ws       (default) the production pod: every turn is a real WebSocket
           connection to the facade process, which calls the runtime process
           over gRPC; the runtime renders the pack, tokenizes and streams from
           its engine-core child on this rank's GPU (``operator/pods.py``).
  runtime  the runtime's Converse handler in-process (no sockets), engine-core
           child process.
  engine   the engine API directly.
``--arrival poisson --rate R`` replaces the closed-loop waves by an open-loop
stream of ``steps x C`` turns per GPU arriving at R turns/s and reports TTFT and
inter-token latency percentiles.
"""
from __future__ import annotations

import time as _time

_T_START = _time.perf_counter()  # process start (phase accounting in the JSON line)

import argparse  # noqa: E402
import asyncio
import json
import os
import random
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "streamed tokens/sec + p50 turn latency, AgentRuntime Llama-3-8B at 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=256, help="concurrent turns per GPU")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--path", choices=["ws", "runtime", "engine"], default="ws")
    ap.add_argument("--stream-interval-ms", type=float, default=0.0,
                    help="runtime text-delta coalescing window (0 = one frame per token)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree per replica")
    ap.add_argument("--arrival", choices=["closed", "poisson"], default="closed")
    ap.add_argument("--rate", type=float, default=0.0, help="poisson: turns/s per replica")
    ap.add_argument("--mixed-budget", type=int, default=None,
                    help="engine mixed steps: decode rows + <= N prefill tokens per forward "
                         "(default: the engine's, gated on the prefill backlog)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-share-prefix", action="store_true",
                    help="engine: no cross-session prefix sharing (every prompt token prefilled)")
    ap.add_argument("--inproc", action="store_true",
                    help="runtime path: engine as a thread of the serving process")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--pod-timeout", type=float, default=900.0)
    ap.add_argument("--pin-cpus", choices=["auto", "on", "off"], default="auto",
                    help="pin each replica's serving tree (client, facade, runtime, "
                         "engine-core) to a disjoint CPU set on its GPU's NUMA node "
                         "(omnia_amd/utils/affinity.py); auto = on when --gpus > 1 and every "
                         "replica gets >= 4 CPUs")
    ap.add_argument("--engine", choices=["gpu", "synthetic"], default="gpu",
                    help="synthetic: ws-path host capacity rehearsal -- the engine-core is a "
                         "token source paced like the measured GPU engine (engine/synthetic.py)")
    ap.add_argument("--tp-shared-device", action="store_true",
                    help="TP rehearsal on fewer GPUs than --tp: the TP ranks of the one "
                         "replica share device(s) over the ipc transport (correctness and "
                         "plumbing, not a scaling number)")
    ap.add_argument("--preflight", choices=["auto", "on", "off"], default="auto",
                    help="multi-GPU first-contact check in a fresh child per rank before any "
                         "pod starts (parallel/preflight.py): peer access, RCCL init + "
                         "all-reduce, IPC all-reduce checked against it; auto = on with GPUs")
    return ap.parse_args(argv)


def job_preflight(a, ws: int, rank: int, local: int, backend: str) -> dict | None:
    """Every rank runs the preflight in a fresh child (rendezvous on a port rank
    0 picks, shared over the bench's gloo group) before its pod starts; rank 0
    gets the job summary.  Outside the timed region."""
    from omnia_amd.parallel import preflight as pf

    if ws > 1:
        import torch.distributed as dist

        box = [_free_port() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        port = box[0]
    else:
        port = _free_port()
    rep = pf.spawn(rank, ws, local, port, backend)
    if ws > 1:
        import torch.distributed as dist

        reps = [None] * ws
        dist.all_gather_object(reps, rep)
    else:
        reps = [rep]
    return pf.summarize(reps)


def tp_preflight(devs: list[int], backend: str = "nccl") -> dict:
    """The preflight over one TP pod's devices, before its engine starts."""
    import concurrent.futures as cf

    from omnia_amd.parallel import preflight as pf

    port = _free_port()
    with cf.ThreadPoolExecutor(len(devs)) as ex:
        reps = list(ex.map(lambda i: pf.spawn(i, len(devs), devs[i], port, backend),
                           range(len(devs))))
    return pf.summarize(reps)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a) -> int:
    """``--gpus N`` outside torchrun: start N rank processes of this script (the
    torchrun env contract) and return the first failing exit code.  Nothing in
    this process initialises a GPU."""
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    failed = []
    for r, p in enumerate(procs):
        p.wait()
        if p.returncode:
            failed.append((r, p.returncode))
            if not rc:
                rc = p.returncode
    for r, code in failed:
        what = f"signal {-code}" if code < 0 else f"exit code {code}"
        print(f"bench: rank {r} of {a.gpus} failed ({what})", file=sys.stderr, flush=True)
    return rc


def _cpulist(cpus) -> str | None:
    """[0, 1, 2, 5] -> "0-2,5" (None: not pinned)."""
    if not cpus:
        return None
    cpus = sorted(cpus)
    out, lo = [], cpus[0]
    for a, b in zip(cpus, cpus[1:] + [None]):
        if b != a + 1:
            out.append(f"{lo}-{a}" if a > lo else str(a))
            lo = b
    return ",".join(out)


def pct(v, q):
    if not v:
        return None
    v = sorted(v)
    return v[min(len(v) - 1, int(round(q * (len(v) - 1))))]


# ============================================================== WebSocket path
class WSDriver:
    """Runs this rank's agent pod (facade + runtime + engine-core processes) and
    drives turns through its WebSocket endpoint."""

    SYSTEM = "You are a benchmark agent."

    def __init__(self, a, rank: int, local: int, use_gpu: bool, world: int):
        from omnia_amd.operator.pods import ProcessPod
        from omnia_amd.runtime.promptpack import PromptPack

        self.a = a
        self.rank = rank
        self.leader = rank % a.tp == 0 or a.tp_shared_device
        self.tmp = tempfile.mkdtemp(prefix=f"omnia-bench-r{rank}-")
        self.rng = random.Random(1234 + rank)
        self.pod = None
        self._ready = []  # pre-opened sessions for the next wave (one per virtual user)
        self._next_contents = None  # the next wave's messages, written during this one
        self.overhead = self._template_overhead()
        if a.prompt_len <= self.overhead:
            raise SystemExit(f"--prompt-len {a.prompt_len} must exceed the chat-template "
                             f"overhead of {self.overhead} tokens")
        if not self.leader:
            return
        pack = PromptPack.minimal(self.SYSTEM).data
        pack["prompts"]["default"]["parameters"] = {
            "max_tokens": a.gen_len, "ignore_eos": True, "temperature": a.temperature,
            "top_p": 1.0}
        pack_path = os.path.join(self.tmp, "pack.json")
        with open(pack_path, "w") as f:
            json.dump(pack, f)
        C = a.concurrency
        renv = {
            "OMNIA_AGENT_NAME": f"bench-{rank}", "OMNIA_PROVIDER_TYPE": "local",
            "OMNIA_PROMPTPACK_PATH": pack_path, "OMNIA_TOOLS_CONFIG_PATH": "",
            "OMNIA_STREAM_INTERVAL_MS": a.stream_interval_ms,
            "OMNIA_ENGINE_MODEL": a.model, "OMNIA_ENGINE_DEVICE": "cuda" if use_gpu else "cpu",
            "OMNIA_ENGINE_MAX_BATCH": max(C, 1),
            "OMNIA_ENGINE_MAX_MODEL_LEN": max(2048, a.prompt_len + a.gen_len + 64),
            "OMNIA_ENGINE_MAX_PREFILL_TOKENS": a.max_prefill_tokens,
            "OMNIA_ENGINE_USE_GRAPHS": "false" if a.no_graphs else "true",
            "OMNIA_ENGINE_SHARE_PREFIX": "false" if a.no_share_prefix else "true",
            "OMNIA_ENGINE_SEED": rank,
            "OMNIA_ENGINE_PROC": "1" if (use_gpu and a.tp == 1) or a.engine == "synthetic" else "0",
            "OMNIA_ENGINE_SYNTHETIC": "1" if a.engine == "synthetic" else "0",
            "OMNIA_ENGINE_TP": a.tp,
            "OMNIA_DEBUG_ENGINE_STATS": "1",  # timed-window device busy (gpu_busy_timed)
            **({"OMNIA_ENGINE_MIXED_BUDGET": a.mixed_budget} if a.mixed_budget is not None
               else {}),
        }
        fenv = {"OMNIA_AGENT_NAME": f"bench-{rank}", "OMNIA_MAX_CONNECTIONS": 4 * C + 64,
                "OMNIA_MSG_RATE": 1000, "OMNIA_MSG_BURST": 1000}
        devs = list(range(local, local + a.tp)) if use_gpu else None
        if devs and a.tp_shared_device:
            import torch

            n = max(1, torch.cuda.device_count())  # no HIP init: counting only
            devs = sorted({d % n for d in devs})  # ranks share these (ipc transport)
        self.tp_preflight = None
        if devs and a.tp > 1 and a.preflight != "off" and a.engine == "gpu":
            self.tp_preflight = tp_preflight(devs)
        self.pod = ProcessPod(f"bench-r{rank}", renv, fenv, device_index=devs,
                              log_dir=os.path.join(self.tmp, "logs"), tp=a.tp)
        self.pod.start(timeout_s=a.pod_timeout)
        self.loop = asyncio.new_event_loop()
        self.http = self.loop.run_until_complete(self._mk_http())

    async def _mk_http(self):
        import aiohttp

        return aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None),
                                     connector=aiohttp.TCPConnector(limit=0))

    def _template_overhead(self) -> int:
        """Tokens the runtime adds around the user text (system prompt + chat
        template), with the engine's tokenizer (byte-level for random-init)."""
        from omnia_amd.engine.tokenizer import make_tokenizer
        from omnia_amd.models.config import resolve
        from omnia_amd.runtime.chat import Message, render_llama3

        self.tok = make_tokenizer(resolve(self.a.model))
        base = render_llama3([Message("system", self.SYSTEM), Message("user", "")])
        return len(self.tok.encode(base))

    def _content(self) -> str:
        n = self.a.prompt_len - self.overhead
        # printable ASCII, one byte token each; fresh per turn (no cross-turn prefix reuse)
        return "".join(self.rng.choices("abcdefghijklmnopqrstuvwxyz ,.", k=n))

    def _contents(self, n: int) -> list[str]:
        return [self._content() for _ in range(n)]

    async def _connect(self):
        from omnia_amd.ee.arena.fleet import FleetSession

        return await FleetSession(self.pod.ws_url, http=self.http, timeout_s=600).__aenter__()

    async def _turn(self, content: str, fs=None, reconnect: bool = False):
        """One turn on a fresh session.  A virtual user keeps its next session
        open while it waits (``reconnect``): the WebSocket handshake of its next
        turn overlaps the rest of this wave instead of stalling the next wave's
        start (turn timing starts at the ``message`` frame either way)."""
        fs = fs or await self._connect()
        # the user's NEXT session opens while this turn streams, so no WebSocket
        # handshake (facade session setup) sits at the wave boundary
        nxt = asyncio.ensure_future(self._connect()) if reconnect else None
        try:
            r = await fs.turn(content)
        finally:
            await fs.__aexit__(None, None, None)
        if nxt is not None:
            self._ready.append(await nxt)
        u = r["usage"] or {}
        return (r["ttft_ms"] / 1e3, r["latency_ms"] / 1e3, int(u.get("output_tokens", 0)),
                int(u.get("input_tokens", 0)), r["chunk_times_s"], int(u.get("cached_tokens", 0)))

    async def _wave(self):
        """One closed-loop wave.  The virtual users' NEXT messages are written on
        a helper thread while this wave runs (as real users type while the agent
        answers), so no client-side text generation sits between two waves."""
        ready, self._ready = self._ready, []
        n = self.a.concurrency
        contents = self._next_contents or self._contents(n)
        nxt = asyncio.get_running_loop().run_in_executor(None, self._contents, n)
        res = await asyncio.gather(*(self._turn(contents[i],
                                                ready[i] if i < len(ready) else None,
                                                reconnect=True)
                                     for i in range(n)))
        self._next_contents = await nxt
        return res

    def wave(self, step: int):
        if self.pod is None:
            return []
        res = self.loop.run_until_complete(self._wave())
        if step < 0:
            ins = {r[3] for r in res}
            if ins != {self.a.prompt_len}:
                raise SystemExit(f"prompt length mismatch: runtime saw {sorted(ins)[:4]} "
                                 f"tokens, expected {self.a.prompt_len}")
        return res

    async def _open_loop(self, n: int, rate: float):
        rng = random.Random(99 + self.rank)
        tasks = []
        t = time.perf_counter()
        for _ in range(n):
            tasks.append(asyncio.ensure_future(self._turn(self._content())))
            t += rng.expovariate(rate)
            d = t - time.perf_counter()
            if d > 0:
                await asyncio.sleep(d)
        return await asyncio.gather(*tasks)

    def open_loop(self, n: int, rate: float):
        if self.pod is None:
            return []
        return self.loop.run_until_complete(self._open_loop(n, rate))

    def _debug(self, method: str):
        if self.pod is None:
            return None
        import urllib.request

        req = urllib.request.Request(
            f"http://127.0.0.1:{self.pod.health_port}/debug/engine-stats", method=method,
            data=b"" if method == "POST" else None)
        try:
            with urllib.request.urlopen(req, timeout=120) as r:
                return json.loads(r.read())
        except (OSError, ValueError):
            return None

    def reset_timing(self):
        """Zero the pod engine's counters and device-busy account (timed window)."""
        self._debug("POST")

    def engine_stats(self) -> dict | None:
        return self._debug("GET")

    def close(self):
        if self.pod is not None:
            ready, self._ready = self._ready, []

            async def _close_ready():
                await asyncio.gather(*(fs.__aexit__(None, None, None) for fs in ready),
                                     return_exceptions=True)

            self.loop.run_until_complete(_close_ready())
            self.loop.run_until_complete(self.http.close())
            self.pod.stop()
            self.pod = None


# ============================================================== in-process paths
class LocalDriver:
    def __init__(self, a, rank: int, local: int, use_gpu: bool, world: int):
        import torch
        import torch.distributed as dist

        from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine
        from omnia_amd.engine.sampling_params import SamplingParams

        self.a = a
        self.rank = rank
        self.proc = a.path == "runtime" and not a.inproc
        self.use_gpu = use_gpu
        C = a.concurrency
        cfg = EngineConfig(model=a.model, device="cuda" if use_gpu else "cpu",
                           max_batch=max(C, 1),
                           max_model_len=max(2048, a.prompt_len + a.gen_len + 64),
                           max_prefill_tokens=a.max_prefill_tokens, use_graphs=not a.no_graphs,
                           seed=rank, share_prefix=not a.no_share_prefix,
                           **({"mixed_budget": a.mixed_budget}
                                         if a.mixed_budget is not None else {}))
        self.cfg = cfg
        self.eng = self.client = None
        if self.proc:
            from omnia_amd.engine.core_proc import EngineCoreClient

            self.client = EngineCoreClient(cfg, device_index=local if use_gpu else None)
            model_cfg = self.client.engine.model_cfg
        else:
            if use_gpu:
                torch.cuda.set_device(local)
            self.eng = LLMEngine(cfg)
            model_cfg = self.eng.model_cfg
        self.vocab = model_cfg.vocab_size
        self.params = SamplingParams(temperature=a.temperature, max_tokens=a.gen_len,
                                     ignore_eos=True, top_p=1.0)
        self.g = torch.Generator().manual_seed(1234 + rank)
        self.runtime = None
        if a.path == "runtime":
            from omnia_amd.runtime.bench_driver import RuntimeBenchDriver

            self.runtime = RuntimeBenchDriver(self.client if self.proc else AsyncLLMEngine(self.eng),
                                              self.params)

    def wave(self, step: int):
        import torch

        a = self.a
        lo = min(1000, self.vocab // 4)
        prompts = torch.randint(lo, self.vocab - lo, (a.concurrency, a.prompt_len),
                                generator=self.g).tolist()
        if self.runtime is not None:
            return [(t, l, n, a.prompt_len, [], None)
                    for t, l, n in self.runtime.run_wave(prompts, step)]
        eng = self.eng
        seqs = [eng.add_request(p, self.params, session_id=f"r{self.rank}-s{step}-{i}")
                for i, p in enumerate(prompts)]
        eng.run_until_done()
        for s in seqs:
            eng.drop_session(s.session_id)  # fresh prompts next wave: no prefix reuse
        return [(s.ttft(), s.latency(), len(s.output), a.prompt_len, [], s.prefix_hit)
                for s in seqs]

    def sync(self):
        import torch

        if self.proc:
            self.client.synchronize()  # torch.cuda.synchronize() in the GPU-owning process
        elif self.use_gpu:
            torch.cuda.synchronize()

    def engine_stats(self) -> dict:
        if self.proc:
            return self.client.stats()
        eng = self.eng
        return {"timing": dict(eng.timing), "counters": dict(eng.counters),
                "runner": dict(eng.runner.stats), "kv_blocks": eng.blocks.num_blocks,
                "block_size": self.cfg.block_size,
                "gpu_busy_s": eng.busy_seconds() if hasattr(eng, "busy_seconds") else None}

    def reset_timing(self):
        if self.proc:
            self.client.call("reset_timing")
        else:
            for k in self.eng.timing:
                self.eng.timing[k] = 0.0
            self.eng.runner.stats["gil_wait_s"] = 0.0
            if hasattr(self.eng, "busy_seconds"):
                self.eng.busy_seconds(reset=True)

    def close(self):
        if self.runtime is not None:
            self.runtime.close()
        elif self.client is not None:
            self.client.shutdown()


# ============================================================== main
def check_streamed(results, gen_len: int, has_frames: bool, strict: bool = True) -> int:
    """The headline counts ``done.usage.output_tokens``; cross-check it against
    what the client actually received.  Every turn must report exactly
    ``gen_len`` tokens (ignore_eos), and on the WS path the streamed chunk frames
    it timed must account for them: never more than one frame per token (plus a
    role frame), and at least half as many frames as tokens (a token may share
    a frame when the detokenizer holds an incomplete UTF-8 sequence -- random-
    init weights emit raw byte tokens -- or when a lagging serving loop drains
    several steps at once).  Returns the total frame count; exits on a violation
    so a drifting count never reaches the JSON line (the exact frames/token ratio
    is reported in it).  ``strict`` False (a tiny test vocabulary) counts only."""
    total = 0
    for r in results:
        n = r[2]
        if n != gen_len:
            raise SystemExit(f"turn reported {n} output tokens, expected {gen_len} (ignore_eos)")
        if has_frames:
            f = len(r[4])
            total += f
            if strict and (f > n + 1 or f < n // 2):
                raise SystemExit(f"turn streamed {f} frames for {n} reported output tokens")
    return total


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a))
    import torch
    import torch.distributed as dist

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but the launcher started {ws} ranks")
    if a.gpus % a.tp and not a.tp_shared_device:
        raise SystemExit(f"--gpus {a.gpus} is not a multiple of --tp {a.tp}")
    if a.tp > 1 and a.path != "ws":
        raise SystemExit("--tp > 1 is served by the ws path (one TP pod per replica)")
    # device_count() does not initialise the GPU: engine children start before any HIP call
    use_gpu = a.device == "cuda" and a.engine == "gpu" and torch.cuda.device_count() > 0
    if a.engine == "synthetic" and a.path != "ws":
        raise SystemExit("--engine synthetic rehearses the ws host path")
    host_only = a.path == "ws" or (a.path == "runtime" and not a.inproc)
    if ws > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # every replica's servers listen in a port window of its own (below the
        # ephemeral range): concurrent bind(0) draws can collide across replicas
        # (OMNIA_BENCH_PORT_BASE moves the job's windows: concurrent bench jobs)
        os.environ.setdefault("OMNIA_PORT_BASE", str(
            int(os.environ.get("OMNIA_BENCH_PORT_BASE", "21000")) + 200 * local))
        # result aggregation only: host-side gloo whenever this process owns no GPU work
        dist.init_process_group("gloo" if (host_only or not use_gpu) else "nccl")

    pinned = None
    if a.pin_cpus == "on" or (a.pin_cpus == "auto" and ws > 1):
        # before any pod process starts: the facade / runtime / engine-core
        # children inherit this process's CPU set
        from omnia_amd.utils import affinity

        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
        phys = [int(x) for x in vis.split(",")] if vis else None
        devs = [phys[r % len(phys)] if phys else r for r in range(ws)]
        pinned = affinity.plan(devs)[rank]
        if a.pin_cpus == "auto" and len(pinned) < affinity.MIN_AUTO_PIN_CPUS:
            # oversubscribed host (e.g. 4 replicas on 8 CPUs): a replica's tree
            # needs ~2.5 cores with bursts above that, and a hard 2-CPU slice
            # starves it (p95 frame gap 63 -> 254 ms measured); share instead
            pinned = None
        else:
            affinity.pin(pinned)
    pre = None
    if a.preflight == "on" or (a.preflight == "auto" and use_gpu and a.engine == "gpu"
                               and host_only):
        # the bench process itself never touches the GPU on these paths: the
        # check runs in fresh children and is gone before any pod starts
        pre = job_preflight(a, ws, rank, local, "nccl" if use_gpu else "gloo")
    drv = WSDriver(a, rank, local, use_gpu, ws) if a.path == "ws" else \
        LocalDriver(a, rank, local, use_gpu, ws)
    drv.preflight = pre
    drv.pinned_cpus = pinned
    try:
        run(a, drv, ws, rank, use_gpu, host_only)
    finally:
        drv.close()
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


def _client_profiler():
    """OMNIA_PYPROFILE=<dir>: profile this client over the timed waves (the pod's
    processes profile themselves, utils/pyprof.py)."""
    if not os.environ.get("OMNIA_PYPROFILE"):
        return None
    import cProfile

    p = cProfile.Profile()
    p.enable()
    return p


def _dump_profiles(prof, drv):
    import signal

    prof.disable()
    d = os.environ["OMNIA_PYPROFILE"]
    os.makedirs(d, exist_ok=True)
    prof.dump_stats(os.path.join(d, f"client-{os.getpid()}.prof"))
    pod = getattr(drv, "pod", None)
    if pod is None:
        return
    import psutil

    pids = [p.pid for p in (pod.runtime, pod.facade) if p is not None]
    for pid in list(pids):
        try:
            pids += [c.pid for c in psutil.Process(pid).children(recursive=True)]
        except psutil.Error:
            pass
    for pid in pids:  # only the processes that installed the SIGUSR1 dump handler
        try:
            cmd = " ".join(psutil.Process(pid).cmdline())
            if any(m in cmd for m in ("omnia_amd.runtime", "omnia_amd.facade",
                                      "omnia_amd.engine.core_proc")):
                os.kill(pid, signal.SIGUSR1)
        except (OSError, psutil.Error):
            pass
    time.sleep(3.0)  # let them write


def _tree_cpu_s() -> float:
    """CPU seconds (user + system) used so far by this rank's process tree: the
    bench client and its agent pod (facade, runtime, engine-core)."""
    import psutil

    me = psutil.Process()
    tot = 0.0
    for p in [me] + me.children(recursive=True):
        try:
            t = p.cpu_times()
            tot += t.user + t.system
        except psutil.Error:
            pass
    return tot


def run(a, drv, ws, rank, use_gpu, host_only):
    import torch
    import torch.distributed as dist

    def sync():
        if isinstance(drv, LocalDriver):
            drv.sync()
        if ws > 1:
            dist.barrier()

    t_ready = time.perf_counter()
    for w in range(a.warmup):
        drv.wave(-1 - w)
    t_warm = time.perf_counter()
    drv.reset_timing()
    sync()
    cpu0 = _tree_cpu_s()
    t0 = time.perf_counter()
    results = []
    wave_ms = []  # this rank's per-wave wall time (closed loop)
    if a.arrival == "poisson":
        if a.rate <= 0:
            raise SystemExit("--arrival poisson needs --rate > 0 (turns/s per replica)")
        results = drv.open_loop(a.steps * a.concurrency, a.rate) if a.path == "ws" else []
    else:
        prof = _client_profiler()
        for k in range(a.steps):
            tw = time.perf_counter()
            results.extend(drv.wave(k))
            wave_ms.append(round(1000 * (time.perf_counter() - tw), 1))
    sync()
    elapsed = time.perf_counter() - t0
    # device time the engine's steps covered over the timed window (hipEvent
    # pairs per step, engine/engine.py busy_seconds) / wall time
    est = drv.engine_stats()
    busy = (est or {}).get("gpu_busy_s")
    my_busy = round(busy / elapsed, 4) if busy is not None and elapsed > 0 else None
    # host cores this replica's serving path kept busy (client included): the
    # CPU a node must supply per replica at this rate
    cores = (_tree_cpu_s() - cpu0) / elapsed if elapsed > 0 else 0.0
    if a.arrival != "poisson" and prof is not None:
        _dump_profiles(prof, drv)

    from omnia_amd.models.config import resolve as _resolve

    # frames track tokens only with a full vocabulary: a tiny test vocab is
    # mostly raw bytes, whose UTF-8 fragments the detokenizer holds back
    # (the host-path rehearsal REPORTS merged frames -- a lagging serving loop
    # drains several steps' tokens at once -- instead of failing on them)
    frames = check_streamed(results, a.gen_len, a.path == "ws",
                            strict=_resolve(a.model).vocab_size >= 32000 and a.engine == "gpu")
    out_tokens = sum(r[2] for r in results)
    ttfts = [r[0] for r in results if r[0] is not None]
    lats = [r[1] for r in results if r[1] is not None]
    # inter-token latency: mean gap per turn (TPOT) and every gap between frames
    tpot = [(r[1] - r[0]) / (r[2] - 1) for r in results if r[2] > 1 and r[0] is not None]
    gaps = []
    for r in results:
        ct = r[4]
        gaps.extend(ct[i] - ct[i - 1] for i in range(1, len(ct)))
    my_rate = out_tokens / elapsed if elapsed > 0 else 0.0
    if ws > 1:
        stats = torch.tensor([elapsed, float(out_tokens)], dtype=torch.float64)
        if not (host_only or not use_gpu):
            stats = stats.cuda()
        mx, sm = stats.clone(), stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, out_tokens = float(mx[0]), float(sm[1])
        gathered = [None] * ws
        dist.all_gather_object(gathered, (ttfts, lats, tpot, gaps[:20000], round(my_rate, 2),
                                          round(cores, 2), getattr(drv, "pinned_cpus", None),
                                          my_busy))
        ttfts = [x for g in gathered for x in g[0]]
        lats = [x for g in gathered for x in g[1]]
        tpot = [x for g in gathered for x in g[2]]
        gaps = [x for g in gathered for x in g[3]]
        per_rank = [g[4] for g in gathered]
        cores_rank = [g[5] for g in gathered]
        pins = [g[6] for g in gathered]
        busy_rank = [g[7] for g in gathered]
    else:
        per_rank = [round(my_rate, 2)]
        cores_rank = [round(cores, 2)]
        pins = [getattr(drv, "pinned_cpus", None)]
        busy_rank = [my_busy]
    value = out_tokens / elapsed
    st = est if isinstance(drv, LocalDriver) else None
    if rank == 0:
        ms = lambda x: round(1000 * x, 2) if x is not None else None  # noqa: E731
        rec = {
            "metric": BASELINE_METRIC,
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            # process start -> serving pod ready (imports, model init, KV pool) and
            # the untimed warmup waves (first-wave graph captures included)
            "startup_s": round(t_ready - _T_START, 2),
            "warmup_s": round(t_warm - t_ready, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random text prompts of exactly prompt_len tokens after the "
                    "chat template, random-init weights of the named architecture, ignore_eos)"
                    if a.engine == "gpu" else
                    "HOST-PATH REHEARSAL: synthetic engine-core paced like the measured GPU "
                    "engine (engine/synthetic.py), no GPU compute",
            "world_size": ws,
            "per_rank_tokens_per_s": per_rank,
            "host_cpu_cores_per_rank": cores_rank,
            # timed-window device busy per rank: engine-step hipEvent intervals / wall
            "gpu_busy_timed": (round(sum(busy_rank) / len(busy_rank), 4)
                               if busy_rank and None not in busy_rank else None),
            "gpu_busy_timed_per_rank": busy_rank,
            "pinned_cpus_per_rank": [_cpulist(p) for p in pins],
            "p50_turn_latency_ms": ms(statistics.median(lats)) if lats else None,
            "p95_turn_latency_ms": ms(pct(lats, 0.95)),
            "p50_ttft_ms": ms(statistics.median(ttfts)) if ttfts else None,
            "p95_ttft_ms": ms(pct(ttfts, 0.95)),
            "p50_tpot_ms": ms(pct(tpot, 0.5)),
            "p95_tpot_ms": ms(pct(tpot, 0.95)),
            "p95_frame_gap_ms": ms(pct(gaps, 0.95)),
            "streamed_frames_rank0": frames if a.path == "ws" else None,
            "frames_per_token_rank0": round(frames / max(1, sum(r[2] for r in results)), 4)
            if a.path == "ws" else None,
            "turns": len(lats),
            # prompt tokens served from KV pages another sequence computed (the
            # shared system-prompt page; engine/kv_manager.py), rank 0's turns
            "prefix_cached_frac": round(sum(r[5] for r in results) / max(1, sum(
                r[3] for r in results)), 4) if results and results[0][5] is not None else None,
            "wave_ms": wave_ms,
            # multi-GPU first contact (parallel/preflight.py), untimed: RCCL world,
            # peer access, RCCL vs IPC all-reduce (checked equal) at 16 KiB / 32 MiB
            "preflight": getattr(drv, "preflight", None),
            "tp_preflight": getattr(drv, "tp_preflight", None),
            "config": {
                "model": a.model,
                "global_batch": a.concurrency * max(1, ws // a.tp),
                "seq_len": a.prompt_len + a.gen_len,
                "prompt_len": a.prompt_len,
                "gen_len": a.gen_len,
                "concurrency_per_replica": a.concurrency,
                "parallelism": f"dp{max(1, ws // a.tp)}" + (f"-tp{a.tp}" if a.tp > 1 else "")
                + ("-shared-device-rehearsal" if a.tp_shared_device else ""),
                "path": a.path,
                "arrival": a.arrival if a.arrival == "closed" else f"poisson@{a.rate}/s",
                "stream_interval_ms": a.stream_interval_ms,
                "mixed_budget": a.mixed_budget if a.mixed_budget is not None else
                "engine default (16384, ungated)",
                "tp": a.tp,
                "hip_graphs": not a.no_graphs,
                "engine": a.engine,
            },
        }
        if st is not None:
            rec["engine"] = {
                "kv_blocks": st["kv_blocks"], "block_size": st["block_size"],
                "prefill_steps": st["counters"]["steps_prefill"],
                "decode_steps": st["counters"]["steps_decode"],
                "graph_captures": st["runner"]["captures"],
                "host_timing_s": {**{k: round(v, 3) for k, v in st["timing"].items()},
                                  "gil_wait_s": round(st["runner"]["gil_wait_s"], 3)},
            }
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
