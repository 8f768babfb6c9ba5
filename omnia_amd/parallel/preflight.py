"""Multi-GPU first-contact preflight (:245-249 / :873-883).

Before a multi-GPU job's serving pods start, every rank runs this module in a
FRESH child process (``python -m omnia_amd.parallel.preflight``) that:

  1. records the peer-access matrix of the devices it can see
     (``hipDeviceCanAccessPeer`` via ``torch.cuda.can_device_access_peer``);
  2. initialises RCCL (the ``nccl`` backend) across all N ranks;
  3. runs one RCCL all-reduce and checks it against the closed form;
  4. runs one IPC one-shot / two-shot all-reduce (``comm.hip`` over xGMI peer
     memory, :class:`~omnia_amd.parallel.custom_allreduce.CustomAllReduce`)
     and checks it bit-for-bit against RCCL's result;
  5. times both at 16 KiB (the decode all-reduce) and 32 MiB (a prefill chunk).

The child exits before any engine touches the device, so the communicator and
IPC buffers it created never coexist with the serving pods.  Each step records
its own failure, so one broken link or peer shows up as a per-rank error line
instead of a hung job.  ``bench.py`` puts ``rccl_world``, ``p2p_ok`` and the
latencies in its JSON (outside the timed region).

On CPU (tests) the same plumbing runs over ``gloo`` with the device steps
skipped.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time
from datetime import timedelta

SIZES = (16 << 10, 32 << 20)


def _label(n: int) -> str:
    return f"{n >> 20}MiB" if n >= 1 << 20 else f"{n >> 10}KiB"


def _time(fn, device, iters: int) -> float:
    import torch

    for _ in range(3):
        fn()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize(device)
        return e0.elapsed_time(e1) * 1000.0 / iters
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t) * 1e6 / iters


def run(rank: int, world: int, local: int, port: int, backend: str = "nccl",
        timeout_s: float = 120.0, sizes=SIZES, iters: int = 20) -> dict:
    """One rank's preflight; returns its report (never raises)."""
    import torch
    import torch.distributed as dist

    rep = {"rank": rank, "world": world, "local_rank": local, "backend": backend,
           "errors": [], "p2p": None, "rccl_world": None, "rccl_ok": None, "ipc_ok": None,
           "rccl_allreduce_us": {}, "ipc_allreduce_us": {}}
    inject = os.environ.get("OMNIA_PREFLIGHT_INJECT", "")  # "<rank>:<step>" (tests)
    fail_at = inject.split(":", 1)[1] if inject.split(":", 1)[0] == str(rank) else ""
    use_gpu = backend == "nccl"
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    t0 = time.perf_counter()
    try:
        if use_gpu:
            torch.cuda.set_device(device)
            n = torch.cuda.device_count()
            rep["device_count"] = n
            rep["p2p"] = [[i == j or bool(torch.cuda.can_device_access_peer(i, j))
                           for j in range(n)] for i in range(n)]
    except Exception as e:  # noqa: BLE001 - reported, not raised
        rep["errors"].append(f"p2p: {e}")
    try:
        if fail_at == "init":
            raise RuntimeError("injected init failure")
        kw = {"device_id": device} if use_gpu else {}
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world, timeout=timedelta(seconds=timeout_s), **kw)
        rep["rccl_world"] = dist.get_world_size()
    except Exception as e:  # noqa: BLE001
        rep["errors"].append(f"init: {e}")
        rep["elapsed_s"] = round(time.perf_counter() - t0, 2)
        return rep
    want_val = world * (world + 1) / 2
    ref = {}
    try:
        ok = True
        for sz in sizes:
            x = torch.full((sz // 2,), float(rank + 1), dtype=torch.bfloat16, device=device)
            y = x.clone()
            dist.all_reduce(y)
            good = bool((y.float() == want_val).all())
            if fail_at == "rccl":
                good = False
            ok &= good
            ref[sz] = y
            buf = x.clone()
            rep["rccl_allreduce_us"][_label(sz)] = round(_time(
                lambda b=buf: dist.all_reduce(b), device, iters), 1)
        rep["rccl_ok"] = ok
        if not ok:
            rep["errors"].append("rccl: all-reduce result mismatch")
    except Exception as e:  # noqa: BLE001
        rep["errors"].append(f"rccl: {e}")
    if use_gpu:
        try:
            from .custom_allreduce import CustomAllReduce

            car = CustomAllReduce(device=device, max_bytes=max(sizes))
            ok = True
            for sz in sizes:
                x = torch.full((sz // 2 // 4096, 4096) if sz >= 1 << 20 else (sz // 2,),
                               float(rank + 1), dtype=torch.bfloat16, device=device)
                out = torch.empty_like(x)
                car.all_reduce(x, out)
                torch.cuda.synchronize(device)
                good = sz in ref and torch.equal(out.view(-1), ref[sz].view(-1))
                if fail_at == "ipc":
                    good = False
                ok &= good
                rep["ipc_allreduce_us"][_label(sz)] = round(_time(
                    lambda a=x, o=out: car.all_reduce(a, o), device, iters), 1)
            car.check()
            car.close()
            rep["ipc_ok"] = ok
            if not ok:
                rep["errors"].append("ipc: one-shot result differs from RCCL")
        except Exception as e:  # noqa: BLE001
            rep["errors"].append(f"ipc: {e}")
    try:
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        rep["errors"].append(f"teardown: {e}")
    rep["elapsed_s"] = round(time.perf_counter() - t0, 2)
    return rep


def spawn(rank: int, world: int, local: int, port: int, backend: str = "nccl",
          timeout_s: float = 120.0, env: dict | None = None) -> dict:
    """Run one rank's preflight in a fresh child process and return its report;
    a child that dies or overruns is reported as that rank's error."""
    import tempfile

    fd, path = tempfile.mkstemp(prefix=f"omnia-preflight-r{rank}-", suffix=".json")
    os.close(fd)
    cmd = [sys.executable, "-m", "omnia_amd.parallel.preflight", "--rank", str(rank),
           "--world", str(world), "--local", str(local), "--port", str(port),
           "--backend", backend, "--timeout", str(timeout_s), "--out", path]
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    penv = dict(os.environ if env is None else env)
    penv["PYTHONPATH"] = root + os.pathsep + penv.get("PYTHONPATH", "")
    try:
        p = subprocess.run(cmd, env=penv, timeout=timeout_s + 60, capture_output=True,
                           text=True)
        rc, tail = p.returncode, (p.stderr or "")[-400:]
    except subprocess.TimeoutExpired:
        rc, tail = None, "timeout"
    except OSError as e:  # the child could not even start
        rc, tail = None, f"spawn failed: {e}"
    rep = None
    try:
        with open(path) as f:
            rep = json.load(f)
    except (OSError, ValueError):
        pass
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
    if rep is None:
        rep = {"rank": rank, "world": world, "local_rank": local, "backend": backend,
               "errors": [f"preflight child exited rc={rc}: {tail.strip()[-300:]}"],
               "rccl_world": None, "rccl_ok": None, "ipc_ok": None, "p2p": None,
               "rccl_allreduce_us": {}, "ipc_allreduce_us": {}}
    elif rc not in (0, None) and not rep["errors"]:
        rep["errors"].append(f"preflight child exited rc={rc}")
    return rep


def summarize(reports: list[dict]) -> dict:
    """The job-level preflight record (bench JSON ``preflight``)."""
    reports = sorted(reports, key=lambda r: r.get("rank", 0))
    worlds = {r.get("rccl_world") for r in reports}
    p2p = [r.get("p2p") for r in reports if r.get("p2p") is not None]
    p2p_ok = None
    if p2p:
        locals_ = [r.get("local_rank", 0) for r in reports if r.get("p2p") is not None]
        p2p_ok = all(m[i][j] for m in p2p for i in locals_ for j in locals_
                     if i < len(m) and j < len(m[i]))

    def worst(key):
        out = {}
        for r in reports:
            for k, v in (r.get(key) or {}).items():
                out[k] = max(out.get(k, 0.0), v)
        return out

    return {
        "ranks": len(reports),
        "rccl_world": worlds.pop() if len(worlds) == 1 else sorted(worlds, key=str),
        "p2p_ok": p2p_ok,
        "rccl_ok": all(r.get("rccl_ok") for r in reports),
        "ipc_ok": (all(r.get("ipc_ok") for r in reports)
                   if any(r.get("ipc_ok") is not None for r in reports) else None),
        "rccl_allreduce_us_max": worst("rccl_allreduce_us"),
        "ipc_allreduce_us_max": worst("ipc_allreduce_us"),
        "failures": [{"rank": r.get("rank"), "errors": r["errors"]} for r in reports
                     if r.get("errors")],
        "p2p_matrix_rank0": reports[0].get("p2p") if reports else None,
    }


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--local", type=int, default=0)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    rep = run(a.rank, a.world, a.local, a.port, a.backend, a.timeout)
    with open(a.out, "w") as f:
        json.dump(rep, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
