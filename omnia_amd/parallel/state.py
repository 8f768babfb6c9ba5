"""Process-group state: one process per GPU, ``torch.distributed`` over RCCL.

Scaling model (MI355X-first):
  * DP  -- independent engine replicas, one per GPU (Llama-3-8B fits one GPU
           with ~250 GB left for KV); sessions are routed session-affine.
  * TP  -- Megatron column/row split (QKV & gate-up column, O & down row),
           two all-reduces per layer.  Decode-size all-reduces use the one-shot
           IPC all-reduce in :mod:`omnia_amd.parallel.custom_allreduce`; RCCL for
           the rest (and as its oracle).
  * EP  -- Mixtral experts spread over the TP group, token dispatch/combine by
           all-to-all (:mod:`omnia_amd.parallel.expert`).
The backend string ``"nccl"`` IS RCCL on ROCm; ``gloo`` drives the CPU tests.

TP device transport (``ParallelState.transport``):
  * ``"rccl"`` -- one GPU per rank: decode-size collectives on the IPC kernels,
    prefill-size all-reduces and gathers on RCCL;
  * ``"ipc"``  -- ranks SHARE devices (more TP ranks than visible GPUs, e.g. a
    TP=8 engine rehearsed on one MI355X, or ``OMNIA_TP_TRANSPORT=ipc``): RCCL
    cannot place two ranks on one device, so the process group is gloo (host
    control only) and EVERY device collective runs on the IPC kernels
    (slot-chunked all-reduce, IPC all-gather).

Transport selection: ``OMNIA_TP_TRANSPORT`` wins; else ``ipc`` when the
launcher's ``LOCAL_WORLD_SIZE`` exceeds the visible device count, else ``rccl``
(also when ``LOCAL_WORLD_SIZE`` is absent: a plain multi-node launch is one
rank per GPU).  The choice is then CHECKED by device identity: every rank
publishes ``(host, device uuid)`` over a gloo side group, and ``rccl`` with two
ranks on one device raises with the fix instead of failing inside RCCL's
communicator init.  The chosen transport is logged once per rank.
"""
from __future__ import annotations

import datetime
import logging
import os
import socket
from dataclasses import dataclass

import torch
import torch.distributed as dist


log = logging.getLogger("omnia.parallel")


def _device_identity() -> str:
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    uid = getattr(props, "uuid", None)
    if uid is not None:
        return str(uid)
    bus = getattr(props, "pci_bus_id", None)
    return f"pci:{getattr(props, 'pci_domain_id', 0)}:{bus}" if bus is not None else \
        f"idx:{os.environ.get('HIP_VISIBLE_DEVICES', '')}:{torch.cuda.current_device()}"


def check_transport(transport: str, idents: list) -> None:
    """Raise if ``transport`` cannot run on the ranks' devices: ``rccl`` needs
    one rank per device.  ``idents`` = every rank's ``(host, device id)``."""
    if transport != "rccl":
        return
    seen: dict = {}
    for r, key in enumerate(idents):
        if tuple(key) in seen:
            raise RuntimeError(
                f"ranks {seen[tuple(key)]} and {r} share device {key[1]} on {key[0]}: RCCL "
                "places one rank per device -- set OMNIA_TP_TRANSPORT=ipc (or launch with "
                "LOCAL_WORLD_SIZE set) to run shared-device ranks on the IPC collectives")
        seen[tuple(key)] = r


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: object = None
    dp_group: object = None
    backend: str = "none"
    custom_ar: object = None  # CustomAllReduce when available
    dp_comm: object = None  # IPC collectives over the DP group (EP all-to-all, CP ring)
    transport: str = "none"  # TP device collectives: "rccl" | "ipc" | "gloo" (CPU)

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def set_state(st: ParallelState) -> None:
    global _STATE
    _STATE = st


def env_world() -> tuple[int, int, int]:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def init_distributed(tp_size: int = 1, backend: str | None = None, device: str | None = None,
                     timeout_s: int = 600) -> ParallelState:
    """Initialise torch.distributed from torchrun env vars and carve TP/DP groups.

    Ranks [k*tp, (k+1)*tp) form TP group k; ranks with equal tp_rank form a DP group.

    RCCL failure detection (SURVEY §5.3 [design]): the ``nccl`` process group's
    watchdog thread polls the communicators' async error state
    (``ncclCommGetAsyncError``, which is RCCL's) and the ``timeout_s`` of every
    collective. PyTorch's default ``TORCH_NCCL_ASYNC_ERROR_HANDLING`` tears the
    rank down on either. The engine's step watchdog (``engine/engine.py``) then
    reports the pod unhealthy, so a lost peer fails the pod instead of hanging
    it.
    """
    ws, rank, local = env_world()
    if ws % tp_size:
        raise ValueError(f"world_size {ws} not divisible by tp_size {tp_size}")
    use_gpu = device != "cpu" and torch.cuda.is_available()
    ndev = torch.cuda.device_count() if use_gpu else 0
    transport = "gloo"
    if use_gpu:
        lws = os.environ.get("LOCAL_WORLD_SIZE")
        shared = lws is not None and ndev < int(lws)
        transport = os.environ.get("OMNIA_TP_TRANSPORT") or ("ipc" if shared else "rccl")
    if backend is None:
        backend = "nccl" if use_gpu and transport == "rccl" else "gloo"
    if use_gpu:
        torch.cuda.set_device(local % max(1, ndev))
    st = ParallelState(world_size=ws, rank=rank, local_rank=local, tp_size=tp_size,
                       tp_rank=rank % tp_size, dp_size=ws // tp_size, dp_rank=rank // tp_size,
                       backend=backend if ws > 1 else "none",
                       transport=transport if ws > 1 else "none")
    if ws > 1:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            kw = {}
            if use_gpu and backend == "nccl":
                kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
            dist.init_process_group(backend=backend, rank=rank, world_size=ws,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        if use_gpu:
            # device identity check over a host-only side group (no RCCL comm yet)
            side = dist.new_group(backend="gloo") if backend != "gloo" else None
            idents = [None] * ws
            dist.all_gather_object(idents, (socket.gethostname(), _device_identity()),
                                   group=side)
            check_transport(transport, idents)
            if transport == "ipc" and len({tuple(x) for x in idents}) == ws and \
                    not os.environ.get("OMNIA_TP_TRANSPORT"):
                log.warning("transport ipc inferred (LOCAL_WORLD_SIZE > visible devices) but "
                            "every rank has its own device (per-rank visibility?): set "
                            "OMNIA_TP_TRANSPORT=rccl to run the large collectives on RCCL")
            if side is not None:
                dist.destroy_process_group(side)
            log.info("rank %d: transport %s (backend %s, %d rank(s) per device)", rank,
                     transport, backend, sum(1 for x in idents if x == idents[rank]))
        for k in range(ws // tp_size):
            ranks = list(range(k * tp_size, (k + 1) * tp_size))
            g = dist.new_group(ranks) if tp_size > 1 else None
            if rank in ranks:
                st.tp_group = g
        for t in range(tp_size):
            ranks = list(range(t, ws, tp_size))
            g = dist.new_group(ranks) if len(ranks) > 1 else None
            if rank in ranks:
                st.dp_group = g
        if use_gpu and tp_size > 1 and (transport == "ipc" or
                                        os.environ.get("OMNIA_CUSTOM_AR", "1") == "1"):
            # one-/two-shot IPC all-reduce for decode-size TP collectives (RCCL for
            # prefill-size messages and as the correctness oracle in the tests)
            from .custom_allreduce import CustomAllReduce

            st.custom_ar = CustomAllReduce(st.tp_group)
        if use_gpu and transport == "ipc" and st.dp_size > 1:
            # DP-attention + EP all-to-all and the context-parallel ring run over the
            # DP group; ranks sharing a device cannot use RCCL, so they get the IPC
            # all-to-all / point-to-point kernels (one region per rank)
            from .custom_allreduce import CustomAllReduce

            st.dp_comm = CustomAllReduce(st.dp_group, max_bytes=16 << 20)
    set_state(st)
    return st


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    if st.custom_ar is not None and x.is_cuda and st.custom_ar.should_use(x):
        return st.custom_ar.all_reduce(x)
    if st.transport == "ipc" and x.is_cuda:
        if x.dtype != torch.bfloat16 or not x.is_contiguous() or x.numel() % 8:
            raise ValueError("ipc TP transport all-reduces contiguous bf16 tensors (n % 8 == 0)")
        return st.custom_ar.all_reduce_any(x)
    dist.all_reduce(x, group=st.tp_group)
    return x


def tp_all_gather(x: torch.Tensor) -> torch.Tensor:
    """``[tp, *x.shape]``: every TP rank's ``x`` in rank order."""
    st = _STATE
    if st.tp_size == 1:
        return x.unsqueeze(0)
    if x.is_cuda and st.custom_ar is not None and (
            st.transport == "ipc" or x.numel() * x.element_size() <= 256 << 10):
        return st.custom_ar.all_gather(x)
    x = x.contiguous()
    if x.is_cuda:
        out = torch.empty((st.tp_size,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out.view(-1), x.view(-1), group=st.tp_group)
        return out
    parts = [torch.empty_like(x) for _ in range(st.tp_size)]
    dist.all_gather(parts, x, group=st.tp_group)
    return torch.stack(parts)


def tp_all_reduce_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                              eps: float) -> torch.Tensor:
    """TP layer boundary: ``residual += allreduce(x)``; returns RMSNorm(residual) * w.
    One fused IPC kernel for decode-size messages, RCCL + the fused add-norm
    kernel otherwise."""
    st = _STATE
    from .. import ops

    if st.tp_size > 1 and st.custom_ar is not None and x.is_cuda and \
            st.custom_ar.can_fuse_norm(x):
        return st.custom_ar.all_reduce_add_rmsnorm(x, residual, w, eps)
    x = tp_all_reduce(x)
    ops.fused_add_rmsnorm(x, residual, w, eps)
    return x


def tp_all_gather_lastdim(x: torch.Tensor) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    g = tp_all_gather(x)  # [tp, ..., n]
    return torch.cat(list(g.unbind(0)), dim=-1)


def shard_range(total: int, parts: int, idx: int) -> tuple[int, int]:
    if total % parts:
        raise ValueError(f"{total} not divisible by {parts}")
    n = total // parts
    return idx * n, (idx + 1) * n


def barrier():
    if dist.is_initialized():
        dist.barrier()


def barrier_group(group):
    if dist.is_initialized():
        dist.barrier(group=group)


def ranks_per_device() -> int:
    """TP ranks sharing one device under the ``ipc`` transport (else 1)."""
    st = _STATE
    if st.transport != "ipc" or not torch.cuda.is_available():
        return 1
    return max(1, -(-st.tp_size // max(1, torch.cuda.device_count())))
