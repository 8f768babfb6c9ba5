"""Tensor-parallel engine: one process per GPU, rank 0 drives.

Process model: every TP rank holds its Megatron shard of the
weights and of the KV cache (``Hkv / tp`` heads per page, same page ids on every
rank).  Only TP-rank 0 runs the scheduler, the block manager and the runtime;
each step it broadcasts the step's packed inputs to the other ranks over the TP
group (RCCL on GPU, gloo on CPU) and every rank then executes the same forward,
meeting in the per-layer all-reduces (IPC one-/two-shot kernels with the
residual add + RMSNorm fused in, ``parallel/custom_allreduce.py``).  Decode
inputs are broadcast straight from rank 0's device staging buffer into the
workers' (one small collective per step, stream-ordered before the graph
replay), so the workers' captured graphs read identical inputs.  Sampling is
distributed (``parallel/tp_sampling.py``): each rank reduces its vocab slice to
candidates, only those are all-gathered, and every rank picks the same token,
which keeps the device-side token feedback of pipelined decode consistent.

Commands (int64 header of 16 words, then an optional payload):
``PREFILL (T,B,maxb,tiles,nsample,len)``, ``DECODE (nrows,ncols)``,
``EAGER (n,ncols)``, ``SWAP_OUT (handle,n)``, ``SWAP_IN (handle,n)``,
``SWAP_DROP (handle)``, ``STOP``.

RCCL and hipGraph capture: decode graphs are captured in lockstep on all ranks
(the capture is itself driven by the broadcast command stream).  Set
``EngineConfig.use_graphs=False`` to run TP decode eagerly.
"""
from __future__ import annotations

import itertools
import logging

import torch
import torch.distributed as dist

from ..parallel import state as pstate
from .model_runner import ModelRunner

log = logging.getLogger("omnia.engine.tp")

STOP, PREFILL, DECODE, EAGER, SWAP_OUT, SWAP_IN, SWAP_DROP = range(7)
HDR = 16


class TPChannel:
    def __init__(self, device):
        st = pstate.get_state()
        self.group = st.tp_group
        self.src = st.rank - st.tp_rank  # global rank of this group's TP-rank 0
        self.device = device
        self.is_gpu = device.type == "cuda"
        self.hdr = torch.zeros(HDR, dtype=torch.int64, device=device)
        self.hdr_host = torch.zeros(HDR, dtype=torch.int64, pin_memory=self.is_gpu)

    def send(self, cmd: int, *vals, payload: torch.Tensor | None = None):
        self.hdr_host.zero_()
        self.hdr_host[0] = cmd
        for i, v in enumerate(vals):
            self.hdr_host[1 + i] = int(v)
        self.hdr.copy_(self.hdr_host, non_blocking=self.is_gpu)
        dist.broadcast(self.hdr, self.src, group=self.group)
        if payload is not None:
            dist.broadcast(payload, self.src, group=self.group)

    def recv(self) -> list[int]:
        dist.broadcast(self.hdr, self.src, group=self.group)
        return self.hdr.tolist()

    def recv_into(self, t: torch.Tensor):
        dist.broadcast(t, self.src, group=self.group)
        return t


class TPModelRunner(ModelRunner):
    """Rank-0 runner: broadcasts every step to the TP workers."""

    fused_launch = False

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.chan = TPChannel(self.device)

    def _prefill_forward(self, t, meta, gather: bool = True):
        # header: T, B, maxb, tiles, n_sample, payload len, gather flag, sampling offset
        self.chan.send(PREFILL, *meta[:5], t.numel(), int(gather),
                       meta[5] if len(meta) > 5 else 0, payload=t)
        return super()._prefill_forward(t, meta, gather)

    def _before_replay(self, nrows, ncols):
        self.chan.send(DECODE, nrows, ncols, payload=self.dec.dev)

    def _before_eager(self, n, ncols):
        self.chan.send(EAGER, n, ncols, payload=self.dec.dev)

    def shutdown(self):
        self.chan.send(STOP)


class TPWorker(ModelRunner):
    """TP ranks > 0: replay rank 0's command stream until STOP."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.chan = TPChannel(self.device)
        self.swapped: dict[int, torch.Tensor] = {}
        self.swap = None

    def run(self):
        while True:
            h = self.chan.recv()
            cmd = h[0]
            if cmd == STOP:
                return
            if cmd == PREFILL:
                T, B, maxb, tiles, ns, n, gather, so = h[1:9]
                t = torch.empty(n, dtype=torch.int64, device=self.device)
                self.chan.recv_into(t)
                meta = (T, B, maxb, tiles, ns, so)
                lg = ModelRunner._prefill_forward(self, t, meta, bool(gather))
                if not gather and ns:
                    self._prefill_tp_sample(t, meta, lg)  # collective: mirror rank 0
            elif cmd == DECODE:
                self.chan.recv_into(self.dec.dev)
                self._replay(h[1], h[2])
            elif cmd == EAGER:
                self.chan.recv_into(self.dec.dev)
                self._eager_forward(h[1], h[2])
            elif cmd == SWAP_OUT:
                blocks = torch.empty(h[2], dtype=torch.int64, device=self.device)
                self.chan.recv_into(blocks)
                self.swapped[h[1]] = self.swap.swap_out(blocks.tolist())
            elif cmd == SWAP_IN:
                blocks = torch.empty(h[2], dtype=torch.int64, device=self.device)
                self.chan.recv_into(blocks)
                self.swap.swap_in(self.swapped.pop(h[1]), blocks.tolist())
            elif cmd == SWAP_DROP:
                self.swap.drop(self.swapped.pop(h[1], None))
            else:
                raise RuntimeError(f"unknown TP command {cmd}")


class TPSwapProxy:
    """Wraps rank 0's SwapSpace so every KV shard moves with it."""

    def __init__(self, swap, chan: TPChannel):
        self.inner = swap
        self.chan = chan
        self.ids = itertools.count(1)
        self.handle_of: dict[int, int] = {}

    def __getattr__(self, k):
        return getattr(self.inner, k)

    def can_hold(self, n_pages):
        while self.inner.used + n_pages > self.inner.capacity_pages and self.inner.parked:
            _, s = self.inner.parked.popitem(last=False)
            self.drop(s.swapped)
        return self.inner.used + n_pages <= self.inner.capacity_pages

    def _blocks(self, blocks):
        return torch.tensor(blocks, dtype=torch.int64, device=self.chan.device)

    def swap_out(self, blocks):
        h = next(self.ids)
        self.chan.send(SWAP_OUT, h, len(blocks), payload=self._blocks(blocks))
        host = self.inner.swap_out(blocks)
        self.handle_of[id(host)] = h
        return host

    def swap_in(self, host, blocks):
        h = self.handle_of.pop(id(host))
        self.chan.send(SWAP_IN, h, len(blocks), payload=self._blocks(blocks))
        self.inner.swap_in(host, blocks)

    def drop(self, host):
        if host is None:
            return
        h = self.handle_of.pop(id(host), None)
        if h is not None:
            self.chan.send(SWAP_DROP, h)
        self.inner.drop(host)


def agree_num_blocks(nb: int, device) -> int:
    """Every TP rank must allocate the same page ids: take the minimum."""
    st = pstate.get_state()
    if st.tp_size == 1:
        return nb
    t = torch.tensor([nb], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.tp_group)
    return int(t.item())


def run_worker(cfg, model_cfg=None, weights=None):
    """Entry point for TP ranks > 0 (returns when rank 0 shuts down)."""
    from ..models import build_model
    from ..models.config import resolve
    from ..models.llama import KVCache
    from .engine import LLMEngine

    model_cfg = model_cfg or resolve(cfg.model)
    dev = LLMEngine._pick_device(cfg)
    dtype = getattr(torch, cfg.dtype)
    if dev.type == "cuda":
        from ..ops.gemm_tuning import enable_tuned_gemms

        enable_tuned_gemms(dev.index or 0)
    model = build_model(model_cfg, device=dev, dtype=dtype, seed=cfg.seed, weights=weights,
                        decode_part_size=cfg.decode_part_size)
    nb = cfg.num_blocks or LLMEngine.kv_pool_blocks(cfg, model_cfg, model.tp, dev, dtype)
    nb = agree_num_blocks(nb, dev)
    kv = KVCache.allocate(model_cfg, nb, cfg.block_size, dev, tp_size=model.tp, dtype=dtype)
    w = TPWorker(model, kv, max_batch=cfg.max_batch, max_model_len=cfg.max_model_len,
                 use_graphs=cfg.use_graphs, max_prefill_tokens=cfg.max_prefill_tokens)
    if cfg.swap_gib > 0 and dev.type == "cuda":
        from .swap import SwapSpace

        w.swap = SwapSpace(kv, cfg.swap_gib)
    log.info("TP worker rank %d ready (%d KV blocks)", pstate.get_state().rank, nb)
    w.run()


def start(cfg, model_cfg=None, weights=None):
    """Process entry: rank 0 gets an ``LLMEngine``; other TP ranks serve as
    workers and get ``None`` once rank 0 shuts down (the caller should exit)."""
    from .engine import LLMEngine

    dev = LLMEngine._pick_device(cfg)
    st = LLMEngine._ensure_parallel(cfg, dev)
    if st.tp_size > 1 and st.tp_rank != 0:
        run_worker(cfg, model_cfg, weights)
        return None
    return LLMEngine(cfg, model_cfg, weights)
