"""Tensor-parallel engine: one process per TP rank, rank 0 drives.

Process model: every TP rank holds its Megatron shard of the
weights and of the KV cache (``Hkv / tp`` heads per page -- one replicated head
per rank when ``Hkv < tp``, e.g. Llama-3-70B at TP=8 -- same page ids on every
rank).  Only TP-rank 0 runs the scheduler, the block manager and the runtime;
every rank executes the same forward and meets the others in the per-layer
all-reduces (IPC one-/two-shot kernels with the residual add + RMSNorm fused in,
``parallel/custom_allreduce.py``).  Sampling is distributed
(``parallel/tp_sampling.py``): each rank reduces its vocab slice to candidates,
only those are all-gathered, and every rank picks the same token, which keeps
the device-side token feedback of pipelined decode consistent.

Step channel (no collective, no device sync on the control path): rank 0 writes
each command -- a 16-word header and the step's packed host inputs (the decode
staging buffer, the prefill upload, swap block lists) -- into a host
shared-memory ring (:class:`ShmRing`, one writer, ``tp - 1`` readers, per-reader
consumed counters for flow control).  A worker polls the ring, copies the
payload into its own pinned staging buffer (double-buffered, reused only after
the H2D copy that read it has completed), enqueues the same H2D copy + graph
replay rank 0 enqueued, and goes straight back to the ring: like rank 0 it runs
ahead of its GPU by a step, and nothing on the decode path waits on the device.
The previous design broadcast header and payload over RCCL every step and read
the header back with ``.tolist()`` (a device -> host sync per step per worker).

Commands: ``PREFILL (T,B,maxb,tiles,nsample,len,gather,sampling offset)``,
``MIXED (T,B,Bd,maxb,mbd,tiles,nsample,launch,len)`` (decode rows + prefill
chunks in one forward, the packed upload of ``ModelRunner._mixed_forward``),
``DECODE (nrows,ncols)``, ``EAGER (n,ncols)``, ``SWAP_OUT (handle,n)``,
``SWAP_IN (handle,n)``, ``SWAP_DROP (handle)``, ``STOP``.

Decode graphs are captured in lockstep on all ranks: a worker captures when it
first sees a ``DECODE`` for a (rows, cols) bucket, exactly when rank 0 does, so
the collectives of the warm-up runs pair up.
"""
from __future__ import annotations

import itertools
import logging
import mmap
import os
import time
import uuid

import numpy as np
import torch
import torch.distributed as dist

from ..parallel import state as pstate
from .model_runner import ModelRunner

log = logging.getLogger("omnia.engine.tp")

# OMNIA_TP_TRACE=1: every command rank 0 publishes and every worker receives is
# logged (flushed) to stderr with a timestamp -- after a device fault, the last
# line of each rank names the step it was in
_TRACE = os.environ.get("OMNIA_TP_TRACE") == "1"


def _trace(what: str, cmd: int, vals) -> None:
    import sys

    names = ("STOP", "PREFILL", "DECODE", "EAGER", "SWAP_OUT", "SWAP_IN", "SWAP_DROP", "MIXED")
    sys.stderr.write(f"[tp {os.getpid()} {time.monotonic():.4f}] {what} "
                     f"{names[cmd] if 0 <= cmd < len(names) else cmd} {list(vals)}\n")
    sys.stderr.flush()

STOP, PREFILL, DECODE, EAGER, SWAP_OUT, SWAP_IN, SWAP_DROP, MIXED = range(8)
HDR = 16


class ShmRing:
    """Single-writer / multi-reader command ring in host shared memory.

    Layout: a 4 KiB control page (int64 ``[0]`` = slots published, ``[8 + r]`` =
    slots consumed by reader ``r``, ``[1]`` slot count, ``[2]`` payload bytes per
    slot, ``[3]`` reader count, ``[4]`` writer pid, ``[72 + r]`` reader pids)
    followed by ``nslots`` slots of ``HDR`` int64 + payload.  Ordering: the
    writer stores payload, header, then the published counter; x86-64 keeps
    stores in order and loads in order, so a reader that sees the counter sees
    the slot (asserted at construction: ``hostsync.check_tso``).  Liveness: a
    blocked reader or writer probes the other side's pid once a second and
    raises if it died, instead of spinning forever."""

    CTRL = 4096
    WRITER_PID, READER_PIDS = 4, 72

    def __init__(self, path: str, create: bool, nslots: int = 8, payload: int = 1 << 20,
                 readers: int = 1, reader: int = -1):
        from ..parallel.hostsync import check_tso

        check_tso()
        if readers > 64:
            raise ValueError("ShmRing supports at most 64 readers")
        self.path = path
        if create:
            size = self.CTRL + nslots * (HDR * 8 + payload)
            fd = os.open(path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
            os.ftruncate(fd, size)
        else:
            fd = os.open(path, os.O_RDWR)
            size = os.fstat(fd).st_size
        self.mm = mmap.mmap(fd, size)
        os.close(fd)
        self.ctrl = np.ndarray((self.CTRL // 8,), dtype=np.int64, buffer=self.mm)
        if create:
            self.ctrl[:] = 0
            self.ctrl[1], self.ctrl[2], self.ctrl[3] = nslots, payload, readers
        self.nslots, self.payload, self.readers = (int(self.ctrl[1]), int(self.ctrl[2]),
                                                   int(self.ctrl[3]))
        if create:
            self.ctrl[self.WRITER_PID] = os.getpid()
        if reader >= 0:
            self.ctrl[self.READER_PIDS + reader] = os.getpid()
        self.stride = HDR * 8 + self.payload
        self.hdrs = [np.ndarray((HDR,), dtype=np.int64, buffer=self.mm,
                                offset=self.CTRL + i * self.stride) for i in range(self.nslots)]
        self.bodies = [np.ndarray((self.payload,), dtype=np.uint8, buffer=self.mm,
                                  offset=self.CTRL + i * self.stride + HDR * 8)
                       for i in range(self.nslots)]
        self.stats = {"puts": 0, "full_waits": 0}

    # ------------------------------------------------------------- writer
    def put(self, hdr: list[int], payload: np.ndarray | None = None, timeout_s: float = 600.0):
        seq = int(self.ctrl[0])
        t0 = probe = None
        while seq - int(self.ctrl[8:8 + self.readers].min()) >= self.nslots:
            now = time.monotonic()
            if t0 is None:
                t0, probe = now, now + 1.0
                self.stats["full_waits"] += 1
            elif now - t0 > timeout_s:
                raise TimeoutError("TP command ring full: a worker stopped consuming")
            elif now > probe:
                probe = now + 1.0
                for r in range(self.readers):
                    if seq - int(self.ctrl[8 + r]) >= self.nslots:
                        self._check_alive(self.READER_PIDS + r, f"TP worker (reader {r})")
            time.sleep(0)
        i = seq % self.nslots
        n = 0
        if payload is not None:
            b = payload.reshape(-1).view(np.uint8)
            n = b.size
            if n > self.payload:
                raise ValueError(f"TP step payload {n} B exceeds the ring slot ({self.payload} B)")
            self.bodies[i][:n] = b
        h = self.hdrs[i]
        h[:] = 0
        h[:len(hdr)] = hdr
        h[HDR - 1] = n
        self.ctrl[0] = seq + 1  # publish last
        self.stats["puts"] += 1

    # ------------------------------------------------------------- reader
    def _check_alive(self, idx: int, who: str):
        from ..parallel.hostsync import _alive

        pid = int(self.ctrl[idx])
        if not _alive(pid):
            raise RuntimeError(f"{who} (pid {pid}) died: TP command ring abandoned")

    def get(self, reader: int, spin_s: float = 0.002,
            timeout_s: float | None = None) -> tuple[list[int], np.ndarray]:
        """Next command for ``reader``.  Spins ``spin_s``, then polls with short
        sleeps; an idle server legitimately waits without bound (``timeout_s``
        None), but a dead writer is detected within a second."""
        mine = int(self.ctrl[8 + reader])
        t0 = time.perf_counter()
        probe = t0 + 1.0
        while int(self.ctrl[0]) <= mine:
            now = time.perf_counter()
            if now - t0 > spin_s:
                time.sleep(0.0002)
                if now > probe:
                    probe = now + 1.0
                    self._check_alive(self.WRITER_PID, "TP rank 0 (ring writer)")
                    if timeout_s is not None and now - t0 > timeout_s:
                        raise TimeoutError("TP command ring: no command within the deadline")
        i = mine % self.nslots
        hdr = self.hdrs[i].tolist()
        return hdr, self.bodies[i][:hdr[HDR - 1]]

    def done(self, reader: int):
        """Release the slot returned by the last :meth:`get` (after copying it)."""
        self.ctrl[8 + reader] += 1

    def close(self, unlink: bool = False):
        try:
            self.hdrs = self.bodies = None
            self.ctrl = None
            self.mm.close()
        except (BufferError, ValueError):  # views still alive: the OS reclaims at exit
            pass
        if unlink:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


def _ring_payload_bytes(runner) -> int:
    """Upper bound of one step's payload: the decode staging buffer or a packed
    prefill upload of ``max_prefill_tokens`` tokens (``ModelRunner._prefill_pack``)."""
    T, B, mb = runner.max_prefill_tokens, runner.max_batch, runner.max_blocks
    # (+ B * mb + 2 * B: a mixed step adds the decode rows' block tables and lengths)
    T = T + B  # mixed steps: decode rows ride in front of the prefill tokens
    prefill = 8 * (3 * T + 2 * (B + 1) + 2 * (T // 64 + B + 1) + B + 2 * B * mb + 8 * B + 64)
    return max(runner.dec.nbytes, prefill, 8 * mb + 64)


class TPChannel:
    """Rank 0 -> workers step channel over a :class:`ShmRing` (created by TP rank
    0, its path handed to the group once over the process group)."""

    def __init__(self, device, runner=None, nslots: int = 8):
        st = pstate.get_state()
        self.group = st.tp_group
        self.src = st.rank - st.tp_rank  # global rank of this group's TP-rank 0
        self.reader = st.tp_rank - 1
        self.device = device
        self.is_gpu = device.type == "cuda"
        create = st.tp_rank == 0
        path = [None]
        if create:
            path[0] = f"/dev/shm/omnia-tp-{os.getpid()}-{uuid.uuid4().hex[:10]}"
            self.ring = ShmRing(path[0], True, nslots, _ring_payload_bytes(runner),
                                st.tp_size - 1)
        dist.broadcast_object_list(path, src=self.src, group=self.group)
        if not create:
            self.ring = ShmRing(path[0], False, reader=self.reader)
        pstate.barrier_group(self.group)  # every reader attached before any unlink
        if create:
            os.unlink(path[0])  # the mappings stay valid; nothing is left in /dev/shm

    def send(self, cmd: int, *vals, payload=None):
        if _TRACE:
            _trace("send", cmd, vals)
        if isinstance(payload, torch.Tensor):
            payload = payload.numpy() if payload.device.type == "cpu" else \
                payload.cpu().numpy()
        self.ring.put([cmd] + [int(v) for v in vals], payload)

    def recv(self) -> tuple[list[int], np.ndarray]:
        return self.ring.get(self.reader)

    def release(self):
        self.ring.done(self.reader)


class TPModelRunner(ModelRunner):
    """Rank-0 runner: publishes every step to the TP workers."""

    fused_launch = False

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.chan = TPChannel(self.device, self)

    def _prefill_forward(self, t, meta, gather: bool = True):
        # header: T, B, maxb, tiles, n_sample, payload len, gather flag, sampling offset
        host = self._prefill_host if self._prefill_host is not None else t.cpu()
        self.chan.send(PREFILL, *meta[:5], t.numel(), int(gather),
                       meta[5] if len(meta) > 5 else 0, payload=host)
        return super()._prefill_forward(t, meta, gather)

    def _mixed_forward_packed(self, t, meta, host=None):
        if host is None:
            host = t.cpu()
        self.chan.send(MIXED, *meta, host.numel(), payload=host)
        return super()._mixed_forward_packed(t, meta, host)

    def _before_replay(self, nrows, ncols, st=None):
        self.chan.send(DECODE, nrows, ncols, payload=(st or self.dec).host)

    def _before_eager(self, n, ncols, st=None):
        self.chan.send(EAGER, n, ncols, payload=(st or self.dec).host)

    def shutdown(self):
        self.chan.send(STOP)


class TPWorker(ModelRunner):
    """TP ranks > 0: replay rank 0's command stream until STOP."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.chan = TPChannel(self.device, self)
        self.swapped: dict[int, torch.Tensor] = {}
        self.swap = None
        self.wflip = 0
        self.wevents = [None, None]

    def _stage_in(self, body: np.ndarray):
        """Payload -> this worker's pinned staging (the buffer of two steps ago,
        once its H2D has completed) -> H2D into the device twin the graphs read."""
        slot = self.wflip
        self.wflip ^= 1
        st = self.stage[slot]
        if self.wevents[slot] is not None:
            self.wevents[slot].synchronize()
        st.host.numpy()[:body.size] = body
        self.chan.release()
        self.dec.dev.copy_(st.host, non_blocking=True)
        if self.is_gpu:
            self.wevents[slot] = self._event()

    def run(self):
        while True:
            h, body = self.chan.recv()
            cmd = h[0]
            if _TRACE:
                _trace("recv", cmd, h[1:10])
            if cmd == STOP:
                self.chan.release()
                return
            if cmd == PREFILL:
                T, B, maxb, tiles, ns, n, gather, so = h[1:9]
                host = torch.from_numpy(body.view(np.int64)[:n].copy())
                self.chan.release()
                t = host.pin_memory().to(self.device, non_blocking=True) if self.is_gpu \
                    else host
                meta = (T, B, maxb, tiles, ns, so)
                lg = ModelRunner._prefill_forward(self, t, meta, bool(gather))
                if not gather and ns:
                    self._prefill_tp_sample(t, meta, lg)  # collective: mirror rank 0
            elif cmd == DECODE:
                self._stage_in(body)
                self._replay(h[1], h[2])
            elif cmd == EAGER:
                self._stage_in(body)
                self._eager_forward(h[1], h[2])
            elif cmd == MIXED:
                meta = tuple(h[1:9])
                n = h[9]
                host = torch.from_numpy(body.view(np.int64)[:n].copy())
                self.chan.release()
                t = host.pin_memory().to(self.device, non_blocking=True) if self.is_gpu \
                    else host
                ModelRunner._mixed_forward_packed(self, t, meta)
            elif cmd in (SWAP_OUT, SWAP_IN):
                blocks = body.view(np.int64)[:h[2]].tolist()
                self.chan.release()
                if cmd == SWAP_OUT:
                    self.swapped[h[1]] = self.swap.swap_out(blocks)
                else:
                    self.swap.swap_in(self.swapped.pop(h[1]), blocks)
            elif cmd == SWAP_DROP:
                self.chan.release()
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

    @staticmethod
    def _blocks(blocks):
        return np.asarray(blocks, dtype=np.int64)

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
    """Every TP rank must allocate the same page ids: take the minimum (a host
    collective: the group may be gloo)."""
    st = pstate.get_state()
    if st.tp_size == 1:
        return nb
    vals = [None] * st.tp_size
    dist.all_gather_object(vals, int(nb), group=st.tp_group)
    return int(min(vals))


def run_worker(cfg, model_cfg=None, weights=None):
    """Entry point for TP ranks > 0 (returns when rank 0 shuts down)."""
    from ..models import build_model
    from ..models.llama import KVCache
    from .engine import LLMEngine, engine_model_config

    model_cfg = engine_model_config(cfg, model_cfg)
    dev = LLMEngine._pick_device(cfg)
    dtype = getattr(torch, cfg.dtype)
    if dev.type == "cuda":
        from ..ops.gemm_tuning import enable_tuned_gemms

        enable_tuned_gemms(dev.index or 0)
    if weights is None and cfg.checkpoint:  # this rank's shard, sliced on load
        from ..models.loader import load_hf_checkpoint

        st = pstate.get_state()
        weights = load_hf_checkpoint(cfg.checkpoint, model_cfg, st.tp_size, st.tp_rank, dev,
                                     dtype)
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
    try:
        w.run()
    finally:
        w.chan.ring.close()


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
