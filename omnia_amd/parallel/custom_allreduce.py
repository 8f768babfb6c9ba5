"""One-shot intra-node all-reduce over xGMI peer memory.

RCCL's ring/tree all-reduce pays per-step link latency that dominates the tiny
decode all-reduces of tensor parallelism (2 per layer, B x d bf16 -- 16 KiB per
sequence for Llama-3-70B).  MI355X nodes are a FULL xGMI mesh (7 links per
GPU), so the latency-optimal algorithm is one hop: every rank publishes its
input in an IPC-exported fine-grained buffer and reads every peer's buffer
directly (kernel + protocol in ``ops/csrc/comm.hip``).  Messages above
``max_bytes`` (prefill) go to RCCL, which is also this op's correctness oracle
in the tests.

Above ``oneshot_max`` (256 KiB) the one-shot read volume ((world-1) x n per
rank) loses to a two-shot reduce-scatter + all-gather (2 (world-1)/world x n),
so 2-D messages switch to the two-shot kernel.  ``all_reduce_add_rmsnorm``
fuses the decoder's residual add + RMSNorm into the two-shot reduce (the rank
that owns a row chunk normalises it; everyone gathers output and residual), so
a tensor-parallel layer boundary is one kernel instead of all-reduce + norm.

Handles are exchanged once over the TP group (any backend: gloo on CPU tests,
RCCL on the node); the per-call path is one kernel launch with no host sync, so
it is captured into the engine's decode hipGraphs.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class CustomAllReduce:
    """One-shot all-reduce for bf16 tensors of at most ``max_bytes``."""

    def __init__(self, group=None, device=None, max_bytes: int = 8 << 20,
                 oneshot_max: int = 256 << 10):
        from .. import ops

        self.k = ops.kernels()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.world > self.k.ar_max_ranks():
            raise ValueError(f"one-shot all-reduce supports <= {self.k.ar_max_ranks()} ranks")
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.slot_bytes = (max_bytes + 15) // 16 * 16
        self.oneshot_max = oneshot_max
        with torch.cuda.device(self.device):
            self.base = self.k.ipc_alloc(self.k.ar_region_bytes(self.slot_bytes))
            handle = self.k.ipc_get_handle(self.base)
            if self.world > 1:
                handles = [None] * self.world
                dist.all_gather_object(handles, handle, group=group)
            else:
                handles = [handle]
            self.opened = []
            ptrs = []
            for p, h in enumerate(handles):
                if p == self.rank:
                    ptrs.append(self.base)
                else:
                    ptr = self.k.ipc_open(h)
                    self.opened.append(ptr)
                    ptrs.append(ptr)
            self.regions = torch.tensor(ptrs, dtype=torch.int64)
            self.epochs = torch.zeros(self.k.ar_blocks(), dtype=torch.int32, device=self.device)
            self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.max_bytes = self.slot_bytes
        self.closed = False

    def should_use(self, x: torch.Tensor) -> bool:
        n = x.numel()
        return (not self.closed and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and n % 8 == 0 and 2 * n <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None,
                   algo: str | None = None) -> torch.Tensor:
        """In place when ``out`` is None (same contract as ``dist.all_reduce``).
        ``algo``: "oneshot" / "twoshot" / None (by size: two-shot above
        ``oneshot_max`` for 2-D tensors)."""
        out = x if out is None else out
        if algo is None:
            algo = "twoshot" if (x.dim() == 2 and 2 * x.numel() > self.oneshot_max) else "oneshot"
        if algo == "twoshot":
            self.k.ar_twoshot(out, x, None, None, self.regions, self.epochs, self.err,
                              self.slot_bytes, self.rank, 0.0)
        else:
            self.k.ar_oneshot(out, x, self.regions, self.epochs, self.err, self.slot_bytes,
                              self.rank)
        return out

    def all_reduce_any(self, x: torch.Tensor) -> torch.Tensor:
        """In-place all-reduce of ANY size: messages above one slot run as a
        sequence of slot-sized one-shot launches over the flat tensor (the
        ``ipc`` TP transport, where ranks may share a device and RCCL cannot be
        used at all)."""
        if 2 * x.numel() <= self.max_bytes:
            return self.all_reduce(x)
        flat = x.view(-1)
        step = (self.max_bytes // 2) // 8 * 8
        for i in range(0, flat.numel(), step):
            self.all_reduce(flat[i:i + step], algo="oneshot")
        return x

    def all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """``[W, *x.shape]`` stack of every rank's ``x`` (rank order), any dtype;
        graph-capturable.  Leading-dim chunks when a rank's bytes exceed a slot."""
        x = x.contiguous()
        out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        nbytes = x.numel() * x.element_size()
        if nbytes % 16:
            raise ValueError("all_gather needs a multiple of 16 bytes per rank")
        if nbytes <= self.max_bytes:
            self.k.ar_allgather(out, x, self.regions, self.epochs, self.err, self.slot_bytes,
                                self.rank)
            return out
        rows = x.shape[0]
        row_bytes = nbytes // rows
        step = max(1, self.max_bytes // row_bytes)
        while step > 1 and (step * row_bytes) % 16:
            step -= 1
        if (step * row_bytes) % 16:
            raise ValueError("all_gather rows do not chunk into 16-byte pieces")
        for r0 in range(0, rows, step):
            piece = x[r0:r0 + step]
            tmp = torch.empty((self.world,) + tuple(piece.shape), dtype=x.dtype, device=x.device)
            self.k.ar_allgather(tmp, piece, self.regions, self.epochs, self.err,
                                self.slot_bytes, self.rank)
            out[:, r0:r0 + piece.shape[0]] = tmp
        return out

    def all_to_all(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """``out[p] = x_of_rank_p[me]`` for ``x`` = ``[W, rows, ...]`` (any dtype,
        the per-peer chunk a multiple of 16 bytes): the IPC all-to-all of the
        EP token dispatch / combine (``comm.hip`` ar_alltoall, one hop per pair
        over the xGMI mesh).  Chunks larger than a slot allows run as row pieces
        (same count on every rank, so the collectives pair up)."""
        x = x.contiguous()
        out = torch.empty_like(x) if out is None else out
        W = self.world
        if x.shape[0] != W:
            raise ValueError(f"all_to_all input must be [world={W}, ...]")
        chunk = x[0].numel() * x.element_size()
        if chunk % 16:
            raise ValueError("all_to_all needs a multiple of 16 bytes per peer")
        if W * chunk <= self.max_bytes:
            self.k.ar_alltoall(out, x, self.regions, self.epochs, self.err, self.slot_bytes,
                               self.rank)
            return out
        rows = x.shape[1]
        row_bytes = chunk // rows
        step = max(1, self.max_bytes // (W * row_bytes))
        while step > 1 and (step * row_bytes) % 16:
            step -= 1
        if (step * row_bytes) % 16:
            raise ValueError("all_to_all rows do not chunk into 16-byte pieces")
        for r0 in range(0, rows, step):
            piece = x[:, r0:r0 + step].contiguous()
            tmp = torch.empty_like(piece)
            self.k.ar_alltoall(tmp, piece, self.regions, self.epochs, self.err,
                               self.slot_bytes, self.rank)
            out[:, r0:r0 + piece.shape[1]] = tmp
        return out

    def send_recv(self, x: torch.Tensor, src: int, out: torch.Tensor | None = None
                  ) -> torch.Tensor:
        """Every rank publishes ``x`` and receives rank ``src``'s (same shape):
        one ring hop of context-parallel attention over IPC (``ar_sendrecv``);
        slot-sized pieces of the flat bytes for larger blocks."""
        x = x.contiguous()
        out = torch.empty_like(x) if out is None else out
        nbytes = x.numel() * x.element_size()
        if nbytes % 16:
            raise ValueError("send_recv needs a multiple of 16 bytes")
        if nbytes <= self.max_bytes:
            self.k.ar_sendrecv(out, x, self.regions, self.epochs, self.err, self.slot_bytes,
                               self.rank, src)
            return out
        fi, fo = x.view(-1).view(torch.uint8), out.view(-1).view(torch.uint8)
        step = self.max_bytes // 16 * 16
        for i in range(0, nbytes, step):
            self.k.ar_sendrecv(fo[i:i + step], fi[i:i + step], self.regions, self.epochs,
                               self.err, self.slot_bytes, self.rank, src)
        return out

    def can_fuse_norm(self, x: torch.Tensor) -> bool:
        return (self.should_use(x) and x.dim() == 2 and x.shape[1] % 8 == 0
                and 4 * x.numel() <= self.slot_bytes)

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                               eps: float, out: torch.Tensor | None = None) -> torch.Tensor:
        """``residual += allreduce(x)`` (bf16, in place); returns ``RMSNorm(residual) * w``."""
        out = x if out is None else out
        self.k.ar_twoshot(out, x, residual, w, self.regions, self.epochs, self.err,
                          self.slot_bytes, self.rank, eps)
        return out

    def check(self) -> None:
        """Raise if any launch timed out waiting for a peer (bounded spin)."""
        if int(self.err.item()):
            raise RuntimeError("custom all-reduce: a peer never arrived (spin bound hit)")

    def close(self) -> None:
        if self.closed:
            return
        torch.cuda.synchronize(self.device)
        for p in self.opened:
            self.k.ipc_close(p)
        self.k.ipc_free(self.base)
        self.closed = True
