"""Expert parallelism with token all-to-all (SURVEY §2.3 EP row, K15; BASELINE
config 5 "expert all-to-all over xGMI").

Two EP layouts exist in the engine (``EngineConfig.ep_mode``):

* ``"tp"`` -- **EP inside TP** (:mod:`omnia_amd.models.mixtral`, the default):
  attention is tensor-parallel, so every rank already holds every token; each
  rank runs only its experts and the all-reduce that dense TP needs anyway
  combines them.  No extra collective.
* ``"a2a"`` -- **DP attention + EP** (this module): every rank is its own
  data-parallel replica for attention (its own batch, KV, scheduler) and the
  expert FFN is sharded E/ep per rank.  Each MoE layer sends every (token, slot)
  assignment to the rank owning its expert, runs the local grouped expert GEMMs
  on what arrives, and sends the results back to be weighted and summed.

The all-to-all is **fixed-capacity and sync-free**, so the whole MoE layer is
static-shaped and hipGraph-capturable:

* send buffer ``[ep, C, d]``: assignment ``(t, j)`` for rank ``r`` lands at slot
  ``r*C + pos`` where ``pos`` is its rank among rank-``r`` assignments -- a
  device-side one-hot cumsum, no ``.tolist()``, no host round trip;
* an expert-id slab ``[ep, C]`` (padding = -1) rides in a second all-to-all;
* ``dist.all_to_all_single`` with equal splits (RCCL over xGMI: each rank talks
  to each peer over its own link, one hop per pair), or -- when the ranks share
  devices (the ``ipc`` transport, e.g. EP=8 rehearsed on one MI355X) -- the IPC
  all-to-all kernel (``ops/csrc/comm.hip`` ar_alltoall: every rank pulls its
  chunk straight out of each peer's exported buffer);
* the receive side runs :func:`omnia_amd.ops.moe_rows` -- the grouped MFMA
  expert kernels with top-1 routing over the received rows; padding rows are
  skipped by ``moe_align`` (no per-expert Python loop);
* the combine all-to-all returns results to the same slots; the source gathers
  its ``r*C + pos`` rows and sums them in fixed slot order, so outputs match the
  single-rank oracle up to GEMM rounding.

Capacity ``C`` must be the same on every rank of a step (it is a collective's
shape); the engine passes the step-global token count (``ForwardBatch.ep_tokens``)
so ``C = T_global * k`` is lossless.  Large (prefill) steps run the layer in
fixed chunks of at most ``chunk_tokens`` (``OMNIA_EP_CHUNK_TOKENS``, default
2048) tokens, the chunk count derived from the step-global token count so every
rank issues the same collectives: transients stay at ``ep * chunk * k`` rows
(at ep = 8, k = 2, I = 14336: ~0.5 GiB of activations for 2048 tokens, instead
of ~15 GiB for an unchunked 16K-token prefill).  The price of static shapes is padding
bandwidth: each rank moves ``ep * C * d`` bytes per direction, of which only
``T*k*d`` are real -- measured and documented against EP-inside-TP in
``docs/PARALLELISM.md``.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..ops import reference as ref


def dispatch_slots(ids: torch.Tensor, e_local: int, ep: int, cap: int) -> torch.Tensor:
    """Send-buffer slot ``rank * cap + pos`` of every (token, slot) assignment,
    ``pos`` = its order among the assignments for ``rank`` (stable)."""
    flat = ids.reshape(-1).long()
    dest = torch.div(flat, e_local, rounding_mode="floor")
    # one-hot by comparison (F.one_hot validates its input with a host sync,
    # which a captured decode graph cannot contain)
    onehot = (dest[:, None] == torch.arange(ep, device=dest.device)[None, :]).to(torch.int32)
    pos = onehot.cumsum(0).gather(1, dest[:, None])[:, 0].long() - 1
    return dest * cap + pos


class ExpertParallelMoE:
    """Top-k MoE FFN with experts sharded over ``group`` (E / ep per rank).

    ``w_gu`` [E_local, 2I, d] and ``w_down`` [E_local, d, I] are this rank's
    experts ``[rank * E_local, (rank + 1) * E_local)``; ``router`` [E, d] is
    replicated."""

    def __init__(self, router: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor, k: int,
                 group=None, renorm: bool = True, comm=None):
        self.router, self.w_gu, self.w_down, self.k = router, w_gu, w_down, k
        self.group = group
        # IPC all-to-all (parallel.state ``dp_comm``) when the ranks share devices
        # (``ipc`` transport: RCCL cannot place two ranks on one GPU); RCCL otherwise
        self.comm = comm
        self.ep = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.e_local = w_gu.shape[0]
        self.n_experts = router.shape[0]
        if self.e_local * self.ep != self.n_experts:
            raise ValueError("experts must split evenly over the EP group")
        self.renorm = renorm
        self.chunk_tokens = max(1, int(os.environ.get("OMNIA_EP_CHUNK_TOKENS", "2048")))
        self.stats = {"calls": 0, "rows_sent": 0, "bytes_sent": 0, "chunks": 0}

    def route(self, x: torch.Tensor):
        if x.is_cuda:
            from .. import ops

            T = x.shape[0]
            ids = torch.empty(T, self.k, dtype=torch.int32, device=x.device)
            wts = torch.empty(T, self.k, dtype=torch.float32, device=x.device)
            ops.kernels().moe_router_topk(ids, wts, x.contiguous(), self.router, self.k,
                                          self.renorm)
            return ids, wts
        return ref.moe_route(F.linear(x.float(), self.router.float()), self.k, self.renorm)

    def _a2a(self, t: torch.Tensor) -> torch.Tensor:
        if self.ep == 1:
            return t
        if self.comm is not None and t.is_cuda:
            return self.comm.all_to_all(t.view(self.ep, -1, *t.shape[1:])).view(t.shape)
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t, group=self.group)
        return out

    def __call__(self, x: torch.Tensor, ids=None, wts=None, tokens: int = 0) -> torch.Tensor:
        """``tokens``: the step-global max token count across the EP group (sets
        the capacity; defaults to this rank's own T, correct for a lone call)."""
        T, d = x.shape
        G = max(tokens, T)
        if G > self.chunk_tokens:
            if ids is None:
                ids, wts = self.route(x)
            c = self.chunk_tokens
            outs = []
            for i in range((G + c - 1) // c):  # same count on every rank (collectives)
                lo, hi = min(i * c, T), min((i + 1) * c, T)
                outs.append(self._layer(x[lo:hi], ids[lo:hi], wts[lo:hi], c))
            return torch.cat(outs) if outs else x.new_empty(0, d)
        return self._layer(x, ids, wts, tokens)

    def _layer(self, x: torch.Tensor, ids, wts, tokens: int) -> torch.Tensor:
        from .. import ops

        T, d = x.shape
        k = self.k
        if ids is None:
            ids, wts = self.route(x)
        # a slot index outside the send buffer would be an out-of-bounds device
        # write; routing always yields [0, E), the clamp keeps it so for any input
        ids = ids.clamp(0, self.n_experts - 1)
        # multiple of 8 rows: the int32 expert-id slab's per-peer chunk stays a
        # multiple of 16 bytes (the IPC all-to-all's vector width)
        cap = -(-max(1, max(tokens, T) * k) // 8) * 8
        slot = dispatch_slots(ids, self.e_local, self.ep, cap)         # [T*k]
        send = x.new_zeros(self.ep * cap, d)
        send.index_copy_(0, slot, x.repeat_interleave(k, dim=0))
        meta = torch.full((self.ep * cap,), -1, dtype=torch.int32, device=x.device)
        meta.index_copy_(0, slot, ids.reshape(-1).to(torch.int32))
        recv, rmeta = self._a2a(send), self._a2a(meta)
        y = ops.moe_rows(recv, rmeta, self.w_gu, self.w_down, self.rank * self.e_local,
                         self.n_experts)
        back = self._a2a(y)
        got = back.index_select(0, slot).float().view(T, k, d)
        out = (got * wts.to(torch.float32).view(T, k, 1)).sum(dim=1)  # fixed slot order
        self.stats["calls"] += 1
        self.stats["chunks"] += 1
        self.stats["rows_sent"] += self.ep * cap
        self.stats["bytes_sent"] += self.ep * cap * d * x.element_size()
        return out.to(x.dtype)
