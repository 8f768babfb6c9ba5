"""Expert parallelism with token all-to-all (SURVEY §2.3 EP row, K15).

Two EP layouts exist in the engine:

* **EP inside TP** (the default, :mod:`omnia_amd.models.mixtral`): attention is
  tensor-parallel, so every rank already holds every token; each rank runs only
  its experts and the all-reduce that dense TP needs anyway combines them.  No
  extra collective.
* **DP-attention + EP** (this module): ranks hold DIFFERENT tokens (data-parallel
  attention, e.g. one replica per GPU), and the expert FFN is sharded E/ep per
  rank.  Tokens travel to their experts' rank and back: dispatch all-to-all ->
  local grouped expert FFN -> combine all-to-all -> weighted sum.  On an 8-GPU
  MI355X node every rank talks to every peer over its own xGMI link, so the
  all-to-all is one hop per pair (RCCL ``alltoall`` over the full mesh).

Wire format per direction: one ``all_to_all_single`` of the counts, then one of
the rows ([n, d] activations) with the (expert, slot) metadata riding in a
second small all-to-all.  Summation order of the combine is fixed (slot order
per token), so the result is identical to the single-rank oracle up to the
GEMM's own rounding.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..ops import reference as ref


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group):
    dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                           input_split_sizes=in_splits, group=group)
    return out


def expert_ffn(x: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor) -> torch.Tensor:
    """SwiGLU FFN of one expert: down(silu(gate x) * up x); w_gu [2I, d], w_down [d, I]."""
    from .. import ops

    if x.shape[0] == 0:
        return x.new_zeros(0, w_down.shape[0])
    return ops.linear(ops.linear_silu(x, w_gu), w_down)


class ExpertParallelMoE:
    """Top-k MoE FFN with experts sharded over ``group`` (E / ep per rank).

    ``w_gu`` [E_local, 2I, d] and ``w_down`` [E_local, d, I] are this rank's
    experts ``[rank * E_local, (rank + 1) * E_local)``; ``router`` [E, d] is
    replicated."""

    def __init__(self, router: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor, k: int,
                 group=None, renorm: bool = True):
        self.router, self.w_gu, self.w_down, self.k = router, w_gu, w_down, k
        self.group = group
        self.ep = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.e_local = w_gu.shape[0]
        self.n_experts = router.shape[0]
        if self.e_local * self.ep != self.n_experts:
            raise ValueError("experts must split evenly over the EP group")
        self.renorm = renorm
        self.stats = {"sent_rows": 0, "recv_rows": 0}

    def route(self, x: torch.Tensor):
        return ref.moe_route(F.linear(x.float(), self.router.float()), self.k, self.renorm)

    def __call__(self, x: torch.Tensor, ids=None, wts=None) -> torch.Tensor:
        T, d = x.shape
        if ids is None:
            ids, wts = self.route(x)
        flat_e = ids.reshape(-1).long()                       # [T*k]
        dest = flat_e // self.e_local                         # owning rank per assignment
        order = torch.argsort(dest, stable=True)               # grouped by rank, stable
        send_counts = torch.bincount(dest, minlength=self.ep)
        rows = x.index_select(0, order // self.k)             # token row per assignment
        meta = flat_e.index_select(0, order).to(torch.int64)  # expert id per row
        if self.ep > 1:
            recv_counts = torch.empty_like(send_counts)
            dist.all_to_all_single(recv_counts, send_counts, group=self.group)
            ins, outs = send_counts.tolist(), recv_counts.tolist()
            r_rows = _a2a(rows.new_empty(sum(outs), d), rows.contiguous(), outs, ins, self.group)
            r_meta = _a2a(meta.new_empty(sum(outs)), meta, outs, ins, self.group)
        else:
            ins = outs = [int(send_counts.sum())]
            r_rows, r_meta = rows, meta
        self.stats["sent_rows"] += int(sum(ins))
        self.stats["recv_rows"] += int(sum(outs))
        # local grouped expert FFN (rows of one expert are processed together)
        y = r_rows.new_empty(r_rows.shape[0], d)
        local = r_meta - self.rank * self.e_local
        for e in range(self.e_local):
            idx = (local == e).nonzero(as_tuple=True)[0]
            if idx.numel():
                y.index_copy_(0, idx, expert_ffn(r_rows.index_select(0, idx), self.w_gu[e],
                                                 self.w_down[e]).to(y.dtype))
        # combine: send results back along the reverse splits
        back = _a2a(y.new_empty(rows.shape[0], d), y, ins, outs, self.group) \
            if self.ep > 1 else y
        per_assign = torch.empty_like(back)
        per_assign.index_copy_(0, order, back)                 # back to (token, slot) order
        w = wts.reshape(-1).to(torch.float32)
        contrib = per_assign.float() * w[:, None]
        out = contrib.view(T, self.k, d).sum(dim=1)            # fixed slot order
        return out.to(x.dtype)
