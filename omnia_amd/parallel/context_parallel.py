"""Context-parallel (ring-attention) prefill for very long prompts.

The reference has no sequence parallelism: it bounds context with
``contextWindow`` + ``truncationStrategy`` before the remote call
(``api/v1alpha1/agentruntime_types.go:417-459``), which
``runtime/agent.py`` keeps as the policy layer. A single prompt longer than
one GPU's prefill budget can still be spread over W ranks:

* **Sharding.** The sequence is cut into 2W equal chunks and rank r holds
  chunks r and 2W-1-r ("zig-zag"). Under a causal mask every rank then does the
  same amount of work.
* **Ring.** Each rank keeps its queries and passes its K/V around the ring with
  ``isend`` / ``irecv`` over RCCL (point-to-point xGMI on a node). The transfer
  of the next K/V block is posted before the current block is computed, so it
  overlaps the math.
* **Merge.** Per-block partial attention is merged with the running
  (max, log-sum-exp) statistics, which is exact.

GQA is native: K/V stay at ``Hkv`` heads on the wire (G x fewer bytes than
expanded heads) and are broadcast to the G query heads of each group inside
the block product.  The block product runs on hipBLASLt (batched matmul in the
activation dtype, fp32 softmax statistics); query rows are processed in tiles
so the score block never exceeds ``q_tile x kv_len`` per head.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


def zigzag_indices(seq_len: int, world: int, rank: int) -> torch.Tensor:
    """Token positions rank ``rank`` holds under zig-zag sharding."""
    if seq_len % (2 * world):
        raise ValueError(f"sequence length {seq_len} not divisible by 2*world={2 * world}")
    c = seq_len // (2 * world)
    a = torch.arange(rank * c, (rank + 1) * c)
    b = torch.arange((2 * world - 1 - rank) * c, (2 * world - rank) * c)
    return torch.cat([a, b])


def shard(x: torch.Tensor, world: int, rank: int, dim: int = 0) -> torch.Tensor:
    return x.index_select(dim, zigzag_indices(x.shape[dim], world, rank).to(x.device))


def unshard(parts: list[torch.Tensor], dim: int = 0) -> torch.Tensor:
    """Inverse of :func:`shard` given every rank's piece (rank order)."""
    world = len(parts)
    L = sum(p.shape[dim] for p in parts)
    out = torch.empty((*parts[0].shape[:dim], L, *parts[0].shape[dim + 1:]),
                      dtype=parts[0].dtype, device=parts[0].device)
    for r, p in enumerate(parts):
        out.index_copy_(dim, zigzag_indices(L, world, r).to(p.device), p)
    return out


def _block(q, k, v, qpos, kpos, scale, causal, q_tile):
    """Partial attention of q [Tq, Hq, D] over one K/V block [Tk, Hkv, D].
    Returns (o [Tq, Hq, D] fp32, lse [Tq, Hq] fp32); rows with no visible key
    get lse = -inf and o = 0."""
    Tq, Hq, D = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    o = torch.zeros(Tq, Hq, D, dtype=torch.float32, device=q.device)
    lse = torch.full((Tq, Hq), -math.inf, dtype=torch.float32, device=q.device)
    kt = k.permute(1, 2, 0)  # [Hkv, D, Tk]
    vv = v.permute(1, 0, 2)  # [Hkv, Tk, D]
    for t0 in range(0, Tq, q_tile):
        qs = q[t0:t0 + q_tile]  # [t, Hq, D]
        t = qs.shape[0]
        qg = qs.reshape(t, Hkv, G, D).permute(1, 0, 2, 3).reshape(Hkv, t * G, D)
        s = torch.bmm(qg, kt).float() * scale  # [Hkv, t*G, Tk]
        s = s.view(Hkv, t, G, -1)
        if causal:
            vis = qpos[t0:t0 + t, None] >= kpos[None, :]  # [t, Tk]
            s = s.masked_fill(~vis[None, :, None, :], -math.inf)
        m = s.amax(-1, keepdim=True)
        m_safe = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
        p = torch.exp(s - m_safe)
        l = p.sum(-1, keepdim=True)
        pv = torch.bmm(p.view(Hkv, t * G, -1).to(v.dtype), vv).float().view(Hkv, t, G, D)
        ob = pv / l.clamp_min(1e-30)
        lb = (m_safe + torch.log(l)).squeeze(-1)  # [Hkv, t, G]
        lb = torch.where(l.squeeze(-1) > 0, lb, torch.full_like(lb, -math.inf))
        o[t0:t0 + t] = ob.permute(1, 0, 2, 3).reshape(t, Hq, D)
        lse[t0:t0 + t] = lb.permute(1, 0, 2).reshape(t, Hq)
    return o, lse


def _merge(o, lse, ob, lb):
    m = torch.maximum(lse, lb)
    m_safe = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    a, b = torch.exp(lse - m_safe), torch.exp(lb - m_safe)
    tot = a + b
    o = (o * a[..., None] + ob * b[..., None]) / tot.clamp_min(1e-30)[..., None]
    return o, torch.where(tot > 0, m_safe + torch.log(tot), torch.full_like(m, -math.inf))


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, seq_len: int,
                   group=None, scale: float | None = None, causal: bool = True,
                   q_tile: int = 2048) -> torch.Tensor:
    """Attention of this rank's zig-zag shard q [T, Hq, D] over the whole
    sequence, whose K/V shards [T, Hkv, D] live on the W ranks of ``group``.
    Returns o [T, Hq, D] in q's dtype."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    scale = scale if scale is not None else q.shape[-1] ** -0.5
    pos = [zigzag_indices(seq_len, world, r).to(q.device) for r in range(world)]
    qpos = pos[rank]
    o = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    lse = torch.full(q.shape[:2], -math.inf, dtype=torch.float32, device=q.device)
    kv = torch.stack([k, v]).contiguous()
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    granks = dist.get_process_group_ranks(group) if group is not None else list(range(world))
    for step in range(world):
        src = (rank - step) % world  # whose K/V ``kv`` holds now
        reqs, recv = [], None
        if step + 1 < world:
            recv = torch.empty_like(kv)
            reqs = dist.batch_isend_irecv([
                dist.P2POp(dist.isend, kv, granks[nxt], group),
                dist.P2POp(dist.irecv, recv, granks[prv], group)])
        ob, lb = _block(q, kv[0], kv[1], qpos, pos[src], scale, causal, q_tile)
        o, lse = _merge(o, lse, ob, lb)
        for r in reqs:
            r.wait()
        if recv is not None:
            kv = recv
    return o.to(q.dtype)


def reference_attention(q, k, v, scale=None, causal=True):
    """Dense causal GQA attention over a whole sequence (fp32), for tests."""
    T, Hq, D = q.shape
    G = Hq // k.shape[1]
    scale = scale if scale is not None else D ** -0.5
    kk = k.repeat_interleave(G, 1).float()
    vv = v.repeat_interleave(G, 1).float()
    s = torch.einsum("qhd,khd->hqk", q.float(), kk) * scale
    if causal:
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1), -math.inf)
    return torch.einsum("hqk,khd->qhd", s.softmax(-1), vv)
