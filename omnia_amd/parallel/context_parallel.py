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
  ``isend`` / ``irecv`` over RCCL (point-to-point xGMI on a node), or -- ranks
  sharing a device, the ``ipc`` transport -- the IPC point-to-point kernel on a
  side stream (``ops/csrc/comm.hip`` ar_sendrecv). The transfer of the next
  K/V block is posted before the current block is computed, so it overlaps
  the math.
* **Merge.** Per-block partial attention is merged with the running
  (max, log-sum-exp) statistics, which is exact.

GQA is native: K/V stay at ``Hkv`` heads on the wire (G x fewer bytes than
expanded heads) and are broadcast to the G query heads of each group inside
the block product.

Two block products:

* :func:`ring_attention` -- generic (any head dim, causal or not) on batched
  matmuls with fp32 statistics; the reference implementation of the ring.
* :func:`ring_attention_paged` -- the serving path (:class:`CPPrefill`, used by
  the engine for prompts over ``EngineConfig.cp_threshold``): K/V travel as
  the engine's paged layout ``[2, pages, Hkv, BS, D]`` and every ring step is
  ONE launch of the hand flash-prefill kernel (``ops/csrc/attention.hip``) over
  the step's zig-zag chunk pairs, with the kernel's LSE output and per-pair key
  bound (``kv_lens``) -- no score matrix is ever materialised.  The rank that
  owns the request copies every K/V block it sees go by into its paged KV
  cache, so after the prefill the owner decodes alone with no extra gather.
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


# ============================================================ serving path
def _pairs(rank: int, src: int) -> list[tuple[int, int, bool]]:
    """(q chunk, k chunk, causal) products of one ring step: chunk 0 = the
    rank's low zig-zag chunk (index r), 1 = its high chunk (2W-1-r).  Chunk
    pairs whose keys all lie after the queries are skipped; every other pair
    is either the causal diagonal or attended in full."""
    if src == rank:
        return [(0, 0, True), (1, 0, False), (1, 1, True)]
    if src < rank:
        return [(0, 0, False), (1, 0, False)]
    return [(1, 0, False), (1, 1, False)]


class _StepLaunch:
    """Kernel metadata of one ring-step pattern (device tensors, built once)."""

    def __init__(self, pairs, c: int, pages: int, device):
        from .. import ops

        n = len(pairs)
        self.pairs = pairs
        self.rows = torch.cat([torch.arange(qc * c, (qc + 1) * c) for qc, _, _ in pairs]).to(device)
        qsl = [i * c for i in range(n + 1)]
        self.q_start_loc = torch.tensor(qsl, dtype=torch.int32, device=device)
        # causal diagonal: queries at relative 0..c-1 over keys 0..c-1; full: queries
        # placed after all c keys (seq_len = 2c, offset c), keys capped at c
        self.seq_lens = torch.tensor([c if causal else 2 * c for _, _, causal in pairs],
                                     dtype=torch.int32, device=device)
        self.kv_lens = torch.full((n,), c, dtype=torch.int32, device=device)
        bt = [list(range(kc * pages, (kc + 1) * pages)) for _, kc, _ in pairs]
        self.block_tables = torch.tensor(bt, dtype=torch.int32, device=device)
        ts, tq = ops.prefill_tiles([c] * n)
        self.tile_seq = torch.tensor(ts, dtype=torch.int32, device=device)
        self.tile_q0 = torch.tensor(tq, dtype=torch.int32, device=device)


def ring_attention_paged(q: torch.Tensor, kv: torch.Tensor, c: int, scale: float, group=None,
                         launches: dict | None = None, on_block=None, comm=None,
                         comm_stream=None) -> torch.Tensor:
    """Causal ring attention of this rank's zig-zag shard.

    q: [2c, Hq, D] (rows 0..c-1 = low chunk, c..2c-1 = high chunk); kv: this
    rank's K/V pages [2, 2c/BS, Hkv, BS, D] (low chunk pages first).
    ``on_block(src, kv_src)`` sees every rank's K/V block once (own included).
    ``comm`` (a :class:`~omnia_amd.parallel.custom_allreduce.CustomAllReduce` over
    ``group``): the ring hop runs on the IPC point-to-point kernel on
    ``comm_stream`` -- ranks sharing a device, where RCCL cannot run -- still
    overlapping the next block's transfer with this block's attention.
    Returns o [2c, Hq, D] in q's dtype."""
    from .. import ops

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    pages = kv.shape[1] // 2
    Hq, D = q.shape[1], q.shape[2]
    o = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    lse = torch.full(q.shape[:2], -math.inf, dtype=torch.float32, device=q.device)
    launches = {} if launches is None else launches
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    granks = (dist.get_process_group_ranks(group) if (group is not None and world > 1)
              else list(range(world)))
    cur = kv.contiguous()
    for step in range(world):
        src = (rank - step) % world
        reqs, recv = [], None
        if step + 1 < world:
            recv = torch.empty_like(cur)
            if comm is not None:
                main = torch.cuda.current_stream()
                side = comm_stream or main
                side.wait_stream(main)  # cur / recv are ready on the side stream
                with torch.cuda.stream(side):
                    comm.send_recv(cur, prv, out=recv)
            else:
                reqs = dist.batch_isend_irecv([
                    dist.P2POp(dist.isend, cur, granks[nxt], group),
                    dist.P2POp(dist.irecv, recv, granks[prv], group)])
        if on_block is not None:
            on_block(src, cur)
        key = (src == rank, src < rank)
        L = launches.get(key)
        if L is None:
            L = launches[key] = _StepLaunch(_pairs(rank, src), c, pages, q.device)
        qb = q.index_select(0, L.rows)
        lb = torch.empty(qb.shape[:2], dtype=torch.float32, device=q.device)
        ob = ops.prefill_attention(qb, cur[0], cur[1], L.block_tables, L.q_start_loc,
                                   L.seq_lens, scale, L.tile_seq, L.tile_q0, lse=lb,
                                   kv_lens=L.kv_lens)
        for i, (qc, _, _) in enumerate(L.pairs):
            sl = slice(qc * c, (qc + 1) * c)
            o[sl], lse[sl] = _merge(o[sl], lse[sl], ob[i * c:(i + 1) * c].float(),
                                    lb[i * c:(i + 1) * c])
        for r in reqs:
            r.wait()
        if recv is not None:
            if comm is not None and comm_stream is not None:
                torch.cuda.current_stream().wait_stream(comm_stream)
            cur = recv
    return o.to(q.dtype)


class CPPrefill:
    """One context-parallel prefill of an ``L``-token prompt over the ranks of
    ``group`` (every rank holds the full model; the request's owner holds its
    KV pages).  The prompt is padded to a multiple of 2W pages; padded rows sit
    after every real token, so causal masking keeps them out of real rows.

    The model's attention (``models/llama.py``) sees ``fb.cp`` and, instead of
    writing K/V into the paged cache, writes them into this rank's scratch pages
    and calls :meth:`attention`."""

    def __init__(self, L: int, world: int, rank: int, group, hkv: int, head_dim: int,
                 block_size: int, device, dtype, owner: bool = False,
                 owner_blocks: list[int] | None = None, max_position: int | None = None):
        self.L, self.world, self.rank, self.group = L, world, rank, group
        unit = 2 * world * block_size
        self.L_pad = -(-L // unit) * unit
        self.c = self.L_pad // (2 * world)
        self.bs = block_size
        self.pages = self.c // block_size  # pages per chunk
        idx = zigzag_indices(self.L_pad, world, rank)
        self.index = idx.to(device)  # rows of the padded prompt this rank holds
        pos = idx.clamp(max=(max_position or self.L_pad) - 1)
        self.positions = pos.to(device=device, dtype=torch.int32)
        self.slots = torch.arange(2 * self.c, dtype=torch.int64, device=device)
        self.scratch = torch.empty(2, 2 * self.pages, hkv, block_size, head_dim, dtype=dtype,
                                   device=device)
        self.owner = owner
        self.owner_blocks = owner_blocks
        self._launches: dict = {}
        self._dst = None
        if owner:
            nreal = -(-L // block_size)  # pages holding real tokens
            if owner_blocks is None or len(owner_blocks) < nreal:
                raise ValueError("owner needs KV blocks for the whole prompt")
            self._dst = torch.tensor(list(owner_blocks[:nreal]), dtype=torch.long, device=device)
            self._nreal = nreal

    def locate(self, p: int) -> tuple[int, int]:
        """(rank, row) holding absolute position ``p`` of the padded prompt."""
        ch = p // self.c
        if ch < self.world:
            return ch, p % self.c
        return 2 * self.world - 1 - ch, self.c + p % self.c

    def _chunk_pages(self, src: int):
        """[(chunk-local page range, first absolute page)] of rank src's chunks."""
        W, P = self.world, self.pages
        return [(0, src * P), (1, (2 * W - 1 - src) * P)]

    def attention(self, kc: torch.Tensor, vc: torch.Tensor, q3: torch.Tensor, scale: float
                  ) -> torch.Tensor:
        """q3: [2c, Hq, D] after RoPE; this rank's K/V already in ``scratch``.
        ``kc`` / ``vc``: the owner's paged cache of this layer."""
        def keep(src, blk):
            if not self.owner:
                return
            for half, first in self._chunk_pages(src):
                lo = first
                hi = min(first + self.pages, self._nreal)
                if hi <= lo:
                    continue
                src_pages = blk[:, half * self.pages: half * self.pages + (hi - lo)]
                dst = self._dst[lo:hi]
                kc.index_copy_(0, dst, src_pages[0])
                vc.index_copy_(0, dst, src_pages[1])

        comm = None
        if q3.is_cuda and self.world > 1:
            from . import state as pstate

            st = pstate.get_state()
            if st.transport == "ipc" and st.dp_comm is not None and self.group is st.dp_group:
                comm = st.dp_comm
                if getattr(self, "_comm_stream", None) is None:
                    self._comm_stream = torch.cuda.Stream(device=q3.device)
        return ring_attention_paged(q3, self.scratch, self.c, scale, self.group,
                                    self._launches, keep, comm=comm,
                                    comm_stream=getattr(self, "_comm_stream", None))
