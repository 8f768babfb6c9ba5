"""Tensor-parallel sampling without gathering the vocabulary.

Under TP the LM head is vocab-parallel: rank r holds logits for its V/tp slice.
Gathering the full [B, V] logits every decode step moves B x V x 2 bytes
(64 MB at B = 256, V = 128256) into every rank; instead each rank reduces its
slice to a few candidates and only those are exchanged (B x tp x (2K + 2)
floats, 0.5 MB at K = 64, tp = 8):

* greedy rows (temperature 0): the global argmax is the argmax of the ranks'
  local top-1s -- exact;
* pure temperature rows (no top-k / top-p): Gumbel-max -- every rank adds
  Gumbel noise to its logits / T and keeps the local winner; the arg-max of the
  winners is an exact sample from softmax(logits / T) over the whole
  vocabulary.  The noise of (row, GLOBAL vocab index v) is a counter-based hash
  of (request seed, step, v): draws are independent across ranks (each hashes
  its own vocab range) without any per-rank RNG state, and a seeded request is
  reproducible whatever the TP degree (``gumbel_uniform`` is the bit-exact
  host reference of the device hash);
* top-k / top-p rows: the fused sampler runs over the union of the ranks'
  local top-K logits (K = 64): exact for top_k <= K; top-p is taken inside that
  candidate set (exact whenever the nucleus has <= K tokens per rank).
Every rank computes the same final token from the same gathered candidates,
which keeps the device-side token feedback of pipelined decode consistent.

On the GPU (:func:`tp_sample_device`) the whole tail is three launches: the
``tp_pack`` kernel (per row: slice arg-max, Gumbel winner, or exact local
top-K by 16-bit radix select, plus the slice's softmax statistics), the IPC
all-gather, and the ``tp_merge`` kernel, whose filtered-row draw uses the
single-GPU fused sampler's noise keyed by the GLOBAL token id and the
full-vocabulary mass for top-p -- so a TP top-k / top-p row draws the token
the single-GPU sampler draws.  No framework op runs in the captured graph.
Penalised / grammar-constrained rows keep the full gather (the runner routes
them to the eager path).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops


_M32 = 0xFFFFFFFF


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    """(x * c) mod 2**32 for int64 x in [0, 2**32) without int64 overflow."""
    return (x * (c & 0xFFFF) + (((x * (c >> 16)) & 0xFFFF) << 16)) & _M32


def _fmix32(h: torch.Tensor) -> torch.Tensor:
    """murmur3 finaliser on int64 tensors holding 32-bit values."""
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    return h ^ (h >> 16)


def gumbel_uniform(seeds: torch.Tensor, steps: torch.Tensor, vocab_start: int, n: int
                   ) -> torch.Tensor:
    """Uniform (0, 1) noise [B, n] for global vocab ids vocab_start .. +n: a pure
    function of (seed, step, vocab id), identical on every device and TP layout."""
    dev = seeds.device
    s = seeds.to(torch.int64)
    row = _fmix32((s & _M32) ^ _fmix32(((s >> 32) & _M32) ^ 0x68BC21EB))
    row = _fmix32(row ^ _fmix32((steps.to(torch.int64) & _M32) ^ 0x02E5BE93))
    v = torch.arange(vocab_start, vocab_start + n, dtype=torch.int64, device=dev)
    h = _fmix32(row[:, None] ^ _fmix32((v + 0x9E3779B9) & _M32)[None, :])
    return (h.to(torch.float64) + 0.5).mul_(1.0 / 4294967296.0).float()


def _gather_packs(pack: torch.Tensor, W: int, group) -> torch.Tensor:
    """``[W, B, ld]``: every TP rank's candidate pack, in rank order."""
    from . import state as pstate

    st = pstate.get_state()
    B = pack.shape[0]
    if st.tp_size == W and (group is None or group is st.tp_group) and st.tp_size > 1:
        return pstate.tp_all_gather(pack)  # IPC kernel on the node (capturable)
    if pack.is_cuda:
        allp = torch.empty(W * B, pack.shape[1], dtype=pack.dtype, device=pack.device)
        dist.all_gather_into_tensor(allp, pack, group=group)
        return allp.view(W, B, -1)
    parts = [torch.empty_like(pack) for _ in range(W)]
    dist.all_gather(parts, pack, group=group)
    return torch.stack(parts)


def tp_sample_device(local_logits: torch.Tensor, vocab_start: int, temperature: torch.Tensor,
                     top_k: torch.Tensor | None, top_p: torch.Tensor | None,
                     seeds: torch.Tensor, steps: torch.Tensor | None = None,
                     out: torch.Tensor | None = None, group=None, K: int = 64,
                     tok_slots: torch.Tensor | None = None,
                     dst: torch.Tensor | None = None) -> torch.Tensor:
    """The GPU sampler: ``tp_pack`` kernel -> all-gather -> ``tp_merge`` kernel
    (``ops/csrc/sampling.hip``), three launches and no framework op, so the
    whole sampling tail of a TP decode step is hand kernels inside its hipGraph.
    With ``tok_slots`` / ``dst`` the merge also scatters each token into its
    sequence's device token slot."""
    from .. import ops

    B, Vl = local_logits.shape
    W = dist.get_world_size(group)
    K = min(K, Vl, 512 // W)
    k = ops.kernels()
    pack = torch.empty(B, 2 * K + 4, dtype=torch.float32, device=local_logits.device)
    temperature = temperature.float()
    top_k = top_k.int() if top_k is not None else None
    top_p = top_p.float() if top_p is not None else None
    seeds = seeds.to(torch.int64)
    steps = steps.to(torch.int64) if steps is not None else None
    k.tp_pack(pack, K, local_logits, vocab_start, temperature, top_k, top_p, seeds, steps)
    allp = _gather_packs(pack, W, group)
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=local_logits.device)
    k.tp_merge(out, tok_slots, dst, allp.contiguous(), K, temperature, top_k, top_p, seeds,
               steps)
    return out


def tp_sample(local_logits: torch.Tensor, vocab_start: int, temperature: torch.Tensor,
              top_k: torch.Tensor, top_p: torch.Tensor, seeds: torch.Tensor | None = None,
              steps: torch.Tensor | None = None, out: torch.Tensor | None = None, group=None,
              K: int = 64, generator: torch.Generator | None = None) -> torch.Tensor:
    B, Vl = local_logits.shape
    W = dist.get_world_size(group)
    if (local_logits.is_cuda and local_logits.dtype == torch.bfloat16 and seeds is not None
            and local_logits.stride(1) == 1 and (out is None or out.dtype == torch.int32)):
        return tp_sample_device(local_logits, vocab_start, temperature, top_k, top_p, seeds,
                                steps, out=out, group=group, K=K)
    # host reference path (CPU / gloo tests, non-bf16 logits): the same candidate
    # pack built from framework ops
    K = min(K, Vl)
    pad = (-(2 * K + 2)) % 4  # 16-byte rows for the IPC all-gather
    pack = torch.zeros(B, 2 * K + 2 + pad, dtype=torch.float32, device=local_logits.device)
    lf = local_logits.float()
    cv, ci = torch.topk(lf, K, dim=1)
    pack[:, :K] = cv
    pack[:, K:2 * K] = ci + vocab_start
    t = temperature.float().clamp(min=1e-6)[:, None]
    if seeds is not None:
        st = steps if steps is not None else torch.zeros(B, dtype=torch.int64, device=lf.device)
        u = gumbel_uniform(seeds.to(lf.device), st.to(lf.device), vocab_start, Vl)
    else:  # no per-request seeds: the caller's generator (must differ per rank)
        u = torch.rand(B, Vl, device=lf.device, generator=generator)
    u = u.clamp_(1e-10, 1.0 - 1e-7)
    gv, gi = (lf / t - torch.log(-torch.log(u))).max(dim=1)
    pack[:, 2 * K] = gv
    pack[:, 2 * K + 1] = gi + vocab_start
    allp = _gather_packs(pack, W, group)
    cand_v = allp[:, :, :K].permute(1, 0, 2).reshape(B, W * K)
    cand_i = allp[:, :, K:2 * K].permute(1, 0, 2).reshape(B, W * K).long()
    gum_v = allp[:, :, 2 * K].t()  # [B, W]
    gum_i = allp[:, :, 2 * K + 1].t().long()
    greedy = cand_i.gather(1, cand_v.argmax(dim=1, keepdim=True))[:, 0]
    gumbel = gum_i.gather(1, gum_v.argmax(dim=1, keepdim=True))[:, 0]
    filt_local = ops.sample(cand_v.to(local_logits.dtype).contiguous(), temperature,
                            top_k, top_p, seeds=seeds, steps=steps).long()
    filtered = cand_i.gather(1, filt_local.clamp(0, W * K - 1)[:, None])[:, 0]
    use_filter = (top_k > 0) | (top_p < 1.0)
    tok = torch.where(temperature <= 0, greedy, torch.where(use_filter, filtered, gumbel))
    if out is None:
        return tok.to(torch.int32)
    out.copy_(tok)
    return out
