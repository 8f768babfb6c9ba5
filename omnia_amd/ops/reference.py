"""Plain-PyTorch fp32 reference implementations of every hand-written kernel.

These are the numerics oracles for ``tests/test_kernels_gpu.py`` and the CPU
execution path used by the CPU test-suite (no GPU in the build container).
They define the exact semantics the HIP kernels must reproduce.
"""
from __future__ import annotations

import math

import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype)


def fused_add_rmsnorm(x, residual, w, eps):
    """residual <- x + residual (rounded to the storage dtype); returns norm(residual)*w."""
    r = (x.float() + residual.float()).to(residual.dtype)
    return rmsnorm(r, w, eps), r


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
                 device="cpu") -> torch.Tensor:
    """[max_pos, head_dim] fp32 table = (cos[D/2] | sin[D/2]) with optional llama3 scaling."""
    half = head_dim // 2
    inv_freq = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2.0 / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        low_wl, high_wl = old / lo, old / hi
        wl = 2 * math.pi / inv_freq
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > low_wl, inv_freq / factor, inv_freq)
        mid = (wl <= low_wl) & (wl >= high_wl)
        scaled = torch.where(mid, (1 - smooth) * inv_freq / factor + smooth * inv_freq, scaled)
        inv_freq = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv_freq)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x: [T, H, D] neox half-rotation."""
    d = x.shape[-1]
    half = d // 2
    cs = cos_sin[positions.long()]
    cos = cs[:, None, :half]
    sin = cs[:, None, half:]
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def write_kv(k_cache, v_cache, k, v, slots):
    """k/v: [T, Hkv, D]; caches [NB, Hkv, BS, D].  Rows with a negative slot
    (padded graph rows) write nothing -- as in the HIP kernels; a -1 would
    otherwise index the LAST page from the end."""
    keep = slots >= 0
    if not bool(keep.all()):
        k, v, slots = k[keep], v[keep], slots[keep]
    bs = k_cache.shape[2]
    blk = (slots // bs).long()
    off = (slots % bs).long()
    k_cache[blk, :, off] = k.to(k_cache.dtype)
    v_cache[blk, :, off] = v.to(v_cache.dtype)


def gather_kv(cache, block_table, length):
    """-> [length, Hkv, D] from paged cache."""
    bs = cache.shape[2]
    nb = (length + bs - 1) // bs
    pages = cache[block_table[:nb].long()]  # [nb, Hkv, BS, D]
    return pages.permute(0, 2, 1, 3).reshape(nb * bs, cache.shape[1], cache.shape[3])[:length]


def paged_attention(q, k_cache, v_cache, block_tables, q_start_loc, seq_lens, scale):
    """Causal attention of each sequence's new queries against its whole paged context.

    q: [T, Hq, D]; returns [T, Hq, D].  Query row i of sequence s sits at absolute
    position ctx - qlen + i.
    """
    out = torch.empty_like(q)
    hq = q.shape[1]
    hkv = k_cache.shape[1]
    g = hq // hkv
    B = seq_lens.numel()
    for s in range(B):
        a, b = int(q_start_loc[s]), int(q_start_loc[s + 1])
        ctx = int(seq_lens[s])
        qlen = b - a
        if qlen == 0:
            continue
        kk = gather_kv(k_cache, block_tables[s], ctx).float().repeat_interleave(g, dim=1)
        vv = gather_kv(v_cache, block_tables[s], ctx).float().repeat_interleave(g, dim=1)
        qq = q[a:b].float()
        scores = torch.einsum("qhd,khd->hqk", qq, kk) * scale
        qpos = torch.arange(ctx - qlen, ctx, device=q.device)[:, None]
        kpos = torch.arange(ctx, device=q.device)[None, :]
        scores = scores.masked_fill((kpos > qpos)[None], float("-inf"))
        p = torch.softmax(scores, dim=-1)
        out[a:b] = torch.einsum("hqk,khd->qhd", p, vv).to(q.dtype)
    return out


def paged_attention_lse(q, k_cache, v_cache, block_tables, q_start_loc, seq_lens, scale,
                        kv_lens=None):
    """:func:`paged_attention` that also returns the fp32 natural-log LSE
    [T, Hq] of every row, with keys of sequence s capped at ``kv_lens[s]``."""
    out = torch.zeros_like(q)
    T, hq = q.shape[0], q.shape[1]
    lse = torch.full((T, hq), float("-inf"), dtype=torch.float32, device=q.device)
    g = hq // k_cache.shape[1]
    for s in range(seq_lens.numel()):
        a, b = int(q_start_loc[s]), int(q_start_loc[s + 1])
        ctx, qlen = int(seq_lens[s]), b - a
        if qlen == 0:
            continue
        klen = min(ctx, int(kv_lens[s])) if kv_lens is not None else ctx
        kk = gather_kv(k_cache, block_tables[s], klen).float().repeat_interleave(g, dim=1)
        vv = gather_kv(v_cache, block_tables[s], klen).float().repeat_interleave(g, dim=1)
        scores = torch.einsum("qhd,khd->hqk", q[a:b].float(), kk) * scale
        qpos = torch.arange(ctx - qlen, ctx, device=q.device)[:, None]
        kpos = torch.arange(klen, device=q.device)[None, :]
        scores = scores.masked_fill((kpos > qpos)[None], float("-inf"))
        l = torch.logsumexp(scores, dim=-1)  # [h, q]
        p = torch.exp(scores - l[..., None]).nan_to_num(0.0)
        out[a:b] = torch.einsum("hqk,khd->qhd", p, vv).to(q.dtype)
        lse[a:b] = l.t()
    return out, lse


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    inter = x.shape[-1] // 2
    g, u = x[..., :inter].float(), x[..., inter:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def apply_penalties(logits, counts, freq, pres, rep):
    x = logits.float().clone()
    if counts is None:
        return x
    seen = counts > 0
    if rep is not None:
        r = rep[:, None].float()
        x = torch.where(seen, torch.where(x > 0, x / r, x * r), x)
    f = freq[:, None].float() if freq is not None else 0.0
    p = pres[:, None].float() if pres is not None else 0.0
    x = torch.where(seen, x - f * counts.float() - p, x)
    return x


def sample_mask(logits, temperature, top_k, top_p):
    """Boolean [B, V] of tokens allowed after temperature / top-k / top-p (exact semantics)."""
    B, V = logits.shape
    x = logits.float() / temperature.clamp_min(1e-6)[:, None]
    allowed = torch.ones_like(x, dtype=torch.bool)
    for r in range(B):
        k = int(top_k[r]) if top_k is not None else 0
        if 0 < k < V:
            kth = torch.topk(x[r], k).values[-1]
            allowed[r] &= x[r] >= kth
        p = float(top_p[r]) if top_p is not None else 1.0
        if p < 1.0:
            xr = torch.where(allowed[r], x[r], torch.tensor(float("-inf")))
            probs = torch.softmax(xr, -1)
            sp, idx = probs.sort(descending=True)
            cum = sp.cumsum(0)
            # smallest prefix with mass >= p
            n = int((cum < p).sum().item()) + 1
            thr = sp[min(n, V) - 1]
            allowed[r] &= probs >= thr
    return allowed


def sample(logits, temperature, top_k=None, top_p=None, generator=None):
    """Greedy when temperature == 0 else a draw from the filtered distribution."""
    B = logits.shape[0]
    out = torch.empty(B, dtype=torch.int32)
    for r in range(B):
        if float(temperature[r]) <= 0:
            out[r] = int(torch.argmax(logits[r].float()))
            continue
        allowed = sample_mask(logits[r:r + 1], temperature[r:r + 1],
                              None if top_k is None else top_k[r:r + 1],
                              None if top_p is None else top_p[r:r + 1])[0]
        x = logits[r].float() / float(temperature[r])
        x = torch.where(allowed, x, torch.tensor(float("-inf")))
        probs = torch.softmax(x, -1)
        out[r] = int(torch.multinomial(probs, 1, generator=generator))
    return out


def mean_pool_l2(hidden: torch.Tensor, cu_seqlens: torch.Tensor) -> torch.Tensor:
    cu = cu_seqlens.tolist()
    h = hidden.float()
    out = torch.zeros(len(cu) - 1, h.shape[1], dtype=torch.float32, device=h.device)
    for b in range(len(cu) - 1):
        if cu[b + 1] > cu[b]:
            v = h[cu[b]:cu[b + 1]].mean(0)
            n = v.norm()
            out[b] = v / n if n > 0 else v
    return out


def cosine_topk(q: torch.Tensor, m: torch.Tensor, k: int, valid: torch.Tensor | None = None):
    s = q.float() @ m.float().t()
    if valid is not None:
        s = s.masked_fill(valid[: m.shape[0]].to(s.device) == 0, float("-inf"))
    # stable order: descending score, ascending index on ties
    idx = torch.arange(m.shape[0], device=s.device).expand_as(s)
    order = torch.argsort(s, dim=1, descending=True, stable=True)[:, :k]
    return torch.gather(s, 1, order), torch.gather(idx, 1, order)


def moe_route(logits: torch.Tensor, k: int, renorm: bool = True):
    """softmax -> top-k (lowest index wins ties) -> optional renormalisation."""
    p = torch.softmax(logits.float(), dim=-1)
    # stable top-k: sort by (-p, index)
    order = torch.argsort(-p, dim=-1, stable=True)[:, :k]
    w = torch.gather(p, 1, order)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return order.to(torch.int32), w


def moe(x: torch.Tensor, router: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor, k: int,
        e_lo: int = 0, renorm: bool = True, ids=None, wts=None,
        act_dtype=None) -> torch.Tensor:
    """fp32 oracle of the MoE FFN over the experts [e_lo, e_lo + w_gu.shape[0]).

    ``ids``/``wts`` pin the routing (so near-tie top-k choices cannot flip between
    implementations); ``act_dtype`` rounds the SwiGLU activation like a kernel
    that stores it (bf16) between the two GEMMs."""
    xf = x.float()
    if ids is None:
        ids, wts = moe_route(xf @ router.float().t(), k, renorm)
    out = torch.zeros_like(xf)
    n_loc = w_gu.shape[0]
    inter = w_down.shape[2]
    for t in range(x.shape[0]):
        for j in range(k):
            e = int(ids[t, j]) - e_lo
            if 0 <= e < n_loc:
                h = w_gu[e].float() @ xf[t]
                a = torch.nn.functional.silu(h[:inter]) * h[inter:]
                if act_dtype is not None:
                    a = a.to(act_dtype).float()
                out[t] += float(wts[t, j]) * (w_down[e].float() @ a)
    return out


def apply_token_mask(logits: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """fp32 reference of K13: unpack the int32 bit rows and fill -inf where clear."""
    B, V = logits.shape
    bits = (mask.to(torch.int64).unsqueeze(-1) >> torch.arange(32, device=mask.device)) & 1
    allow = bits.reshape(B, -1)[:, :V].to(torch.bool).to(logits.device)
    logits.masked_fill_(~allow, float("-inf"))
    return logits


def dense_forward(cfg, w: dict, tokens: list[int]) -> torch.Tensor:
    """fp32 whole-model oracle: dense causal forward of ONE sequence.

    Independent of the engine's paged-KV / batching machinery (no block tables,
    no slots, no chunking, no graphs): embedding -> per layer RMSNorm, QKV,
    RoPE, causal GQA softmax attention, O, residual, RMSNorm, SwiGLU MLP (or
    top-k MoE), residual -> final norm -> LM head.  ``w`` holds the model's
    weights in its natural [out, in] layout (``LlamaModel.w``, any device /
    dtype; computed in fp32 on the CPU).  Returns fp32 logits [T, vocab].
    """
    f = lambda t: t.detach().to("cpu", torch.float32)  # noqa: E731
    T = len(tokens)
    D, hq, hkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    ids = torch.tensor(tokens, dtype=torch.long)
    pos = torch.arange(T)
    cs = rope_cos_sin(max(T, 1), D, cfg.rope_theta, cfg.rope_scaling)
    x = f(w["embed"])[ids]
    causal = torch.ones(T, T, dtype=torch.bool).tril()
    scale = 1.0 / math.sqrt(D)
    for layer in w["layers"]:
        h = rmsnorm(x, f(layer["in_norm"]), cfg.rms_eps)
        qkv = h @ f(layer["qkv"]).t()
        q = qkv[:, : hq * D].view(T, hq, D)
        k = qkv[:, hq * D: (hq + hkv) * D].view(T, hkv, D)
        v = qkv[:, (hq + hkv) * D:].view(T, hkv, D)
        q, k = apply_rope(q, pos, cs), apply_rope(k, pos, cs)
        g = hq // hkv
        kk, vv = k.repeat_interleave(g, dim=1), v.repeat_interleave(g, dim=1)
        s = torch.einsum("qhd,khd->hqk", q, kk) * scale
        s = s.masked_fill(~causal[None], float("-inf"))
        o = torch.einsum("hqk,khd->qhd", torch.softmax(s, dim=-1), vv).reshape(T, hq * D)
        x = x + o @ f(layer["o"]).t()
        h = rmsnorm(x, f(layer["post_norm"]), cfg.rms_eps)
        if "router" in layer:
            m = moe(h, f(layer["router"]), f(layer["experts_gate_up"]),
                    f(layer["experts_down"]), cfg.experts_per_token)
        else:
            m = silu_mul(h @ f(layer["gate_up"]).t()) @ f(layer["down"]).t()
        x = x + m
    x = rmsnorm(x, f(w["final_norm"]), cfg.rms_eps)
    return x @ f(w["lm_head"]).t()
