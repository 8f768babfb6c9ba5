"""Numerics of every hand-written gfx950 kernel against the plain-PyTorch fp32
reference of the same op (omnia_amd.ops.reference).  GPU only."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from omnia_amd import ops
from omnia_amd.ops import reference as ref

DEV = "cuda"


def _close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


def test_extension_is_native():
    k = ops.kernels()
    assert k.arch == "gfx950"
    assert k.__file__.endswith("_omnia_kernels.so")


@pytest.mark.parametrize("rows,d", [(1, 4096), (37, 4096), (256, 8192), (5, 2048)])
def test_rmsnorm(rows, d):
    torch.manual_seed(0)
    x = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(d, device=DEV, dtype=torch.bfloat16)
    y = ops.rmsnorm(x, w, 1e-5)
    _close(y, ref.rmsnorm(x, w, 1e-5), 0.05, 0.01)


def test_fused_add_rmsnorm():
    torch.manual_seed(1)
    x = torch.randn(33, 4096, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(33, 4096, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(4096, device=DEV, dtype=torch.bfloat16)
    ey, er = ref.fused_add_rmsnorm(x, r, w, 1e-5)
    ops.fused_add_rmsnorm(x, r, w, 1e-5)
    _close(r, er, 0.0)
    _close(x, ey, 0.05, 0.01)


def test_silu_mul():
    x = torch.randn(19, 2 * 14336, device=DEV, dtype=torch.bfloat16)
    _close(ops.silu_mul(x), ref.silu_mul(x), 0.02, 0.01)


def test_embedding():
    w = torch.randn(1000, 4096, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, 1000, (57,), device=DEV, dtype=torch.int32)
    _close(ops.embedding(ids, w), w[ids.long()], 0.0)
    # vocab-parallel shard: ids outside [500, 1000) give zero rows
    y = ops.embedding(ids, w[500:].contiguous(), vocab_start=500)
    exp = torch.where((ids >= 500)[:, None], w[ids.long()], torch.zeros_like(w[ids.long()]))
    _close(y, exp, 0.0)


def _make_cache(nb, hkv, bs, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    kc = torch.randn(nb, hkv, bs, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(nb, hkv, bs, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    return kc, vc


@pytest.mark.parametrize("bs", [16, 32])
def test_rope_kv(bs):
    T, hq, hkv = 23, 32, 8
    qkv = torch.randn(T, (hq + 2 * hkv) * 128, device=DEV, dtype=torch.bfloat16)
    q = qkv[:, : hq * 128]
    k = qkv[:, hq * 128: (hq + hkv) * 128]
    v = qkv[:, (hq + hkv) * 128:]
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(8192, 128, 500000.0, device=DEV)
    kc, vc = _make_cache(16, hkv, bs)
    kc0, vc0 = kc.clone(), vc.clone()
    slots = torch.randperm(16 * bs, device=DEV)[:T].long()
    eq = ref.apply_rope(q.reshape(T, hq, 128).clone(), pos, cs)
    ek = ref.apply_rope(k.reshape(T, hkv, 128).clone(), pos, cs)
    ev = v.reshape(T, hkv, 128).clone()
    ref.write_kv(kc0, vc0, ek, ev, slots)
    ops.rope_kv(q, k, v, pos, cs, kc, vc, slots, hq, hkv, bs)
    _close(q.reshape(T, hq, 128), eq, 0.02, 0.01)
    _close(kc, kc0, 0.02, 0.01)
    _close(vc, vc0, 0.0)


def _tables(lens, bs, nb_total):
    maxb = max((l + bs - 1) // bs for l in lens)
    perm = torch.randperm(nb_total)
    bt = torch.zeros(len(lens), maxb + 2, dtype=torch.int32)
    p = 0
    for i, l in enumerate(lens):
        nb = (l + bs - 1) // bs
        bt[i, :nb] = perm[p:p + nb].int()
        p += nb
    return bt.to(DEV)


@pytest.mark.parametrize("uv", ["4", "8", "g8"])
@pytest.mark.parametrize("nw", ["2", "4"])
@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 8)])
@pytest.mark.parametrize("bs", [16, 32])
def test_decode_attention(hq, hkv, bs, nw, uv, monkeypatch):
    # both workgroup shapes (2 / 4 waves; the launcher picks by grid size) and
    # both V prefetch depths
    monkeypatch.setenv("OMNIA_DECODE_NW", nw)
    monkeypatch.setenv("OMNIA_DECODE_U", "8" if uv == "g8" else uv)
    monkeypatch.setenv("OMNIA_DECODE_UG", "8" if uv == "g8" else "4")
    torch.manual_seed(3)
    lens = [1, 17, 64, 513, 1500, 3000]
    B = len(lens)
    nb_total = sum((l + bs - 1) // bs for l in lens) + 8
    kc, vc = _make_cache(nb_total, hkv, bs, seed=3)
    bt = _tables(lens, bs, nb_total)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = torch.randn(B, hq, 128, device=DEV, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(128)
    out = ops.decode_attention(q, kc, vc, bt, sl, scale, part_size=512)
    qsl = torch.arange(B + 1, dtype=torch.int32)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl, sl.cpu(), scale)
    _close(out.cpu(), exp, 0.02, 0.02)


@pytest.mark.parametrize("splits,split_min", [(2, 64), (4, 64), (8, 32), (64, 64)])
@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 1)])
def test_decode_attention_length_balanced_split(hq, hkv, splits, split_min):
    """Device-side split (splits > 0): every context cut into up to `splits`
    equal page-aligned partitions (>= split_min keys, <= part_size) and merged
    -- against the fp32 oracle and the fixed-partition kernel."""
    torch.manual_seed(5)
    bs = 32
    lens = [1, 31, 32, 33, 200, 513, 640, 1500, 3000]
    B = len(lens)
    nb_total = sum((l + bs - 1) // bs for l in lens) + 8
    kc, vc = _make_cache(nb_total, hkv, bs, seed=5)
    bt = _tables(lens, bs, nb_total)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = torch.randn(B, hq, 128, device=DEV, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(128)
    out = ops.decode_attention(q, kc, vc, bt, sl, scale, part_size=512, splits=splits,
                               split_min=split_min)
    qsl = torch.arange(B + 1, dtype=torch.int32)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl, sl.cpu(), scale)
    _close(out.cpu(), exp, 0.02, 0.02)
    fixed = ops.decode_attention(q, kc, vc, bt, sl, scale, part_size=512)
    _close(out.float().cpu(), fixed.float().cpu(), 0.02, 0.02)


@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("hq,hkv,hp,qt", [(32, 8, 1, 64), (32, 8, 2, 64), (32, 8, 4, 64),
                                          (64, 8, 4, 64), (8, 8, 0, 64), (32, 8, 1, 128),
                                          (8, 8, 1, 128), (32, 8, 0, 32), (64, 8, 0, 32),
                                          (16, 8, 0, 32), (8, 8, 0, 32), (8, 1, 0, 32)])
def test_prefill_attention(bs, hq, hkv, hp, qt):
    torch.manual_seed(4)
    # (new tokens, cached prefix) per sequence: ragged + page-boundary edges
    specs = [(1, 0), (64, 0), (100, 37), (257, 0), (5, 600), (130, 64)]
    lens = [q + c for q, c in specs]
    qlens = [q for q, _ in specs]
    nb_total = sum((l + bs - 1) // bs for l in lens) + 8
    kc, vc = _make_cache(nb_total, hkv, bs, seed=4)
    bt = _tables(lens, bs, nb_total)
    T = sum(qlens)
    q = torch.randn(T, hq, 128, device=DEV, dtype=torch.bfloat16)
    qsl = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(128)
    out = ops.prefill_attention(q, kc, vc, bt, qsl, sl, scale, heads_per_wave=hp, q_tile=qt)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl.cpu(), sl.cpu(), scale)
    _close(out.cpu(), exp, 0.03, 0.02)


def test_sample_greedy_matches_argmax():
    logits = torch.randn(7, 128256, device=DEV)
    temp = torch.zeros(7, device=DEV)
    tok = ops.sample(logits, temp)
    assert torch.equal(tok.long().cpu(), logits.argmax(-1).cpu())
    tok16 = ops.sample(logits.bfloat16(), temp)
    assert torch.equal(tok16.long().cpu(), logits.bfloat16().float().argmax(-1).cpu())


def test_sample_bf16_vector_path_logprob_and_masked():
    """bf16 rows take the fused one-pass max/argmax/partition sweep (16-B
    loads): token, log-prob and -inf (grammar-masked) entries vs fp32 torch."""
    torch.manual_seed(11)
    B, V = 9, 128256
    logits = (torch.randn(B, V, device=DEV) * 4).bfloat16()
    logits[0, :1000] = float("-inf")
    logits[1, 5] = 30.0
    logits[2, 7] = 25.0
    logits[2, 9] = 25.0  # tie -> lowest index, like argmax
    temp = torch.zeros(B, device=DEV)
    lp = torch.empty(B, device=DEV)
    tok = ops.sample(logits, temp, out_logprob=lp).long().cpu()
    f = logits.float().cpu()
    assert torch.equal(tok, f.argmax(-1))
    exp_lp = torch.log_softmax(f, -1)[torch.arange(B), tok]
    assert (lp.cpu() - exp_lp).abs().max() < 1e-3
    # temperature path (same fused sweep feeds its max / partition function)
    temp = torch.full((B,), 0.9, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV)
    tok = ops.sample(logits, temp, seeds=seeds, steps=seeds, out_logprob=lp).long().cpu()
    exp_lp = torch.log_softmax(f / 0.9, -1)[torch.arange(B), tok]
    assert (lp.cpu() - exp_lp).abs().max() < 1e-3
    assert bool(torch.isfinite(f[torch.arange(B), tok]).all())


def test_sample_topk_topp_support():
    torch.manual_seed(5)
    B, V = 6, 32000
    logits = torch.randn(B, V, device=DEV) * 3
    temp = torch.full((B,), 0.8, device=DEV)
    top_k = torch.tensor([0, 1, 5, 50, 0, 20], dtype=torch.int32, device=DEV)
    top_p = torch.tensor([1.0, 1.0, 1.0, 0.9, 0.5, 0.3], device=DEV)
    allowed = ref.sample_mask(logits.cpu(), temp.cpu(), top_k.cpu(), top_p.cpu())
    for step in range(20):
        seeds = torch.full((B,), 1234, dtype=torch.int64, device=DEV)
        steps = torch.full((B,), step, dtype=torch.int64, device=DEV)
        tok = ops.sample(logits, temp, top_k, top_p, seeds=seeds, steps=steps).long().cpu()
        assert allowed[torch.arange(B), tok].all(), (step, tok)
    # top_k = 1 is greedy
    assert int(tok[1]) == int(logits[1].argmax())


def test_sample_distribution_temperature():
    """Gumbel-max draw matches softmax(logits / T) in distribution."""
    V = 8
    logits = torch.tensor([[2.0, 1.0, 0.5, 0.0, -1.0, -2.0, 0.3, 1.5]], device=DEV)
    temp = torch.full((4096,), 0.7, device=DEV)
    big = logits.expand(4096, V).contiguous()
    seeds = torch.arange(4096, dtype=torch.int64, device=DEV)
    tok = ops.sample(big, temp, seeds=seeds, steps=torch.zeros(4096, dtype=torch.int64,
                                                                  device=DEV)).long().cpu()
    freq = torch.bincount(tok, minlength=V).float() / 4096
    exp = torch.softmax(logits[0].cpu() / 0.7, -1)
    assert (freq - exp).abs().max() < 0.03


def test_sample_penalties():
    B, V = 2, 1000
    logits = torch.zeros(B, V, device=DEV)
    logits[:, 10] = 5.0
    logits[:, 20] = 4.0
    counts = torch.zeros(B, V, dtype=torch.int32, device=DEV)
    counts[0, 10] = 3
    temp = torch.zeros(B, device=DEV)
    freq = torch.tensor([1.0, 1.0], device=DEV)
    pres = torch.tensor([0.0, 0.0], device=DEV)
    tok = ops.sample(logits, temp, counts=counts, freq_pen=freq, pres_pen=pres).cpu()
    assert tok.tolist() == [20, 10]
    assert int(counts[0, 20]) == 1 and int(counts[1, 10]) == 1


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("V", [1000, 128256])
def test_apply_token_mask_matches_reference(dtype, V):
    g = torch.Generator().manual_seed(5)
    B, W = 5, (V + 31) // 32
    logits = torch.randn(B, V, generator=g).to(dtype)
    mask = torch.randint(-2**31, 2**31 - 1, (B, W), generator=g, dtype=torch.int64).to(torch.int32)
    mask[2] = -1  # an unconstrained row stays untouched
    want = ref.apply_token_mask(logits.float().clone(), mask)
    got = ops.apply_token_mask(logits.cuda(), mask.cuda()).float().cpu()
    assert torch.equal(torch.isinf(got), torch.isinf(want))
    fin = torch.isfinite(want)
    assert torch.equal(got[fin], want[fin])
    # masked greedy sampling picks the best ALLOWED token
    tok = ops.sample(ops.apply_token_mask(logits.cuda(), mask.cuda()),
                     torch.zeros(B, device="cuda"))
    assert torch.equal(tok.cpu().long(), want.argmax(-1))
