"""Prefill GEMM with fused epilogues (ops/csrc/pgemm.hip) against fp32 PyTorch
references of the same ops: plain / row-scaled GEMM, gate_up + SwiGLU, residual
add + row sum of squares, QKV + RoPE + paged KV write.  Ragged M (not a multiple
of the 256-row tile) and K > one iteration are covered; every check has a
negative control (a deliberately wrong reference must FAIL the same tolerance)."""
import pytest
import torch

from omnia_amd import ops
from omnia_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rand(*shape, std=1.0, gen=None):
    return (torch.randn(*shape, device=DEV, generator=gen) * std).to(torch.bfloat16)


def _close(got, want, tol):
    err = (got.float() - want.float()).abs().max().item()
    scale = want.float().abs().max().item()
    return err <= tol * scale, err / max(scale, 1e-30)


@pytest.fixture(autouse=True, params=[0, 1], ids=["8wave", "4wave"])
def schedule(request):
    """Every check runs on both main loops: the 8-wave ping-pong and the 4-wave
    one-wave-per-SIMD schedule (same epilogues)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.kernels().pgemm_set_schedule(request.param)
    yield request.param
    ops.kernels().pgemm_set_schedule(0)


@pytest.fixture(scope="module")
def gen():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device=DEV)
    g.manual_seed(1234)
    return g


@pytest.mark.parametrize("M,N,K", [(256, 512, 128), (300, 768, 512), (1000, 1024, 1280)])
def test_plain_and_row_scaled(gen, M, N, K):
    x = _rand(M, K, gen=gen)
    w = _rand(N, K, std=0.05, gen=gen)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.pgemm(0, x, w, out=out)
    want = x.float() @ w.float().t()
    ok, e = _close(out, want, 1e-2)
    assert ok, e
    # asymmetric negative control: the transposed-operand product must not match
    bad = x.float() @ w.float().flip(0).t()
    assert not _close(out, bad, 1e-2)[0]
    # row scale from 3 partial sums of squares
    ss = torch.rand(M, 3, device=DEV, generator=gen) * K
    ops.pgemm(0, x, w, out=out, ss_in=ss, inv_d=1.0 / K, eps=1e-5)
    rs = torch.rsqrt(ss.sum(1) / K + 1e-5)
    ok, e = _close(out, want * rs[:, None], 1e-2)
    assert ok, e
    assert not _close(out, want, 1e-2)[0]


@pytest.mark.parametrize("M,F,K", [(256, 256, 256), (517, 384, 640)])
def test_swiglu(gen, M, F, K):
    x = _rand(M, K, gen=gen)
    w = _rand(2 * F, K, std=0.05, gen=gen)
    ss = torch.rand(M, 2, device=DEV, generator=gen) * K
    out = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    ops.pgemm(1, x, w, out=out, ss_in=ss, inv_d=1.0 / K, eps=1e-6)
    rs = torch.rsqrt(ss.sum(1) / K + 1e-6)[:, None]
    h = (x.float() @ w.float().t()) * rs
    g, u = h[:, :F], h[:, F:]
    want = torch.nn.functional.silu(g) * u
    ok, e = _close(out, want, 1.5e-2)
    assert ok, e
    swapped = torch.nn.functional.silu(u) * g
    assert not _close(out, swapped, 1.5e-2)[0]


@pytest.mark.parametrize("M,N,K", [(256, 512, 256), (389, 1024, 384)])
def test_residual_sumsq(gen, M, N, K):
    x = _rand(M, K, gen=gen)
    w = _rand(N, K, std=0.05, gen=gen)
    res = _rand(M, N, gen=gen)
    res0 = res.clone()
    ss = torch.full((M, N // 256), -1.0, device=DEV)
    ops.pgemm(2, x, w, out=res, ss_out=ss)
    g = (x.float() @ w.float().t()).to(torch.bfloat16)
    want = (res0.float() + g.float()).to(torch.bfloat16)
    ok, e = _close(res, want, 1e-2)
    assert ok, e
    want_ss = want.float().pow(2).view(M, N // 256, 256).sum(-1)
    ok, e = _close(ss, want_ss, 1e-3)
    assert ok, e
    assert not _close(res, res0, 1e-2)[0]


def test_qkv_rope_kv_write(gen):
    hq, hkv, D, bs = 8, 2, 128, 16
    M, K = 300, 512
    N = (hq + 2 * hkv) * D
    x = _rand(M, K, gen=gen)
    w = _rand(N, K, std=0.05, gen=gen)
    ss = torch.rand(M, 1, device=DEV, generator=gen) * K
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32, generator=gen)
    cos_sin = ref.rope_cos_sin(8192, D, 5e5, {"rope_type": "llama3", "factor": 8.0}, device=DEV)
    nb = 64
    kc = torch.zeros(nb, hkv, bs, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    perm = torch.randperm(nb * bs, device=DEV, generator=gen)[:M]
    slots = perm.to(torch.int64)
    slots[5] = -1  # padding row: no KV write
    q = torch.empty(M, hq * D, dtype=torch.bfloat16, device=DEV)
    ops.pgemm(3, x, w, out=q, ss_in=ss, inv_d=1.0 / K, eps=1e-5, positions=positions,
              cos_sin=cos_sin, k_cache=kc, v_cache=vc, slots=slots, hq=hq, hkv=hkv,
              block_size=bs)
    rs = torch.rsqrt(ss.sum(1) / K + 1e-5)[:, None]
    qkv = ((x.float() @ w.float().t()) * rs).to(torch.bfloat16)
    qq = ref.apply_rope(qkv[:, : hq * D].view(M, hq, D), positions, cos_sin)
    kk = ref.apply_rope(qkv[:, hq * D:(hq + hkv) * D].view(M, hkv, D), positions, cos_sin)
    vv = qkv[:, (hq + hkv) * D:].view(M, hkv, D)
    ok, e = _close(q.view(M, hq, D), qq, 2e-2)
    assert ok, e
    unrotated = qkv[:, : hq * D]
    assert not _close(q, unrotated, 2e-2)[0]
    kc_want = torch.zeros_like(kc)
    vc_want = torch.zeros_like(vc)
    keep = slots >= 0
    ref.write_kv(kc_want, vc_want, kk[keep], vv[keep], slots[keep])
    ok, e = _close(kc, kc_want, 2e-2)
    assert ok, e
    ok, e = _close(vc, vc_want, 2e-2)
    assert ok, e


def test_row_sumsq(gen):
    x = _rand(333, 4096, gen=gen)
    ss = torch.empty(333, device=DEV)
    ops.row_sumsq(x, out=ss)
    ok, e = _close(ss, x.float().pow(2).sum(1), 1e-4)
    assert ok, e


def test_rejects_bad_shapes(gen):
    x = _rand(256, 192, gen=gen)  # K not a multiple of 128
    w = _rand(256, 192, gen=gen)
    with pytest.raises(RuntimeError):
        ops.pgemm(0, x, w, out=torch.empty(256, 256, dtype=torch.bfloat16, device=DEV))


@pytest.mark.parametrize("epi", [0, 1, 2])
def test_schedules_are_bit_identical(gen, schedule, epi):
    """Both main loops accumulate every output element over K in the same order
    with the same instruction: identical bits, ragged M included."""
    M, K = 777, 1024
    N = 512
    x = _rand(M, K, gen=gen)
    w = _rand(2 * N if epi == 1 else N, K, std=0.05, gen=gen)
    ss = torch.rand(M, 2, device=DEV, generator=gen) * K
    outs = []
    for sched in (0, 1):
        ops.kernels().pgemm_set_schedule(sched)
        if epi == 2:
            o = _rand(M, N, gen=torch.Generator(device=DEV).manual_seed(5))
            sso = torch.zeros(M, N // 256, device=DEV)
            ops.pgemm(2, x, w, out=o, ss_out=sso)
            outs.append((o, sso))
        else:
            o = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            ops.pgemm(epi, x, w, out=o, ss_in=ss, inv_d=1.0 / K, eps=1e-5)
            outs.append((o,))
    ops.kernels().pgemm_set_schedule(schedule)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,K,S", [(256, 512, 1024, 4), (192, 768, 2048, 8), (77, 256, 512, 2),
                                     (300, 512, 896, 7)])
def test_splitk_slabs(gen, schedule, M, N, K, S):
    """EPI 4: fp16 slab s holds x[:, Ks] @ w[:, Ks]^T of K-slice s; decode sizes
    (one m-tile, ragged) and prefill sizes (two m-tiles) against fp32 matmuls."""
    x = _rand(M, K, gen=gen)
    w = _rand(N, K, std=0.05, gen=gen)
    parts = torch.full((S, M, N), float("nan"), dtype=torch.float16, device=DEV)
    ops.pgemm_splitk(x, w, S, parts, schedule)
    ks = K // S
    for s in range(S):
        want = x[:, s * ks:(s + 1) * ks].float() @ w[:, s * ks:(s + 1) * ks].float().t()
        ok, e = _close(parts[s], want, 2e-3)
        assert ok, (s, e)
    total = x.float() @ w.float().t()
    ok, e = _close(parts.float().sum(0), total, 5e-3)
    assert ok, e
    # negative control: the slabs in the wrong K order do not match slice 0
    want0 = x[:, :ks].float() @ w[:, :ks].float().t()
    assert not _close(parts[S - 1], want0, 2e-3)[0]


def test_splitk_saturates_fp16(gen, schedule):
    """A K-slice partial beyond the fp16 range saturates to +-65504 (finite), so
    the consumer never sees inf / NaN (unclamped casts)."""
    M, N, K, S = 256, 256, 512, 2
    x = torch.full((M, K), 16.0, dtype=torch.bfloat16, device=DEV)
    w = torch.full((N, K), 16.0, dtype=torch.bfloat16, device=DEV)  # partial = 256*256 = 65536
    w[: N // 2] = -16.0
    parts = torch.empty(S, M, N, dtype=torch.float16, device=DEV)
    ops.pgemm_splitk(x, w, S, parts, schedule)
    assert torch.isfinite(parts).all()
    assert (parts[:, :, N // 2:] == 65504).all() and (parts[:, :, : N // 2] == -65504).all()


def test_splitk_feeds_consumer(gen, schedule):
    """pgemm split-K slabs through splitk_swiglu == SwiGLU of the fp32 product."""
    M, F, K, S = 256, 512, 2048, 4
    x = _rand(M, K, gen=gen)
    w = _rand(2 * F, K, std=0.05, gen=gen)
    act = ops.splitk_swiglu(ops.pgemm_splitk(x, w, S, sched=schedule))
    h = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    want = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
    ok, e = _close(act, want, 2e-2)
    assert ok, e


def test_splitk_rejects_bad_split(gen):
    x = _rand(256, 1024, gen=gen)
    w = _rand(256, 1024, gen=gen)
    with pytest.raises(RuntimeError):  # K / S = 341.33
        ops.pgemm_splitk(x, w, 3)
    with pytest.raises(RuntimeError):  # K / S = 64: not whole iterations of two K-tiles
        ops.pgemm_splitk(x, w, 16)


@pytest.mark.parametrize("hq,hkv", [(8, 1), (4, 1), (6, 1)])
def test_qkv_epilogue_tp_shard_heads(gen, schedule, hq, hkv):
    """TP shards' QKV: one KV head per rank (Llama-3-70B at TP=8: hq 8, hkv 1 ->
    10 heads = 5 tiles) -- 256-column tiles straddle the q / k / v boundaries;
    the per-head epilogue still routes q, k and v correctly."""
    D, bs, M, K = 128, 16, 300, 512
    N = (hq + 2 * hkv) * D
    x = _rand(M, K, gen=gen)
    w = _rand(N, K, std=0.05, gen=gen)
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32, generator=gen)
    cos_sin = ref.rope_cos_sin(8192, D, 5e5, None, device=DEV)
    nb = 64
    kc = torch.zeros(nb, hkv, bs, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(nb * bs, device=DEV, generator=gen)[:M].to(torch.int64)
    q = torch.empty(M, hq * D, dtype=torch.bfloat16, device=DEV)
    ops.pgemm(3, x, w, out=q, positions=positions, cos_sin=cos_sin, k_cache=kc, v_cache=vc,
              slots=slots, hq=hq, hkv=hkv, block_size=bs)
    qkv = (x.float() @ w.float().t()).to(torch.bfloat16)
    qq = ref.apply_rope(qkv[:, : hq * D].view(M, hq, D), positions, cos_sin)
    kk = ref.apply_rope(qkv[:, hq * D:(hq + hkv) * D].view(M, hkv, D), positions, cos_sin)
    vv = qkv[:, (hq + hkv) * D:].view(M, hkv, D)
    ok, e = _close(q.view(M, hq, D), qq, 2e-2)
    assert ok, e
    kw, vw = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.write_kv(kw, vw, kk, vv, slots)
    assert _close(kc, kw, 2e-2)[0] and _close(vc, vw, 2e-2)[0]
    assert not _close(vc, kw, 2e-2)[0]  # k and v not swapped
