"""Split-K consumer kernels (ops/csrc/splitk.hip) vs their fp32 PyTorch
semantics (the CPU fallbacks in omnia_amd.ops, built on ops/reference.py)."""
import pytest
import torch

from omnia_amd import ops
from omnia_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _parts(S, M, N, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(S, M, N, device="cuda", generator=g) * 0.5


@pytest.mark.parametrize("S,M,d", [(1, 3, 4096), (4, 256, 4096), (8, 17, 8192), (2, 64, 2048)])
def test_splitk_add_rmsnorm(S, M, d):
    p = _parts(S, M, d, S + M)
    res = torch.randn(M, d, device="cuda").to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(d, device="cuda")).to(torch.bfloat16)
    res_ref = res.clone().cpu()
    out = ops.splitk_add_rmsnorm(p, res, w, 1e-5)
    want = ops.splitk_add_rmsnorm(p.cpu(), res_ref, w.cpu(), 1e-5)
    torch.testing.assert_close(res.cpu().float(), res_ref.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(out.cpu().float(), want.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("S,T,hq,hkv", [(1, 5, 4, 2), (4, 256, 32, 8), (8, 33, 8, 1)])
def test_splitk_rope_kv(S, T, hq, hkv):
    D, BS, NB = 128, 16, 64
    p = _parts(S, T, (hq + 2 * hkv) * D, T)
    pos = torch.randint(0, 2000, (T,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(NB * BS, device="cuda")[:T].to(torch.int64)
    slots[0] = -1  # a padded row: no KV write
    cs = ref.rope_cos_sin(4096, D, 500000.0, device="cuda")
    kc = torch.zeros(NB, hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc_r, vc_r = kc.cpu(), vc.cpu()
    q = ops.splitk_rope_kv(p, pos, cs, kc, vc, slots, hq, hkv, BS)
    m = slots.cpu() >= 0
    q_r = ops.splitk_rope_kv(p.cpu()[:, m], pos.cpu()[m], cs.cpu(), kc_r, vc_r, slots.cpu()[m],
                             hq, hkv, BS)
    torch.testing.assert_close(q.cpu()[m].float(), q_r.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(kc.cpu().float(), kc_r.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(vc.cpu().float(), vc_r.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("S,M,I", [(1, 7, 512), (4, 256, 14336), (16, 9, 3584)])
def test_splitk_swiglu_and_reduce(S, M, I):
    p = _parts(S, M, 2 * I, I)
    torch.testing.assert_close(ops.splitk_swiglu(p).cpu().float(),
                               ops.splitk_swiglu(p.cpu()).float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(ops.splitk_reduce(p).cpu().float(),
                               p.sum(0).cpu().to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("S,M", [(5, 256), (8, 33)])
def test_consumers_read_half_slabs(S, M):
    """fp16 slabs (tgemm mode 3) through every consumer give the same result as
    the same values held in fp32 slabs."""
    d, I, hq, hkv, D, BS, NB = 4096, 1024, 8, 2, 128, 16, 64
    p16 = _parts(S, M, d, S * M).half()
    res = torch.randn(M, d, device="cuda").to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(d, device="cuda")).to(torch.bfloat16)
    r16, r32 = res.clone(), res.clone()
    o16 = ops.splitk_add_rmsnorm(p16, r16, w, 1e-5)
    o32 = ops.splitk_add_rmsnorm(p16.float(), r32, w, 1e-5)
    torch.testing.assert_close(r16, r32, rtol=0, atol=0)
    torch.testing.assert_close(o16.float(), o32.float(), rtol=1e-2, atol=1e-2)
    g16 = _parts(S, M, 2 * I, M).half()
    torch.testing.assert_close(ops.splitk_swiglu(g16).float(),
                               ops.splitk_swiglu(g16.float()).float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(ops.splitk_reduce(g16).float(),
                               ops.splitk_reduce(g16.float()).float(), rtol=1e-2, atol=1e-2)
    q16 = _parts(S, M, (hq + 2 * hkv) * D, M + 1).half()
    pos = torch.randint(0, 2000, (M,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(NB * BS, device="cuda")[:M].to(torch.int64)
    cs = ref.rope_cos_sin(4096, D, 500000.0, device="cuda")
    caches = [torch.zeros(NB, hkv, BS, D, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
    qa = ops.splitk_rope_kv(q16, pos, cs, caches[0], caches[1], slots, hq, hkv, BS)
    qb = ops.splitk_rope_kv(q16.float(), pos, cs, caches[2], caches[3], slots, hq, hkv, BS)
    torch.testing.assert_close(qa.float(), qb.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(caches[0].float(), caches[2].float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(caches[1].float(), caches[3].float(), rtol=1e-2, atol=1e-2)
