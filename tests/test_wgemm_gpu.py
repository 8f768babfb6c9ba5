"""Weight-streaming decode GEMM (ops/csrc/wgemm.hip) vs the fp32 PyTorch oracle:
bf16 output, fused SwiGLU, and fp32 split-K partial slabs, across batch sizes
that exercise every M-fragment count and the clamped tail rows."""
import pytest
import torch

from omnia_amd import ops
from omnia_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _mk(M, N, K, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    return x, w


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 100, 128, 200, 256])
@pytest.mark.parametrize("nw,nwaves", [(1, 4), (2, 4), (4, 4), (2, 2)])
def test_mode0_matches_fp32(M, nw, nwaves):
    if nw == 4 and M > 128:
        pytest.skip("NW=4 covers M <= 128")
    x, w = _mk(M, 1024, 512, seed=M)
    out = ops.wgemm(0, x, w, 1, nw, nwaves)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M", [3, 48, 160, 256])
@pytest.mark.parametrize("nw", [2, 4])
def test_mode1_swiglu_matches_fp32(M, nw):
    if nw == 4 and M > 128:
        pytest.skip("NW=4 covers M <= 128")
    I = 512
    x, w = _mk(M, 2 * I, 1024, seed=7 + M)
    out = ops.wgemm(1, x, w, 1, nw, 4)
    want = ref.silu_mul((x.float() @ w.float().t()))
    torch.testing.assert_close(out.float(), want.float(), rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("M,S", [(5, 2), (77, 4), (256, 8), (256, 1)])
def test_mode2_splitk_slabs_sum_to_product(M, S):
    x, w = _mk(M, 768, 2048, seed=M + S)
    part = ops.wgemm(2, x, w, S, 1, 4)
    assert part.shape == (S, M, 768) and part.dtype == torch.float32
    want = x.float() @ w.float().t()
    torch.testing.assert_close(part.sum(0), want, rtol=1e-3, atol=2e-3)


def test_llama3_8b_shapes():
    """The five Llama-3-8B decode projections at the serving batch."""
    M = 256
    for N, K, mode, S, nw in ((6144, 4096, 2, 4, 2), (4096, 4096, 2, 4, 1),
                              (14336, 4096, 1, 1, 2), (4096, 14336, 2, 4, 1)):
        x, w = _mk(M, 2 * N if mode == 1 else N, K, seed=N + K)
        out = ops.wgemm(mode, x, w, S, nw, 4)
        full = x.float() @ w.float().t()
        want = ref.silu_mul(full) if mode == 1 else full
        got = out.sum(0) if mode == 2 else out.float()
        torch.testing.assert_close(got, want.float(), rtol=3e-2, atol=3e-2)


def test_rejects_bad_shapes_before_launch():
    x, w = _mk(16, 1000, 512)
    with pytest.raises(RuntimeError, match="wgemm"):
        ops.wgemm(0, x, w, 1, 2, 4)  # 1000 rows not a multiple of the block's 128
    x, w = _mk(300, 1024, 512)
    with pytest.raises(RuntimeError):
        ops.wgemm(0, x, w, 1, 2, 4)  # M > 256


# ------------------------------------------- wide-batch kernel (wgemm_wide.hip)
@pytest.mark.parametrize("M", [129, 160, 192, 200, 256])
@pytest.mark.parametrize("wt", [1, 2])
def test_wide_mode0_matches_fp32(M, wt):
    x, w = _mk(M, 1024, 1024, seed=M + wt)
    out = ops.wgemm_wide(0, x, w, 1, wt)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M", [130, 256])
def test_wide_mode1_swiglu_matches_fp32(M):
    I = 512
    x, w = _mk(M, 2 * I, 1024, seed=11 + M)
    out = ops.wgemm_wide(1, x, w, 1, 2)
    want = ref.silu_mul((x.float() @ w.float().t()))
    torch.testing.assert_close(out.float(), want.float(), rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("M,S,wt", [(256, 2, 2), (177, 4, 1), (256, 8, 1)])
def test_wide_mode2_splitk_slabs(M, S, wt):
    x, w = _mk(M, 1024, 8192, seed=M * S)
    part = ops.wgemm_wide(2, x, w, S, wt)
    assert part.shape == (S, M, 1024)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(part.sum(0), want, rtol=1e-3, atol=3e-3)


def test_wide_llama3_8b_shapes():
    M = 256
    for N, K, mode, S, wt in ((6144, 4096, 2, 2, 2), (4096, 4096, 2, 4, 2),
                              (14336, 4096, 1, 1, 2), (4096, 14336, 2, 7, 2)):
        x, w = _mk(M, 2 * N if mode == 1 else N, K, seed=N + K)
        out = ops.wgemm_wide(mode, x, w, S, wt)
        full = x.float() @ w.float().t()
        want = ref.silu_mul(full) if mode == 1 else full
        got = out.sum(0) if mode == 2 else out.float()
        torch.testing.assert_close(got, want.float(), rtol=3e-2, atol=3e-2)


def test_wide_rejects_bad_shapes_before_launch():
    x, w = _mk(100, 1024, 1024)
    with pytest.raises(RuntimeError, match="wgemm_wide"):
        ops.wgemm_wide(0, x, w, 1, 2)  # M <= 128 belongs to wgemm
    x, w = _mk(256, 1024, 1000)
    with pytest.raises(RuntimeError, match="wgemm_wide"):
        ops.wgemm_wide(0, x, w, 1, 2)  # K not a whole number of ring turns
