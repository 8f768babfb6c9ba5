"""Full-batch tile decode GEMM (ops/csrc/tgemm.hip) vs the fp32 PyTorch oracle:
bf16 output, fused SwiGLU and fp32 split-K slabs (even and uneven splits), for
every block width, with and without non-temporal weight loads, across batch
sizes that exercise the clamped tail rows.  The asymmetric random operands
catch a transposed or row/column-swapped epilogue."""
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


@pytest.mark.parametrize("M", [1, 77, 129, 200, 256])
@pytest.mark.parametrize("bn,pipe", [(64, 0), (128, 0), (256, 0), (64, 4), (128, 4)])
def test_mode0_matches_fp32(M, bn, pipe):
    x, w = _mk(M, 1024, 512, seed=M + bn)
    out = ops.tgemm(0, x, w, 1, bn, int(bn == 128) | pipe)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M", [3, 190, 256])
@pytest.mark.parametrize("bn,wnt", [(64, 1), (128, 1), (256, 1), (128, 2), (256, 3), (128, 4),
                                    (64, 5)])
def test_mode1_swiglu_matches_fp32(M, bn, wnt):
    I = 512
    x, w = _mk(M, 2 * I, 1024, seed=7 + M + bn)
    out = ops.tgemm(1, x, w, 1, bn, wnt)
    want = ref.silu_mul((x.float() @ w.float().t()))
    torch.testing.assert_close(out.float(), want.float(), rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("M,S,bn,wnt", [(256, 1, 128, 0), (256, 3, 128, 0), (256, 5, 64, 0),
                                         (201, 7, 256, 0), (256, 16, 64, 0), (130, 2, 256, 0),
                                         (256, 3, 128, 4), (256, 5, 64, 5), (256, 16, 128, 4),
                                         (77, 7, 128, 5)])
def test_mode2_splitk_slabs_sum_to_product(M, S, bn, wnt):
    """Uneven splits; with the pipelined variant also slices of 1-3 k-steps (odd
    and even step counts through its two-step unrolled loop)."""
    x, w = _mk(M, 1024, 2048, seed=M + S + bn)  # 32 k-steps: S = 3, 5, 7 split unevenly
    part = ops.tgemm(2, x, w, S, bn, wnt)
    assert part.shape == (S, M, 1024) and part.dtype == torch.float32
    want = x.float() @ w.float().t()
    torch.testing.assert_close(part.sum(0), want, rtol=1e-3, atol=3e-3)


@pytest.mark.parametrize("wnt", [1, 2, 3, 4, 5])
def test_llama3_8b_shapes(wnt):
    """The four Llama-3-8B decode projections at the serving batch (64-k and
    32-k ring stages)."""
    M = 256
    for N, K, mode, S, bn in ((6144, 4096, 2, 5, 128), (4096, 4096, 2, 8, 128),
                              (14336, 4096, 1, 1, 128), (4096, 14336, 2, 7, 128),
                              (4096, 4096, 2, 4, 256 if wnt < 4 else 64)):
        x, w = _mk(M, 2 * N if mode == 1 else N, K, seed=N + K)
        out = ops.tgemm(mode, x, w, S, bn, wnt)
        full = x.float() @ w.float().t()
        want = ref.silu_mul(full) if mode == 1 else full
        got = out.sum(0) if mode == 2 else out.float()
        torch.testing.assert_close(got, want.float(), rtol=3e-2, atol=3e-2)


def test_repeat_launches_are_deterministic():
    x, w = _mk(256, 2048, 4096, seed=3)
    a = ops.tgemm(2, x, w, 4, 128, 1).clone()
    for _ in range(3):
        b = ops.tgemm(2, x, w, 4, 128, 1)
        assert torch.equal(a, b)


def test_rejects_bad_shapes_before_launch():
    x, w = _mk(16, 1000, 512)
    with pytest.raises(RuntimeError, match="tgemm"):
        ops.tgemm(0, x, w, 1, 128, 0)  # 1000 rows not a multiple of the block's 128
    x, _ = _mk(300, 1024, 512)
    _, w = _mk(300, 1024, 256)
    with pytest.raises(RuntimeError, match="K mismatch"):
        ops.tgemm(0, x, w, 1, 128, 0)  # K mismatch (M > 256 is valid: 256-row tiles)
    x, w = _mk(64, 1024, 512)
    with pytest.raises(RuntimeError, match="tgemm"):
        ops.tgemm(2, x, w, 9, 128, 0)  # more splits than 64-k steps
    with pytest.raises(RuntimeError, match="tgemm"):
        ops.tgemm(0, x, w, 1, 96, 0)  # unsupported block width
    with pytest.raises(RuntimeError, match="tgemm"):
        ops.tgemm(0, x, w, 1, 64, 2)  # 32-k stages need BN >= 128
    with pytest.raises(RuntimeError, match="tgemm"):
        ops.tgemm(0, x, w, 1, 256, 4)  # register-pipelined variant needs BN <= 128


@pytest.mark.parametrize("M,mode,bn,S,wnt", [(257, 0, 128, 1, 0), (600, 0, 256, 1, 0),
                                              (1024, 1, 256, 1, 0), (777, 1, 128, 1, 2),
                                              (1000, 2, 128, 3, 2), (4096, 1, 256, 1, 0)])
def test_prefill_row_tiles_match_fp32(M, mode, bn, S, wnt):
    """M > 256: 256-row tiles in grouped order (the prefill path), ragged last tile."""
    N = 512
    x, w = _mk(M, 2 * N if mode == 1 else N, 1024, seed=M + mode)
    out = ops.tgemm(mode, x, w, S, bn, wnt)
    full = x.float() @ w.float().t()
    if mode == 1:
        torch.testing.assert_close(out.float(), ref.silu_mul(full).float(), rtol=3e-2,
                                   atol=3e-2)
    elif mode == 2:
        assert out.shape == (S, M, N)
        torch.testing.assert_close(out.sum(0), full, rtol=1e-3, atol=3e-3)
    else:
        torch.testing.assert_close(out.float(), full, rtol=2e-2, atol=2e-2)
