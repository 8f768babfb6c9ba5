"""Decode projection GEMM (ops/csrc/gemm.hip) vs a plain PyTorch fp32 reference.

Covers every (wm, wn) tile instance, split-K with the in-launch combine
(S = 1..8), the fused SwiGLU epilogue, ragged batch sizes (rows past M are
computed from a clamped row and never stored), a strided output, and bitwise
determinism of the split-K combine across repeated launches.  GPU only."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from omnia_amd import ops

DEV = "cuda"


def _ref(x, w, mode):
    y = F.linear(x.float(), w.float())
    if mode == 1:
        n = w.shape[0] // 2
        y = F.silu(y[:, :n]) * y[:, n:]
    return y


def _run(mode, M, N, K, S, wm, wn, out=None, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(M, K, device=DEV, dtype=torch.float32, generator=g).bfloat16()
    rows = N if mode == 0 else 2 * N
    w = (torch.randn(rows, K, device=DEV, dtype=torch.float32, generator=g) * 0.05).bfloat16()
    ops.dgemm_prepare(DEV)
    ws, cnt = ops._dgemm_ws[torch.cuda.current_device()]
    o = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16) if out is None else out
    ops.kernels().dgemm(mode, o, x, w, ws, cnt, S, wm, wn)
    return o, _ref(x, w, mode)


def _check(o, r):
    o = o.float()
    assert torch.isfinite(o).all()
    err = (o - r).abs().max().item()
    assert err <= 2e-2 * r.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("wm,wn", [(1, 1), (1, 2), (1, 4), (2, 1), (2, 2), (2, 4), (4, 1), (4, 2)])
@pytest.mark.parametrize("mode", [0, 1])
def test_tiles(wm, wn, mode):
    M = 64 * wm - 3
    N = 64 * wn * 3
    o, r = _run(mode, M, N, 512, 1, wm, wn)
    _check(o, r)


@pytest.mark.parametrize("S", [2, 4, 8])
@pytest.mark.parametrize("mode", [0, 1])
def test_split_k(S, mode):
    o, r = _run(mode, 256, 1024, 4096, S, 4, 2)
    _check(o, r)


@pytest.mark.parametrize("M", [1, 7, 64, 100, 129, 256])
def test_front_end_shapes(M, monkeypatch):
    monkeypatch.setattr(ops, "_dgemm_force", True)
    ops.dgemm_prepare(DEV)
    x = torch.randn(M, 4096, device=DEV).bfloat16()
    w = (torch.randn(6144, 4096, device=DEV) * 0.02).bfloat16()
    _check(ops.linear(x, w), _ref(x, w, 0))
    wgu = (torch.randn(2 * 1024, 4096, device=DEV) * 0.02).bfloat16()
    _check(ops.linear_silu(x, wgu), _ref(x, wgu, 1))


def test_strided_out_and_determinism():
    big = torch.zeros(256, 2048, device=DEV, dtype=torch.bfloat16)
    view = big[:, 512:1536]
    o1, r = _run(0, 256, 1024, 4096, 4, 4, 2, out=view)
    _check(o1, r)
    assert big[:, :512].abs().max().item() == 0 and big[:, 1536:].abs().max().item() == 0
    first = o1.clone()
    for _ in range(5):
        o2, _ = _run(0, 256, 1024, 4096, 4, 4, 2, out=view)
        assert torch.equal(first, o2)


def test_counters_reset():
    ops.dgemm_prepare(DEV)
    _run(0, 200, 4096, 4096, 8, 4, 2)
    torch.cuda.synchronize()
    assert int(ops._dgemm_ws[torch.cuda.current_device()][1].abs().sum().item()) == 0


def test_rejects_bad_shapes():
    ops.dgemm_prepare(DEV)
    ws, cnt = ops._dgemm_ws[torch.cuda.current_device()]
    x = torch.randn(300, 512, device=DEV).bfloat16()
    w = torch.randn(128, 512, device=DEV).bfloat16()
    o = torch.empty(300, 128, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.kernels().dgemm(0, o, x, w, ws, cnt, 1, 4, 2)  # M > 256
    x = torch.randn(16, 576, device=DEV).bfloat16()
    w = torch.randn(128, 576, device=DEV).bfloat16()
    o = torch.empty(16, 128, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.kernels().dgemm(0, o, x, w, ws, cnt, 2, 1, 2)  # K % (64*S)


@pytest.mark.parametrize("wm,S,M", [(1, 1, 256), (2, 2, 200), (1, 4, 130), (2, 1, 129)])
def test_multiple_row_tiles(wm, S, M):
    for mode in (0, 1):
        o, r = _run(mode, M, 512, 1024, S, wm, 2)
        _check(o, r)
