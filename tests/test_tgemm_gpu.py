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


@pytest.mark.parametrize("M,S,bn,wnt", [(256, 5, 128, 0), (201, 7, 256, 0), (256, 8, 128, 9),
                                         (77, 4, 64, 5)])
def test_mode3_half_slabs_match_fp32_slabs(M, S, bn, wnt):
    """fp16 slabs (mode 3): each slab is the fp32 slab rounded to fp16, so the
    slab-by-slab error is within fp16's half-ulp; packed weights (wnt bit 3) too."""
    x, w = _mk(M, 1024, 2048, seed=3 * M + S)
    if wnt & 8:
        wp = ops.tgemm_pack(w, bn, 0)
        p32, p16 = ops.tgemm(2, x, wp, S, bn, wnt), ops.tgemm(3, x, wp, S, bn, wnt)
    else:
        p32, p16 = ops.tgemm(2, x, w, S, bn, wnt), ops.tgemm(3, x, w, S, bn, wnt)
    assert p16.shape == (S, M, 1024) and p16.dtype == torch.float16
    torch.testing.assert_close(p16.float(), p32.half().float(), rtol=0, atol=0)
    torch.testing.assert_close(p16.float().sum(0), x.float() @ w.float().t(),
                               rtol=3e-3, atol=1e-2)


def test_mode3_half_slabs_saturate():
    """A K-slice partial beyond fp16's range saturates to +-65504 instead of
    turning inf (then NaN in the consumer); the fp32 slabs keep the true value."""
    M, N, K, S = 256, 256, 1024, 2
    x = torch.full((M, K), 16.0, dtype=torch.bfloat16, device="cuda")
    w = torch.full((N, K), 16.0, dtype=torch.bfloat16, device="cuda")  # slice sum 131072
    w[: N // 2] = -16.0
    p16 = ops.tgemm(3, x, w, S, 128, 0)
    assert torch.isfinite(p16).all()
    assert (p16[:, :, N // 2:] == 65504).all() and (p16[:, :, : N // 2] == -65504).all()
    p32 = ops.tgemm(2, x, w, S, 128, 0)
    assert (p32[:, :, N // 2:] == 131072).all()


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


@pytest.mark.parametrize("mode,bn,S,wnt", [(0, 128, 1, 0), (0, 64, 1, 0), (0, 256, 1, 0),
                                           (2, 128, 5, 0), (2, 64, 4, 4), (2, 128, 8, 4),
                                           (1, 128, 1, 0), (1, 64, 1, 1), (2, 256, 3, 1),
                                           (0, 128, 1, 4), (1, 256, 1, 0)])
@pytest.mark.parametrize("M", [1, 130, 256, 600])
def test_tile_packed_weights_match_row_major(M, mode, bn, S, wnt):
    """wnt bit 3: the weights re-laid by ops.tgemm_pack (stage-contiguous, chunks
    pre-swizzled) give the row-major kernel's result bit for bit -- every tile
    width, SwiGLU tile order, split-K slices and prefill row tiles (M > 256)."""
    N, K = 1024, 2048
    x, w = _mk(M, 2 * N if mode == 1 else N, K, seed=M + bn + S)
    ref = ops.tgemm(mode, x, w, S, bn, wnt)
    wp = ops.tgemm_pack(w, bn, 1 if mode == 1 else 0)
    assert not torch.equal(wp, w)  # really re-laid
    got = ops.tgemm(mode, x, wp, S, bn, wnt | 8)
    assert torch.equal(got, ref)
    # negative control: the packed weights read as row-major are wrong
    bad = ops.tgemm(mode, x, wp, S, bn, wnt)
    assert not torch.equal(bad, ref)


def test_model_decode_on_packed_weights_is_bit_identical():
    """The Llama decode forward at the serving batch (M = 256, the tuned table's
    tgemm configs) on the prepacked copies equals the row-major forward."""
    from omnia_amd.models import build_model
    from omnia_amd.models.config import resolve

    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    model = build_model(mc, device=torch.device("cuda"), dtype=torch.bfloat16, seed=3)
    model.pack_budget_frac = 1.0
    import os

    os.environ["OMNIA_TGEMM_PACK"] = "1"
    h = (torch.randn(256, mc.hidden_size, device="cuda") * 0.5).to(torch.bfloat16)
    layer = model.w["layers"][0]
    model._packed = {}
    ref_mlp = model.mlp(layer, h, is_decode=True)
    ref_qkv = model._proj("qkv", h, layer["qkv"], True)
    ref_mlp = ref_mlp.t.clone() if hasattr(ref_mlp, "t") else ref_mlp.clone()
    ref_qkv = ref_qkv.t.clone() if hasattr(ref_qkv, "t") else ref_qkv.clone()
    packed = model.prepack_decode(256)
    if not packed:
        pytest.skip("the tuned table sends no Llama-3-8B decode projection to tgemm")
    os.environ.pop("OMNIA_TGEMM_PACK", None)
    got_mlp = model.mlp(layer, h, is_decode=True)
    got_qkv = model._proj("qkv", h, layer["qkv"], True)
    got_mlp = got_mlp.t if hasattr(got_mlp, "t") else got_mlp
    got_qkv = got_qkv.t if hasattr(got_qkv, "t") else got_qkv
    assert torch.equal(got_mlp, ref_mlp) and torch.equal(got_qkv, ref_qkv)


def test_every_tgemm_table_entry_matches_fp32():
    """Every tile-kernel entry of the tuned decode table (the shapes the serving
    engine dispatches to it: Llama-3-8B, Llama-3-70B TP=1 / TP=8 shards) run as
    the engine runs it -- fp16 slabs (mode 3) or fused SwiGLU (mode 1) --
    against the fp32 product, at the bucket's batch size."""
    import json
    import os

    path = os.path.join(os.path.dirname(ops.__file__), "tuned", "wgemm_mi355x.json")
    table = json.load(open(path))
    checked = 0
    for key, (bn, nwaves, S) in sorted(table.items()):
        if nwaves >= 0 or nwaves == ops.PGEMM_SPLIT:
            continue
        mode, M, N, K = (int(v) for v in key.split(":"))
        rows = 2 * N if mode == 1 else N
        x, w = _mk(M, rows, K, seed=M + N + K)
        want = x.float() @ w.float().t()
        if mode == 1 and S == 1:
            got = ops.tgemm(1, x, w, 1, bn, -1 - nwaves)
            torch.testing.assert_close(got.float(), ref.silu_mul(want).float(),
                                       rtol=3e-2, atol=3e-2)
        else:
            got = ops.tgemm(3, x, w, S, bn, -1 - nwaves).float().sum(0)
            torch.testing.assert_close(got, want, rtol=1e-2, atol=2e-2)
        checked += 1
        del x, w
    assert checked >= 10
