"""MoE kernels (K14) vs the fp32 oracle; Mixtral engine on the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from omnia_amd import ops
from omnia_amd.ops import reference as ref


def _weights(E, d, I, g, dev="cuda"):
    wgu = (torch.randn(E, 2 * I, d, generator=g) * 0.05).to(torch.bfloat16)
    wd = (torch.randn(E, d, I, generator=g) * 0.05).to(torch.bfloat16)
    router = (torch.randn(E, d, generator=g) * 0.2).to(torch.bfloat16)
    return router.to(dev), wgu.to(dev), wd.to(dev)


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (37, 8, 2), (256, 8, 2), (64, 16, 4)])
def test_moe_topk_matches_reference(T, E, k):
    g = torch.Generator().manual_seed(T * E)
    logits = torch.randn(T, E, generator=g)
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    w = torch.empty(T, k, dtype=torch.float32, device="cuda")
    ops.kernels().moe_topk(ids, w, logits.cuda(), k, True)
    rid, rw = ref.moe_route(logits, k)
    assert torch.equal(ids.cpu(), rid)
    torch.testing.assert_close(w.cpu(), rw, atol=1e-5, rtol=1e-5)


def test_moe_topk_nan_and_padding_rows_route_to_valid_distinct_experts():
    """A NaN row (e.g. a padded decode row) or an all -inf row must still yield k
    distinct ids in [0, E) and finite weights: the expert-parallel dispatch turns
    ids into send-buffer slots, so a -1 there would be an out-of-bounds write."""
    E, k = 8, 2
    logits = torch.randn(6, E)
    logits[1] = float("nan")
    logits[2] = float("-inf")
    logits[3, :5] = float("nan")  # partially NaN: the finite experts win
    ids = torch.full((6, k), -7, dtype=torch.int32, device="cuda")
    w = torch.empty(6, k, dtype=torch.float32, device="cuda")
    ops.kernels().moe_topk(ids, w, logits.cuda(), k, True)
    ids, w = ids.cpu(), w.cpu()
    assert ((ids >= 0) & (ids < E)).all() and (ids[:, 0] != ids[:, 1]).all()
    assert torch.isfinite(w).all()
    assert set(ids[3].tolist()) <= {5, 6, 7}
    torch.testing.assert_close(w[1], torch.full((k,), 1.0 / k))
    rid, rw = ref.moe_route(logits[[0, 4, 5]], k)
    assert torch.equal(ids[[0, 4, 5]], rid)


@pytest.mark.parametrize("T,d,I,E,k,e_lo,e_n", [
    (1, 256, 256, 8, 2, 0, 8), (13, 512, 256, 8, 2, 0, 8), (256, 512, 512, 8, 2, 0, 8),
    (100, 256, 256, 8, 2, 4, 4),  # expert-parallel shard: experts 4..7 only
])
def test_moe_grouped_path_matches_reference(T, d, I, E, k, e_lo, e_n):
    g = torch.Generator().manual_seed(T + d)
    router, wgu, wd = _weights(E, d, I, g)
    x = (torch.randn(T, d, generator=g)).to(torch.bfloat16).cuda()
    wgu_l, wd_l = wgu[e_lo:e_lo + e_n].contiguous(), wd[e_lo:e_lo + e_n].contiguous()
    out = ops.moe(x, router, wgu_l, wd_l, k, E, e_lo, graph_safe=True)
    # pin the oracle to the kernel's routing (bf16 router logits, as in ops.moe)
    logits = torch.nn.functional.linear(x, router)
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    w = torch.empty(T, k, dtype=torch.float32, device="cuda")
    ops.kernels().moe_topk(ids, w, logits, k, True)
    rid, rw = ref.moe_route(logits.float().cpu(), k)
    assert torch.equal(ids.cpu(), rid)
    exp = ref.moe(x.cpu(), router.cpu(), wgu_l.cpu(), wd_l.cpu(), k, e_lo, ids=rid, wts=rw,
                  act_dtype=torch.bfloat16)
    torch.testing.assert_close(out.float().cpu(), exp, atol=1e-2, rtol=1e-2)


def test_moe_library_path_matches_grouped(monkeypatch):
    g = torch.Generator().manual_seed(5)
    E, d, I, k, T = 4, 256, 512, 2, 2048
    router, wgu, wd = _weights(E, d, I, g)
    x = torch.randn(T, d, generator=g).to(torch.bfloat16).cuda()
    monkeypatch.setattr(ops, "MOE_TILE256_ROWS", 1 << 30)  # the 64-row grouped kernels
    a = ops.moe(x, router, wgu, wd, k, E, 0, graph_safe=True)
    monkeypatch.setenv("OMNIA_MOE_LIBRARY", "1")
    b = ops.moe(x, router, wgu, wd, k, E, 0, graph_safe=False)  # hipBLASLt per expert
    torch.testing.assert_close(a.float(), b.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,d,I,E,k,e_lo,e_n", [
    (2048, 512, 512, 8, 2, 0, 8),    # prefill-sized: 256x256-tile grouped GEMMs
    (2500, 256, 384, 8, 2, 0, 8),    # ragged expert segments, I not a multiple of 256
    (4096, 512, 256, 8, 2, 4, 4),    # expert-parallel shard: experts 4..7 only
])
def test_moe_tile256_prefill_matches_reference(T, d, I, E, k, e_lo, e_n):
    """Large batches run the 256-row-segment grouped GEMMs (pgemm.hip EPI 5 / 6)
    without a host sync: against the fp32 oracle pinned to the kernel's routing,
    and against the 64-row grouped kernels (a different tiling of the same sums)."""
    g = torch.Generator().manual_seed(T + I)
    router, wgu, wd = _weights(E, d, I, g)
    x = (torch.randn(T, d, generator=g)).to(torch.bfloat16).cuda()
    wgu_l, wd_l = wgu[e_lo:e_lo + e_n].contiguous(), wd[e_lo:e_lo + e_n].contiguous()
    assert T * k >= ops.MOE_TILE256_ROWS * e_n  # the 256-tile path is the one under test
    out = ops.moe(x, router, wgu_l, wd_l, k, E, e_lo, graph_safe=True)
    logits = torch.nn.functional.linear(x, router)
    rid, rw = ref.moe_route(logits.float().cpu(), k)
    exp = ref.moe(x.cpu(), router.cpu(), wgu_l.cpu(), wd_l.cpu(), k, e_lo, ids=rid, wts=rw,
                  act_dtype=torch.bfloat16)
    torch.testing.assert_close(out.float().cpu(), exp, atol=1e-2, rtol=1e-2)
    saved = ops.MOE_TILE256_ROWS
    try:
        ops.MOE_TILE256_ROWS = 1 << 30
        small = ops.moe(x, router, wgu_l, wd_l, k, E, e_lo, graph_safe=True)
    finally:
        ops.MOE_TILE256_ROWS = saved
    torch.testing.assert_close(out.float(), small.float(), atol=1e-2, rtol=1e-2)
    # negative control: dropping the routing weights must not pass
    assert not torch.allclose(out.float().cpu(), exp * 2, atol=1e-2, rtol=1e-2)


def test_moe_tile256_is_graph_capturable():
    """No host sync: the prefill-sized grouped path captures into a hipGraph and
    replays to the eager result."""
    g = torch.Generator().manual_seed(11)
    E, d, I, k, T = 8, 512, 512, 2, 2048
    router, wgu, wd = _weights(E, d, I, g)
    x = torch.randn(T, d, generator=g).to(torch.bfloat16).cuda()
    want = ops.moe(x, router, wgu, wd, k, E, 0, graph_safe=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.moe(x, router, wgu, wd, k, E, 0, graph_safe=True)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        got = ops.moe(x, router, wgu, wd, k, E, 0, graph_safe=True)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(got, want)


def test_mixtral_engine_graphs_match_eager():
    from omnia_amd.engine.engine import EngineConfig, LLMEngine
    from omnia_amd.engine.sampling_params import SamplingParams

    def run(graphs):
        e = LLMEngine(EngineConfig(model="tiny-mixtral", device="cuda", num_blocks=128,
                                   max_batch=8, max_model_len=1024, use_graphs=graphs))
        p = SamplingParams(temperature=0, max_tokens=10, ignore_eos=True)
        return [s.output for s in e.generate([list(range(3, 90)), list(range(40, 60))], p)]

    assert run(True) == run(False)


def test_moe_decode_layer_bandwidth_report():
    """Mixtral-8x7B-shaped MoE layer at decode batch 256 (prints achieved HBM rate)."""
    g = torch.Generator(device="cuda").manual_seed(0)
    E, d, I, k, T = 8, 4096, 14336, 2, 256
    router = (torch.randn(E, d, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    wgu = (torch.randn(E, 2 * I, d, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    wd = (torch.randn(E, d, I, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    x = torch.randn(T, d, device="cuda", generator=g).to(torch.bfloat16)
    for _ in range(3):
        ops.moe(x, router, wgu, wd, k, E)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    n = 10
    for _ in range(n):
        ops.moe(x, router, wgu, wd, k, E)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    gb = (wgu.numel() + wd.numel()) * 2 / 1e9
    print(f"\nMoE decode layer T={T}: {ms:.3f} ms, weights {gb:.2f} GB -> {gb / ms:.2f} TB/s")
    assert ms > 0


@pytest.mark.parametrize("T,d,E,k", [(1, 4096, 8, 2), (333, 4096, 8, 2), (4096, 1024, 16, 4),
                                     (64, 512, 64, 6)])
def test_router_topk_fused_matches_linear_then_topk(T, d, E, k):
    """The fused router GEMM + top-k (no logits tensor, no library GEMM) routes
    like bf16 F.linear followed by moe_topk -- up to bf16 rounding ties of the
    logits, which may order near-equal experts differently (<= 0.5 % of rows
    against the library GEMM; 2-6 % against fp32 at E=16-64, k=4-6)."""
    g = torch.Generator().manual_seed(T * E + d)
    x = torch.randn(T, d, generator=g).to(torch.bfloat16).cuda()
    router = (torch.randn(E, d, generator=g) * 0.02).to(torch.bfloat16).cuda()
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    w = torch.empty(T, k, dtype=torch.float32, device="cuda")
    ops.kernels().moe_router_topk(ids, w, x, router, k, True)
    ids2 = torch.empty_like(ids)
    w2 = torch.empty_like(w)
    ops.kernels().moe_topk(ids2, w2, torch.nn.functional.linear(x, router), k, True)
    same = (ids == ids2).all(1)
    assert same.float().mean().item() >= 0.995, same.float().mean().item()
    torch.testing.assert_close(w[same], w2[same], atol=1e-2, rtol=1e-2)
    # against the fp32 oracle: every chosen expert's fp32 logit, in the kernel's
    # order, equals the fp32 top-k value at that rank up to bf16 rounding (the
    # kernel, like the library GEMM, rounds logits to bf16, so near-ties may swap)
    lf = torch.nn.functional.linear(x.float(), router.float()).cpu()
    rid, rw = ref.moe_route(lf, k)
    sel = lf.gather(1, ids.cpu().long())
    top = lf.topk(k, dim=1).values
    tol = 2.0 ** -7 * lf.abs().amax(1, keepdim=True)
    assert ((sel - top).abs() <= tol).all()
    m = (ids.cpu() == rid).all(1)  # rows whose order no near-tie swapped
    assert m.float().mean().item() >= 0.9
    torch.testing.assert_close(w.cpu()[m], rw[m], atol=1e-2, rtol=1e-2)
