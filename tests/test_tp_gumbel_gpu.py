"""The fused TP Gumbel kernel (``sampling.hip`` tp_gumbel) against its host
reference (``tp_sampling.gumbel_uniform`` + fp32 log-log arg-max): same winner
for pure-temperature rows, untouched logits (-inf, vocab_start) for greedy and
top-k / top-p rows, and a vocab slice that is not a multiple of 8 / unaligned."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("V,off", [(16032, 0), (4003, 1)])
def test_tp_gumbel_matches_reference(V, off):
    from omnia_amd import ops
    from omnia_amd.parallel.tp_sampling import gumbel_uniform

    torch.manual_seed(0)
    B, vs = 64, 48096
    base = torch.randn(B, V + off, device="cuda").to(torch.bfloat16) * 3
    logits = base[:, off:]  # off = 1: rows not 16-byte aligned -> scalar path
    temp = torch.rand(B, device="cuda") + 0.3
    temp[::7] = 0.0
    top_k = torch.zeros(B, dtype=torch.int32, device="cuda")
    top_k[3::11] = 40
    top_p = torch.ones(B, device="cuda")
    top_p[5::13] = 0.9
    seeds = torch.randint(0, 2**62, (B,), dtype=torch.int64, device="cuda")
    steps = torch.randint(0, 10000, (B,), dtype=torch.int64, device="cuda")
    pack = torch.zeros(B, 6, device="cuda")
    ops.kernels().tp_gumbel(pack, 2, logits, vs, temp, top_k, top_p, seeds, steps)
    torch.cuda.synchronize()
    u = gumbel_uniform(seeds.cpu(), steps.cpu(), vs, V).clamp_(1e-10, 1 - 1e-7)
    g = logits.float().cpu() / temp.cpu().clamp(min=1e-6)[:, None] - torch.log(-torch.log(u))
    gv, gi = g.max(dim=1)
    pure = (temp > 0) & (top_k <= 0) & (top_p >= 1)
    pure = pure.cpu()
    got_v, got_i = pack[:, 2].cpu(), pack[:, 3].cpu().long()
    assert torch.all(got_v[~pure] == float("-inf")) and torch.all(got_i[~pure] == vs)
    agree = (got_i[pure] == gi[pure] + vs).float().mean().item()
    assert agree >= 0.98, agree  # ulp-level log differences may flip a near tie
    assert torch.allclose(got_v[pure], gv[pure], rtol=1e-4, atol=1e-4)
    assert torch.all(pack[:, [0, 1, 4, 5]] == 0)  # other columns untouched
