"""The GPU tensor-parallel sampler (``sampling.hip`` tp_pack + tp_merge) on one
device: W vocab slices of the same logits are packed as W ranks would, the packs
stacked as the all-gather would, and the merge's token compared with the
single-GPU references of the FULL row:

* greedy rows: the full-row arg-max (ties -> lowest id) -- exact;
* pure-temperature rows: the host Gumbel reference (``gumbel_uniform``);
* top-k / top-p rows: the single-GPU fused sampler ``ops.sample`` on the full
  row, which draws with the same noise keyed by the global token id -- exact
  whenever the kept set lies inside the W x K candidates (peaked rows here).

Plus: each rank's pack holds exactly its slice's top-K (as a value multiset),
the merge scatters the tokens into the device token slots, and a negative
control (every rank's greedy id off by one) moves every greedy token."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _packs(k, logits, W, K, temp, top_k, top_p, seeds, steps):
    B, V = logits.shape
    Vl = V // W
    packs = []
    for w in range(W):
        pk = torch.full((B, 2 * K + 4), float("nan"), device=DEV)
        k.tp_pack(pk, K, logits[:, w * Vl:(w + 1) * Vl], w * Vl, temp, top_k, top_p, seeds, steps)
        packs.append(pk)
    return torch.stack(packs)


@pytest.mark.parametrize("W,V", [(2, 128256), (4, 128256), (8, 128256), (3, 4002 * 3)])
def test_tp_pack_merge_matches_single_gpu_sampler(W, V):
    from omnia_amd import ops
    from omnia_amd.parallel.tp_sampling import gumbel_uniform

    k = ops.kernels()
    K = min(64, 512 // W)
    torch.manual_seed(W)
    B = 96
    logits = torch.randn(B, V, device=DEV) * 1.5
    # peaked rows: a few dominant tokens so every top-p nucleus sits in the candidates
    hot = torch.randint(0, V, (B, 6), device=DEV)
    logits.scatter_(1, hot, torch.randn(B, 6, device=DEV) * 2 + 25)
    logits = logits.bfloat16()
    kind = torch.arange(B, device=DEV) % 6  # 0 greedy 1 pure 2 top-k 3 top-p 4 both 5 k=1
    temp = torch.where(kind == 0, 0.0, 0.7 + torch.rand(B, device=DEV)).float()
    top_k = torch.where(kind == 2, 40, torch.where(kind == 4, 20, torch.where(kind == 5, 1, 0)))
    top_k = top_k.to(torch.int32)
    top_p = torch.where((kind == 3) | (kind == 4), 0.9, 1.0).float()
    seeds = torch.randint(0, 2**62, (B,), dtype=torch.int64, device=DEV)
    steps = torch.randint(0, 5000, (B,), dtype=torch.int64, device=DEV)
    allp = _packs(k, logits, W, K, temp, top_k, top_p, seeds, steps)
    assert torch.isfinite(allp[:, :, 2 * K + 3]).all()  # every column defined
    out = torch.full((B,), -7, dtype=torch.int32, device=DEV)
    slots = torch.zeros(2 * B + 8, dtype=torch.int32, device=DEV)
    dst = torch.randperm(2 * B, device=DEV)[:B] + 1
    k.tp_merge(out, slots, dst, allp, K, temp, top_k, top_p, seeds, steps)
    torch.cuda.synchronize()
    got = out.long().cpu()
    assert torch.equal(slots[dst].long().cpu(), got)  # fused token-slot scatter

    kc = kind.cpu()
    full = logits.float().cpu()
    # greedy: exact full-row arg-max
    g = kc == 0
    assert torch.equal(got[g], full[g].argmax(1))
    # pure temperature: host Gumbel reference over the whole vocabulary
    p = kc == 1
    u = gumbel_uniform(seeds.cpu(), steps.cpu(), 0, V).clamp_(1e-10, 1 - 1e-7)
    gum = (full / temp.cpu().clamp(min=1e-6)[:, None] - torch.log(-torch.log(u))).argmax(1)
    assert (got[p] == gum[p]).float().mean().item() >= 0.97
    # filtered rows: the single-GPU fused sampler on the full row
    ref = ops.sample(logits, temp, top_k, top_p, seeds=seeds, steps=steps).long().cpu()
    for kk, need in ((2, 1.0), (5, 1.0), (3, 0.95), (4, 0.95)):
        m = kc == kk
        agree = (got[m] == ref[m]).float().mean().item()
        assert agree >= need, (kk, agree)
    # each rank's pack: exactly its slice's top-K values (filtered rows)
    Vl = V // W
    fr = ((kc >= 2) & (kc <= 5)).nonzero()[:, 0]
    for w in range(W):
        vals = allp[w][fr][:, :K].cpu()
        want = full[fr][:, w * Vl:(w + 1) * Vl].topk(K, dim=1).values
        assert torch.equal(vals.sort(1).values, want.sort(1).values), w
        ids = allp[w][fr][:, K:2 * K].cpu().long() - w * Vl
        assert torch.equal(full[fr][:, w * Vl:(w + 1) * Vl].gather(1, ids), vals)
    # negative control: every rank's greedy id off by one -> every greedy answer moves
    bad = allp.clone()
    bad[:, :, K] += 1
    out2 = torch.empty_like(out)
    k.tp_merge(out2, None, None, bad, K, temp, top_k, top_p, seeds, steps)
    assert torch.equal(out2.long().cpu()[g], got[g] + 1)


def test_tp_pack_merge_graph_replay_is_stable():
    """The three-launch tail captured in a hipGraph and replayed many times gives
    the eager tokens every time (fresh inputs copied in between replays)."""
    from omnia_amd import ops

    k = ops.kernels()
    W, V, B, K = 2, 64128 * 2, 8, 64
    logits = (torch.randn(B, V, device=DEV) * 3).bfloat16()
    temp = torch.tensor([0, 0.8, 1.0, 0, 0.9, 1.2, 0, 0.7], device=DEV).float()
    top_k = torch.tensor([0, 0, 20, 0, 0, 40, 0, 0], device=DEV, dtype=torch.int32)
    top_p = torch.tensor([1, 1, 1, 1, 0.95, 1, 1, 0.8], device=DEV).float()
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 7 + 1
    steps = torch.zeros(B, dtype=torch.int64, device=DEV)
    out = torch.zeros(B, dtype=torch.int32, device=DEV)

    def body():
        allp = _packs(k, logits, W, K, temp, top_k, top_p, seeds, steps)
        k.tp_merge(out, None, None, allp, K, temp, top_k, top_p, seeds, steps)

    body()
    eager = out.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for i in range(20):
        steps.fill_(i % 3)
        g.replay()
        torch.cuda.synchronize()
        if i % 3 == 0:
            assert torch.equal(out, eager)
