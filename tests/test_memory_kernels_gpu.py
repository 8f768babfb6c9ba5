"""K17 (mean-pool + L2) and K18 (cosine scores + exact top-k) vs fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from omnia_amd import ops
from omnia_amd.ops import reference as ref


@pytest.mark.parametrize("D", [384, 1024, 4096])
def test_mean_pool_l2(D):
    g = torch.Generator().manual_seed(D)
    lens = [1, 7, 0, 130, 33]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    h = torch.randn(int(cu[-1]), D, generator=g).to(torch.bfloat16)
    out = ops.mean_pool_l2(h.cuda(), cu.cuda()).cpu()
    exp = ref.mean_pool_l2(h, cu)
    torch.testing.assert_close(out, exp, atol=2e-5, rtol=1e-4)
    assert torch.all(out[2] == 0)


@pytest.mark.parametrize("nq,N,D,k", [(1, 1000, 768, 10), (3, 50_000, 1024, 400),
                                      (8, 7777, 256, 1024), (5, 200_001, 384, 100)])
def test_cosine_topk_matches_reference(nq, N, D, k):
    g = torch.Generator().manual_seed(N)
    m = torch.nn.functional.normalize(torch.randn(N, D, generator=g), dim=1).to(torch.bfloat16)
    q = torch.nn.functional.normalize(torch.randn(nq, D, generator=g), dim=1)
    valid = (torch.rand(N, generator=g) > 0.1).to(torch.uint8)
    v, i = ops.cosine_topk(q.cuda(), m.cuda(), k, valid.cuda())
    rv, ri = ref.cosine_topk(q, m, k, valid)
    # scores agree to fp32-accumulation tolerance; the selected sets agree except
    # possibly at near-ties on the boundary
    torch.testing.assert_close(v.cpu(), rv, atol=1e-5, rtol=1e-5)
    for r in range(nq):
        a, b = set(i[r].tolist()), set(ri[r].tolist())
        assert len(a ^ b) <= 2, (r, len(a ^ b))
        assert all(valid[j] for j in a)
    # each returned score is the true score of the returned index
    s_true = (q.cuda() @ m.cuda().float().t()).gather(1, i)
    torch.testing.assert_close(v, s_true, atol=1e-5, rtol=1e-5)
    assert torch.all(v[:, :-1] >= v[:, 1:])


def test_topk_ties_prefer_lower_index():
    N, D = 4096, 128
    m = torch.zeros(N, D, dtype=torch.bfloat16)
    m[:, 0] = 1.0  # every row identical -> all ties
    q = torch.zeros(1, D)
    q[0, 0] = 1.0
    v, i = ops.cosine_topk(q.cuda(), m.cuda(), 50)
    assert i[0].tolist() == list(range(50))
    assert torch.all(v == 1.0)


def test_vector_index_gpu_agrees_with_cpu():
    from omnia_amd.memory.vector_index import VectorIndex

    g = torch.Generator().manual_seed(1)
    vecs = torch.randn(3000, 256, generator=g)
    items = [(f"k{i}", v.tolist()) for i, v in enumerate(vecs)]
    gi, ci = VectorIndex(256, device="cuda"), VectorIndex(256, device="cpu")
    gi.upsert(items)
    ci.upsert(items)
    gi.remove(["k5", "k6"])
    ci.remove(["k5", "k6"])
    qs = [vecs[5].tolist(), vecs[100].tolist()]
    a, b = gi.search(qs, 20), ci.search(qs, 20)
    for ra, rb in zip(a, b):
        assert [k for k, _ in ra][:10] == [k for k, _ in rb][:10]
        assert "k5" not in [k for k, _ in ra]


def test_local_embedder_gpu_batch_invariant():
    from omnia_amd.memory.embedding import LocalModelEmbedder

    e = LocalModelEmbedder("tiny-embed", device="cuda", max_tokens_per_batch=1024)
    texts = ["hello world", "memory tier on gfx950 " * 30, "x"]
    v = torch.tensor(e.embed_sync(texts))
    assert torch.allclose(v.norm(dim=1), torch.ones(3), atol=1e-4)
    solo = torch.tensor(e.embed_sync([texts[1]]))
    assert torch.allclose(solo[0], v[1], atol=2e-3)
