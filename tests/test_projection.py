"""Memory Galaxy projection: basis choice, TF-IDF/LSA, PCA, exact t-SNE on
torch (cluster separation), Procrustes alignment, render decision, stored
layouts served by memory-api, and the render worker.

Parity: ``ee/pkg/memory/projection/*_test.go``,
``ee/pkg/memory/projectionworker/*_test.go`` (behaviour)."""
import math
import time

import numpy as np
import pytest
import torch

from omnia_amd.ee import projection as P
from omnia_amd.memory.model import Memory
from omnia_amd.memory.store import MemoryStore

WS = "ws1"


def _inp(i, emb=None, content="", t=0.0):
    return P.Input(f"e{i:04d}", content or f"doc {i}", emb, observed_at=t)


def test_basis_selection_and_cap():
    with_emb = [_inp(i, np.ones(4)) for i in range(7)] + [_inp(i + 7) for i in range(3)]
    assert P.choose_basis(with_emb, 0.7) == P.BASIS_DENSE
    assert P.choose_basis(with_emb, 0.8) == P.BASIS_LEXICAL
    used, unemb = P.select_inputs(with_emb, P.BASIS_DENSE)
    assert len(used) == 7 and unemb == 3
    ins = [_inp(i, t=float(i)) for i in range(10)]
    capped, flag = P.apply_cap(ins, 4)
    assert flag and [i.observed_at for i in capped] == [9.0, 8.0, 7.0, 6.0]


def test_tokenize_and_tfidf():
    assert P.tokenize("The VPN, on 2FA-keys!") == ["the", "vpn", "2fa", "keys"]
    red = P.tfidf_lsa(["alpha beta gamma", "alpha beta delta", "omega sigma tau"], 2, "cpu")
    assert red.shape == (3, 2)
    d01 = torch.dist(red[0], red[1])
    d02 = torch.dist(red[0], red[2])
    assert d01 < d02
    assert P.tfidf_lsa(["a b", "c"], 2, "cpu").shape == (2, 1)  # empty vocabulary


def test_tsne_separates_clusters():
    g = torch.Generator().manual_seed(0)
    centers = torch.randn(3, 16, generator=g) * 10
    x = torch.cat([c + torch.randn(20, 16, generator=g) for c in centers])
    y = P.tsne_2d(x, iters=300, seed=1)
    assert y.shape == (60, 2) and torch.isfinite(y).all()
    lab = torch.arange(60) // 20
    cent = torch.stack([y[lab == k].mean(0) for k in range(3)])
    within = torch.stack([(y[lab == k] - cent[k]).norm(dim=1).mean() for k in range(3)]).mean()
    between = torch.pdist(cent).min()
    assert between > 2.0 * within


def test_procrustes_recovers_rotation():
    ref_pts = torch.randn(10, 2, generator=torch.Generator().manual_seed(2))
    th = 0.7
    rot = torch.tensor([[math.cos(th), -math.sin(th)], [math.sin(th), math.cos(th)]])
    cur = ref_pts @ rot.T + torch.tensor([3.0, -1.0])
    ids = [f"e{i}" for i in range(10)]
    out = P.align(cur, ids, {i: ref_pts[k].tolist() for k, i in enumerate(ids)})
    assert torch.allclose(out, ref_pts, atol=1e-5)
    assert torch.equal(P.align(cur, ids, {"e0": [0, 0]}), cur)  # < 2 shared points


def test_should_render_rules():
    cfg = {"changeThreshold": 5}
    assert P.should_render(None, "3:1:3", cfg, 0)
    st = {"fingerprint": "10:5:10", "computed_at": 1000.0}
    assert not P.should_render(st, "10:5:10", cfg, 2000)  # unchanged
    assert not P.should_render(st, "12:9:10", cfg, 2000)  # below threshold
    assert P.should_render(st, "12:9:11", cfg, 2000)  # eligibility changed
    assert P.should_render(st, "15:9:10", cfg, 2000)
    sch = {"schedule": "@every 1h"}
    assert not P.should_render(st, "15:9:10", sch, 1000 + 1800)  # rendered too recently
    assert P.should_render(st, "15:9:10", sch, 1000 + 3601)


def _seed(store, n_per=12, dim=32):
    rng = np.random.default_rng(0)
    centers = rng.standard_normal((3, dim)) * 8
    for k in range(3):
        for j in range(n_per):
            res = store.save(Memory(content=f"topic{k} fact {j}", scope={
                "workspace_id": WS, "virtual_user_id": f"u{j % 4}"}))
            store.set_embedding(res["observation_id"],
                                (centers[k] + rng.standard_normal(dim)).astype(np.float32), "m")


def test_render_store_and_serve():
    store = MemoryStore()
    _seed(store)
    res = P.render(store, WS, opts=P.Options(tsne_iters=250), device="cpu")
    assert res["basis"] == P.BASIS_DENSE and res["model"] == P.MODEL_TSNE
    assert res["total"] == 36
    xs = torch.tensor([[p["x"], p["y"]] for p in res["points"]])
    assert float(xs.abs().max()) == pytest.approx(1.0)
    stored = P.ProjectionStore(store).load(P.scope_key(WS))
    assert stored["fingerprint"].startswith("36:") and len(stored["coords"]) == 36
    # a re-render aligns to the stored layout: shared points barely move
    res2 = P.render(store, WS, opts=P.Options(tsne_iters=250), device="cpu")
    a = {p["id"]: (p["x"], p["y"]) for p in res["points"]}
    moved = np.mean([math.dist(a[p["id"]], (p["x"], p["y"])) for p in res2["points"]])
    assert moved < 0.05
    served = P.from_stored(P.ProjectionStore(store).load(P.scope_key(WS)),
                           P.gather_inputs(store, WS))
    assert served["total"] == 36 and served["basis"] == P.BASIS_DENSE


def test_worker_renders_on_change_only():
    store = MemoryStore()
    _seed(store, n_per=4)
    clock = [time.time()]
    w = P.ProjectionWorker(store, [("pol", {"projection": {"enabled": True,
                                                           "changeThreshold": 2}})],
                           workspaces=lambda p: [WS], opts=P.Options(tsne_iters=50),
                           device="cpu", now=lambda: clock[0])
    assert w.run_once() == [(WS, "rendered")]
    assert w.run_once() == [(WS, "skipped")]
    store.save(Memory(content="one more", scope={"workspace_id": WS, "virtual_user_id": "u1"}))
    assert w.run_once() == [(WS, "skipped")]  # one new row < changeThreshold 2
    store.save(Memory(content="two more", scope={"workspace_id": WS, "virtual_user_id": "u1"}))
    assert w.run_once() == [(WS, "rendered")]
    ok, release = w.locks.try_lock(WS, "projection")
    other = P.ProjectionWorker(store, [("pol", {"projection": {"enabled": True}})],
                               workspaces=lambda p: [WS])
    for _ in range(2):
        store.save(Memory(content="x", scope={"workspace_id": WS, "virtual_user_id": "u2"}))
    assert other.run_once() == [(WS, "lock_held")]
    release()
    assert P.ProjectionWorker(store, [("pol", {"projection": {"enabled": False}})]).run_once() \
        == []


@pytest.mark.gpu
def test_tsne_on_device_at_render_cap():
    """The full 2,000-point cap, 1,000 iterations, on the MI355X."""
    g = torch.Generator().manual_seed(0)
    centers = torch.randn(4, 50, generator=g) * 10
    x = torch.cat([c + torch.randn(500, 50, generator=g) for c in centers]).cuda()
    t0 = time.time()
    y = P.tsne_2d(x, iters=1000)
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"t-SNE n=2000 x 1000 iters on {torch.cuda.get_device_name()}: {dt:.2f} s")
    lab = torch.arange(2000, device="cuda") // 500
    cent = torch.stack([y[lab == k].mean(0) for k in range(4)])
    within = torch.stack([(y[lab == k] - cent[k]).norm(dim=1).mean() for k in range(4)]).mean()
    assert torch.pdist(cent).min() > 2.0 * within
    assert dt < 30.0
