"""Expert-parallel and context-parallel serving with 2-8 ranks on ONE MI355X.

RCCL cannot place two ranks on one device, so the ranks run the ``ipc``
transport (parallel/state.py): gloo for host bootstrap only, the host
shared-memory lockstep agreement (parallel/hostsync.py), and every device
collective on the IPC kernels -- the EP token dispatch / combine on the IPC
all-to-all (``comm.hip`` ar_alltoall), the CP ring hops on the IPC
point-to-point kernel (ar_sendrecv) on a side stream.

* EP (BASELINE config 5's ``epMode: a2a`` path, DP attention + EP): world 2, 4
  and 8 over tiny-mixtral-e8 (8 experts, one per rank at world 8), every rank
  its own engine with its own prompts (one rank idle at world >= 4: it still
  serves the others' all-to-alls).  Every logit row each rank sampled from is
  checked against the fp32 dense oracle ``ops.reference.dense_forward`` of the
  FULL expert set; negative control: the oracle with two experts swapped.
* CP (``EngineConfig.cp_threshold``): world 2 and 4 over tiny-llama, a prompt
  over the threshold owned by rank 0 is prefilled by the whole group with ring
  attention, then decoded by its owner; oracle check + negative control (a
  swapped kv-head slice).
"""
import os
import random
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROUTER_SCALE = 30.0  # sharpen routing so bf16 vs fp32 top-k cannot tie


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rows(tap):
    out = {}
    for ids, rows in tap:
        for i, sid in enumerate(ids):
            out.setdefault(sid, []).append(rows[i])
    return out


def _check(mc, w, seqs, rows_by_seq, tol):
    from omnia_amd.ops import reference as ref

    ok = total = 0
    worst = 0.0
    for sid, prompt, output in seqs:
        got = rows_by_seq[sid]
        # pipelined decode may run one speculative step past the finish (dropped
        # token, recorded row): trailing, at most one
        assert len(output) <= len(got) <= len(output) + 1, (sid, len(got), len(output))
        got = got[:len(output)]
        want = ref.dense_forward(mc, w, (prompt + output)[:-1])[len(prompt) - 1:]
        for g, r in zip(got, want):
            err = float((g.float().cpu() - r).abs().max() / r.abs().max())
            worst = max(worst, err)
            ok += err < tol
            total += 1
    return ok / max(1, total), worst, total


def _full_mixtral(mc, seed):
    """The whole model (every expert) from the same per-(layer, expert)
    generators the EP ranks draw their shards from -- drawn on the DEVICE in
    the ranks' dtype (CPU and HIP generators produce different streams), then
    moved to the CPU in fp32 for the oracle."""
    from omnia_amd.models.mixtral import MixtralModel
    from omnia_amd.parallel import state as pstate

    saved = pstate.get_state()
    pstate.set_state(pstate.ParallelState())
    try:
        m = MixtralModel(mc, device="cuda", dtype=torch.bfloat16, seed=seed, ep_mode="tp")
    finally:
        pstate.set_state(saved)

    def cpu(x):
        if isinstance(x, torch.Tensor):
            return x.float().cpu()
        if isinstance(x, dict):
            return {k: cpu(v) for k, v in x.items()}
        if isinstance(x, list):
            return [cpu(v) for v in x]
        return x

    return cpu(m.w)


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      OMNIA_LOGIT_TAP="1")


def _ep_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from omnia_amd.engine.engine import EngineConfig, LLMEngine
        from omnia_amd.engine.sampling_params import SamplingParams
        from omnia_amd.models.config import resolve
        from omnia_amd.parallel import state as pstate

        torch.cuda.set_device(0)
        mc = resolve("tiny-mixtral-e8")
        eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", ep_mode="a2a",
                                     num_blocks=128, block_size=16, max_batch=8,
                                     max_model_len=512, max_prefill_tokens=64, seed=5))
        st = pstate.get_state()
        assert st.transport == "ipc" and st.backend == "gloo" and st.dp_comm is not None
        assert eng.ep_lockstep and eng.model.e_local == mc.num_experts // world
        for layer in eng.model.w["layers"]:
            layer["router"].mul_(ROUTER_SCALE)
        eng.runner.enable_logit_tap()
        rng = random.Random(100 + rank)
        V = mc.vocab_size
        idle = world >= 4 and rank == world - 1
        lens = [] if idle else [(37, 90, 15)[i % 3] + rank for i in range(1 + rank % 3)]
        prompts = [[rng.randrange(10, V - 10) for _ in range(n)] for n in lens]
        greedy = SamplingParams(temperature=0.0, max_tokens=5 + rank % 4, ignore_eos=True)
        if prompts:
            seqs = eng.generate(prompts, greedy)
        else:
            seqs = []
            eng.run_until_done()
        plain = [(s.seq_id, list(s.prompt), list(s.output)) for s in seqs]
        rows = _rows(eng.runner.logit_tap or [])
        stats = dict(eng.runner.ep_stats)
        ag = dict(eng.runner.agreement.stats)
        err = int(st.dp_comm.err.item())
        full = _full_mixtral(mc, 5)
        for layer in full["layers"]:
            layer["router"].mul_(ROUTER_SCALE)
        frac, worst, n = _check(mc, full, plain, rows, 0.04) if plain else (1.0, 0.0, 0)
        bad = {k: v for k, v in full.items() if k != "layers"}
        bad["layers"] = [dict(x) for x in full["layers"]]
        gu = bad["layers"][0]["experts_gate_up"].clone()
        gu[[0, 1]] = gu[[1, 0]]
        bad["layers"][0]["experts_gate_up"] = gu
        bfrac, bworst, _ = _check(mc, bad, plain, rows, 0.04) if plain else (0.0, 1.0, 0)
        q.put(("ok", rank, {"frac": frac, "worst": worst, "rows": n, "neg_frac": bfrac,
                            "neg_worst": bworst, "idle": idle, "stats": stats, "agree": ag,
                            "ipc_err": err}))
        import torch.distributed as dist

        dist.barrier()
    except Exception:  # pragma: no cover - surfaced through the queue
        import traceback

        q.put(("err", rank, traceback.format_exc()))


def _ep_worker_mixtral(rank, world, port, q):
    """Mixtral-8x7B layer shapes (d 4096, 8 experts x 14336, 32 q / 8 kv heads,
    vocab 32000), 2 layers: rows go back to the parent, which builds the full
    model once for the oracle."""
    _env(rank, world, port)
    try:
        from omnia_amd.engine.engine import EngineConfig, LLMEngine
        from omnia_amd.engine.sampling_params import SamplingParams
        from omnia_amd.models.config import resolve

        torch.cuda.set_device(0)
        mc = resolve("mixtral-8x7b").replace(num_layers=2)
        eng = LLMEngine(EngineConfig(model="mixtral-8x7b", device="cuda", ep_mode="a2a",
                                     num_blocks=128, block_size=16, max_batch=8,
                                     max_model_len=512, max_prefill_tokens=128, seed=5),
                        model_cfg=mc)
        assert eng.model.e_local == mc.num_experts // world
        for layer in eng.model.w["layers"]:
            layer["router"].mul_(ROUTER_SCALE)
        eng.runner.enable_logit_tap()
        rng = random.Random(300 + rank)
        lens = [(29, 61)[i % 2] + 3 * rank for i in range(1 + rank % 2)]
        prompts = [[rng.randrange(10, mc.vocab_size - 10) for _ in range(n)] for n in lens]
        seqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=4,
                                                    ignore_eos=True))
        plain = [(s.seq_id, list(s.prompt), list(s.output)) for s in seqs]
        # numpy (pickled by value): torch CPU tensors would travel as shared-memory
        # handles that die with this process
        rows = {k: [r.float().cpu().numpy() for r in v] for k, v in
                _rows(eng.runner.logit_tap or []).items()}
        q.put(("ok", rank, {"plain": plain, "rows": rows,
                            "stats": dict(eng.runner.ep_stats)}))
        import torch.distributed as dist

        dist.barrier()
    except Exception:  # pragma: no cover
        import traceback

        q.put(("err", rank, traceback.format_exc()))


def _cp_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from omnia_amd.engine.engine import EngineConfig, LLMEngine
        from omnia_amd.engine.sampling_params import SamplingParams
        from omnia_amd.models.config import resolve
        from omnia_amd.parallel import state as pstate

        torch.cuda.set_device(0)
        mc = resolve("tiny-llama")
        eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=256,
                                     block_size=16, max_batch=8, max_model_len=2048,
                                     max_prefill_tokens=256, cp_threshold=200, seed=9))
        st = pstate.get_state()
        assert st.transport == "ipc" and st.dp_comm is not None and eng.cp_lockstep
        eng.runner.enable_logit_tap()
        rng = random.Random(7)
        V = mc.vocab_size
        greedy = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
        plain = []
        if rank == 0:  # one long prompt (ring-attention prefill) + one short local one
            prompts = [[rng.randrange(10, V - 10) for _ in range(n)] for n in (700, 40)]
            seqs = eng.generate(prompts, greedy)
            plain = [(s.seq_id, list(s.prompt), list(s.output)) for s in seqs]
        else:
            eng.run_until_done()
        rows = _rows(eng.runner.logit_tap or [])
        cp = int(eng.counters.get("cp_prefills", 0))
        err = int(st.dp_comm.err.item())
        w = eng.model.w
        frac, worst, n = _check(mc, w, plain, rows, 0.03) if plain else (1.0, 0.0, 0)
        bfrac, bworst = 0.0, 1.0
        if plain:
            bad = {k: v for k, v in w.items() if k != "layers"}
            bad["layers"] = [dict(x) for x in w["layers"]]
            D, hq = mc.head_dim, mc.num_heads
            qkv = bad["layers"][0]["qkv"].clone()
            k0 = hq * D
            qkv[k0:k0 + D], qkv[k0 + D:k0 + 2 * D] = (qkv[k0 + D:k0 + 2 * D].clone(),
                                                      qkv[k0:k0 + D].clone())
            bad["layers"][0]["qkv"] = qkv
            bfrac, bworst, _ = _check(mc, bad, plain, rows, 0.03)
        q.put(("ok", rank, {"frac": frac, "worst": worst, "rows": n, "neg_frac": bfrac,
                            "neg_worst": bworst, "cp_prefills": cp, "ipc_err": err}))
        import torch.distributed as dist

        dist.barrier()
    except Exception:  # pragma: no cover
        import traceback

        q.put(("err", rank, traceback.format_exc()))


def _spawn(target, world, timeout=420):
    from conftest import release_gpu_memory

    release_gpu_memory()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            status, rank, val = q.get(timeout=timeout)
            assert status == "ok", val
            res[rank] = val
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ep_a2a_on_one_gpu_matches_dense_oracle(world):
    res = _spawn(_ep_worker, world)
    print(f"EP={world}: {res}")
    busy = [r for r in res.values() if not r["idle"]]
    assert all(r["ipc_err"] == 0 for r in res.values())
    assert all(r["rows"] > 0 and r["frac"] >= 0.97 for r in busy), res
    assert any(r["neg_frac"] < 0.97 and r["neg_worst"] > 0.04 for r in busy), res
    # every rank stepped together, with host agreements and graph decode steps
    steps = {r["stats"]["steps"] for r in res.values()}
    assert len(steps) == 1, steps
    assert all(r["agree"]["calls"] >= r["stats"]["steps"] for r in res.values())
    assert all(r["stats"]["graph_steps"] > 0 for r in res.values())
    # steady-state decode ran one step ahead of the host (launch N+1, then collect N)
    assert any(r["stats"]["pipelined_steps"] > 0 for r in busy), res
    if world >= 4:
        assert res[world - 1]["stats"]["idle_fill"] > 0


def test_ep8_mixtral_layer_shapes_on_one_gpu_matches_dense_oracle():
    """BASELINE config 5's EP = 8 with Mixtral-8x7B's exact layer shapes (2
    layers): one expert per rank, IPC all-to-all of 4096-wide rows."""
    from omnia_amd.models.config import resolve

    res = _spawn(_ep_worker_mixtral, 8, timeout=600)
    mc = resolve("mixtral-8x7b").replace(num_layers=2)
    full = _full_mixtral(mc, 5)
    for layer in full["layers"]:
        layer["router"].mul_(ROUTER_SCALE)
    bad = {k: v for k, v in full.items() if k != "layers"}
    bad["layers"] = [dict(x) for x in full["layers"]]
    gu = bad["layers"][0]["experts_gate_up"].clone()
    gu[[0, 1]] = gu[[1, 0]]
    bad["layers"][0]["experts_gate_up"] = gu
    ok = total = 0
    negs = []
    for rank, r in sorted(res.items()):
        rows = {k: [torch.from_numpy(x) for x in v] for k, v in r["rows"].items()}
        frac, worst, n = _check(mc, full, r["plain"], rows, 0.04)
        bfrac, bworst, _ = _check(mc, bad, r["plain"], rows, 0.04)
        print(f"EP=8 mixtral rank {rank}: frac {frac:.3f} worst {worst:.4f} rows {n} "
              f"neg {bfrac:.3f}/{bworst:.3f} stats {r['stats']}")
        ok += round(frac * n)
        total += n
        negs.append((bfrac, bworst))
        assert n > 0
    # at d = 4096 with random routers a bf16 top-2 near-tie flips an expert for a
    # few rows (measured 5 of 48 at 0.05-0.15 rel.); the swapped-expert oracle
    # fails EVERY row on every rank
    assert ok / total >= 0.85, (ok, total)
    assert all(b < 0.5 for b, _ in negs), negs
    assert len({r["stats"]["steps"] for r in res.values()}) == 1


@pytest.mark.parametrize("world", [2, 4])
def test_cp_ring_on_one_gpu_matches_dense_oracle(world):
    res = _spawn(_cp_worker, world)
    print(f"CP={world}: {res}")
    assert all(r["ipc_err"] == 0 for r in res.values())
    assert all(r["cp_prefills"] >= 1 for r in res.values())  # every rank joined the ring
    own = res[0]
    assert own["rows"] > 0 and own["frac"] == 1.0, own
    assert own["neg_frac"] < 1.0 and own["neg_worst"] > 0.03, own
