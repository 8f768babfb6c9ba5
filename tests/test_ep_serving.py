"""DP-attention + expert-parallel serving (``EngineConfig.ep_mode="a2a"``): every
rank is its own engine with its own prompts, the Mixtral MoE layers exchange
tokens through the fixed-capacity all-to-all, and the ranks step in lockstep
(prefill on one rank while another decodes or idles).  Outputs must equal a
single-rank engine with all experts local on the same prompts (gloo, world 2,
4 and 8; the same weights by construction: experts are drawn per global id)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

PROMPTS = {  # rank -> prompts of different counts and lengths (unequal load)
    0: [[5, 9, 2, 7, 3, 11, 4], [8, 1, 6]],
    1: [[13, 2, 9, 9, 1, 4, 4, 4, 7, 2, 5, 12]],
    2: [],  # an idle rank still serves the group's all-to-alls
    3: [[3, 3, 3], [14, 15, 2, 1], [6, 7, 8, 9, 10]],
}
MAX_TOKENS = {0: 6, 1: 9, 2: 0, 3: 4}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(model="tiny-mixtral", **kw):
    from omnia_amd.engine.engine import EngineConfig

    return EngineConfig(model=model, device="cpu", dtype="float32", num_blocks=64,
                        block_size=4, max_batch=8, max_model_len=128, use_graphs=False,
                        seed=5, **kw)


def _model(world):
    return "tiny-mixtral-e8" if world > 4 else "tiny-mixtral"


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    try:
        from omnia_amd.engine.engine import LLMEngine
        from omnia_amd.engine.sampling_params import SamplingParams

        eng = LLMEngine(_cfg(_model(world), ep_mode="a2a"))
        assert eng.ep_lockstep and eng.model.e_local == eng.model_cfg.num_experts // world
        prompts, mt = PROMPTS[rank % 4], MAX_TOKENS[rank % 4]
        outs = []
        if prompts:
            seqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=mt,
                                                        ignore_eos=True))
            outs = [s.output for s in seqs]
        else:
            eng.run_until_done()
        q.put(("ok", rank, outs, dict(eng.runner.ep_stats)))
        import torch.distributed as dist

        dist.barrier()
    except Exception:  # pragma: no cover
        import traceback

        q.put(("err", rank, traceback.format_exc(), None))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_attention_ep_engine_matches_single_rank(world):
    from omnia_amd.engine.engine import LLMEngine
    from omnia_amd.engine.sampling_params import SamplingParams

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[1])
    for p in procs:
        p.join(60)
    for status, rank, val, _ in res:
        assert status == "ok", val
    oracle = LLMEngine(_cfg(_model(world), ep_mode="tp"))  # one rank, every expert local
    for _, rank, outs, stats in res:
        prompts = PROMPTS[rank % 4]
        if not prompts:
            assert outs == [] and stats["idle_fill"] > 0  # served the others' MoE layers
            continue
        want = oracle.generate(prompts, SamplingParams(temperature=0.0,
                                                       max_tokens=MAX_TOKENS[rank % 4],
                                                       ignore_eos=True))
        assert outs == [s.output for s in want], (rank, outs)
        assert stats["steps"] >= MAX_TOKENS[rank % 4]


def test_capacity_is_step_global_and_lossless():
    """Single-process view of the dispatch plan: slots are unique per rank
    buffer and every assignment fits (capacity = global tokens x k)."""
    from omnia_amd.parallel.expert import dispatch_slots

    ids = torch.tensor([[0, 3], [3, 1], [2, 0], [3, 2]], dtype=torch.int32)
    slot = dispatch_slots(ids, e_local=2, ep=2, cap=4 * 2)
    dest = ids.reshape(-1).long() // 2
    assert len(set(slot.tolist())) == slot.numel()
    assert torch.equal(slot // 8, dest)
    # order within a destination follows (token, slot) order
    assert (slot[dest == 0] % 8).tolist() == [0, 1, 2]
    assert (slot[dest == 1] % 8).tolist() == [0, 1, 2, 3, 4]
