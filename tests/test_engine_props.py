"""Property test of the continuous-batching engine on the CPU (tiny-llama, fp32,
greedy): for random arrival schedules, prompt / output lengths, batch and
prefill limits, mixed steps on or off, the synchronous or the pipelined loop
(graph replays simulated on the CPU, ``OMNIA_SIM_GRAPHS``: device token
slots, placeholders, padded graph rows), and KV pools small enough to force
preemption with recompute, every request finishes with exactly its token
budget and the tokens equal generating that request alone.  Each scheduled
step also respects the batch and prefill-token limits.

It found two bugs: partially prefilled prompts kept their pages while a running
sequence was cut off at the pool limit (the scheduler now preempts them first),
and the CPU KV write sent padded rows' slot -1 to the last page's last slot."""
import functools
import os

import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams


@functools.lru_cache(maxsize=None)
def _weights():
    from omnia_amd.models import build_model
    from omnia_amd.models.config import resolve

    return build_model(resolve("tiny-llama"), device="cpu", dtype=torch.float32, seed=5).w


def _engine(sim: bool = False, **kw):
    base = dict(model="tiny-llama", device="cpu", dtype="float32", block_size=8,
                max_model_len=256, use_graphs=sim, pipeline=sim)
    base.update(kw)
    old = os.environ.get("OMNIA_SIM_GRAPHS")
    os.environ["OMNIA_SIM_GRAPHS"] = "1" if sim else "0"
    try:
        return LLMEngine(EngineConfig(**base), weights=_weights())
    finally:
        if old is None:
            os.environ.pop("OMNIA_SIM_GRAPHS", None)
        else:
            os.environ["OMNIA_SIM_GRAPHS"] = old


@functools.lru_cache(maxsize=None)
def _alone(prompt: tuple, max_tokens: int) -> tuple:
    e = _engine(num_blocks=64, max_batch=4, max_prefill_tokens=256)
    p = SamplingParams(temperature=0, max_tokens=max_tokens, ignore_eos=True)
    return tuple(e.generate([list(prompt)], p)[0].output)


REQ = st.tuples(st.integers(1, 90), st.integers(1, 10), st.integers(0, 6), st.integers(0, 3))


@given(st.lists(REQ, min_size=1, max_size=5), st.integers(2, 4), st.sampled_from([16, 32, 64]),
       st.sampled_from([0, 24]), st.integers(14, 40), st.booleans())
@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
def test_engine_matches_single_requests(reqs, max_batch, max_prefill, mixed, num_blocks, sim):
    e = _engine(sim, num_blocks=num_blocks, max_batch=max_batch, max_prefill_tokens=max_prefill,
                mixed_budget=mixed)
    plan = []
    for i, (plen, mt, at, salt) in enumerate(reqs):
        prompt = tuple((7 * i + 3 * salt + j) % 200 + 10 for j in range(plen))
        plan.append((at, prompt, mt))
    seqs, steps, pending = [], 0, sorted(range(len(plan)), key=lambda i: plan[i][0])
    sch = e.scheduler
    orig = sch.schedule

    def checked():
        p = orig()
        if p.kind in ("decode", "mixed"):
            assert len(p.decode) <= max_batch
            assert len({s.seq_id for s in p.decode}) == len(p.decode)
        if p.kind in ("prefill", "mixed"):
            assert sum(n for _, n in p.prefill) <= max_prefill
            assert all(n > 0 for _, n in p.prefill)
        return p

    sch.schedule = checked
    while pending or e.has_work():
        while pending and plan[pending[0]][0] <= steps:
            i = pending.pop(0)
            at, prompt, mt = plan[i]
            s = e.add_request(list(prompt), SamplingParams(temperature=0, max_tokens=mt,
                                                           ignore_eos=True))
            seqs.append((i, s))
        e.step()
        steps += 1
        assert steps < 2000, "engine did not drain"
    for i, s in seqs:
        at, prompt, mt = plan[i]
        assert len(s.output) == mt
        assert tuple(s.output) == _alone(prompt, mt), (i, e.counters)


TURN = st.tuples(st.sampled_from(["s0", "s1", "s2"]), st.integers(1, 30), st.integers(1, 6))


@given(st.lists(TURN, min_size=1, max_size=6), st.integers(14, 40), st.booleans(),
       st.sampled_from([0, 24]), st.sampled_from([0.0, 0.0004]))
@settings(max_examples=20, deadline=None, suppress_health_check=[HealthCheck.too_slow])
def test_multi_turn_sessions_match_stateless_generation(turns, num_blocks, sim, mixed, swap):
    """Session KV reuse (prefix hits, parked pages, LRU eviction under a small
    pool, the host swap tier holding a few evicted pages): turn k of a session
    -- history + its reply + a new message -- equals generating that whole
    prompt with no cache."""
    e = _engine(sim, num_blocks=num_blocks, max_batch=3, max_prefill_tokens=32,
                mixed_budget=mixed, swap_gib=swap)
    hist: dict = {}
    p = lambda n: SamplingParams(temperature=0, max_tokens=n, ignore_eos=True)  # noqa: E731
    for k, (sid, nmsg, gen) in enumerate(turns):
        prompt = hist.get(sid, []) + [(11 * k + j) % 180 + 20 for j in range(nmsg)]
        if len(prompt) + gen > min(250, (num_blocks - 1) * 8):
            continue  # larger than the whole pool: that turn cannot run at all
        s = e.generate([prompt], p(gen), session_ids=[sid])[0]
        assert tuple(s.output) == _alone(tuple(prompt), gen), (k, sid, s.prefix_hit)
        hist[sid] = prompt + s.output
