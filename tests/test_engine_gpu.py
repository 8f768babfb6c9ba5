"""Engine on the GPU: hipGraph decode, async (pipelined) scheduling, session KV."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams


def eng(**kw):
    base = dict(model="tiny-llama", device="cuda", num_blocks=256, block_size=32, max_batch=16,
                max_model_len=2048)
    base.update(kw)
    return LLMEngine(EngineConfig(**base))


def _run(e, prompts, max_toks):
    seqs = [e.add_request(p, SamplingParams(temperature=0, max_tokens=m, ignore_eos=True),
                          session_id=f"s{i}") for i, (p, m) in enumerate(zip(prompts, max_toks))]
    e.run_until_done()
    return [s.output for s in seqs]


def test_pipelined_equals_synchronous_greedy():
    prompts = [list(range(10 + i, 60 + 3 * i)) for i in range(9)]
    max_toks = [5, 17, 33, 1, 40, 8, 25, 3, 12]  # ragged finishes change batch composition
    a = _run(eng(pipeline=True), prompts, max_toks)
    b = _run(eng(pipeline=False), prompts, max_toks)
    c = _run(eng(use_graphs=False), prompts, max_toks)
    assert a == b == c
    assert [len(x) for x in a] == max_toks


def test_pipelined_chunked_prefill_equals_synchronous_sampled():
    """Many small pipelined prefill steps (chunked prompts finishing in different
    steps) + seeded sampling: identical to the synchronous engine and to eager."""
    prompts = [list(range(5 + i, 5 + i + 30 + 23 * i)) for i in range(8)]

    def run(temp=0.8, **kw):
        e = eng(max_prefill_tokens=64, **kw)
        seqs = [e.add_request(p, SamplingParams(temperature=temp, top_k=20, seed=100 + i,
                                                max_tokens=6 + i, ignore_eos=True),
                              session_id=f"c{i}") for i, p in enumerate(prompts)]
        e.run_until_done()
        return [s.output for s in seqs], e.runner.stats["prefill_steps"]

    a, na = run(pipeline=True)
    b, nb = run(pipeline=False)
    assert a == b
    assert na == nb and na > 5
    g = [run(0.0, **kw)[0] for kw in (dict(pipeline=True), dict(use_graphs=False))]
    assert g[0] == g[1]


def test_decode_matches_fresh_prefill_on_gpu():
    e = eng()
    s = e.generate([list(range(3, 200))], SamplingParams(temperature=0, max_tokens=20,
                                                          ignore_eos=True))[0]
    full = s.prompt + s.output[:-1]
    s2 = eng().generate([full], SamplingParams(temperature=0, max_tokens=1,
                                               ignore_eos=True))[0]
    assert s2.output[0] == s.output[-1]


def test_session_prefix_reuse_gpu_equivalence():
    e = eng()
    p = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)
    t1 = e.generate([list(range(5, 100))], p, session_ids=["x"])[0]
    turn2 = t1.prompt + t1.output + list(range(300, 340))
    t2 = e.generate([turn2], p, session_ids=["x"])[0]
    assert t2.prefix_hit >= len(t1.prompt)
    t2_fresh = eng().generate([turn2], p)[0]
    assert t2.output == t2_fresh.output


def test_sampled_decode_with_topk_topp_runs():
    e = eng()
    seqs = e.generate([list(range(1, 50))] * 4,
                      SamplingParams(temperature=0.9, top_k=50, top_p=0.9, max_tokens=16,
                                     seed=7, ignore_eos=True))
    assert all(len(s.output) == 16 for s in seqs)
    assert all(0 <= t < 512 for s in seqs for t in s.output)


def test_llama3_8b_shapes_one_step():
    """Real 8B architecture: prefill + a few graph decode steps."""
    e = LLMEngine(EngineConfig(model="llama-3-8b", device="cuda", num_blocks=512,
                               block_size=32, max_batch=8, max_model_len=4096))
    seqs = e.generate([list(range(1000, 1600)), list(range(2000, 2100))],
                      SamplingParams(temperature=0, max_tokens=8, ignore_eos=True))
    assert all(len(s.output) == 8 for s in seqs)
    assert e.runner.stats["graph_replays"] > 0
    del e
    torch.cuda.empty_cache()


def test_guided_json_mixed_with_pipelined_batch():
    """Grammar-constrained requests (synchronous steps with GPU token masks) share
    the engine with ordinary requests; every guided output is schema-valid JSON."""
    import json

    from omnia_amd.utils import jsonschema as js

    schema = {"type": "object", "properties": {"n": {"type": "integer"},
                                               "tag": {"enum": ["x", "yy"]}},
              "required": ["n", "tag"]}
    e = eng()
    guided = [e.add_request(list(range(20, 60 + i)), SamplingParams(
        temperature=0.9, seed=i, max_tokens=200, json_schema=schema)) for i in range(4)]
    free = [e.add_request(list(range(30, 70)), SamplingParams(temperature=0, max_tokens=20,
                                                              ignore_eos=True))
            for _ in range(3)]
    e.run_until_done()
    for s in guided:
        assert s.finish_reason.value == "stop"
        js.validate(json.loads(e.tokenizer.decode(s.output)), schema)
    assert all(len(s.output) == 20 for s in free)
    assert free[0].output == free[1].output == free[2].output
