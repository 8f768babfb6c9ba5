"""Engine behaviour on CPU (tiny random model, reference ops)."""
import torch

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.kv_manager import BlockManager, common_prefix
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.engine.tokenizer import Detokenizer, SyntheticTokenizer
from omnia_amd.models.config import TINY_LLAMA
from omnia_amd.ops import reference as ref


def make_engine(**kw):
    base = dict(model="tiny-llama", device="cpu", num_blocks=96, block_size=16, max_batch=8,
                max_model_len=1024)
    base.update(kw)
    return LLMEngine(EngineConfig(**base))


def test_greedy_is_deterministic_and_batch_invariant():
    e = make_engine()
    p = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)
    a = e.generate(["abc def", "xyz"], p)
    b = e.generate(["abc def"], p)
    assert a[0].output == b[0].output
    assert len(a[1].output) == 6


def test_incremental_decode_matches_full_prefill():
    """Logits of the KV-cached decode path equal a fresh full prefill."""
    e = make_engine()
    p = SamplingParams(temperature=0, max_tokens=5, ignore_eos=True)
    s = e.generate(["the cache must agree"], p)[0]
    full = s.prompt + s.output[:-1]
    e2 = make_engine()
    s2 = e2.generate([full], SamplingParams(temperature=0, max_tokens=1, ignore_eos=True))[0]
    assert s2.output[0] == s.output[-1]


def test_session_prefix_reuse_and_equivalence():
    e = make_engine()
    p = SamplingParams(temperature=0, max_tokens=4, ignore_eos=True)
    t1 = e.generate(["system: be brief. user: hi"], p, session_ids=["sess"])[0]
    conv = "system: be brief. user: hi" + e.tokenizer.decode(t1.output) + " user: more"
    t2 = e.generate([conv], p, session_ids=["sess"])[0]
    assert t2.prefix_hit >= len(t1.prompt)
    fresh = make_engine().generate([conv], p)[0]
    # synthetic tokenizer decode/encode of generated ids is not invertible for ids>255,
    # so compare against the same token ids
    e3 = make_engine()
    ids = t2.prompt
    again = e3.generate([ids], p)[0]
    assert again.output == t2.output
    assert fresh.prefix_hit == 0


def test_chunked_prefill_equals_single_shot():
    p = SamplingParams(temperature=0, max_tokens=3, ignore_eos=True)
    prompt = list(range(1, 300))
    a = make_engine(max_prefill_tokens=64).generate([prompt], p)[0]
    b = make_engine(max_prefill_tokens=4096).generate([prompt], p)[0]
    assert a.output == b.output


def test_preemption_recovers():
    # tiny pool: two long sequences cannot both fit -> one is preempted and recomputed
    e = make_engine(num_blocks=24, block_size=16)
    p = SamplingParams(temperature=0, max_tokens=120, ignore_eos=True)
    seqs = e.generate([list(range(5, 105)), list(range(7, 107))], p)
    assert all(len(s.output) == 120 for s in seqs)
    ref_out = make_engine(num_blocks=200).generate([list(range(5, 105))], p)[0].output
    assert seqs[0].output == ref_out


def test_single_sequence_capped_at_pool_capacity():
    # one sequence alone outgrows the pool (max_model_len > pool): it finishes
    # "length" at capacity instead of faulting the engine; the next request runs
    from omnia_amd.engine.sequence import FinishReason

    e = make_engine(num_blocks=8, block_size=16, max_model_len=1024)
    p = SamplingParams(temperature=0, max_tokens=500, ignore_eos=True)
    s = e.generate([list(range(5, 45))], p)[0]
    assert s.finish_reason == FinishReason.LENGTH and 0 < len(s.output) < 500
    assert s.length <= 8 * 16
    s2 = e.generate([list(range(5, 25))], SamplingParams(temperature=0, max_tokens=4))[0]
    assert len(s2.output) == 4


def test_stop_conditions():
    e = make_engine()
    s = e.generate(["x"], SamplingParams(temperature=0, max_tokens=3))[0]
    assert s.finish_reason.value in ("length", "stop")
    s = e.generate(["x"], SamplingParams(temperature=0, max_tokens=50,
                                         stop_token_ids=[]), )[0]
    assert len(s.output) <= 50


def test_block_manager_lru_eviction():
    bm = BlockManager(9, 4)
    a = bm.allocate(3)
    bm.retain("s1", a, list(range(10)))
    b = bm.allocate(3)
    bm.retain("s2", b, list(range(10)))
    c = bm.allocate(4)  # evicts s1 (LRU)
    assert not bm.has_session("s1") and bm.has_session("s2")
    assert len(set(c)) == 4 and 0 not in c
    blocks, n = bm.acquire_prefix("s2", list(range(6)) + [99])
    assert n == 6 and len(blocks) == 2


def test_common_prefix():
    assert common_prefix(list(range(1000)), list(range(1000))) == 1000
    assert common_prefix(list(range(600)), list(range(300)) + [-1]) == 300


def test_detokenizer_utf8_split():
    tk = SyntheticTokenizer(512, 256, (257,))
    ids = tk.encode("héllo ✓")
    d = Detokenizer(tk)
    out = "".join(d.push(i) for i in ids) + d.flush()
    assert out == "héllo ✓"


def test_sampler_reference_mask():
    logits = torch.tensor([[3.0, 2.0, 1.0, 0.0, -1.0]])
    m = ref.sample_mask(logits, torch.tensor([1.0]), torch.tensor([2]), torch.tensor([1.0]))
    assert m.tolist() == [[True, True, False, False, False]]
    m = ref.sample_mask(logits, torch.tensor([1.0]), torch.tensor([0]), torch.tensor([0.5]))
    assert m[0, 0] and not m[0, 2]


def test_model_param_count():
    from omnia_amd.models.config import LLAMA3_8B, LLAMA3_70B

    assert abs(LLAMA3_8B.num_params() / 1e9 - 8.03) < 0.05
    assert abs(LLAMA3_70B.num_params() / 1e9 - 70.6) < 0.2
    assert LLAMA3_8B.kv_bytes_per_token() == 128 * 1024


def test_mixed_steps_match_separate_steps():
    """Mixed decode+prefill steps (mixed_budget) produce the same greedy tokens
    as separate prefill / decode steps, with staggered arrivals."""
    from omnia_amd.engine.engine import EngineConfig, LLMEngine
    from omnia_amd.engine.sampling_params import SamplingParams

    outs = {}
    for budget in (0, 48):
        eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=256,
                                     block_size=16, max_batch=8, max_model_len=1024,
                                     max_prefill_tokens=256, mixed_budget=budget, seed=1))
        p = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
        first = [eng.add_request(list(range(10, 90)), p), eng.add_request(list(range(5, 40)), p)]
        for _ in range(4):
            eng.step()
        later = [eng.add_request(list(range(100, 230)), p), eng.add_request([7] * 61, p)]
        eng.run_until_done()
        outs[budget] = [s.output for s in first + later]
        if budget:
            assert eng.counters.get("steps_mixed", 0) >= 2
    assert outs[0] == outs[48]


def test_mixed_steps_only_for_a_trickle_backlog():
    """``mixed_backlog``: a burst of prompts is prefilled first (full prefill
    steps); once the backlog fits, decode rows ride along the prefill chunks."""
    from omnia_amd.engine.kv_manager import BlockManager
    from omnia_amd.engine.sampling_params import SamplingParams
    from omnia_amd.engine.scheduler import Scheduler, SchedulerConfig
    from omnia_amd.engine.sequence import Sequence

    sch = Scheduler(SchedulerConfig(max_batch=16, max_prefill_tokens=64, mixed_budget=64,
                                    mixed_backlog=100), BlockManager(256, 4))
    p = SamplingParams(max_tokens=4)
    first = Sequence(prompt=list(range(1, 9)), params=p)
    sch.add(first)
    plan = sch.schedule()
    assert plan.kind == "prefill"
    sch.on_prefill_done(plan.prefill, {first.seq_id: 5})
    for _ in range(5):  # a burst: 5 x 40 = 200 backlog tokens > 100
        sch.add(Sequence(prompt=list(range(1, 41)), params=p))
    assert sch.backlog_tokens() == 200
    assert sch.schedule().kind == "prefill"  # prefill-first while the burst drains
    while sch.backlog_tokens() > 100:
        plan = sch.schedule()
        assert plan.kind == "prefill"
        sch.on_prefill_done(plan.prefill, {s.seq_id: 5 for s, _ in plan.prefill})
    assert sch.schedule().kind == "mixed"  # a trickle: decoders keep streaming


def test_shared_prefix_pages_equivalence_cpu():
    """Cross-session prefix sharing on the CPU engine: the common system prompt's
    full pages are computed once; later prompts map them, and greedy outputs
    equal an engine without sharing.  Fault recovery forgets them."""
    p = SamplingParams(temperature=0, max_tokens=5, ignore_eos=True)
    sysp = list(range(11, 61))  # 50 tokens: 3 full pages of 16
    w1 = [sysp + [70 + i, 71 + i] for i in range(3)]
    w2 = [sysp + list(range(100 + i, 110 + 2 * i)) for i in range(3)]
    from omnia_amd.observability import metrics as M

    shared0 = M.KV_SHARED_HIT_TOKENS._value.get()
    e = make_engine(dtype="float32")
    e.generate(w1, p)
    got = e.generate(w2, p)
    assert [s.prefix_hit for s in got] == [48] * 3
    assert M.KV_SHARED_HIT_TOKENS._value.get() - shared0 == 3 * 48
    want = make_engine(dtype="float32", share_prefix=False).generate(w2, p)
    assert [s.output for s in got] == [s.output for s in want]
    e.recover(RuntimeError("test"))
    assert not e.blocks.table and not e.blocks.ref
    assert e.generate(w2[:1], p)[0].prefix_hit == 0
