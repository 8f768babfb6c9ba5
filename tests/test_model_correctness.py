"""Whole-model correctness gate: the engine's logits at every generated position
(chunked ragged prefill, hipGraph decode, session prefix reuse, multi-sequence
batches) against an independent fp32 dense forward of the same weights
(``ops.reference.dense_forward``: no paging, no batching, no graphs).

The GPU variants run tiny-llama, a 2-layer model with Llama-3-8B's exact layer
shapes (hidden 4096, 32 q / 8 kv heads, MLP 14336, vocab 128256) and
tiny-mixtral.  A negative control corrupts one weight slice of the oracle and
asserts the gate then fails -- so a wrong slice or stride in any engine path
cannot pass silently."""
import random

import pytest
import torch

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.models.config import resolve
from omnia_amd.ops import reference as ref


def _engine(device, mc, chunk, **kw):
    kw.setdefault("mixed_budget", 0)  # the paths under test; mixed steps have their own test
    eng = LLMEngine(EngineConfig(model=mc.name, device=device, num_blocks=512, block_size=16,
                                 max_batch=8, max_model_len=1024, max_prefill_tokens=chunk,
                                 pipeline=False, seed=3, **kw), model_cfg=mc)
    eng.runner.enable_logit_tap()
    return eng


def _run(eng, mc, rng, prompt_lens=(150, 70, 33), gen=10):
    V = mc.vocab_size
    greedy = SamplingParams(temperature=0.0, max_tokens=gen, ignore_eos=True)
    prompts = [[rng.randrange(10, V - 10) for _ in range(n)] for n in prompt_lens]
    seqs = eng.generate(prompts, greedy, session_ids=["a", "b", "c"])
    # turn 2 of session "a": resident KV prefix + 20 new tokens
    p2 = prompts[0] + seqs[0].output + [rng.randrange(10, V - 10) for _ in range(20)]
    s2 = eng.generate([p2], greedy, session_ids=["a"])[0]
    assert s2.prefix_hit > 0
    return seqs + [s2]


def _rows_by_seq(tap):
    out = {}
    for ids, rows in tap:
        for i, sid in enumerate(ids):
            out.setdefault(sid, []).append(rows[i])
    return out


def _check(mc, w, seqs, tap, rel_tol, min_pass=1.0):
    """-> (fraction of rows within tolerance, worst relative error)."""
    rows = _rows_by_seq(tap)
    ok = total = 0
    worst = 0.0
    for s in seqs:
        got = rows[s.seq_id]
        assert len(got) == len(s.output)
        full = s.prompt + s.output
        want = ref.dense_forward(mc, w, full[:-1])[len(s.prompt) - 1:]
        for g, r in zip(got, want):
            err = float((g - r).abs().max() / r.abs().max())
            worst = max(worst, err)
            ok += err < rel_tol
            total += 1
    return ok / total, worst


def _gate(device, mc, chunk, rel_tol, min_pass=1.0, router_scale=None, prompt_lens=None,
          **kw):
    rng = random.Random(7)
    torch.manual_seed(0)
    eng = _engine(device, mc, chunk, **kw)
    w = eng.model.w
    if router_scale is not None:  # sharpen routing so bf16 vs fp32 top-k cannot tie
        for layer in w["layers"]:
            layer["router"].mul_(router_scale)
    seqs = _run(eng, mc, rng, **({"prompt_lens": prompt_lens} if prompt_lens else {}))
    c = eng.counters  # prompts really were chunked (prefill or mixed steps)
    assert c["steps_prefill"] + c.get("steps_mixed", 0) + c.get("steps_mixed_sync", 0) > \
        len(seqs), dict(c)
    frac, worst = _check(mc, w, seqs, eng.runner.logit_tap, rel_tol)
    assert frac >= min_pass, f"{mc.name}: {frac:.3f} of rows within {rel_tol}, worst {worst:.4f}"
    # negative control: a wrong kv-head slice in the oracle must fail the gate
    bad = {"embed": w["embed"], "lm_head": w["lm_head"], "final_norm": w["final_norm"],
           "layers": [dict(x) for x in w["layers"]]}
    D, hq, hkv = mc.head_dim, mc.num_heads, mc.num_kv_heads
    qkv = bad["layers"][0]["qkv"].clone()
    k0 = hq * D
    qkv[k0:k0 + D], qkv[k0 + D:k0 + 2 * D] = qkv[k0 + D:k0 + 2 * D].clone(), qkv[k0:k0 + D].clone()
    bad["layers"][0]["qkv"] = qkv
    bfrac, bworst = _check(mc, bad, seqs, eng.runner.logit_tap, rel_tol)
    assert bfrac < min_pass and bworst > rel_tol
    return frac, worst


def test_cpu_engine_matches_dense_oracle():
    """CPU build of the same engine paths (reference ops, eager decode)."""
    _gate("cpu", resolve("tiny-llama"), chunk=64, rel_tol=0.03)


@pytest.mark.gpu
def test_gpu_tiny_llama_matches_dense_oracle():
    frac, worst = _gate("cuda", resolve("tiny-llama"), chunk=64, rel_tol=0.03)
    print(f"tiny-llama worst rel err {worst:.4f}")


@pytest.mark.gpu
def test_gpu_llama3_8b_shaped_two_layers_matches_dense_oracle():
    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    frac, worst = _gate("cuda", mc, chunk=64, rel_tol=0.04)
    print(f"llama-3-8b-2l worst rel err {worst:.4f}")


@pytest.mark.gpu
def test_gpu_llama3_8b_shaped_fused_prefill_matches_dense_oracle():
    """Prefill chunks of 384 rows run the fused-epilogue prefill layer (pgemm.hip:
    QKV+RoPE+KV write, O/down + residual + row sumsq, gate_up + SwiGLU with the
    folded RMSNorm row scale); decode and the second turn's 20-token prefill run
    the split-K / tile paths.  Chunks are not a multiple of the 256-row tile."""
    from omnia_amd.models.llama import LlamaModel

    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    saved = LlamaModel.PGEMM_MIN_ROWS
    LlamaModel.PGEMM_MIN_ROWS = 257  # serving default 2049: 384-row chunks take split-K
    try:
        frac, worst = _gate("cuda", mc, chunk=384, rel_tol=0.04, prompt_lens=(600, 300, 280))
    finally:
        LlamaModel.PGEMM_MIN_ROWS = saved
    print(f"llama-3-8b-2l fused prefill worst rel err {worst:.4f}")


def test_norm_folding_is_exact_reparametrisation():
    """fold_norms moves non-unit RMSNorm weights into the QKV / gate_up rows: the
    dense oracle of the folded weights equals the oracle of the original ones."""
    from omnia_amd.models.llama import LlamaModel

    mc = resolve("tiny-llama")
    torch.manual_seed(0)
    base = LlamaModel(mc, device="cpu", seed=5)
    orig = {"embed": base.w["embed"], "lm_head": base.w["lm_head"],
            "final_norm": base.w["final_norm"], "layers": []}
    for layer in base.w["layers"]:
        l2 = {k: v.clone() for k, v in layer.items()}
        l2["in_norm"] = (1 + 0.5 * torch.rand_like(l2["in_norm"].float())).to(l2["in_norm"].dtype)
        l2["post_norm"] = (1 + 0.5 * torch.rand_like(l2["post_norm"].float())).to(l2["post_norm"].dtype)
        orig["layers"].append(l2)
    keep = {"layers": [{k: v.clone() for k, v in l.items()} for l in orig["layers"]],
            **{k: v for k, v in orig.items() if k != "layers"}}
    folded = LlamaModel(mc, device="cpu", seed=5, weights=orig)
    for l in folded.w["layers"]:
        assert bool(torch.all(l["in_norm"] == 1)) and bool(torch.all(l["post_norm"] == 1))
    ids = list(range(100, 140))
    want = ref.dense_forward(mc, keep, ids)
    got = ref.dense_forward(mc, folded.w, ids)
    err = float((got - want).abs().max() / want.abs().max())
    assert err < 0.02, err
    # negative control: dropping the norm weights entirely is visibly different
    plain = {"layers": [dict(l, in_norm=torch.ones_like(l["in_norm"]),
                             post_norm=torch.ones_like(l["post_norm"])) for l in keep["layers"]],
             **{k: v for k, v in keep.items() if k != "layers"}}
    bad = ref.dense_forward(mc, plain, ids)
    assert float((bad - want).abs().max() / want.abs().max()) > 0.05


@pytest.mark.gpu
def test_gpu_tiny_mixtral_matches_dense_oracle():
    frac, worst = _gate("cuda", resolve("tiny-mixtral"), chunk=64, rel_tol=0.04,
                        min_pass=0.97, router_scale=30.0)
    print(f"tiny-mixtral: {frac:.3f} rows within tol, worst rel err {worst:.4f}")


def test_cpu_mixtral_a2a_expert_parallel_path_matches_dense_oracle():
    """ep_mode a2a (DP attention + EP) on one rank: the dispatch -> row-routed
    expert FFN -> combine path of every MoE layer against the dense oracle."""
    _gate("cpu", resolve("tiny-mixtral"), chunk=64, rel_tol=0.04, min_pass=0.97,
          router_scale=30.0, ep_mode="a2a")


@pytest.mark.gpu
def test_gpu_tiny_mixtral_a2a_expert_parallel_path_matches_dense_oracle():
    """Same on the GPU: the static-capacity dispatch / combine and the row-routed
    grouped MFMA expert kernels (ops.moe_rows) inside captured decode graphs."""
    frac, worst = _gate("cuda", resolve("tiny-mixtral"), chunk=64, rel_tol=0.04,
                        min_pass=0.97, router_scale=30.0, ep_mode="a2a")
    print(f"tiny-mixtral a2a EP: {frac:.3f} rows within tol, worst rel err {worst:.4f}")


@pytest.mark.gpu
def test_gpu_llama3_8b_shaped_large_batch_decode():
    """160 concurrent sequences: the decode GEMMs run at M=160 (the hand MFMA
    dgemm / tuned hipBLASLt dispatch of the serving batch sizes), checked on a
    sample of the sequences."""
    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=2048, block_size=16,
                                 max_batch=192, max_model_len=512, max_prefill_tokens=1024,
                                 pipeline=False, seed=5), model_cfg=mc)
    eng.runner.enable_logit_tap()
    rng = random.Random(11)
    prompts = [[rng.randrange(10, mc.vocab_size - 10) for _ in range(24 + (i % 7))]
               for i in range(160)]
    seqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))
    assert eng.runner.stats["graph_replays"] >= 4
    sample = [seqs[i] for i in (0, 31, 77, 128, 159)]
    frac, worst = _check(mc, eng.model.w, sample, eng.runner.logit_tap, 0.04)
    print(f"llama-3-8b-2l B=160: worst rel err {worst:.4f}")
    assert frac == 1.0


@pytest.fixture
def forced_wgemm(monkeypatch):
    """Route every decode projection through wgemm + the split-K consumers."""
    from omnia_amd import ops

    def cfg(M, N, K, mode):
        if M > 256:
            return None
        S = 2 if K % 256 == 0 else 1
        if mode == 1:
            return (2, 2, S)
        return (1, 2, S)

    monkeypatch.setattr(ops, "wgemm_config", cfg)


@pytest.mark.gpu
def test_gpu_fused_splitk_decode_path_matches_dense_oracle(forced_wgemm):
    """QKV -> splitk_rope_kv, O / down -> splitk_add_rmsnorm, gate_up split-K ->
    splitk_swiglu, all inside the captured decode graphs."""
    for mc in (resolve("tiny-llama"),
               resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)):
        frac, worst = _gate("cuda", mc, chunk=64, rel_tol=0.04)
        print(f"{mc.name} fused split-K decode: worst rel err {worst:.4f}")


@pytest.mark.gpu
def test_gpu_mixed_steps_match_dense_oracle():
    """Mixed decode + prefill steps (split decode / prefill attention in one
    forward) with staggered arrivals, against the dense oracle."""
    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=512, block_size=16,
                                 max_batch=8, max_model_len=1024, max_prefill_tokens=256,
                                 pipeline=False, seed=9, mixed_budget=40), model_cfg=mc)
    eng.runner.enable_logit_tap()
    rng = random.Random(3)
    V = mc.vocab_size
    p = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    seqs = [eng.add_request([rng.randrange(10, V - 10) for _ in range(n)], p) for n in (70, 33)]
    for _ in range(3):
        eng.step()
    seqs += [eng.add_request([rng.randrange(10, V - 10) for _ in range(n)], p) for n in (120, 9)]
    eng.run_until_done()
    assert eng.counters.get("steps_mixed", 0) >= 3
    frac, worst = _check(mc, eng.model.w, seqs, eng.runner.logit_tap, 0.04)
    print(f"mixed steps: {eng.counters['steps_mixed']}, worst rel err {worst:.4f}")
    assert frac == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [False, True])
def test_gpu_fused_mixed_steps_match_dense_oracle(pipeline):
    """Mixed steps of >= 257 rows run the fused-epilogue prefill layer (pgemm.hip,
    the decode rows riding the prefill GEMMs; split decode / prefill attention
    in between) -- against the dense oracle, synchronous and pipelined."""
    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=512, block_size=16,
                                 max_batch=8, max_model_len=1024, max_prefill_tokens=640,
                                 pipeline=pipeline, seed=11, mixed_budget=640,
                                 mixed_backlog=2048), model_cfg=mc)
    eng.runner.enable_logit_tap()
    model = eng.model
    model.PGEMM_MIXED_MIN_ROWS = 257  # the serving default (4096) skips these small steps
    fused = {"mixed": 0}
    orig = model._fused_residual

    def counted(fb, kv):
        if fb.num_decode:
            fused["mixed"] += 1
        return orig(fb, kv)

    model._fused_residual = counted
    rng = random.Random(5)
    V = mc.vocab_size
    p = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
    seqs = [eng.add_request([rng.randrange(10, V - 10) for _ in range(n)], p) for n in (90, 41)]
    for _ in range(3):
        eng.step()
    seqs += [eng.add_request([rng.randrange(10, V - 10) for _ in range(n)], p) for n in (420, 330)]
    eng.run_until_done()
    assert fused["mixed"] >= 1, eng.counters
    frac, worst = _check(mc, eng.model.w, seqs, eng.runner.logit_tap, 0.04)
    print(f"fused mixed steps: {fused['mixed']}, worst rel err {worst:.4f}")
    assert frac == 1.0


@pytest.mark.gpu
def test_gpu_midsize_mixed_steps_split_k_match_dense_oracle():
    """Mixed steps of 257..4095 rows (the open loop's) take the 256x256 tile with
    split-K + the slab consumers for qkv / o / down and the unsplit fused tile for
    gate_up wherever ops/tuned/midm_mi355x.json lists a win -- against the dense
    oracle, pipelined."""
    from omnia_amd import ops

    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=512, block_size=16,
                                 max_batch=8, max_model_len=1024, max_prefill_tokens=640,
                                 seed=12, mixed_budget=640, mixed_backlog=2048), model_cfg=mc)
    eng.runner.enable_logit_tap()
    seen = []
    orig = ops.midm_config

    def spy(M, N, K, mode):
        cfg = orig(M, N, K, mode)
        if cfg is not None:
            seen.append((M, N, K, mode, cfg[2]))
        return cfg

    ops.midm_config = spy
    try:
        rng = random.Random(6)
        V = mc.vocab_size
        p = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
        # a pure 520-row prefill chunk (below the fused layer's 2049 rows), then
        # mixed steps of 257..640 rows
        seqs = [eng.add_request([rng.randrange(10, V - 10) for _ in range(n)], p)
                for n in (300, 220)]
        for _ in range(3):
            eng.step()
        seqs += [eng.add_request([rng.randrange(10, V - 10) for _ in range(n)], p)
                 for n in (420, 330)]
        eng.run_until_done()
    finally:
        ops.midm_config = orig
    assert {m for *_, m, _ in seen} >= {0}, seen  # split-K projections ran
    assert any(S > 1 for *_, S in seen), seen
    frac, worst = _check(mc, eng.model.w, seqs, eng.runner.logit_tap, 0.04)
    print(f"mid-size split-K steps: {len(seen)} projections, worst rel err {worst:.4f}")
    assert frac == 1.0


@pytest.mark.gpu
def test_gpu_70b_shaped_midsize_prefill_split_k_matches_dense_oracle():
    """Llama-3-70B-shaped (2 layers) 520-row prefill below the fused layer's
    threshold: qkv / o split-K and gate_up on the unsplit fused tile from the
    70B rows of ops/tuned/midm_mi355x.json -- against the dense oracle."""
    from omnia_amd import ops

    mc = resolve("llama-3-70b").replace(name="llama-3-70b-2l", num_layers=2)
    eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=256, block_size=16,
                                 max_batch=4, max_model_len=1024, max_prefill_tokens=640,
                                 seed=14, mixed_budget=0), model_cfg=mc)
    eng.runner.enable_logit_tap()
    seen = []
    orig = ops.midm_config

    def spy(M, N, K, mode):
        cfg = orig(M, N, K, mode)
        if cfg is not None:
            seen.append((M, N, K, mode, cfg[2]))
        return cfg

    ops.midm_config = spy
    try:
        rng = random.Random(8)
        V = mc.vocab_size
        p = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)
        seqs = eng.generate([[rng.randrange(10, V - 10) for _ in range(n)] for n in (300, 220)],
                            p)
    finally:
        ops.midm_config = orig
    assert any(S > 1 for *_, S in seen) and any(m == 1 for *_, m, _ in seen), seen
    frac, worst = _check(mc, eng.model.w, seqs, eng.runner.logit_tap, 0.04)
    print(f"70b-shaped mid-size prefill: worst rel err {worst:.4f}")
    assert frac == 1.0


@pytest.mark.gpu
def test_gpu_shared_prefix_pages_match_dense_oracle():
    """Cross-session prefix sharing (kv_manager.py): the second wave's prompts map
    the 6 full 16-token pages of the 100-token system prompt the first wave
    computed; every logit row of the second wave (prefill from token 96 over the
    shared pages, then decode) stays within the dense oracle's tolerance."""
    mc = resolve("llama-3-8b").replace(name="llama-3-8b-2l", num_layers=2)
    eng = LLMEngine(EngineConfig(model=mc.name, device="cuda", num_blocks=512, block_size=16,
                                 max_batch=8, max_model_len=1024, seed=13), model_cfg=mc)
    eng.runner.enable_logit_tap()
    rng = random.Random(9)
    V = mc.vocab_size
    sysp = [rng.randrange(10, V - 10) for _ in range(100)]
    p = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    eng.generate([sysp + [rng.randrange(10, V - 10) for _ in range(n)] for n in (20, 57, 3)], p)
    eng.runner.logit_tap.clear()
    seqs = eng.generate([sysp + [rng.randrange(10, V - 10) for _ in range(n)]
                         for n in (40, 1, 90, 13)], p)
    assert [s.prefix_hit for s in seqs] == [96] * 4
    frac, worst = _check(mc, eng.model.w, seqs, eng.runner.logit_tap, 0.04)
    print(f"shared-prefix rows: worst rel err {worst:.4f}")
    assert frac == 1.0
