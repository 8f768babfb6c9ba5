"""Context-parallel prefill on the serving path (``EngineConfig.cp_threshold``):
DP engine replicas step in lockstep; a prompt at or over the threshold is
prefilled by the whole group (zig-zag shards, ring attention through the
paged-attention op with its LSE output), the owner keeps the K/V it saw go by
and decodes alone.  Outputs must equal a single-rank engine on the same prompts
(gloo, world 2 and 4, fp32 on CPU), and the paged ring must equal dense causal
attention."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from omnia_amd.parallel import context_parallel as cp

LONG = [(7 * i + 3) % 97 + 1 for i in range(53)]
LONG2 = [(11 * i + 5) % 89 + 1 for i in range(41)]
PROMPTS = {  # rank -> prompts (long ones go context-parallel; unequal load)
    0: [LONG, [8, 1, 6]],
    1: [[13, 2, 9, 9, 1, 4, 4, 4, 7, 2, 5, 12]],
    2: [],
    3: [LONG2, [6, 7, 8, 9, 10]],
}
MAX_TOKENS = {0: 6, 1: 5, 2: 0, 3: 4}
THRESHOLD = 32


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(**kw):
    from omnia_amd.engine.engine import EngineConfig

    return EngineConfig(model="tiny-llama", device="cpu", dtype="float32", num_blocks=96,
                        block_size=4, max_batch=8, max_model_len=256, use_graphs=False,
                        seed=3, **kw)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    try:
        from omnia_amd.engine.engine import LLMEngine
        from omnia_amd.engine.sampling_params import SamplingParams

        eng = LLMEngine(_cfg(cp_threshold=THRESHOLD))
        assert eng.cp_lockstep and eng.lockstep
        prompts, mt = PROMPTS[rank % 4], MAX_TOKENS[rank % 4]
        outs = []
        if prompts:
            seqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=mt,
                                                        ignore_eos=True))
            outs = [s.output for s in seqs]
        else:
            eng.run_until_done()
        q.put(("ok", rank, outs, eng.counters.get("cp_prefills", 0),
               eng.runner.stats.get("cp_prefills", 0)))
        import torch.distributed as dist

        dist.barrier()
    except Exception:  # pragma: no cover
        import traceback

        q.put(("err", rank, traceback.format_exc(), 0, 0))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cp_engine_matches_single_rank(world):
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
    for status, rank, val, _, _ in res:
        assert status == "ok", val
    n_long = sum(1 for r in range(world) for p in PROMPTS[r % 4] if len(p) >= THRESHOLD)
    oracle = LLMEngine(_cfg())
    for _, rank, outs, cp_steps, cp_runs in res:
        assert cp_runs == n_long  # every rank took part in every CP prefill
        prompts = PROMPTS[rank % 4]
        if not prompts:
            assert outs == []
            continue
        want = oracle.generate(prompts, SamplingParams(temperature=0.0,
                                                       max_tokens=MAX_TOKENS[rank % 4],
                                                       ignore_eos=True))
        assert outs == [s.output for s in want], (rank, outs)


def _pack_pages(k, v, bs):
    """[T, Hkv, D] x2 -> the engine's paged layout [2, T/bs, Hkv, bs, D]."""
    T, H, D = k.shape
    kv = torch.stack([k, v]).view(2, T // bs, bs, H, D).permute(0, 1, 3, 2, 4)
    return kv.contiguous()


def test_paged_ring_single_rank_matches_dense():
    torch.manual_seed(0)
    bs, W = 4, 1
    L = 2 * W * bs * 3
    Hq, Hkv, D = 4, 2, 8
    q = torch.randn(L, Hq, D)
    k = torch.randn(L, Hkv, D)
    v = torch.randn(L, Hkv, D)
    c = L // 2
    o = cp.ring_attention_paged(q, _pack_pages(k, v, bs), c, D ** -0.5)
    ref = cp.reference_attention(q, k, v)
    assert (o - ref).abs().max() < 1e-5


def test_lse_output_and_kv_cap_cpu():
    from omnia_amd import ops
    from omnia_amd.ops import reference as ref

    torch.manual_seed(2)
    bs, Hq, Hkv, D = 4, 4, 2, 8
    k = torch.randn(16, Hkv, D)
    v = torch.randn(16, Hkv, D)
    kv = _pack_pages(k, v, bs)
    q = torch.randn(8, Hq, D)
    bt = torch.tensor([[0, 1, 2, 3]], dtype=torch.int32)
    # "full" block: 8 queries after all 16 keys, keys capped at 16 of a 24 context
    qsl = torch.tensor([0, 8], dtype=torch.int32)
    lens = torch.tensor([24], dtype=torch.int32)
    lse = torch.empty(8, Hq)
    o = ops.prefill_attention(q, kv[0], kv[1], bt, qsl, lens, D ** -0.5, lse=lse,
                              kv_lens=torch.tensor([16], dtype=torch.int32))
    s = torch.einsum("qhd,khd->hqk", q, k.repeat_interleave(2, 1)) * D ** -0.5
    want = torch.einsum("hqk,khd->qhd", s.softmax(-1), v.repeat_interleave(2, 1))
    assert (o - want).abs().max() < 1e-5
    assert (lse - torch.logsumexp(s, -1).t()).abs().max() < 1e-5
    o2, l2 = ref.paged_attention_lse(q, kv[0], kv[1], bt, qsl, torch.tensor([8], dtype=torch.int32),
                                     D ** -0.5)
    assert torch.isfinite(l2).all() and o2.shape == q.shape


@pytest.mark.gpu
def test_paged_ring_kernel_lse_on_gpu():
    """The hand prefill kernel's LSE output and key cap (ring-step pairs) on the
    MI355X against fp32 dense attention, merged over a 2-rank ring simulated on
    one device (bf16 operands, fp32 statistics)."""
    from omnia_amd import ops

    torch.manual_seed(1)
    dev = "cuda"
    bs, W = 32, 2
    Hq, Hkv, D = 32, 8, 128
    L = 2 * W * bs * 6  # 768 tokens, c = 192
    c = L // (2 * W)
    q = torch.randn(L, Hq, D, device=dev).bfloat16()
    k = torch.randn(L, Hkv, D, device=dev).bfloat16()
    v = torch.randn(L, Hkv, D, device=dev).bfloat16()
    ref = cp.reference_attention(q.float(), k.float(), v.float())
    # lse of the kernel over one causal pass equals logsumexp of the dense scores
    kv_all = _pack_pages(k, v, bs)
    pages = L // bs
    lse = torch.empty(L, Hq, device=dev)
    o = ops.prefill_attention(q, kv_all[0], kv_all[1],
                              torch.arange(pages, dtype=torch.int32, device=dev)[None],
                              torch.tensor([0, L], dtype=torch.int32, device=dev),
                              torch.tensor([L], dtype=torch.int32, device=dev), D ** -0.5,
                              lse=lse)
    kk = k.float().repeat_interleave(Hq // Hkv, 1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kk) * D ** -0.5
    s = s.masked_fill(torch.ones(L, L, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    assert (lse - torch.logsumexp(s, -1).t()).abs().max().item() < 2e-2
    assert (o.float() - ref).abs().max().item() < 3e-2
    # every rank's ring, with the K/V blocks of the other rank fed in order
    shards = [cp.zigzag_indices(L, W, r).to(dev) for r in range(W)]
    blocks = [_pack_pages(k[idx], v[idx], bs) for idx in shards]
    for r in range(W):
        out = torch.zeros(2 * c, Hq, D, device=dev)
        acc_l = torch.full((2 * c, Hq), float("-inf"), device=dev)
        qr = q[shards[r]]
        for step in range(W):
            src = (r - step) % W
            L_ = cp._StepLaunch(cp._pairs(r, src), c, c // bs, q.device)
            lb = torch.empty(len(L_.pairs) * c, Hq, device=dev)
            ob = ops.prefill_attention(qr.index_select(0, L_.rows), blocks[src][0],
                                       blocks[src][1], L_.block_tables, L_.q_start_loc,
                                       L_.seq_lens, D ** -0.5, L_.tile_seq, L_.tile_q0,
                                       lse=lb, kv_lens=L_.kv_lens)
            for i, (qc, _, _) in enumerate(L_.pairs):
                sl = slice(qc * c, (qc + 1) * c)
                out[sl], acc_l[sl] = cp._merge(out[sl], acc_l[sl], ob[i * c:(i + 1) * c].float(),
                                               lb[i * c:(i + 1) * c])
        err = (out - ref[shards[r]]).abs().max().item()
        assert err < 3e-2, (r, err)


def _cp_oracle(device):
    """A long prompt prefilled through the CP path (ring of one rank: scratch
    pages, prefill kernel with LSE + key cap, owner page copy, last-hidden
    pick), then decoded normally from the copied KV; every logit row is checked
    against the fp32 dense forward of the same weights."""
    import random
    import socket as _s
    import time as _time

    import torch.distributed as dist

    from omnia_amd.engine.cp import run_cp_prefill
    from omnia_amd.engine.sampling_params import SamplingParams
    from omnia_amd.models.config import resolve
    import sys as _sys

    _sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_model_correctness import _check, _engine

    if not dist.is_initialized():
        with _s.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=1)
    try:
        mc = resolve("tiny-llama")
        torch.manual_seed(0)
        eng = _engine(device, mc, 256)
        eng.scheduler.cfg.cp_threshold = 64
        rng = random.Random(11)
        prompt = [rng.randrange(10, mc.vocab_size - 10) for _ in range(709)]
        s = eng.add_request(prompt, SamplingParams(temperature=0.0, max_tokens=6,
                                                   ignore_eos=True))
        assert eng.scheduler.cp_candidate() is s
        tok = run_cp_prefill(eng.runner, s, s.length, 0, dist.group.WORLD)
        for x, t in eng.scheduler.cp_done(s, tok):
            eng._append(x, t, _time.perf_counter())
        eng.run_until_done()
        assert len(s.output) == 6 and eng.runner.stats["cp_prefills"] == 1
        frac, worst = _check(mc, eng.model.w, [s], eng.runner.logit_tap, 0.03)
        assert frac == 1.0, worst
        return worst
    finally:
        dist.destroy_process_group()


def test_cp_prefill_matches_dense_oracle_cpu():
    _cp_oracle("cpu")


@pytest.mark.gpu
def test_cp_prefill_matches_dense_oracle_gpu():
    _cp_oracle("cuda")
