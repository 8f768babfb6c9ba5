#!/usr/bin/env python3
"""Headline benchmark: streamed tokens/sec + p50 turn latency of an AgentRuntime
serving Llama-3-8B (BASELINE.json metric) on 1/2/4/8 MI355X GPUs.

One process per GPU (torchrun), each rank an independent engine replica
(DP = N, weak scaling: per-GPU concurrency is fixed as N grows).  A "step" is
one wave of C concurrent agent turns per GPU: each turn submits a fresh
synthetic ``--prompt-len``-token message (no KV prefix reuse across waves) and
streams ``--gen-len`` tokens with ignore_eos, exactly the reference's arena
load-test definitions (``ee/pkg/arena/fleet/client.go:124-157``): TTFT = first
streamed token, turn latency = done.  Weights are random-init bf16 of the exact
Llama-3-8B architecture (no checkpoints offline); data is synthetic.

``--path runtime`` drives every turn through the omnia.runtime.v1 Converse
handler (agent loop + PromptPack rendering + chunk framing) in-process instead
of calling the engine directly.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "streamed tokens/sec + p50 turn latency, AgentRuntime Llama-3-8B at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=256, help="concurrent turns per GPU")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--path", choices=["engine", "runtime"], default="runtime",
                    help="runtime = full AgentRuntime turn path (default); engine = engine only")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--device", default="cuda")
    return ap.parse_args()


def main():
    a = parse()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = a.device == "cuda" and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local)
    if ws > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if use_gpu else "gloo")

    from omnia_amd.engine.engine import EngineConfig, LLMEngine
    from omnia_amd.engine.sampling_params import SamplingParams

    C = a.concurrency
    cfg = EngineConfig(model=a.model, device="cuda" if use_gpu else "cpu",
                       max_batch=max(C, 1), max_model_len=max(2048, a.prompt_len + a.gen_len + 64),
                       max_prefill_tokens=a.max_prefill_tokens, use_graphs=not a.no_graphs,
                       seed=rank)
    eng = LLMEngine(cfg)
    vocab = eng.model_cfg.vocab_size
    params = SamplingParams(temperature=a.temperature, max_tokens=a.gen_len, ignore_eos=True,
                            top_p=1.0)
    g = torch.Generator().manual_seed(1234 + rank)

    runtime = None
    if a.path == "runtime":
        from omnia_amd.runtime.bench_driver import RuntimeBenchDriver

        runtime = RuntimeBenchDriver(eng, params)

    def one_wave(step: int):
        lo = min(1000, vocab // 4)
        prompts = torch.randint(lo, vocab - lo, (C, a.prompt_len), generator=g).tolist()
        if runtime is not None:
            return runtime.run_wave(prompts, step)
        seqs = [eng.add_request(p, params, session_id=f"r{rank}-s{step}-{i}")
                for i, p in enumerate(prompts)]
        eng.run_until_done()
        for s in seqs:
            eng.drop_session(s.session_id)  # fresh prompts next wave: no prefix reuse
        return [(s.ttft(), s.latency(), len(s.output)) for s in seqs]

    def sync():
        if use_gpu:
            torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()

    for w in range(a.warmup):
        one_wave(-1 - w)
    sync()
    t0 = time.perf_counter()
    results = []
    for k in range(a.steps):
        results.extend(one_wave(k))
    sync()
    elapsed = time.perf_counter() - t0

    out_tokens = sum(r[2] for r in results)
    ttfts = [r[0] for r in results if r[0] is not None]
    lats = [r[1] for r in results if r[1] is not None]
    stats = torch.tensor([elapsed, float(out_tokens)], dtype=torch.float64)
    if ws > 1:
        t = stats.clone().cuda() if use_gpu else stats.clone()
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        out_tokens = float(sm[1])
        gathered = [None] * ws
        dist.all_gather_object(gathered, (ttfts, lats))
        ttfts = [x for gg in gathered for x in gg[0]]
        lats = [x for gg in gathered for x in gg[1]]
    value = out_tokens / elapsed
    if rank == 0:
        rec = {
            "metric": BASELINE_METRIC,
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random prompt token ids, random-init weights of the named "
                    "architecture, ignore_eos)",
            "p50_turn_latency_ms": round(1000 * statistics.median(lats), 2) if lats else None,
            "p95_turn_latency_ms": round(1000 * sorted(lats)[int(0.95 * (len(lats) - 1))], 2)
            if lats else None,
            "p50_ttft_ms": round(1000 * statistics.median(ttfts), 2) if ttfts else None,
            "config": {
                "model": a.model,
                "global_batch": C * ws,
                "seq_len": a.prompt_len + a.gen_len,
                "prompt_len": a.prompt_len,
                "gen_len": a.gen_len,
                "concurrency_per_gpu": C,
                "parallelism": f"dp{ws}",
                "path": a.path,
                "tp": 1,
                "hip_graphs": not a.no_graphs,
            },
            "engine": {
                "kv_blocks": eng.blocks.num_blocks,
                "block_size": cfg.block_size,
                "prefill_steps": eng.counters["steps_prefill"],
                "decode_steps": eng.counters["steps_decode"],
                "graph_captures": eng.runner.stats["captures"],
            },
        }
        print(json.dumps(rec), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
