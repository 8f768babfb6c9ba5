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

``--path runtime`` (default) drives every turn through the omnia.runtime.v1
Converse handler (agent loop + PromptPack rendering + chunk framing) with the
engine in its own engine-core process (``omnia_amd.engine.core_proc``, the
production layout); ``--inproc`` runs it as a thread of the serving process and
``--path engine`` calls the engine directly.
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
    ap.add_argument("--inproc", action="store_true",
                    help="runtime path: run the engine as a thread of the serving process "
                         "instead of its own engine-core process")
    ap.add_argument("--device", default="cuda")
    return ap.parse_args()


def main():
    a = parse()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # device_count() does not initialise the GPU: the engine-core child must be
    # started before this process touches it
    use_gpu = a.device == "cuda" and torch.cuda.device_count() > 0
    proc = a.path == "runtime" and not a.inproc

    from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine
    from omnia_amd.engine.sampling_params import SamplingParams

    C = a.concurrency
    cfg = EngineConfig(model=a.model, device="cuda" if use_gpu else "cpu",
                       max_batch=max(C, 1), max_model_len=max(2048, a.prompt_len + a.gen_len + 64),
                       max_prefill_tokens=a.max_prefill_tokens, use_graphs=not a.no_graphs,
                       seed=rank)
    eng = client = None
    if proc:
        from omnia_amd.engine.core_proc import EngineCoreClient

        client = EngineCoreClient(cfg, device_index=local if use_gpu else None)
        if ws > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")  # host-side result aggregation only
        model_cfg = client.engine.model_cfg
    else:
        if use_gpu:
            torch.cuda.set_device(local)
        if ws > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl" if use_gpu else "gloo")
        eng = LLMEngine(cfg)
        model_cfg = eng.model_cfg
    vocab = model_cfg.vocab_size
    params = SamplingParams(temperature=a.temperature, max_tokens=a.gen_len, ignore_eos=True,
                            top_p=1.0)
    g = torch.Generator().manual_seed(1234 + rank)

    runtime = None
    if a.path == "runtime":
        from omnia_amd.runtime.bench_driver import RuntimeBenchDriver

        runtime = RuntimeBenchDriver(client if proc else AsyncLLMEngine(eng), params)

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
        if proc:
            client.synchronize()  # torch.cuda.synchronize() in the GPU-owning process
        elif use_gpu:
            torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()

    def engine_stats() -> dict:
        if proc:
            return client.stats()
        return {"timing": dict(eng.timing), "counters": dict(eng.counters),
                "runner": dict(eng.runner.stats), "kv_blocks": eng.blocks.num_blocks,
                "block_size": cfg.block_size}

    def reset_timing():
        if proc:
            client.call("reset_timing")
        else:
            for k in eng.timing:
                eng.timing[k] = 0.0
            eng.runner.stats["gil_wait_s"] = 0.0

    gc_pauses = None
    if os.environ.get("OMNIA_STEP_TRACE"):
        import gc

        gc_pauses = {0: [0, 0.0], 1: [0, 0.0], 2: [0, 0.0]}
        _gc_t = {}

        def _gc_cb(phase, info):
            if phase == "start":
                _gc_t["t"] = time.perf_counter()
            else:
                e = gc_pauses[info["generation"]]
                e[0] += 1
                e[1] += time.perf_counter() - _gc_t.get("t", time.perf_counter())

        gc.callbacks.append(_gc_cb)
    for w in range(a.warmup):
        one_wave(-1 - w)
    sync()
    reset_timing()
    t0 = time.perf_counter()
    results = []
    for k in range(a.steps):
        results.extend(one_wave(k))
    sync()
    elapsed = time.perf_counter() - t0
    if gc_pauses is not None:
        print("[gc]", {g: (n, round(t * 1e3, 1)) for g, (n, t) in gc_pauses.items()},
              file=sys.stderr)
    if eng is not None and eng.step_trace is not None and rank == 0:
        import json as _json

        gt = eng.gpu_trace
        gpu = [(a.elapsed_time(b), (gt[i - 1][1].elapsed_time(a) if i else 0.0))
               for i, (a, b) in enumerate(gt)]
        with open(os.environ["OMNIA_STEP_TRACE"], "w") as f:
            _json.dump({"host": eng.step_trace, "gpu_ms_and_gap": gpu}, f)

    out_tokens = sum(r[2] for r in results)
    ttfts = [r[0] for r in results if r[0] is not None]
    lats = [r[1] for r in results if r[1] is not None]
    stats = torch.tensor([elapsed, float(out_tokens)], dtype=torch.float64)
    if ws > 1:
        t = stats.clone().cuda() if (use_gpu and not proc) else stats.clone()
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
    st = engine_stats()
    if runtime is not None:
        runtime.close()
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
                "engine_process": proc,
                "tp": 1,
                "hip_graphs": not a.no_graphs,
            },
            "engine": {
                "kv_blocks": st["kv_blocks"],
                "block_size": st["block_size"],
                "prefill_steps": st["counters"]["steps_prefill"],
                "decode_steps": st["counters"]["steps_decode"],
                "graph_captures": st["runner"]["captures"],
                "host_timing_s": {**{k: round(v, 3) for k, v in st["timing"].items()},
                                  "gil_wait_s": round(st["runner"]["gil_wait_s"], 3)},
            },
        }
        print(json.dumps(rec), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
