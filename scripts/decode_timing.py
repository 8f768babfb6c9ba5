"""Break down host vs device time of one bench wave (engine path)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams

C = int(os.environ.get("C", "256"))
eng = LLMEngine(EngineConfig(model=os.environ.get("MODEL", "llama-3-8b"), max_batch=C, max_model_len=2048))
params = SamplingParams(temperature=0, max_tokens=128, ignore_eos=True)
g = torch.Generator().manual_seed(0)
for wave in range(2):
    prompts = torch.randint(1000, 100000, (C, 512), generator=g).tolist()
    seqs = [eng.add_request(p, params) for p in prompts]
    T = {"sched": 0, "inputs": 0, "replay": 0, "sync": 0, "post": 0, "prefill": 0}
    nd = 0
    t_wave = time.perf_counter()
    r = eng.runner
    while eng.has_work():
        t0 = time.perf_counter()
        plan = eng.scheduler.schedule()
        t1 = time.perf_counter(); T["sched"] += t1 - t0
        if plan.kind == "prefill":
            sampled = r.run_prefill(plan.prefill)
            done = eng.scheduler.on_prefill_done(plan.prefill, sampled)
            torch.cuda.synchronize()
            T["prefill"] += time.perf_counter() - t1
        else:
            seqs_d = plan.decode
            import bisect
            n = len(seqs_d)
            ncols = r._ctx_bucket(max(s.length for s in seqs_d))
            nrows = r.buckets[bisect.bisect_left(r.buckets, n)]
            r._decode_inputs(seqs_d, nrows, ncols)
            t2 = time.perf_counter(); T["inputs"] += t2 - t1
            gr = r.graphs.get((nrows, ncols)) or r._capture(nrows, ncols)
            gr.replay()
            t3 = time.perf_counter(); T["replay"] += t3 - t2
            r.out_host[:n].copy_(r.out_tok[:n], non_blocking=True)
            torch.cuda.current_stream().synchronize()
            toks = r.out_host[:n].tolist()
            t4 = time.perf_counter(); T["sync"] += t4 - t3
            done = eng.scheduler.on_decode_done(seqs_d, toks)
            nd += 1
        t5 = time.perf_counter()
        now = time.perf_counter()
        for s, tok in done:
            eng._append(s, tok, now)
        T["post"] += time.perf_counter() - t5
    wall = time.perf_counter() - t_wave
    print(f"wave {wave}: wall {wall*1000:.0f}ms decode_steps {nd} " + " ".join(f"{k}={v*1000:.0f}ms" for k, v in T.items()), flush=True)
