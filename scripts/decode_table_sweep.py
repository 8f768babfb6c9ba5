#!/usr/bin/env python3
"""Decode-projection table sweep for a model's shapes (BASELINE configs 4 / 5:
Llama-3-70B at TP=1, Mixtral's attention): for each projection and batch
bucket, time the library path (ops.linear / linear_silu), every tgemm
configuration (BN x splits x weight-load flags, fp16 slabs + the consumer
kernel) and the pgemm 256x256 split-K tile (+ consumer), and write the winners
as ``ops/tuned/wgemm_mi355x.json`` entries (``mode:M:N:K -> [nw, nwaves, S]``;
tgemm = ``[bn, -1 - flags, S]``, pgemm split-K = ``[256, -64, S]``).  An entry
is written only when it beats the library path by >= 5 %.  Weights rotate over
>= 1.5 GiB so every call streams them from HBM.

    python scripts/decode_table_sweep.py --model llama-3-70b --m 128,256 --out x.json
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from omnia_amd import ops  # noqa: E402
from omnia_amd.models.config import resolve  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

dev = "cuda"


def timeit(fn, reps=25):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--m", default="128,256")
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="decode_table_sweep.json")
    a = ap.parse_args()
    cfg = resolve(a.model)
    d, I, hq, hkv = cfg.hidden_size, cfg.intermediate_size, cfg.num_heads, cfg.num_kv_heads
    shapes = {"qkv": ((hq + 2 * hkv) * 128, d, 0), "o": (d, hq * 128, 0),
              "gate_up": (I, d, 1), "down": (d, I, 0)}
    if a.only:
        shapes = {k: v for k, v in shapes.items() if k in a.only.split(",")}
    cs = ref.rope_cos_sin(8192, 128, 500000.0, device=dev)
    kc = torch.zeros(64, hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    nw_ = torch.ones(d, device=dev, dtype=torch.bfloat16)
    results, table = {}, {}
    for name, (N, K, mode) in shapes.items():
        rows = 2 * N if mode == 1 else N
        ncopy = max(2, int(1.5 * 2**30 // (rows * K * 2)) + 1)
        ws = [(torch.randn(rows, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]

        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            pos = torch.arange(M, device=dev, dtype=torch.int32) + 600
            slots = torch.arange(M, device=dev, dtype=torch.int64)
            res = torch.randn(M, d, device=dev).to(torch.bfloat16)

            def consume(p):
                if name == "gate_up":
                    ops.splitk_swiglu(p)
                elif name == "qkv":
                    ops.splitk_rope_kv(p, pos, cs, kc, vc, slots, hq, hkv, 32)
                else:
                    ops.splitk_add_rmsnorm(p, res, nw_, 1e-5)

            out = {}
            lib = (lambda: ops.linear_silu(x, nxt())) if mode == 1 else \
                (lambda: ops.linear(x, nxt()))
            out["lib"] = timeit(lib)
            for bn in (64, 128, 256):
                for S in (1, 2, 3, 4, 5, 6, 8, 12, 16):
                    for fl in (0, 1):
                        try:
                            if mode == 1 and S == 1:
                                fn = lambda bn=bn, fl=fl: ops.tgemm(1, x, nxt(), 1, bn, fl)  # noqa
                            else:
                                parts = torch.empty(S, M, rows, device=dev, dtype=torch.float16)

                                def fn(bn=bn, S=S, fl=fl, parts=parts):
                                    consume(ops.tgemm(3, x, nxt(), S, bn, fl, parts))
                            out[f"t:{bn}:{S}:{fl}"] = timeit(fn)
                        except RuntimeError:
                            continue
            for S in (1, 2, 4, 8, 16):
                if K % S or (K // S) % 128 or rows % 256:
                    continue
                parts = torch.empty(S, M, rows, device=dev, dtype=torch.float16)
                out[f"p:{S}"] = timeit(lambda S=S, parts=parts: consume(
                    ops.pgemm_splitk(x, nxt(), S, parts)))
            best_k, best_t = min(((k, v) for k, v in out.items() if k != "lib"),
                                 key=lambda kv: kv[1])
            results[f"{name}:{M}"] = out
            key = f"{mode}:{M}:{N}:{K}"
            if best_t < 0.95 * out["lib"]:
                f = best_k.split(":")
                table[key] = ([int(f[1]), -1 - int(f[3]), int(f[2])] if f[0] == "t"
                              else [256, -64, int(f[1])])
            print(f"{a.model} {name} M{M}: lib {out['lib']:.1f}us best {best_k} "
                  f"{best_t:.1f}us -> {table.get(key, 'lib')}", flush=True)
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump({"results": results, "table": table}, f, indent=1)


if __name__ == "__main__":
    main()
