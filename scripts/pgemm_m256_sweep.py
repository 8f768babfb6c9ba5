#!/usr/bin/env python3
"""Decode projections at M <= 256 on the 256x256 MFMA tile with split-K
(pgemm.hip EPI 4, fp16 slabs) against the tuned table's current choice.

Every candidate is timed WITH the consumer kernel that reduces its slabs
(splitk_rope_kv / splitk_add_rmsnorm / splitk_swiglu), the same pair the
decode step runs.  Weights rotate over >= 1.5 GiB so every call streams them
from HBM (Llama-3-8B shapes; ``--shapes 70b`` for the Llama-3-70B TP=1 ones).
Each candidate's slab sum is also checked against an fp32 matmul once.

    python scripts/pgemm_m256_sweep.py out.json [--m 128,192,256] [--shapes 8b]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

dev = "cuda"
SHAPES = {
    "8b": dict(d=4096, I=14336, hq=32, hkv=8),
    "70b": dict(d=8192, I=28672, hq=64, hkv=8),
}


def timeit(fn, reps=30):
    for _ in range(4):
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
    ap.add_argument("out", nargs="?", default="pgemm_m256_sweep.json")
    ap.add_argument("--m", default="256,192,128")
    ap.add_argument("--shapes", default="8b")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    sh = SHAPES[a.shapes]
    d, I, hq, hkv = sh["d"], sh["I"], sh["hq"], sh["hkv"]
    shapes = {"gate_up": (2 * I, d), "down": (d, I), "qkv": ((hq + 2 * hkv) * 128, d),
              "o": (d, hq * 128)}
    if a.only:
        shapes = {k: v for k, v in shapes.items() if k in a.only.split(",")}
    cs = ref.rope_cos_sin(8192, 128, 500000.0, device=dev)
    kc = torch.zeros(64, hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    nw = torch.ones(d, device=dev, dtype=torch.bfloat16)
    res_all = {}
    for M in [int(m) for m in a.m.split(",")]:
        pos = torch.arange(M, device=dev, dtype=torch.int32) + 600
        slots = torch.arange(M, device=dev, dtype=torch.int64)
        res = torch.randn(M, d, device=dev).to(torch.bfloat16)
        for name, (N, K) in shapes.items():
            ncopy = max(2, int(1.5 * 2**30 // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws[it[0]]

            def consume(p):
                if name == "gate_up":
                    ops.splitk_swiglu(p)
                elif name == "qkv":
                    ops.splitk_rope_kv(p, pos, cs, kc, vc, slots, hq, hkv, 32)
                else:
                    ops.splitk_add_rmsnorm(p, res, nw, 1e-5)

            exact = x.float() @ ws[0].float().t()
            scale = exact.abs().max().item()
            out = {}
            # the tuned table's current choice (tgemm / wgemm + consumer)
            mode = 1 if name == "gate_up" else 0
            cfg = ops.wgemm_config(M, N // 2 if mode else N, K, mode)
            if cfg is not None:
                bn, nwv, S = cfg
                if mode == 1 and S == 1:
                    fn = lambda: ops.wgemm(1, x, nxt(), 1, bn, nwv)  # noqa: E731
                else:
                    dt = torch.float16 if nwv < 0 else torch.float32
                    parts = torch.empty(S, M, N, device=dev, dtype=dt)

                    def fn(bn=bn, nwv=nwv, S=S, parts=parts):
                        m = 3 if dt == torch.float16 else 2
                        if nwv < 0:
                            p = ops.tgemm(m, x, nxt(), S, bn, -1 - nwv, parts)
                        else:
                            p = ops.wgemm(2, x, nxt(), S, bn, nwv, out=parts)
                        consume(p)
                out[f"table:{cfg}"] = timeit(fn)
            for sched in (0, 1):
                for S in (1, 2, 3, 4, 6, 7, 8, 12, 14, 16):
                    if K % S or (K // S) % 128:
                        continue
                    nblk = (N // 256) * S
                    if nblk > 2048:
                        continue
                    parts = torch.empty(S, M, N, device=dev, dtype=torch.float16)
                    ops.pgemm_splitk(x, ws[0], S, parts, sched)
                    torch.cuda.synchronize()
                    err = (parts.float().sum(0) - exact).abs().max().item() / scale
                    if err > 2e-2:
                        print(f"  BAD {name} M{M} S{S} sched{sched} rel err {err:.3g}", flush=True)
                        out[f"pgemm:s{sched}:S{S}:BAD"] = err
                        continue

                    def fn(S=S, sched=sched, parts=parts):
                        consume(ops.pgemm_splitk(x, nxt(), S, parts, sched))
                    out[f"pgemm:s{sched}:S{S}"] = timeit(fn)
                    out[f"pgemm:s{sched}:S{S}:noconsumer"] = timeit(
                        lambda S=S, sched=sched, parts=parts: ops.pgemm_splitk(x, nxt(), S, parts,
                                                                               sched))
            if name == "gate_up" and M > 0:  # the fused-SwiGLU prefill tile, unsplit
                act = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
                out["pgemm:epi1"] = timeit(lambda: ops.pgemm(1, x, nxt(), out=act))
            best = sorted((v, k) for k, v in out.items()
                          if not k.endswith("noconsumer") and not k.endswith("BAD"))[:5]
            tab = next((v for k, v in out.items() if k.startswith("table")), None)
            print(f"M{M} {name} table {tab if tab is None else round(tab, 1)}us | "
                  + " | ".join(f"{k} {v:.1f}" for v, k in best), flush=True)
            res_all[f"{M}:{name}"] = out
            del ws
            torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res_all, f, indent=1)


if __name__ == "__main__":
    main()
