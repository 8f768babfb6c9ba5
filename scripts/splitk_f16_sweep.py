#!/usr/bin/env python3
"""Decode projections at M = 256 with fp16 split-K slabs: tile GEMM (tgemm
mode 1 / 3) + the consumer kernel that reduces the slabs, per (BN, splits, flags),
against the tuned table's current choice.  Weights rotate over >= 1.5 GiB so
every call streams them from HBM (Llama-3-8B shapes)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

M, d, I, hq, hkv = 256, 4096, 14336, 32, 8
dev = "cuda"


def timeit(fn, reps=40):
    for _ in range(5):
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
    x = torch.randn(M, d, device=dev).to(torch.bfloat16)
    xa = torch.randn(M, I, device=dev).to(torch.bfloat16)
    res = torch.randn(M, d, device=dev).to(torch.bfloat16)
    nw = torch.ones(d, device=dev, dtype=torch.bfloat16)
    pos = torch.arange(M, device=dev, dtype=torch.int32) + 600
    cs = ref.rope_cos_sin(4096, 128, 500000.0, device=dev)
    kc = torch.zeros(64, hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.arange(M, device=dev, dtype=torch.int64)
    shapes = {"gate_up": (2 * I, d), "down": (d, I), "qkv": ((hq + 2 * hkv) * 128, d),
              "o": (d, d)}
    out = {}
    for name, (N, K) in shapes.items():
        ncopy = max(2, int(1.5 * 2**30 // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]

        inp = xa if name == "down" else x
        cands = []
        for bn in (64, 128, 256):
            for S in (1, 2, 3, 4, 5, 6, 8, 12, 16):
                for fl in (0, 1, 4):
                    cands.append((bn, S, fl))
        for bn, S, fl in cands:
            if name == "gate_up" and S == 1:
                fn = lambda: ops.tgemm(1, inp, nxt(), 1, bn, fl)  # noqa: E731
            else:
                NN = N
                parts = torch.empty(S, M, NN, device=dev, dtype=torch.float16)

                def fn(bn=bn, S=S, fl=fl, parts=parts):
                    p = ops.tgemm(3, inp, nxt(), S, bn, fl, parts)
                    if name == "gate_up":
                        ops.splitk_swiglu(p)
                    elif name == "qkv":
                        ops.splitk_rope_kv(p, pos, cs, kc, vc, slots, hq, hkv, 32)
                    else:
                        ops.splitk_add_rmsnorm(p, res, nw, 1e-5)
            try:
                t = timeit(fn)
            except Exception as e:  # noqa: BLE001 - rejected shapes
                continue
            out[f"{name}:{bn}:{S}:{fl}"] = t
        best = sorted((v, k) for k, v in out.items() if k.startswith(name + ":"))[:6]
        print(name, " | ".join(f"{k} {v:.1f}us" for v, k in best), flush=True)
        del ws
        torch.cuda.empty_cache()
    with open(sys.argv[1] if len(sys.argv) > 1 else "splitk_f16_sweep.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
