#!/usr/bin/env python3
"""Mid-size projections (M = 257..4095 rows: the open loop's mixed steps) --
the library path the engine takes there against the 256x256 prefill tile.

Per Llama-3-8B projection, each candidate is timed WITH its epilogue, the way
a mixed step runs it:

* ``lib``: hipBLASLt (``ops.linear``) + the separate epilogue kernel:
  ``rope_kv`` (qkv), ``silu_mul`` (gate_up), ``fused_add_rmsnorm`` (o, down);
* ``epi``: pgemm with the epilogue fused (EPI 3 / 1 / 2), unsplit;
* ``S<n>``: pgemm split-K (EPI 4, fp16 slabs) + the slab consumer
  (``splitk_rope_kv`` / ``splitk_swiglu`` / ``splitk_add_rmsnorm``).

Weights rotate over >= 1.5 GiB so every call streams them from HBM.

    python scripts/midm_sweep.py [--m 512,1024,2048] [--out x.json] [--shapes 70b]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

dev = "cuda"


def timeit(fn, reps=20):
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
    ap.add_argument("--m", default="512,768,1024,1536,2048,3072")
    ap.add_argument("--out", default="midm_sweep.json")
    ap.add_argument("--shapes", default="8b", choices=["8b", "70b"])
    a = ap.parse_args()
    d, I, hq, hkv = (4096, 14336, 32, 8) if a.shapes == "8b" else (8192, 28672, 64, 8)
    shapes = {"qkv": ((hq + 2 * hkv) * 128, d), "o": (d, hq * 128), "gate_up": (2 * I, d),
              "down": (d, I)}
    cs = ref.rope_cos_sin(8192, 128, 500000.0, device=dev)
    results = {}
    for M in [int(m) for m in a.m.split(",")]:
        pos = torch.arange(M, device=dev, dtype=torch.int32) + 600
        nblk = (M + 31) // 32 + 8
        kc = torch.zeros(nblk, hkv, 32, 128, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        slots = torch.arange(M, device=dev, dtype=torch.int64)
        nw = torch.ones(d, device=dev, dtype=torch.bfloat16)
        res = torch.randn(M, d, device=dev).to(torch.bfloat16)
        ss = torch.empty(M, d // 256, device=dev, dtype=torch.float32)
        for name, (N, K) in shapes.items():
            ncopy = max(2, int(1.5 * 2**30 // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws[it[0]]

            out = {}
            if name == "qkv":
                def lib():
                    y = ops.linear(x, nxt())
                    ops.rope_kv(y[:, :hq * 128], y[:, hq * 128:(hq + hkv) * 128],
                                y[:, (hq + hkv) * 128:], pos, cs, kc, vc, slots, hq, hkv, 32)
                q = torch.empty(M, hq * 128, device=dev, dtype=torch.bfloat16)

                def epi():
                    ops.pgemm(3, x, nxt(), out=q, positions=pos, cos_sin=cs, k_cache=kc,
                              v_cache=vc, slots=slots, hq=hq, hkv=hkv, block_size=32)

                def consume(p):
                    ops.splitk_rope_kv(p, pos, cs, kc, vc, slots, hq, hkv, 32)
            elif name == "gate_up":
                def lib():
                    ops.linear_silu(x, nxt())
                act = torch.empty(M, I, device=dev, dtype=torch.bfloat16)

                def epi():
                    ops.pgemm(1, x, nxt(), out=act)

                def consume(p):
                    ops.splitk_swiglu(p)
            else:
                def lib():
                    y = ops.linear(x, nxt())
                    ops.fused_add_rmsnorm(y, res, nw, 1e-5)

                def epi():
                    ops.pgemm(2, x, nxt(), out=res, ss_out=ss)

                def consume(p):
                    ops.splitk_add_rmsnorm(p, res, nw, 1e-5)
            out["lib"] = timeit(lib)
            out["epi"] = timeit(epi)
            for S in (2, 3, 4, 6, 8):
                if K % S or (K // S) % 128:
                    continue
                parts = torch.empty(S, M, N, device=dev, dtype=torch.float16)
                out[f"S{S}"] = timeit(lambda S=S, parts=parts: consume(
                    ops.pgemm_splitk(x, nxt(), S, parts)))
            best = min(out, key=out.get)
            flops = 2 * M * N * K
            print(f"M{M:5d} {name:7s} lib {out['lib']:7.1f}us ({flops / out['lib'] / 1e6:5.0f} TF) "
                  f"| epi {out['epi']:7.1f} | "
                  + " ".join(f"{k} {v:.1f}" for k, v in out.items() if k.startswith("S"))
                  + f" -> {best} ({out['lib'] / out[best]:.2f}x)", flush=True)
            results[f"{M}:{name}"] = out
            del ws
            torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
