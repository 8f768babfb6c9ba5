"""Decode-GEMM sweep on one MI355X: tuned hipBLASLt (+ silu_mul), the LDS-staged
hand kernel (gemm.hip) and the weight-streaming kernel (wgemm.hip, every
(NW, waves, S) variant) for the Llama-3-8B / 70B projection shapes.

Weights rotate over copies totalling >= 1 GiB so the 256 MiB MALL cannot serve
them; x is re-used (it is L2-resident in the real step too).  Mode-2 (split-K
partial) variants are charged for writing their fp32 slabs but not for the
consumer's reduction (that kernel exists anyway: RoPE / add+RMSNorm).
Prints one line per (shape, M) and writes JSON to --out."""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402

SHAPES = {  # name: (N, K, mode)
    "qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (14336, 4096, 1),
    "down": (4096, 14336, 0), "lm_head": (128256, 4096, 0),
    # Llama-3-70B per-GPU shards at TP=8
    "70b_qkv_tp8": (1280, 8192, 0), "70b_o_tp8": (8192, 1024, 0),
    "70b_gu_tp8": (3584, 8192, 1), "70b_down_tp8": (8192, 3584, 0),
}


def bench(fn, iters=30):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="256,128,64,16")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--out", default="gpurun_out/wgemm_sweep.json")
    a = ap.parse_args()
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    print("tuned hipBLASLt table:", enable_tuned_gemms(0))
    res = {}
    for name in a.shapes.split(","):
        N, K, mode = SHAPES[name]
        rows = 2 * N if mode == 1 else N
        nbytes = rows * K * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.randn(rows, K, device="cuda").mul_(0.02).to(torch.bfloat16)
              for _ in range(copies)]
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)

            def lib(i):
                y = F.linear(x, ws[i % copies])
                return ops.silu_mul(y) if mode == 1 else y

            t_lib = bench(lib)
            best = None
            cands = []
            for nw in (1, 2, 4):
                if mode == 1 and nw == 1:
                    continue
                if nw == 4 and M > 128:
                    continue
                for nwaves in (4, 2):
                    per_block = 16 * nw * nwaves
                    if rows % per_block:
                        continue
                    for S in (1, 2, 4, 8, 16):
                        if K % (128 * S):
                            continue
                        # mode 1 with S > 1: split-K slabs of all 2I rows, SwiGLU in the consumer
                        md = 2 if S > 1 else mode
                        ncol = rows if md == 2 else N
                        outb = (torch.empty(S, M, ncol, device="cuda") if md == 2
                                else torch.empty(M, N, device="cuda", dtype=torch.bfloat16))

                        def f(i, md=md, S=S, nw=nw, nwaves=nwaves, outb=outb):
                            ops.wgemm(md, x, ws[i % copies], S, nw, nwaves, out=outb)

                        try:
                            t = bench(f)
                        except RuntimeError as e:
                            print("skip", name, M, nw, nwaves, S, e, file=sys.stderr)
                            continue
                        cands.append((round(t, 2), nw, nwaves, S))
            cands.sort()
            best = cands[0] if cands else None
            gbs = lambda t: nbytes / t / 1e3  # noqa: E731
            print(f"{name:8s} M={M:3d} lib {t_lib:7.1f} us ({gbs(t_lib):5.0f} GB/s)  "
                  f"wgemm {best[0]:7.1f} us ({gbs(best[0]):5.0f} GB/s) nw={best[1]} "
                  f"waves={best[2]} S={best[3]}  x{t_lib / best[0]:.2f}  top3={cands[:3]}",
                  flush=True)
            s1 = [c for c in cands if c[3] == 1]
            if s1:
                print(f"{'':8s}       best S=1 (no slab reduce): {s1[0]}", flush=True)
            res[f"{name}:{M}"] = {"lib_us": t_lib, "best": best, "top": cands[:12],
                                  "best_s1": s1[0] if s1 else None, "weight_bytes": nbytes,
                                  "N": N, "K": K, "mode": mode, "M": M,
                                  "slab_bytes_per_split": M * rows * 4}
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
