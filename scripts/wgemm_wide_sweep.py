"""Wide-batch decode GEMM sweep (M in 160..256) on one MI355X: tuned hipBLASLt
(+ silu_mul) vs wgemm_wide.hip for every (wt, S) variant, Llama-3-8B and
Llama-3-70B (TP=1 and TP=8 shard) projection shapes.  Weights rotate over copies
totalling >= 1 GiB (the 256 MiB MALL cannot serve them); split-K variants are
charged for writing their fp32 slabs AND for one extra read of them (the
consumer kernel's reduction), so the comparison is end to end.  One line per
(shape, M); JSON to --out."""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402

SHAPES = {  # name: (N, K, mode)
    "qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (14336, 4096, 1),
    "down": (4096, 14336, 0),
    "70b_qkv": (10240, 8192, 0), "70b_o": (8192, 8192, 0), "70b_gu": (28672, 8192, 1),
    "70b_down": (8192, 28672, 0),
    "70b_qkv_tp8": (1280, 8192, 0), "70b_o_tp8": (8192, 1024, 0),
    "70b_gu_tp8": (3584, 8192, 1), "70b_down_tp8": (8192, 3584, 0),
}
HBM_READ_GBS = 5500.0  # slab re-read charge for the consumer reduction


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
    ap.add_argument("--m", default="256,192")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--out", default="gpurun_out/wgemm_wide_sweep.json")
    a = ap.parse_args()
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    print("tuned hipBLASLt table:", enable_tuned_gemms(0), flush=True)
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
            want = lib(0).float()
            cands = []
            for wt in (2, 1):
                if mode == 1 and wt != 2:
                    continue
                if rows % (128 * wt):
                    continue
                for S in (1, 2, 3, 4, 6, 7, 8, 12, 14, 16):
                    if K % (256 * S):
                        continue
                    if mode == 1 and S > 1:
                        continue  # SwiGLU needs the whole K in-kernel
                    md = 2 if S > 1 else mode
                    outb = (torch.empty(S, M, N, device="cuda") if md == 2
                            else torch.empty(M, N, device="cuda", dtype=torch.bfloat16))

                    def f(i, md=md, S=S, wt=wt, outb=outb):
                        ops.wgemm_wide(md, x, ws[i % copies], S, wt, out=outb)

                    try:
                        t = bench(f)
                    except RuntimeError as e:
                        print("skip", name, M, wt, S, e, file=sys.stderr)
                        continue
                    f(0)
                    got = outb.sum(0) if md == 2 else outb.float()
                    err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
                    charge = (S * M * N * 4 / HBM_READ_GBS / 1e3) if md == 2 else 0.0
                    cands.append((round(t + charge, 2), wt, S, round(t, 2), round(err, 4)))
            cands.sort()
            best = cands[0]
            gbs = lambda t: nbytes / t / 1e3  # noqa: E731
            print(f"{name:12s} M={M:3d} lib {t_lib:7.1f} us ({gbs(t_lib):5.0f} GB/s)  "
                  f"wide {best[0]:7.1f} us ({gbs(best[0]):5.0f} GB/s) wt={best[1]} S={best[2]}"
                  f" raw={best[3]} err={best[4]}  x{t_lib / best[0]:.2f}  top3={cands[:3]}",
                  flush=True)
            res[f"{name}:{M}"] = {"lib_us": t_lib, "best": best, "top": cands[:12],
                                  "weight_bytes": nbytes, "N": N, "K": K, "mode": mode, "M": M}
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
