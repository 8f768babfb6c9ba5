"""A/B the pgemm.hip main-loop variants (bare GEMM, EPI 0) against tuned
hipBLASLt, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule
24).  Variant bits: 1 no wave-row stagger, 2 WITH s_setprio (v0 is the default build), 4/8/12 = 4/16/32
m-tiles per L2 group (default 8)."""
import argparse
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
          "down": (4096, 14336)}
VARIANTS = (0, 1, 2, 3, 4, 8, 12)
# 32 = 32x32x16 MFMA (VAR bit 4), 33 / 34 = with no stagger / with s_setprio


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="gate_up:16384,qkv:16384,o:16384,down:16384,qkv:4096,o:4096")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default=",".join(str(v) for v in VARIANTS))
    a = ap.parse_args()
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms(0)
    kk = ops.kernels()
    for case in a.cases.split(","):
        name, M = case.split(":")
        M = int(M)
        N, K = SHAPES[name]
        w = torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        want = (x[:64].float() @ w.float().t())
        fns = {"lib": lambda: F.linear(x, w)}
        for v in [int(x) for x in a.variants.split(",")]:
            fns[f"v{v}"] = (lambda v=v: kk.pgemm_variant(v, out, x, w))
            fns[f"v{v}"]()
            torch.cuda.synchronize()
            err = ((out[:64].float() - want).abs().max() / want.abs().max()).item()
            assert err < 1e-2, (name, v, err)
        iters = max(3, int(2e5 / (2.0 * M * N * K / 1.4e12 * 1e6 + 1)))
        iters = min(iters, 50)
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                res[k].append(timed(f, iters))
        flops = 2.0 * M * N * K
        lib = statistics.median(res["lib"])
        line = " ".join(f"{k}={statistics.median(v):7.1f}us/{flops / statistics.median(v) / 1e6:4.0f}TF"
                        for k, v in res.items())
        best = min((statistics.median(v), k) for k, v in res.items() if k != "lib")
        print(f"{name:8s} M={M:6d} {line} | best {best[1]} x{lib / best[0]:.3f}", flush=True)
        del w, x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
