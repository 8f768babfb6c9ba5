"""Prefill-chunk GEMMs on one MI355X: hipBLASLt (F.linear; + the silu_mul pass
for gate_up) vs tgemm.hip tiled over 256-row blocks (MODE 1 fuses SwiGLU into
the gate_up epilogue).  Llama-3-8B shapes, M = prefill chunk rows.  Every tgemm
variant is checked against an fp32 reference on a row subset.  Prints TFLOP/s."""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

SHAPES = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (14336, 4096, 1),
          "down": (4096, 14336, 0)}


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="4096,8192,16384")
    ap.add_argument("--shapes", default="gate_up,qkv,o,down")
    ap.add_argument("--out", default="gpurun_out/prefill_sweep.json")
    a = ap.parse_args()
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    print("tuned hipBLASLt table:", enable_tuned_gemms(0), flush=True)
    res = {}
    for name in a.shapes.split(","):
        N, K, mode = SHAPES[name]
        rows = 2 * N if mode == 1 else N
        w = torch.randn(rows, K, device="cuda").mul_(0.02).to(torch.bfloat16)
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            flops = 2.0 * M * rows * K
            if mode == 1:
                t_lib = bench(lambda: ops.silu_mul(F.linear(x, w)))
                t_gemm = bench(lambda: F.linear(x, w))
            else:
                t_lib = t_gemm = bench(lambda: F.linear(x, w))
            sub = torch.arange(0, M, max(1, M // 64), device="cuda")
            want = x[sub].float() @ w.float().t()
            if mode == 1:
                want = ref.silu_mul(want.to(torch.bfloat16)).float()
            cands = []
            for bn in (128, 256):
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                try:
                    t = bench(lambda bn=bn, out=out: ops.tgemm(mode, x, w, 1, bn, 0, out=out))
                except RuntimeError as e:
                    print("skip", name, M, bn, e, file=sys.stderr)
                    continue
                ops.tgemm(mode, x, w, 1, bn, 0, out=out)
                torch.cuda.synchronize()
                err = ((out[sub].float() - want).abs().max() / want.abs().max()).item()
                cands.append((round(t, 1), bn, round(flops / t / 1e6, 0), round(err, 4)))
            cands.sort()
            best = cands[0]
            print(f"{name:8s} M={M:6d} lib {t_lib:8.1f} us ({flops / t_gemm / 1e6:5.0f} TF gemm"
                  f"{' + silu_mul' if mode == 1 else ''}) | tgemm {best[0]:8.1f} us "
                  f"({best[2]:5.0f} TF) bn={best[1]} err={best[3]} x{t_lib / best[0]:.2f}  "
                  f"all={cands}", flush=True)
            res[f"{name}:{M}"] = {"lib_us": t_lib, "lib_gemm_us": t_gemm, "tgemm": cands}
        del w
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
