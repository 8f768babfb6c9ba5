"""LM head at the decode batch (M = 256, N = 128256, K = 4096, bf16 out): tuned
hipBLASLt (F.linear) against tgemm.hip tile widths / flags, weights rotated over
copies larger than the 256 MB MALL.  Prints us and TB/s per config.

    python scripts/lm_head_sweep.py"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402


def bench(fn, iters=30):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    print("tuned hipBLASLt table:", enable_tuned_gemms(0), flush=True)
    N, K = 128256, 4096
    copies = 3
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
    nbytes = N * K * 2
    for M in (256, 192, 128):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        want = F.linear(x, ws[0]).float()
        t = bench(lambda i: F.linear(x, ws[i % copies]))
        print(f"M={M:3d} hipBLASLt        {t:7.1f} us  {nbytes / t / 1e6:5.2f} TB/s", flush=True)
        for bn in (128, 256):
            for wnt in (0, 1, 4, 5):
                if wnt & 4 and bn > 128:
                    continue
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                t = bench(lambda i: ops.tgemm(0, x, ws[i % copies], 1, bn, wnt, out=out))
                ops.tgemm(0, x, ws[0], 1, bn, wnt, out=out)
                err = ((out.float() - want).abs().max() / want.abs().max()).item()
                print(f"M={M:3d} tgemm bn={bn:3d} wnt={wnt} {t:7.1f} us  {nbytes / t / 1e6:5.2f} TB/s"
                      f"  err {err:.4f}", flush=True)


if __name__ == "__main__":
    main()
