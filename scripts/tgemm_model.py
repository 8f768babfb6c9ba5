"""Decode-GEMM intake model check (tgemm.hip): kernel-only time of the gate_up /
down projections at the bench's M = 256 against the batch size (x bytes per
CU) and the tile width / split count (x re-reads vs weight bytes per CU).

    python scripts/tgemm_model.py

The wnt codes >= 8 (split x / W rings, bits 3-4) and >= 32 (measurement-only
pipelines: 32 staging alone, 64 W alone, 96 x alone, 128 / 160 tile-packed W)
exist in tgemm.hip at commit 1a05c5a only; at other commits they are rejected
and print "skip".  Findings: profiles/r5/decode_gemm/README.md."""
import sys

import torch

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402


def bench(fn, iters=40):
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
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--all-m", action="store_true", help="also M = 192 / 128 / 64")
    a = ap.parse_args()
    shapes = {"gate_up": (28672, 4096), "down": (4096, 14336), "qkv": (6144, 4096),
              "o": (4096, 4096)}
    print(f"{'shape':8s} {'M':>4s} {'mode':>4s} {'bn':>4s} {'S':>3s} {'wnt':>3s} {'blocks':>6s} "
          f"{'us':>7s} {'W KB/cu':>8s} {'x KB/cu':>8s} {'GB/s W':>7s}", flush=True)
    for name, (rows, K) in shapes.items():
        nbytes = rows * K * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.randn(rows, K, device="cuda").mul_(0.02).to(torch.bfloat16)
              for _ in range(copies)]
        packed = {}
        for M in (256, 192, 128, 64):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            if M != 256 and not a.all_m:
                continue
            cfgs = []
            # (mode, bn, S, wnt); wnt bit 3 = tile-packed weights (ops.tgemm_pack)
            base = {"gate_up": [(1, 128, 1, 0), (1, 128, 1, 4), (1, 64, 1, 0), (2, 256, 2, 0)],
                    "down": [(2, 128, 8, 4), (2, 128, 8, 0), (2, 128, 7, 4), (2, 64, 4, 4)],
                    "qkv": [(2, 128, 5, 0), (2, 128, 4, 0), (2, 64, 4, 4), (2, 128, 6, 4)],
                    "o": [(2, 64, 4, 0), (2, 64, 4, 4), (2, 128, 8, 0), (2, 64, 8, 0)]}[name]
            for c in base:
                cfgs += [c, c[:3] + (c[3] | 8,)]
            for mode, bn, S, wnt in cfgs:
                N = rows // 2 if mode == 1 else rows
                cols = bn // 2 if mode == 1 else bn
                ntiles = N // cols
                blocks = ntiles * S
                out = (torch.empty(S, M, N, device="cuda") if mode == 2 else
                       torch.empty(M, N, device="cuda", dtype=torch.bfloat16))
                wsrc = ws
                if wnt & 8:
                    key = (bn, 1 if mode == 1 else 0)
                    if key not in packed:
                        packed[key] = [ops.tgemm_pack(w_, bn, key[1]) for w_ in ws]
                    wsrc = packed[key]
                try:
                    t = bench(lambda i: ops.tgemm(mode, x, wsrc[i % copies], S, bn, wnt, out=out))
                except RuntimeError as e:
                    print("skip", name, M, mode, bn, S, e, flush=True)
                    continue
                ops.tgemm(mode, x, wsrc[0], S, bn, wnt, out=out)
                full = x.float() @ ws[0].float().t()
                if mode == 1:
                    want = torch.nn.functional.silu(full[:, :N]) * full[:, N:]
                    got = out.float()
                else:
                    want, got = full, out.sum(0)
                err = ((got - want).abs().max() / want.abs().max()).item() 
                wcu = bn * (K // S) * 2 / 1024
                xcu = M * (K // S) * 2 / 1024
                print(f"{name:8s} {M:4d} {mode:4d} {bn:4d} {S:3d} {wnt:3d} {blocks:6d} {t:7.1f} "
                      f"{wcu:8.0f} {xcu:8.0f} {nbytes / t / 1e3:7.0f}  err {err:.4f}", flush=True)
        del ws, packed
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
