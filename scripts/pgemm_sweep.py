"""Prefill-chunk GEMMs on one MI355X: the hand 256x256 8-phase kernel with fused
epilogues (ops/csrc/pgemm.hip) against tuned hipBLASLt (F.linear) plus the
unfused follow-up pass the fused epilogue replaces:
  qkv      pgemm epi 3 (RoPE + paged KV write)    vs  F.linear + rope_kv
  o, down  pgemm epi 2 (residual add + sumsq)     vs  F.linear + fused_add_rmsnorm
  gate_up  pgemm epi 1 (SwiGLU)                   vs  F.linear + silu_mul
and the bare GEMM (pgemm epi 0 vs F.linear).  Llama-3-8B shapes, M = prefill chunk
rows, random operands.  Prints TFLOP/s; every variant is error-checked."""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
          "down": (4096, 14336)}


def bench(fn, iters=10, rounds=3):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000 / iters)
    return best  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="4096,8192,16384")
    ap.add_argument("--shapes", default="gate_up,qkv,o,down")
    ap.add_argument("--out", default="gpurun_out/pgemm_sweep.json")
    ap.add_argument("--schedule", type=int, default=0,
                    help="pgemm main loop: 0 = 8-wave ping-pong, 1 = 4-wave")
    a = ap.parse_args()
    ops.kernels().pgemm_set_schedule(a.schedule)
    print("pgemm schedule:", a.schedule, flush=True)
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    print("tuned hipBLASLt table:", enable_tuned_gemms(0), flush=True)
    res = {}
    hq, hkv, bs = 32, 8, 16
    cos_sin = ref.rope_cos_sin(8192, 128, 5e5, None, device="cuda")
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        w = torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            flops = 2.0 * M * N * K
            t_gemm = bench(lambda: F.linear(x, w))
            o0 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            t_p0 = bench(lambda: ops.pgemm(0, x, w, out=o0))
            sub = torch.arange(0, M, max(1, M // 64), device="cuda")
            want = x[sub].float() @ w.float().t()
            err0 = ((o0[sub].float() - want).abs().max() / want.abs().max()).item()
            line = {"gemm_lib_us": t_gemm, "gemm_pgemm_us": t_p0, "err0": err0}
            if name == "gate_up":
                I = N // 2
                t_lib = bench(lambda: ops.silu_mul(F.linear(x, w)))
                o1 = torch.empty(M, I, device="cuda", dtype=torch.bfloat16)
                t_f = bench(lambda: ops.pgemm(1, x, w, out=o1))
                wref = ref.silu_mul(want.to(torch.bfloat16)).float()
                errf = ((o1[sub].float() - wref).abs().max() / wref.abs().max()).item()
            elif name == "qkv":
                nb = (M + bs - 1) // bs + 1
                kc = torch.empty(nb, hkv, bs, 128, device="cuda", dtype=torch.bfloat16)
                vc = torch.empty_like(kc)
                pos = torch.arange(M, device="cuda", dtype=torch.int32) % 8192
                slots = torch.arange(M, device="cuda", dtype=torch.int64)

                def lib():
                    y = F.linear(x, w)
                    ops.rope_kv(y[:, :hq * 128], y[:, hq * 128:(hq + hkv) * 128],
                                y[:, (hq + hkv) * 128:], pos, cos_sin, kc, vc, slots, hq, hkv, bs)
                t_lib = bench(lib)
                q = torch.empty(M, hq * 128, device="cuda", dtype=torch.bfloat16)
                t_f = bench(lambda: ops.pgemm(3, x, w, out=q, positions=pos, cos_sin=cos_sin,
                                              k_cache=kc, v_cache=vc, slots=slots, hq=hq,
                                              hkv=hkv, block_size=bs))
                qr = ref.apply_rope(want[:, :hq * 128].to(torch.bfloat16).view(-1, hq, 128),
                                    pos[sub], cos_sin).float().view(-1, hq * 128)
                errf = ((q[sub].float() - qr).abs().max() / qr.abs().max()).item()
            else:
                res_t = torch.randn(M, N, device="cuda").to(torch.bfloat16)
                nw = torch.ones(N, device="cuda", dtype=torch.bfloat16)
                ss = torch.empty(M, N // 256, device="cuda")

                def lib():
                    y = F.linear(x, w)
                    ops.fused_add_rmsnorm(y, res_t, nw, 1e-5)
                t_lib = bench(lib)
                t_f = bench(lambda: ops.pgemm(2, x, w, out=res_t, ss_out=ss))
                errf = 0.0
            line.update({"lib_fused_us": t_lib, "pgemm_fused_us": t_f, "err_fused": errf})
            res[f"{name}:{M}"] = line
            print(f"{name:8s} M={M:6d} GEMM lib {t_gemm:8.1f} us {flops / t_gemm / 1e6:5.0f} TF | "
                  f"pgemm {t_p0:8.1f} us {flops / t_p0 / 1e6:5.0f} TF x{t_gemm / t_p0:.2f} "
                  f"err {err0:.4f} || +epilogue lib {t_lib:8.1f} us | pgemm {t_f:8.1f} us "
                  f"x{t_lib / t_f:.2f} err {errf:.4f}", flush=True)
        del w
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
