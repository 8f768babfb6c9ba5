"""Full-batch decode GEMM sweep (M = 256 / 224 / 192) on one MI355X.

Compares, END TO END (projection + the kernel that consumes it, because the
split-K variants move their reduction into that consumer):
  lib      tuned hipBLASLt + the unfused consumer
           (qkv: rope_kv, o/down: fused_add_rmsnorm, gate_up: silu_mul)
  current  what the engine dispatches today (ops.dgemm for gate_up; lib otherwise)
  tgemm    tgemm.hip (every bn / S / nt variant) + the fused split-K consumer
           (splitk_rope_kv / splitk_add_rmsnorm / splitk_swiglu; mode 1 SwiGLU
           needs none)
Weights rotate over copies totalling >= 1 GiB (the 256 MiB MALL cannot serve
them).  Every tgemm variant is checked against an fp32 reference of the
projection.  One line per (shape, M); JSON to --out; --table writes the winning
configs as ops/tuned/wgemm_mi355x.json entries (nwaves = -1 / -2)."""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops import reference as ref  # noqa: E402

SHAPES = {  # name: (N, K, mode)   (Llama-3-8B; 70B TP=8 shard)
    "qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (14336, 4096, 1),
    "down": (4096, 14336, 0), "lm_head": (128256, 4096, 0),
    "70b_qkv_tp8": (1280, 8192, 0), "70b_o_tp8": (8192, 1024, 0),
    "70b_gu_tp8": (3584, 8192, 1), "70b_down_tp8": (8192, 3584, 0),
}


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
    return e0.elapsed_time(e1) * 1000 / iters  # us


class Consumer:
    """The kernel after the projection, in its unfused and split-K-fused forms."""

    def __init__(self, name, M, N):
        dev = "cuda"
        self.name, self.M, self.N = name, M, N
        if name.startswith("qkv") or name.endswith("qkv_tp8"):
            self.kind = "rope"
            self.hq, self.hkv = (32, 8) if N == 6144 else (8, 1)
            bs = 32
            nb = (M + bs - 1) // bs + 1
            self.kc = torch.zeros(nb, self.hkv, bs, 128, dtype=torch.bfloat16, device=dev)
            self.vc = torch.zeros_like(self.kc)
            self.pos = torch.arange(M, dtype=torch.int32, device=dev) + 100
            self.slots = torch.arange(M, dtype=torch.int64, device=dev)
            self.cs = ref.rope_cos_sin(4096, 128, 500000.0, None, device=dev)
            self.bs = bs
        elif name.startswith("gate") or name.endswith("gu_tp8"):
            self.kind = "swiglu"
        elif name == "lm_head":  # the sampler reads the bf16 logits as they are
            self.kind = "none"
        else:
            self.kind = "norm"
            self.res = torch.randn(M, N, device=dev).to(torch.bfloat16)
            self.w = torch.ones(N, dtype=torch.bfloat16, device=dev)

    def unfused(self, y):
        if self.kind == "none":
            return y
        if self.kind == "rope":
            D = 128
            q = y[:, : self.hq * D]
            k = y[:, self.hq * D: (self.hq + self.hkv) * D]
            v = y[:, (self.hq + self.hkv) * D:]
            ops.rope_kv(q, k, v, self.pos, self.cs, self.kc, self.vc, self.slots, self.hq,
                        self.hkv, self.bs)
        elif self.kind == "swiglu":
            return ops.silu_mul(y)
        else:
            ops.fused_add_rmsnorm(y, self.res, self.w, 1e-5)
        return y

    def fused(self, parts):
        if self.kind == "rope":
            return ops.splitk_rope_kv(parts, self.pos, self.cs, self.kc, self.vc, self.slots,
                                      self.hq, self.hkv, self.bs)
        if self.kind == "swiglu":
            return ops.splitk_swiglu(parts)
        return ops.splitk_add_rmsnorm(parts, self.res, self.w, 1e-5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="256,224,192")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--bn", default="64,128,256")
    ap.add_argument("--out", default="gpurun_out/tgemm_sweep.json")
    ap.add_argument("--table", default="", help="merge winners into this wgemm table json")
    ap.add_argument("--min-gain", type=float, default=1.03)
    ap.add_argument("--bk32", action="store_true", help="also try the 32-k-stage variants")
    a = ap.parse_args()
    from omnia_amd.ops.gemm_tuning import enable_tuned_gemms

    print("tuned hipBLASLt table:", enable_tuned_gemms(0), flush=True)
    res = {}
    table_upd = {}
    for name in a.shapes.split(","):
        N, K, mode = SHAPES[name]
        rows = 2 * N if mode == 1 else N
        nbytes = rows * K * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.randn(rows, K, device="cuda").mul_(0.02).to(torch.bfloat16)
              for _ in range(copies)]
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            cons = Consumer(name, M, N)
            want = (x.float() @ ws[0].float().t())
            if mode == 1:
                want = ref.silu_mul(want.to(torch.bfloat16)).float()

            def lib(i):
                y = F.linear(x, ws[i % copies])
                return cons.unfused(y)

            t_lib = bench(lib)
            t_cur = None
            if mode == 1 and ops.dgemm_config(M, N, K, 1) is not None:
                t_cur = bench(lambda i: ops.linear_silu(x, ws[i % copies]))
            t_gemm_only = bench(lambda i: F.linear(x, ws[i % copies]))
            cands = []
            for bn in [int(b) for b in a.bn.split(",")]:
                cols = bn // 2 if mode == 1 else bn
                if N % cols:
                    continue
                ntiles = N // cols
                for S in (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16):
                    if cons.kind == "none":  # bf16 output straight to its reader
                        if S > 1:
                            continue
                    elif S > K // 64 or ntiles * S > 640 or (ntiles * S < 96 and S < 16):
                        continue
                    md = mode if S == 1 and mode == 1 or cons.kind == "none" else 2
                    # bit 0 nt W loads, bit 1 32-k stages (lost everywhere, --bk32),
                    # bit 2 register-pipelined fragment reads (BN <= 128)
                    flags = [0, 1] + ([4, 5] if bn <= 128 else []) + \
                        ([2, 3] if a.bk32 and bn >= 128 else [])
                    for wnt in flags:
                        outb = (torch.empty(S, M, rows, device="cuda") if md == 2 else
                                torch.empty(M, N, device="cuda", dtype=torch.bfloat16))

                        def f(i, md=md, S=S, bn=bn, wnt=wnt, outb=outb):
                            ops.tgemm(md, x, ws[i % copies], S, bn, wnt, out=outb)
                            return cons.fused(outb) if md == 2 else outb

                        def g(i, md=md, S=S, bn=bn, wnt=wnt, outb=outb):
                            ops.tgemm(md, x, ws[i % copies], S, bn, wnt, out=outb)

                        try:
                            t = bench(f)
                            tg = bench(g)
                        except RuntimeError as e:
                            print("skip", name, M, bn, S, e, file=sys.stderr)
                            continue
                        g(0)
                        torch.cuda.synchronize()
                        if md == 2:
                            got = outb.sum(0)
                            if mode == 1:
                                got = ref.silu_mul(got.to(torch.bfloat16)).float()
                        else:
                            got = outb.float()
                        err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
                        cands.append((round(t, 2), bn, S, wnt, round(tg, 2), round(err, 4)))
            cands.sort()
            best = cands[0]
            gbs = lambda t: nbytes / t / 1e3  # noqa: E731
            tflops = lambda t: 2 * M * rows * K / t / 1e6  # noqa: E731
            cur = f" cur {t_cur:6.1f}" if t_cur is not None else ""
            print(f"{name:12s} M={M:3d} lib+cons {t_lib:6.1f} (gemm {t_gemm_only:6.1f} us "
                  f"{gbs(t_gemm_only):5.0f} GB/s){cur} | tgemm+cons {best[0]:6.1f} "
                  f"(gemm {best[4]:6.1f} us {gbs(best[4]):5.0f} GB/s {tflops(best[4]):5.0f} TF) "
                  f"bn={best[1]} S={best[2]} nt={best[3]} err={best[5]} "
                  f"x{(t_cur or t_lib) / best[0]:.2f}  top4={cands[:4]}", flush=True)
            res[f"{name}:{M}"] = {"lib_us": t_lib, "lib_gemm_us": t_gemm_only, "cur_us": t_cur,
                                  "best": best, "top": cands[:16], "weight_bytes": nbytes,
                                  "N": N, "K": K, "mode": mode, "M": M}
            if best[5] < 0.02 and (t_cur or t_lib) / best[0] >= a.min_gain:
                bucket = next(b for b in ops.WGEMM_BUCKETS if M <= b)
                table_upd[f"{mode}:{bucket}:{N}:{K}"] = [best[1], -1 - best[3], best[2]]
        del ws
        torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    if a.table:
        try:
            with open(a.table) as f:
                tab = json.load(f)
        except FileNotFoundError:
            tab = {}
        tab.update(table_upd)
        with open(a.table, "w") as f:
            json.dump(dict(sorted(tab.items())), f, indent=1)
        print("table entries:", json.dumps(table_upd), flush=True)


if __name__ == "__main__":
    main()
