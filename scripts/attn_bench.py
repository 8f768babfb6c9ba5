#!/usr/bin/env python3
"""Decode-attention micro-benchmark on one MI355X: Llama-3-8B head geometry
(32 q / 8 kv heads x 128, bf16 paged KV, 32-token pages), B sequences of
context ``ctx`` scattered over a large page pool (no cache reuse between
launches: every call streams B*ctx*2*8*128*2 bytes of K/V), per partition size.
Reports us/call and effective HBM GB/s (KV bytes / time)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnia_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--ctx", default="576,1024,2048")
    ap.add_argument("--parts", default="512,1024,2048")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--bs", type=int, default=32)
    a = ap.parse_args()
    dev = "cuda"
    hq, hkv, D, bs = 32, 8, 128, a.bs
    for ctx in [int(c) for c in a.ctx.split(",")]:
        nbp = (ctx + bs - 1) // bs
        max_blocks = max(64, nbp)
        nblk = a.B * nbp * 2  # pool twice the working set
        k = torch.randn(nblk, hkv, bs, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(nblk, hkv, bs, D, device=dev, dtype=torch.bfloat16)
        perm = torch.randperm(nblk, device=dev)[: a.B * nbp].view(a.B, nbp).int()
        bt = torch.zeros(a.B, max_blocks, dtype=torch.int32, device=dev)
        bt[:, :nbp] = perm
        sl = torch.full((a.B,), ctx, dtype=torch.int32, device=dev)
        q = torch.randn(a.B, hq, D, device=dev, dtype=torch.bfloat16)
        kv_bytes = a.B * ctx * hkv * D * 2 * 2
        ref = None
        for part in [int(p) for p in a.parts.split(",")]:
            ws = ops.decode_workspace(a.B, hq, max_blocks, bs, part, dev)
            out = torch.empty(a.B, hq, D, device=dev, dtype=torch.bfloat16)
            f = lambda: ops.decode_attention(q, k, v, bt, sl, D ** -0.5, part, ws, out)
            f()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.iters):
                f()
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 1e3 / a.iters
            print(f"B={a.B} ctx={ctx} bs={bs} part={part}: {us:8.1f} us  "
                  f"{kv_bytes / us / 1e3:7.0f} GB/s  maxdiff={err:.2e}", flush=True)
        del k, v
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
