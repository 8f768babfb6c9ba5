#!/usr/bin/env python3
"""Decode-attention micro-benchmark on one MI355X: Llama-3-8B head geometry
(32 q / 8 kv heads x 128, bf16 paged KV, 32-token pages), B sequences of
context ``ctx`` scattered over a large page pool (no cache reuse between
launches: every call streams B*ctx*2*8*128*2 bytes of K/V), per partition size.
Consecutive calls rotate over R disjoint page sets (>= 1.5 GiB of K/V in total)
so no call is served from the 256 MiB Infinity Cache left warm by the previous
one -- in a decode step every layer streams its own KV.  ``--jitter J`` draws
the context lengths uniformly from [ctx-J, ctx+J] (a continuous batch).
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
    ap.add_argument("--jitter", type=int, default=0)
    a = ap.parse_args()
    dev = "cuda"
    hq, hkv, D, bs = 32, 8, 128, a.bs
    for ctx in [int(c) for c in a.ctx.split(",")]:
        cmax = ctx + a.jitter
        nbp = (cmax + bs - 1) // bs
        max_blocks = max(64, nbp)
        call_bytes = a.B * cmax * hkv * D * 2 * 2
        R = max(2, -(-(3 << 29) // call_bytes))
        nblk = a.B * nbp * R
        k = torch.randn(nblk, hkv, bs, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(nblk, hkv, bs, D, device=dev, dtype=torch.bfloat16)
        perm = torch.randperm(nblk, device=dev).int().view(R, a.B, nbp)
        bts = []
        for r in range(R):
            bt = torch.zeros(a.B, max_blocks, dtype=torch.int32, device=dev)
            bt[:, :nbp] = perm[r]
            bts.append(bt)
        gen = torch.Generator().manual_seed(0)
        sl = torch.randint(ctx - a.jitter, ctx + a.jitter + 1, (a.B,), generator=gen) \
            if a.jitter else torch.full((a.B,), ctx)
        kv_bytes = int(sl.sum()) * hkv * D * 2 * 2
        sl = sl.int().to(dev)
        q = torch.randn(a.B, hq, D, device=dev, dtype=torch.bfloat16)
        ref = None
        for part in [int(p) for p in a.parts.split(",")]:
            ws = ops.decode_workspace(a.B, hq, max_blocks, bs, part, dev)
            out = torch.empty(a.B, hq, D, device=dev, dtype=torch.bfloat16)
            f = lambda i=0: ops.decode_attention(q, k, v, bts[i % R], sl, D ** -0.5, part,
                                                 ws, out)
            f()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for i in range(a.iters):
                f(i)
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 1e3 / a.iters
            print(f"B={a.B} ctx={ctx}+-{a.jitter} R={R} bs={bs} part={part}: {us:8.1f} us  "
                  f"{kv_bytes / us / 1e3:7.0f} GB/s  maxdiff={err:.2e}", flush=True)
        del k, v
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
