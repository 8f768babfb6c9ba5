#!/usr/bin/env python3
"""Prefill-attention micro-benchmark: one 16K-token prefill chunk (32 sequences x
512 new tokens, no cached prefix, causal), Llama-3-8B heads, per GQA packing
(heads per wave).  Reports us/call and achieved TFLOP/s (causal FLOPs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnia_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    hq, hkv, D, bs = 32, 8, 128, 32
    for nseq, qlen in ((32, 512), (8, 2048)):
        nbp = qlen // bs
        nblk = nseq * nbp
        k = torch.randn(nblk, hkv, bs, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(nblk, hkv, bs, D, device=dev, dtype=torch.bfloat16)
        bt = torch.arange(nblk, dtype=torch.int32, device=dev).view(nseq, nbp)
        q = torch.randn(nseq * qlen, hq, D, device=dev, dtype=torch.bfloat16)
        qsl = torch.arange(0, nseq * qlen + 1, qlen, dtype=torch.int32, device=dev)
        sl = torch.full((nseq,), qlen, dtype=torch.int32, device=dev)
        tiles = {}
        for qt in (32, 64, 128):
            s, q0 = ops.prefill_tiles([qlen] * nseq, qt)
            tiles[qt] = (torch.tensor(s, dtype=torch.int32, device=dev),
                         torch.tensor(q0, dtype=torch.int32, device=dev))
        flops = nseq * hq * (qlen * (qlen + 1) / 2) * D * 4
        ref = None
        for hp, qt in ((1, 64), (1, 128), (0, 32)):
            out = torch.empty_like(q)
            ts, tq = tiles[qt]
            f = lambda: ops.prefill_attention(q, k, v, bt, qsl, sl, D ** -0.5, ts, tq, out, hp,
                                              qt)
            f()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(20):
                f()
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 1e3 / 20
            print(f"seqs={nseq} qlen={qlen} hp={hp} qtile={qt}: {us:8.1f} us  "
                  f"{flops / us / 1e6:7.1f} "
                  f"TFLOP/s  maxdiff={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
