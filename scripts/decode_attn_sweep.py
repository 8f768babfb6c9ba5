"""Decode attention sweep at the WS bench's decode shape (Llama-3-8B, 256
sequences, one query each, 32 q / 8 kv heads, 32-token pages, contexts
513..640): kernel time and KV stream rate per partition size, with the
partition-merge kernel included.  The K+V stream (>= 545 MB) exceeds the
256 MB Infinity Cache, so back-to-back runs read HBM (no flush kernel: its
dirty lines would be written back under the measured kernel).

    python scripts/decode_attn_sweep.py [--nw 2,4] [--parts 256,512,1024]
    python scripts/decode_attn_sweep.py --batch 128 --hq 64   # Llama-3-70B, TP=1
    python scripts/decode_attn_sweep.py --hq 8 --hkv 1        # one Llama-3-70B TP=8 rank

Rows ``mix`` draw every sequence's length uniformly from 513..640, as in a
closed-loop wave (the partition split then varies per sequence).

``--nw`` runs each shape with the 2- and the 4-wave workgroup
(``OMNIA_DECODE_NW``, read per launch) and checks them against each other.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nw", default="0")
    ap.add_argument("--parts", default="128,192,256,320,384,512,640,1024")
    ap.add_argument("--u", default="4", help="V rows in flight per lane (OMNIA_DECODE_U); "
                    "g8 = 8 K groups and 8 V rows (OMNIA_DECODE_UG=8)")
    ap.add_argument("--splits", default="0",
                    help="0 = fixed partitions of --parts keys; n > 0 = length-balanced "
                         "split into up to n partitions (--parts is then the cap)")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8, help="1 = a Llama-3-70B TP=8 shard")
    a = ap.parse_args()
    nws = [int(x) for x in a.nw.split(",")]
    parts = [int(x) for x in a.parts.split(",")]
    torch.manual_seed(0)
    dev = "cuda"
    B, hq, hkv, D, BS = a.batch, a.hq, a.hkv, 128, 32
    max_len = 1024
    mb = max_len // BS
    nblk = B * mb + 8
    # cache copies rotated per launch: the working set stays above the 256 MB
    # Infinity Cache at the smaller shapes too
    ncopy = max(2, -(-768 * 2**20 // (2 * nblk * hkv * BS * D * 2)))  # > 2x the MALL
    kcs = [torch.randn(nblk, hkv, BS, D, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    vcs = [torch.randn(nblk, hkv, BS, D, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    kc, vc = kcs[0], vcs[0]
    perm = torch.randperm(nblk - 8, device=dev)[:B * mb].to(torch.int32)
    bt = perm.view(B, mb).contiguous()
    q = torch.randn(B, hq, D, device=dev, dtype=torch.bfloat16)
    scale = D ** -0.5
    print(f"{'len':>5} {'part':>5} {'sp':>3} {'nw':>3} {'u':>2} {'us':>8} {'TB/s':>6}  err", flush=True)
    for L in (520, 576, 640, "mix"):
        if L == "mix":
            g = torch.Generator().manual_seed(1)
            sl = torch.randint(513, 641, (B,), generator=g, dtype=torch.int32).to(dev)
        else:
            sl = torch.full((B,), L, dtype=torch.int32, device=dev)
        ref = None
        for part, nw, uv, sp in [(p, w, u, int(x)) for p in parts for w in nws
                                 for u in a.u.split(",") for x in a.splits.split(",")]:
            os.environ["OMNIA_DECODE_U"] = "8" if uv == "g8" else uv
            os.environ["OMNIA_DECODE_UG"] = "8" if uv == "g8" else "4"
            if nw:
                os.environ["OMNIA_DECODE_NW"] = str(nw)
            else:
                os.environ.pop("OMNIA_DECODE_NW", None)
            ws = ops.decode_workspace(B, hq, mb, BS, part, dev, sp)
            out = ops.decode_attention(q, kc, vc, bt, sl, scale, part_size=part, workspace=ws,
                                       splits=sp)
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            ts = []
            for i in range(30):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.decode_attention(q, kcs[i % ncopy], vcs[i % ncopy], bt, sl, scale, part_size=part,
                                     workspace=ws, out=out, splits=sp)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            us = ts[len(ts) // 2]
            nbytes = int(sl.sum().item()) * hkv * D * 2 * 2
            print(f"{L!s:>5} {part:5d} {sp:3d} {nw:3d} {uv:>2} {us:8.1f} {nbytes / us / 1e6:6.2f}  {err:.2e}", flush=True)
    time.sleep(0.1)


if __name__ == "__main__":
    main()
