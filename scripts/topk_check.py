"""Vocab-slice top-k as the TP sampler runs it (bf16 [B, V/tp], k = 64), eager
and inside a captured graph, for the batch sizes the TP engine tests hit;
checked against fp32 top-k after a device synchronize per case.

    python scripts/topk_check.py
"""
import torch


def main():
    dev = "cuda"
    torch.manual_seed(0)
    for V in (64128, 32064, 16032):
        for B in (1, 2, 3, 4, 8, 64):
            x = torch.randn(B, V, device=dev, dtype=torch.bfloat16)
            v, i = torch.topk(x, 64, dim=1)
            torch.cuda.synchronize()
            vr, _ = torch.topk(x.float(), 64, dim=1)
            ok_e = torch.equal(v.float(), vr)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                torch.topk(x, 64, dim=1)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gv, gi = torch.topk(x, 64, dim=1)
            g.replay()
            torch.cuda.synchronize()
            ok_g = torch.equal(gv.float(), vr)
            print(f"V={V} B={B}: eager {ok_e} graph {ok_g}", flush=True)


if __name__ == "__main__":
    main()
