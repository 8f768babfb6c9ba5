"""Run one tgemm configuration back to back (for rocprofv3 --pmc passes):
python scripts/tgemm_pmc.py <shape> <M> <bn> <S> <wnt> [iters]"""
import sys

import torch

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (14336, 4096, 1),
          "down": (4096, 14336, 0)}


def main():
    name, M, bn, S, wnt = sys.argv[1], *map(int, sys.argv[2:6])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 50
    N, K, mode = SHAPES[name]
    rows = 2 * N if mode == 1 else N
    copies = max(2, (1 << 30) // (rows * K * 2) + 1)
    ws = [torch.randn(rows, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(copies)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    md = 1 if (mode == 1 and S == 1) else 2
    out = (torch.empty(S, M, rows, device="cuda") if md == 2 else
           torch.empty(M, N, device="cuda", dtype=torch.bfloat16))
    for i in range(iters):
        ops.tgemm(md, x, ws[i % copies], S, bn, wnt, out=out)
    torch.cuda.synchronize()
    print("ok", name, M, bn, S, wnt)


if __name__ == "__main__":
    main()
