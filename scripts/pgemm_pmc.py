"""Short fixed workload for PMC passes over the prefill GEMM: the hand pgemm
(default build) and tuned hipBLASLt on the same random operands, 10 launches
each (o projection shape, M = 16384)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from omnia_amd import ops  # noqa: E402
from omnia_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
M, N, K = 16384, 4096, 4096
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = torch.randn(N, K, device="cuda").mul_(0.02).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
kk = ops.kernels()
for _ in range(10):
    kk.pgemm_variant(0, out, x, w)
for _ in range(10):
    F.linear(x, w)
torch.cuda.synchronize()
print("ok")
