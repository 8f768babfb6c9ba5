"""Tune hipBLASLt solutions for the engine's GEMM shapes with TunableOp and
write omnia_amd/ops/tuned/tunableop_gfx950_0.csv (run on an MI355X)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from omnia_amd.models.config import resolve
from omnia_amd.ops import gemm_tuning

models = os.environ.get("MODELS", "llama-3-8b").split(",")
batches = [int(x) for x in os.environ.get("BATCHES", "1,8,16,32,64,128,256,512").split(",")]
prefill = [int(x) for x in os.environ.get("PREFILL", "16384").split(",") if x]
gemm_tuning.enable_tuned_gemms(0, tuning=True)
t0 = time.time()
shapes = []
for m in models:
    cfg = resolve(m)
    shapes += gemm_tuning.decode_shapes(cfg, batches=tuple(batches + prefill))
seen = set()
vocab = {resolve(m).vocab_size for m in models}
for (M, N, K) in shapes:
    if (M, N, K) in seen or (M in prefill and N in vocab):
        continue  # the LM head only sees the last token of each prefill
    seen.add((M, N, K))
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    F.linear(x, w)
    torch.cuda.synchronize()
    print(f"tuned {M}x{N}x{K} t={time.time()-t0:.0f}s", flush=True)
torch.cuda.tunable.write_file() if hasattr(torch.cuda.tunable, "write_file") else None
print("written", torch.cuda.tunable.get_filename())
