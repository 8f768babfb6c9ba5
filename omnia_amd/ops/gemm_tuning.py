"""hipBLASLt solution selection for the engine's plain GEMMs.

The dense projections (QKV, O, gate_up, down, lm_head) are plain bf16 GEMMs and
stay on hipBLASLt.  Its default heuristic picks poor tiles for the skinny decode
shapes (M = batch <= 512), so we pin per-shape solutions found by PyTorch's
TunableOp (``scripts/tune_gemms.py`` benchmarks every hipBLASLt/rocBLAS candidate
on the MI355X) and ship the table in-tree (``omnia_amd/ops/tuned/``).  At engine
start the table is loaded read-only: no tuning happens on the serving path.
"""
from __future__ import annotations

import os
from pathlib import Path

TUNED_DIR = Path(__file__).resolve().parent / "tuned"


def table_path(device_index: int = 0) -> Path:
    return TUNED_DIR / f"tunableop_gfx950_{device_index}.csv"


def enable_tuned_gemms(device_index: int = 0, tuning: bool = False) -> bool:
    """Load the shipped solution table (and optionally keep tuning new shapes)."""
    if os.environ.get("OMNIA_GEMM_TUNING", "1") == "0":
        return False
    import torch

    if not torch.cuda.is_available():
        return False
    src = table_path(0)
    if not src.exists() and not tuning:
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(tuning)
    if src.exists():
        try:
            tun.read_file(str(src))
        except Exception:
            return False
    if tuning:
        TUNED_DIR.mkdir(exist_ok=True)
        tun.set_filename(str(TUNED_DIR / "tunableop_gfx950_0.csv"))
        tun.set_max_tuning_duration(int(os.environ.get("OMNIA_TUNE_MS", "200")))
    return True


def decode_shapes(cfg, tp: int = 1, batches=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512)):
    """(M, N, K) of every projection the engine runs for a model config."""
    d, D = cfg.hidden_size, cfg.head_dim
    hq, hkv, inter = cfg.num_heads // tp, max(1, cfg.num_kv_heads // tp), cfg.intermediate_size // tp
    nk = [((hq + 2 * hkv) * D, d), (d, hq * D), (2 * inter, d), (d, inter),
          (cfg.vocab_size // tp, d)]
    return [(m, n, k) for m in batches for n, k in nk]
