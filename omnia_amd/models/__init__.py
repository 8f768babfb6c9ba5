"""Model families served by the in-node engine (Llama-3 dense, Mixtral MoE)."""
from .config import REGISTRY, ModelConfig, resolve  # noqa: F401


def build_model(cfg: ModelConfig, device="cpu", dtype=None, seed: int = 0, **kw):
    import torch

    dtype = dtype or torch.bfloat16
    if kw.get("weights") is None:
        kw.pop("weights", None)
    if cfg.arch == "llama":
        from .llama import LlamaModel

        kw.pop("ep_mode", None)
        return LlamaModel(cfg, device=device, dtype=dtype, seed=seed, **kw)
    if cfg.arch == "mixtral":
        from .mixtral import MixtralModel

        return MixtralModel(cfg, device=device, dtype=dtype, seed=seed, **kw)
    raise ValueError(f"unsupported arch {cfg.arch}")
