"""Model architecture configs (public HF shapes, random-init weights in this repo).

The reference (AltairaLabs/Omnia) never runs a model -- its Provider CRD points
at remote vendors (``api/v1alpha1/provider_types.go:273-413``).  These configs
are the in-node engine's model registry; the Provider CRD ``spec.model`` name is
resolved here (``resolve``).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str = "llama"  # llama | mixtral
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    # MoE
    num_experts: int = 0
    experts_per_token: int = 0
    # tokenizer special ids (llama-3 layout)
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128009)

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def num_params(self) -> int:
        d, i, L = self.hidden_size, self.intermediate_size, self.num_layers
        attn = d * (self.q_size + 2 * self.kv_size) + self.q_size * d
        mlp = 3 * d * i * max(1, self.num_experts) + (d * self.num_experts if self.is_moe else 0)
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * d) + emb + d

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


LLAMA3_8B = ModelConfig(name="llama-3-8b")
LLAMA31_8B = ModelConfig(
    name="llama-3.1-8b",
    max_position=131072,
    rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                  "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
)
LLAMA3_70B = ModelConfig(name="llama-3-70b", hidden_size=8192, intermediate_size=28672,
                         num_layers=80, num_heads=64, num_kv_heads=8)
MIXTRAL_8X7B = ModelConfig(name="mixtral-8x7b", arch="mixtral", vocab_size=32000,
                           hidden_size=4096, intermediate_size=14336, num_layers=32,
                           num_heads=32, num_kv_heads=8, rope_theta=1e6, max_position=32768,
                           num_experts=8, experts_per_token=2, bos_token_id=1,
                           eos_token_ids=(2,))
# in-node embedding model for the memory tier (K17): a small Llama-shaped encoder
# whose last hidden states are mean-pooled + L2-normalised (1024-d vectors)
EMBED_1B = ModelConfig(name="omnia-embed-1b", vocab_size=128256, hidden_size=1024,
                       intermediate_size=4096, num_layers=16, num_heads=8, num_kv_heads=8,
                       max_position=8192, tie_embeddings=True)
TINY_EMBED = ModelConfig(name="tiny-embed", vocab_size=512, hidden_size=256,
                         intermediate_size=512, num_layers=2, num_heads=2, num_kv_heads=2,
                         max_position=4096, tie_embeddings=True, bos_token_id=256,
                         eos_token_ids=(257,))
# tiny shapes for CPU tests / smoke (same code paths, head_dim fixed at 128)
TINY_LLAMA = ModelConfig(name="tiny-llama", vocab_size=512, hidden_size=256,
                         intermediate_size=512, num_layers=2, num_heads=4, num_kv_heads=2,
                         max_position=4096, bos_token_id=256, eos_token_ids=(257,))
# TP=4/8 rehearsal shape: 8 q heads over 2 kv heads, so at TP 4 and 8 every rank
# holds ONE replicated kv head -- the per-rank layout of Llama-3-70B at TP=8
TINY_LLAMA_H8 = ModelConfig(name="tiny-llama-h8", vocab_size=512, hidden_size=1024,
                            intermediate_size=1024, num_layers=2, num_heads=8, num_kv_heads=2,
                            max_position=4096, bos_token_id=256, eos_token_ids=(257,))
TINY_MIXTRAL = ModelConfig(name="tiny-mixtral", arch="mixtral", vocab_size=512,
                           hidden_size=256, intermediate_size=256, num_layers=2, num_heads=4,
                           num_kv_heads=2, max_position=4096, num_experts=4,
                           experts_per_token=2, bos_token_id=256, eos_token_ids=(257,))
# 8 experts: one per rank of an 8-way expert-parallel group (EP world-8 tests)
TINY_MIXTRAL_E8 = ModelConfig(name="tiny-mixtral-e8", arch="mixtral", vocab_size=512,
                              hidden_size=256, intermediate_size=128, num_layers=2,
                              num_heads=4, num_kv_heads=2, max_position=4096, num_experts=8,
                              experts_per_token=2, bos_token_id=256, eos_token_ids=(257,))

REGISTRY: dict[str, ModelConfig] = {
    c.name: c for c in [LLAMA3_8B, LLAMA31_8B, LLAMA3_70B, MIXTRAL_8X7B, TINY_LLAMA, TINY_MIXTRAL,
                   TINY_MIXTRAL_E8, EMBED_1B, TINY_EMBED, TINY_LLAMA_H8]
}
ALIASES = {
    "meta-llama/Meta-Llama-3-8B": "llama-3-8b",
    "meta-llama/Meta-Llama-3-8B-Instruct": "llama-3-8b",
    "llama3-8b": "llama-3-8b",
    "meta-llama/Llama-3.1-8B-Instruct": "llama-3.1-8b",
    "meta-llama/Meta-Llama-3-70B-Instruct": "llama-3-70b",
    "llama3-70b": "llama-3-70b",
    "mistralai/Mixtral-8x7B-Instruct-v0.1": "mixtral-8x7b",
    "mixtral": "mixtral-8x7b",
}


def resolve(name: str, **overrides) -> ModelConfig:
    key = ALIASES.get(name, name)
    if key not in REGISTRY:
        raise KeyError(f"unknown model {name!r}; known: {sorted(REGISTRY)}")
    cfg = REGISTRY[key]
    return cfg.replace(**overrides) if overrides else cfg
