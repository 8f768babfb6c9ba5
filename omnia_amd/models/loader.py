"""Weight layout, TP sharding and checkpoint loading.

Our layout per layer (natural ``[out, in]`` so ``F.linear`` is one hipBLASLt GEMM):
``qkv`` = [q (Hq*D) ; k (Hkv*D) ; v (Hkv*D)] rows, ``o`` [d, Hq*D],
``gate_up`` = [gate (I) ; up (I)] rows, ``down`` [d, I]; MoE layers hold
``router`` [E, d] and per-expert ``experts_gate_up`` [E, 2I, d] / ``experts_down``
[E, d, I].  Megatron sharding: QKV/gate_up column-parallel (output rows), O/down
row-parallel (input columns), vocab-parallel embedding/lm_head; KV heads are
replicated when ``Hkv < tp`` (each rank keeps head ``r * Hkv // tp``).  Experts are
sharded across the TP group (expert parallel).

``load_hf_checkpoint`` reads HF Llama / Mixtral safetensors directly (no torch
pickle: ``safetensors`` only) and slices each rank's shard with ``get_slice`` so a
rank never materialises the full tensor.
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import torch

from .config import ModelConfig


def _kv_head_range(cfg: ModelConfig, tp: int, rank: int) -> tuple[int, int]:
    if cfg.num_kv_heads >= tp:
        n = cfg.num_kv_heads // tp
        return rank * n, (rank + 1) * n
    h = rank * cfg.num_kv_heads // tp
    return h, h + 1


def shard_layer(layer: dict, cfg: ModelConfig, tp: int, rank: int) -> dict:
    if tp == 1:
        return dict(layer)
    D = cfg.head_dim
    hq = cfg.num_heads // tp
    q0 = rank * hq * D
    k0, k1 = _kv_head_range(cfg, tp, rank)
    out = {"in_norm": layer["in_norm"], "post_norm": layer["post_norm"]}
    qkv = layer["qkv"]
    Q, K = cfg.num_heads * D, cfg.num_kv_heads * D
    out["qkv"] = torch.cat([qkv[q0:q0 + hq * D], qkv[Q + k0 * D:Q + k1 * D],
                            qkv[Q + K + k0 * D:Q + K + k1 * D]]).contiguous()
    out["o"] = layer["o"][:, q0:q0 + hq * D].contiguous()
    if "gate_up" in layer:
        inter = cfg.intermediate_size
        n = inter // tp
        gu = layer["gate_up"]
        out["gate_up"] = torch.cat([gu[rank * n:(rank + 1) * n],
                                    gu[inter + rank * n:inter + (rank + 1) * n]]).contiguous()
        out["down"] = layer["down"][:, rank * n:(rank + 1) * n].contiguous()
    if "router" in layer:
        E = cfg.num_experts
        ne = E // tp
        out["router"] = layer["router"]
        out["experts_gate_up"] = layer["experts_gate_up"][rank * ne:(rank + 1) * ne].contiguous()
        out["experts_down"] = layer["experts_down"][rank * ne:(rank + 1) * ne].contiguous()
    return out


def shard_weights(full: dict, cfg: ModelConfig, tp: int, rank: int) -> dict:
    """Full (tp=1) weight dict -> this rank's shard."""
    if tp == 1:
        return full
    v = cfg.vocab_size // tp
    w = {"final_norm": full["final_norm"],
         "embed": full["embed"][rank * v:(rank + 1) * v].contiguous(),
         "layers": [shard_layer(l, cfg, tp, rank) for l in full["layers"]]}
    w["lm_head"] = w["embed"] if cfg.tie_embeddings else \
        full["lm_head"][rank * v:(rank + 1) * v].contiguous()
    return w


# ------------------------------------------------------------------ HF checkpoints
_HF_LLAMA = {
    "q": "model.layers.{i}.self_attn.q_proj.weight",
    "k": "model.layers.{i}.self_attn.k_proj.weight",
    "v": "model.layers.{i}.self_attn.v_proj.weight",
    "o": "model.layers.{i}.self_attn.o_proj.weight",
    "gate": "model.layers.{i}.mlp.gate_proj.weight",
    "up": "model.layers.{i}.mlp.up_proj.weight",
    "down": "model.layers.{i}.mlp.down_proj.weight",
    "in_norm": "model.layers.{i}.input_layernorm.weight",
    "post_norm": "model.layers.{i}.post_attention_layernorm.weight",
    "router": "model.layers.{i}.block_sparse_moe.gate.weight",
    "w1": "model.layers.{i}.block_sparse_moe.experts.{e}.w1.weight",  # gate
    "w3": "model.layers.{i}.block_sparse_moe.experts.{e}.w3.weight",  # up
    "w2": "model.layers.{i}.block_sparse_moe.experts.{e}.w2.weight",  # down
}


class _Reader:
    """Lazy safetensors reader over a (possibly sharded) checkpoint directory."""

    def __init__(self, path: str | Path):
        from safetensors import safe_open

        p = Path(path)
        idx = p / "model.safetensors.index.json"
        if idx.exists():
            wm = json.loads(idx.read_text())["weight_map"]
            files = sorted(set(wm.values()))
        else:
            files = [f.name for f in sorted(p.glob("*.safetensors"))]
            wm = None
        self.handles = {f: safe_open(str(p / f), framework="pt") for f in files}
        self.where = wm or {k: f for f, h in self.handles.items() for k in h.keys()}

    def has(self, name):
        return name in self.where

    def slice(self, name, rows=None, cols=None) -> torch.Tensor:
        s = self.handles[self.where[name]].get_slice(name)
        if rows is None and cols is None:
            return s[:]
        r = slice(None) if rows is None else slice(*rows)
        if cols is None:
            return s[r]
        return s[r, slice(*cols)]


def load_hf_checkpoint(path: str | Path, cfg: ModelConfig, tp: int = 1, rank: int = 0,
                       device="cpu", dtype=torch.bfloat16) -> dict:
    rd = _Reader(path)
    D = cfg.head_dim
    hq = cfg.num_heads // tp
    k0, k1 = _kv_head_range(cfg, tp, rank)
    vn = cfg.vocab_size // tp
    vr = (rank * vn, (rank + 1) * vn)

    def t(x):
        return x.to(device=device, dtype=dtype).contiguous()

    w = {"embed": t(rd.slice("model.embed_tokens.weight", vr)),
         "final_norm": t(rd.slice("model.norm.weight")), "layers": []}
    if cfg.tie_embeddings or not rd.has("lm_head.weight"):
        w["lm_head"] = w["embed"]
    else:
        w["lm_head"] = t(rd.slice("lm_head.weight", vr))
    for i in range(cfg.num_layers):
        n = {k: v.format(i=i, e="{e}") for k, v in _HF_LLAMA.items()}
        q = rd.slice(n["q"], (rank * hq * D, (rank + 1) * hq * D))
        k = rd.slice(n["k"], (k0 * D, k1 * D))
        v = rd.slice(n["v"], (k0 * D, k1 * D))
        layer = {"in_norm": t(rd.slice(n["in_norm"])), "post_norm": t(rd.slice(n["post_norm"])),
                 "qkv": t(torch.cat([q, k, v])),
                 "o": t(rd.slice(n["o"], None, (rank * hq * D, (rank + 1) * hq * D)))}
        if cfg.is_moe:
            E = cfg.num_experts
            ne = E // tp
            layer["router"] = t(rd.slice(n["router"]))
            gus, downs = [], []
            for e in range(rank * ne, (rank + 1) * ne):
                gus.append(torch.cat([rd.slice(n["w1"].format(e=e)),
                                      rd.slice(n["w3"].format(e=e))]))
                downs.append(rd.slice(n["w2"].format(e=e)))
            layer["experts_gate_up"] = t(torch.stack(gus))
            layer["experts_down"] = t(torch.stack(downs))
        else:
            inter = cfg.intermediate_size // tp
            ir = (rank * inter, (rank + 1) * inter)
            layer["gate_up"] = t(torch.cat([rd.slice(n["gate"], ir), rd.slice(n["up"], ir)]))
            layer["down"] = t(rd.slice(n["down"], None, ir))
        w["layers"].append(layer)
    return w


def config_from_hf(path: str | Path, name: str | None = None) -> ModelConfig:
    """Build a ModelConfig from an HF ``config.json`` (Llama / Mixtral)."""
    c = json.loads((Path(path) / "config.json").read_text())
    arch = "mixtral" if "mixtral" in c.get("model_type", "") else "llama"
    eos = c.get("eos_token_id", 2)
    heads = c["num_attention_heads"]
    return ModelConfig(
        name=name or Path(path).name, arch=arch, vocab_size=c["vocab_size"],
        hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"],
        num_layers=c["num_hidden_layers"], num_heads=heads,
        num_kv_heads=c.get("num_key_value_heads", heads),
        head_dim=c.get("head_dim", c["hidden_size"] // heads),
        rope_theta=float(c.get("rope_theta", 10000.0)), rope_scaling=c.get("rope_scaling"),
        rms_eps=float(c.get("rms_norm_eps", 1e-5)),
        max_position=c.get("max_position_embeddings", 8192),
        tie_embeddings=bool(c.get("tie_word_embeddings", False)),
        num_experts=c.get("num_local_experts", 0),
        experts_per_token=c.get("num_experts_per_tok", 0),
        bos_token_id=c.get("bos_token_id", 1),
        eos_token_ids=tuple(eos) if isinstance(eos, list) else (eos,))


def save_hf_checkpoint(w: dict, cfg: ModelConfig, path: str | Path):
    """Write a tp=1 weight dict as an HF-named safetensors checkpoint (round-trip
    testing and exporting random-init models)."""
    from safetensors.torch import save_file

    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    D, Q, K = cfg.head_dim, cfg.num_heads * cfg.head_dim, cfg.num_kv_heads * cfg.head_dim
    out = {"model.embed_tokens.weight": w["embed"], "model.norm.weight": w["final_norm"]}
    if not cfg.tie_embeddings:
        out["lm_head.weight"] = w["lm_head"]
    for i, l in enumerate(w["layers"]):
        n = {k: v.format(i=i, e="{e}") for k, v in _HF_LLAMA.items()}
        out[n["q"]], out[n["k"]], out[n["v"]] = l["qkv"][:Q], l["qkv"][Q:Q + K], l["qkv"][Q + K:]
        out[n["o"]] = l["o"]
        out[n["in_norm"]], out[n["post_norm"]] = l["in_norm"], l["post_norm"]
        if "router" in l:
            out[n["router"]] = l["router"]
            I = l["experts_down"].shape[2]
            for e in range(l["experts_gate_up"].shape[0]):
                out[n["w1"].format(e=e)] = l["experts_gate_up"][e, :I]
                out[n["w3"].format(e=e)] = l["experts_gate_up"][e, I:]
                out[n["w2"].format(e=e)] = l["experts_down"][e]
        else:
            I = l["down"].shape[1]
            out[n["gate"]], out[n["up"]] = l["gate_up"][:I], l["gate_up"][I:]
            out[n["down"]] = l["down"]
    save_file({k: v.contiguous().cpu() for k, v in out.items()}, str(p / "model.safetensors"))
    hf = {"model_type": "mixtral" if cfg.is_moe else "llama", "vocab_size": cfg.vocab_size,
          "hidden_size": cfg.hidden_size, "intermediate_size": cfg.intermediate_size,
          "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
          "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
          "rope_theta": cfg.rope_theta, "rope_scaling": cfg.rope_scaling,
          "rms_norm_eps": cfg.rms_eps, "max_position_embeddings": cfg.max_position,
          "tie_word_embeddings": cfg.tie_embeddings, "num_local_experts": cfg.num_experts,
          "num_experts_per_tok": cfg.experts_per_token, "bos_token_id": cfg.bos_token_id,
          "eos_token_id": list(cfg.eos_token_ids)}
    (p / "config.json").write_text(json.dumps(hf, indent=1))
