"""Mixtral-family sparse MoE forward (config 5).

Attention is the Llama block (TP-sharded heads, paged KV, same kernels); the FFN
is a top-2 router over E experts.  Experts are sharded across the TP group
(expert parallelism): after TP attention every rank holds the full hidden state,
runs its local experts on the tokens routed to them (device-side routing +
grouped MFMA GEMMs, :func:`omnia_amd.ops.moe`) and the per-layer all-reduce
that a dense TP MLP needs anyway combines the experts' contributions -- so EP
costs no extra collective over dense TP.  (Token all-to-all for DP-attention +
EP lives in :mod:`omnia_amd.parallel.expert`.)
"""
from __future__ import annotations

import math

import torch

from .. import ops
from .llama import LlamaModel, _init


class MixtralModel(LlamaModel):
    def __init__(self, cfg, *a, **kw):
        if not cfg.is_moe:
            raise ValueError("MixtralModel needs num_experts > 0")
        super().__init__(cfg, *a, **kw)
        if cfg.num_experts % self.tp:
            raise ValueError("num_experts must be divisible by the TP/EP size")
        self.e_local = cfg.num_experts // self.tp
        self.e_lo = self.tpr * self.e_local
        self.graph_safe = True  # flipped off by the runner for eager prefill

    def _random_mlp(self, g) -> dict:
        cfg, dev, dt, d = self.cfg, self.device, self.dtype, self.cfg.hidden_size
        E = cfg.num_experts // self.tp
        I = cfg.intermediate_size
        return {
            "router": _init((cfg.num_experts, d), 0.02, dev, dt, g),
            "experts_gate_up": _init((E, 2 * I, d), 0.02, dev, dt, g),
            "experts_down": _init((E, d, I), 0.02 / math.sqrt(2 * cfg.num_layers), dev, dt, g),
        }

    def mlp(self, layer: dict, h: torch.Tensor, is_decode: bool = False) -> torch.Tensor:
        return ops.moe(h, layer["router"], layer["experts_gate_up"], layer["experts_down"],
                       self.cfg.experts_per_token, self.cfg.num_experts, self.e_lo,
                       graph_safe=self.graph_safe or h.shape[0] < 64)

    def forward(self, fb, kv, gather: bool = True):
        # decode batches are captured into hipGraphs: keep the MoE path sync-free
        self.graph_safe = fb.is_decode
        return super().forward(fb, kv, gather)
