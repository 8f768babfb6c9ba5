"""Mixtral-family sparse MoE forward (config 5).

Attention is the Llama block (paged KV, same kernels); the FFN is a top-2
router over E experts on the grouped MFMA kernels (``ops/csrc/moe.hip``).
Two expert-parallel layouts (``ep_mode``):

* ``"tp"`` (default) -- EP inside TP: attention is TP-sharded, so after it every
  rank holds the full hidden state; each rank runs its local experts on the
  tokens routed to them and the per-layer all-reduce a dense TP MLP needs anyway
  combines the experts' contributions -- EP costs no extra collective.
* ``"a2a"`` -- DP attention + EP: every rank is a data-parallel replica for
  attention (tp = 1, its own batch / KV / scheduler) and holds E/ep experts;
  tokens travel to their experts' rank and back through the fixed-capacity,
  sync-free all-to-all of :mod:`omnia_amd.parallel.expert` (graph-safe decode).
  The engine runs the replicas in lockstep (``engine/ep.py``).

Expert weights are drawn per (layer, global expert) and the router per layer,
so any sharding of the same seed is a slice of one model: the EP ranks compose
exactly to the single-rank oracle.
"""
from __future__ import annotations

import math

import torch

from .. import ops
from ..parallel import state as pstate
from .llama import LlamaModel, _init


class MixtralModel(LlamaModel):
    fold_post_norm = False  # the post-attention norm feeds the router and every expert

    def __init__(self, cfg, *a, ep_mode: str = "tp", **kw):
        if not cfg.is_moe:
            raise ValueError("MixtralModel needs num_experts > 0")
        st = pstate.get_state()
        self.ep_mode = ep_mode
        if ep_mode == "a2a":
            if st.tp_size != 1:
                raise ValueError("ep_mode a2a runs data-parallel attention (tp must be 1)")
            self.ep, self.ep_rank, self.ep_group = st.dp_size, st.dp_rank, st.dp_group
        elif ep_mode == "tp":
            self.ep, self.ep_rank, self.ep_group = st.tp_size, st.tp_rank, st.tp_group
        else:
            raise ValueError(f"unknown ep_mode {ep_mode!r}")
        if cfg.num_experts % self.ep:
            raise ValueError("num_experts must be divisible by the EP size")
        self.e_local = cfg.num_experts // self.ep
        self.e_lo = self.ep_rank * self.e_local
        self.ep_tokens = 0  # step-global token count (a2a capacity), set by the EP runner
        self._ep_layers: dict = {}
        super().__init__(cfg, *a, **kw)
        self.graph_safe = True  # flipped off by the runner for eager prefill

    def _random_mlp(self, g, li: int = 0) -> dict:
        cfg, dev, dt, d = self.cfg, self.device, self.dtype, self.cfg.hidden_size
        I = cfg.intermediate_size

        def gen(tag: int):
            return torch.Generator(device=dev).manual_seed(
                (self.seed * 1_000_003 + li * 4099 + tag) & 0x7FFFFFFF)

        gu = torch.empty(self.e_local, 2 * I, d, dtype=dt, device=dev)
        dn = torch.empty(self.e_local, d, I, dtype=dt, device=dev)
        for j in range(self.e_local):
            ge = gen(1 + self.e_lo + j)
            gu[j] = _init((2 * I, d), 0.02, dev, dt, ge)
            dn[j] = _init((d, I), 0.02 / math.sqrt(2 * cfg.num_layers), dev, dt, ge)
        return {"router": _init((cfg.num_experts, d), 0.02, dev, dt, gen(0)),
                "experts_gate_up": gu, "experts_down": dn}

    def mlp(self, layer: dict, h: torch.Tensor, is_decode: bool = False) -> torch.Tensor:
        if self.ep_mode == "a2a":
            from ..parallel.expert import ExpertParallelMoE

            key = id(layer)
            moe = self._ep_layers.get(key)
            if moe is None:
                moe = self._ep_layers[key] = ExpertParallelMoE(
                    layer["router"], layer["experts_gate_up"], layer["experts_down"],
                    self.cfg.experts_per_token, group=self.ep_group,
                    comm=pstate.get_state().dp_comm)
            return moe(h, tokens=self.ep_tokens)
        return ops.moe(h, layer["router"], layer["experts_gate_up"], layer["experts_down"],
                       self.cfg.experts_per_token, self.cfg.num_experts, self.e_lo,
                       graph_safe=self.graph_safe or h.shape[0] < 64)

    def forward(self, fb, kv, gather: bool = True):
        # decode batches are captured into hipGraphs: keep the MoE path sync-free
        self.graph_safe = fb.is_decode
        return super().forward(fb, kv, gather)
