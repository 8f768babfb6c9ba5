"""Llama-3 family forward on the engine's paged KV cache (TP-aware).

Per layer (T tokens, hidden d):
    fused_add_rmsnorm -> QKV GEMM -> RoPE + paged KV write (HIP) ->
    paged attention (HIP prefill / decode) -> O GEMM [-> TP all-reduce] ->
    fused_add_rmsnorm -> gate_up GEMM + SwiGLU -> down GEMM [-> all-reduce]
GEMMs go through :func:`omnia_amd.ops.linear`: the hand MFMA decode kernel
(``ops/csrc/gemm.hip``, SwiGLU fused in its epilogue) on the shapes where the
MI355X sweep measured it faster, tuned hipBLASLt everywhere else.
Weights are kept in their natural [out, in] layout so ``F.linear`` maps onto a
single hipBLASLt GEMM; column-parallel shards (QKV, gate_up) and row-parallel
shards (O, down) follow Megatron.  The reference has no model code at all
(SURVEY §0.2); this replaces its remote Provider (``internal/runtime/provider.go:95-151``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as ref
from ..parallel import overlap
from ..parallel import state as pstate
from .config import ModelConfig

# decode attention: below this many (sequence, kv head) pairs a step splits every
# live context on the device (``LlamaModel.decode_part``)
DECODE_SPLIT_PAIRS = int(os.environ.get("OMNIA_DECODE_SPLIT_PAIRS", "256"))


@dataclass
class ForwardBatch:
    """Flattened step inputs.  All tensors live on the model device."""

    input_ids: torch.Tensor  # int32 [T]
    positions: torch.Tensor  # int32 [T]
    slots: torch.Tensor  # int64 [T]  flat KV slot of each token
    block_tables: torch.Tensor  # int32 [B, max_blocks]
    seq_lens: torch.Tensor  # int32 [B] total context incl. this step's tokens
    logits_indices: torch.Tensor  # int64 [B] rows of T whose logits are needed
    is_decode: bool = True
    q_start_loc: torch.Tensor | None = None  # int32 [B+1] (prefill)
    tile_seq: torch.Tensor | None = None  # int32 [n_tiles] (prefill)
    tile_q0: torch.Tensor | None = None
    num_seqs: int = 0
    # mixed step: the first ``num_decode`` tokens are decode rows (one token of a
    # running sequence each, attended by the decode kernel over dec_*), the rest
    # are prefill chunks described by q_start_loc / seq_lens / block_tables
    num_decode: int = 0
    dec_block_tables: torch.Tensor | None = None  # int32 [Bd, max_blocks]
    dec_seq_lens: torch.Tensor | None = None  # int32 [Bd]
    # decode rows whose input token is still on the device: tok_slots[ids_src[r]]
    # where ids_src[r] >= 0 (resolved inside the embedding kernel)
    ids_src: torch.Tensor | None = None
    tok_slots: torch.Tensor | None = None
    # context-parallel prefill (parallel/context_parallel.py CPPrefill): this
    # rank's zig-zag shard of one long prompt; K/V go to the CP scratch pages and
    # attention is the ring over the CP group
    cp: object = None


class Parts:
    """fp32 split-K partial slabs [S, M, N] of a projection (wgemm.hip MODE 2)."""

    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        self.t = t


class RowPar:
    """A deferred TP row-parallel projection ``x @ w.T`` (prefill): ``add_norm``
    runs it chunked along M with each chunk's all-reduce + residual + RMSNorm
    overlapped on a side stream (``parallel/overlap.py``)."""

    __slots__ = ("x", "w")

    def __init__(self, x: torch.Tensor, w: torch.Tensor):
        self.x, self.w = x, w


@dataclass
class KVCache:
    k: list  # per layer [NB, Hkv_local, BS, D]
    v: list
    block_size: int
    num_blocks: int

    @staticmethod
    def allocate(cfg: ModelConfig, num_blocks: int, block_size: int, device, tp_size: int = 1,
                 dtype=torch.bfloat16) -> "KVCache":
        hkv = max(1, cfg.num_kv_heads // tp_size)
        buf = torch.empty(cfg.num_layers, 2, num_blocks, hkv, block_size, cfg.head_dim,
                          dtype=dtype, device=device)
        return KVCache(k=[buf[i, 0] for i in range(cfg.num_layers)],
                       v=[buf[i, 1] for i in range(cfg.num_layers)],
                       block_size=block_size, num_blocks=num_blocks)


def _init(shape, std, device, dtype, gen):
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=gen)
    return t.to(dtype)


class LlamaModel:
    def __init__(self, cfg: ModelConfig, device="cpu", dtype=torch.bfloat16, seed: int = 0,
                 weights: dict | None = None, decode_part_size: int = 512):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        st = pstate.get_state()
        self.tp, self.tpr = st.tp_size, st.tp_rank
        if cfg.num_heads % self.tp:
            raise ValueError("num_heads not divisible by tp")
        self.hq = cfg.num_heads // self.tp
        self.hkv = max(1, cfg.num_kv_heads // self.tp)
        self.inter = cfg.intermediate_size // self.tp
        self.vocab_local = cfg.vocab_size // self.tp if cfg.vocab_size % self.tp == 0 else None
        if self.vocab_local is None:
            raise ValueError("vocab not divisible by tp")
        self.vocab_start = self.tpr * self.vocab_local
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.seed = seed
        self.decode_part_size = decode_part_size
        self.cos_sin = ref.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                        cfg.rope_scaling, device=self.device)
        self.w = weights if weights is not None else self._random_weights(seed)
        self.fold_norms()
        self._ws = {}
        ops.dgemm_prepare(self.device)  # split-K workspace, before any graph capture

    # ------------------------------------------------------------ weights
    def _random_weights(self, seed: int) -> dict:
        """Random-init shard of this TP rank (no checkpoint available offline).

        Std 0.02 like HF init; norms at 1.  Initialised directly on the device."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed * 1000 + self.tpr)
        d, D = cfg.hidden_size, cfg.head_dim
        w = {
            "embed": _init((self.vocab_local, d), 0.02, dev, dt, g),
            "final_norm": torch.ones(d, dtype=dt, device=dev),
            "layers": [],
        }
        w["lm_head"] = w["embed"] if cfg.tie_embeddings else _init((self.vocab_local, d), 0.02,
                                                                   dev, dt, g)
        for li in range(cfg.num_layers):
            layer = {
                "in_norm": torch.ones(d, dtype=dt, device=dev),
                "post_norm": torch.ones(d, dtype=dt, device=dev),
                "qkv": _init(((self.hq + 2 * self.hkv) * D, d), 0.02, dev, dt, g),
                "o": _init((d, self.hq * D), 0.02 / math.sqrt(2 * cfg.num_layers), dev, dt, g),
            }
            layer.update(self._random_mlp(g, li))
            w["layers"].append(layer)
        return w

    def _random_mlp(self, g, li: int = 0) -> dict:
        cfg, dev, dt, d = self.cfg, self.device, self.dtype, self.cfg.hidden_size
        return {
            "gate_up": _init((2 * self.inter, d), 0.02, dev, dt, g),
            "down": _init((d, self.inter), 0.02 / math.sqrt(2 * cfg.num_layers), dev, dt, g),
        }

    def weight_bytes(self) -> int:
        n = 0
        seen = set()

        def add(t):
            nonlocal n
            if isinstance(t, torch.Tensor) and t.data_ptr() not in seen:
                seen.add(t.data_ptr())
                n += t.numel() * t.element_size()

        for k, v in self.w.items():
            if k == "layers":
                for layer in v:
                    for t in layer.values():
                        if isinstance(t, list):
                            for x in t:
                                add(x)
                        else:
                            add(t)
            else:
                add(v)
        return n

    # RMSNorm(h) @ W^T == rsqrt(mean(h^2) + eps) * (h @ (W diag(w))^T): the norm
    # weight folds into the consumer's weight rows once at load, after which
    # every norm of the model is weightless.  The prefill path (pgemm.hip) then
    # applies the row scale in the QKV / gate_up epilogue from the row sums of
    # squares its producer (O / down residual epilogue) emits, and the decode /
    # TP / CP paths run their existing norm kernels with a ones weight.
    fold_post_norm = True  # Mixtral's post-attention norm also feeds the router

    def fold_norms(self) -> None:
        for layer in self.w["layers"]:
            pairs = [("in_norm", "qkv")]
            if self.fold_post_norm:
                pairs.append(("post_norm", "gate_up"))
            for nk, wk in pairs:
                nw = layer[nk]
                if bool(torch.all(nw == 1)):
                    continue
                W = layer[wk]
                layer[wk] = (W.float() * nw.float()[None, :]).to(W.dtype)
                layer[nk] = torch.ones_like(nw)

    # ------------------------------------------------------------ forward
    # Projections return either a bf16 tensor (library / gemm.hip path, not yet
    # TP-reduced) or :class:`Parts` (fp32 split-K slabs of the weight-streaming
    # kernel, wgemm.hip), which the NEXT kernel reduces while doing its own work:
    # QKV parts -> splitk_rope_kv (RoPE + paged KV write), O / down parts ->
    # splitk_add_rmsnorm (residual add + RMSNorm), gate_up parts -> splitk_swiglu.
    def _wcfg(self, M: int, N: int, K: int, mode: int, is_decode: bool):
        if self.device.type != "cuda":
            return None
        if not is_decode:
            # mid-size steps below the prefill tile's row threshold: split-K on
            # the 256x256 tile where the table lists a win (ops.midm_config)
            if self.tp == 1 and self.use_pgemm and M < self._min_rows:
                return ops.midm_config(M, N, K, mode)
            return None
        return ops.wgemm_config(M, N, K, mode)

    # tile-packed decode weights (ops.tgemm_pack): a second, stage-contiguous copy
    # of each projection the tuned table sends to tgemm.  Streamed alone, row-major
    # weights (128-B pieces of rows 2*K bytes apart) reach ~4.5 TB/s and packed
    # ones ~6.0 TB/s; inside the full kernel, next to the x re-reads and the
    # MFMAs, the gain is 0-3 % per projection (profiles/r5/decode_gemm/); end to
    # end the closed-loop bench gains +0.8 % tok/s and -2 % TPOT, 3 of 3
    # interleaved pairs (profiles/r6/bench/tgemm_pack/).  The copy (~14 GB for
    # Llama-3-8B, 5 % of HBM) is built before the KV pool is sized, by default
    # whenever it fits pack_budget_frac of HBM (70B TP=1 and MoE models: never);
    # OMNIA_TGEMM_PACK=0 turns it off.
    pack_budget_frac = 0.10  # of the device's HBM

    def prepack_decode(self, max_batch: int) -> int:
        """Pack the decode projections for every batch bucket up to ``max_batch``;
        returns the bytes packed (0: off / nothing on tgemm / over budget)."""
        self._packed = {}
        env = os.environ.get("OMNIA_TGEMM_PACK", "1")
        if env not in ("1", "force") or self.device.type != "cuda" or self.tp != 1 \
                or self.cfg.is_moe:
            return 0
        want = {}
        top = next((b for b in ops.WGEMM_BUCKETS if b >= max_batch), ops.WGEMM_BUCKETS[-1])
        for b in (b for b in ops.WGEMM_BUCKETS if b <= top):
            for layer in self.w["layers"]:
                for key, mode in (("qkv", 0), ("o", 0), ("down", 0), ("gate_up", 1)):
                    w = layer[key]
                    N = w.shape[0] // 2 if mode == 1 else w.shape[0]
                    cfg = ops.wgemm_config(b, N, w.shape[1], mode)
                    if cfg is None or cfg[1] >= 0 or (-1 - cfg[1]) & 2:
                        continue  # not tgemm, or its 32-k stage form
                    pmode = 1 if mode == 1 and cfg[2] == 1 else 0
                    want[(w.data_ptr(), cfg[0], pmode)] = w
        total = sum(w.numel() * w.element_size() for w in want.values())
        cap = torch.cuda.get_device_properties(self.device).total_memory * self.pack_budget_frac
        if not want or (env != "force" and total > cap):
            return 0
        for (ptr, bn, pmode), w in want.items():
            self._packed[(ptr, bn, pmode)] = ops.tgemm_pack(w, bn, pmode)
        return total

    # split-K slabs of the tile GEMM in fp16 (tgemm mode 3): half the slab bytes
    # the producer writes and the consumer (splitk.hip) reads; each slab is one
    # K-slice's fp32 sum rounded to 11 bits, finer than the bf16 rounding of the
    # projection output itself.  OMNIA_SPLITK_FP32=1 keeps fp32 slabs.
    splitk_half = os.environ.get("OMNIA_SPLITK_FP32", "0") != "1"

    def _slab_dtype(self, nwaves: int) -> torch.dtype:
        if nwaves == ops.PGEMM_SPLIT:
            return torch.float16  # the 256x256 split-K tile writes fp16 slabs only
        return torch.float16 if (self.splitk_half and nwaves < 0) else torch.float32

    def _wgemm(self, mode: int, x: torch.Tensor, w: torch.Tensor, S: int, nw: int, nwaves: int,
               out: torch.Tensor | None = None) -> torch.Tensor:
        """ops.wgemm, on the tile-packed copy of ``w`` when one exists for this
        tgemm config; split-K slabs in fp16 on the tile GEMM (``out``'s dtype)."""
        if nwaves == ops.PGEMM_SPLIT:
            return ops.pgemm_splitk(x, w, S, out)
        if nwaves < 0 and mode == 2 and out is not None and out.dtype == torch.float16:
            mode = 3
        packed = getattr(self, "_packed", None)
        if packed and nwaves < 0:
            wp = packed.get((w.data_ptr(), nw, 1 if mode == 1 else 0))
            if wp is not None:
                return ops.tgemm(mode, x, wp, S, nw, (-1 - nwaves) | 8, out)
        if mode == 3:
            return ops.tgemm(3, x, w, S, nw, -1 - nwaves, out)
        return ops.wgemm(mode, x, w, S, nw, nwaves, out=out)

    def _parts(self, tag, S: int, M: int, N: int,
               dtype: torch.dtype = torch.float32) -> torch.Tensor:
        if M > ops.WGEMM_MAX_M:  # mid-size steps: M varies per step, do not pin one per M
            return torch.empty(S, M, N, dtype=dtype, device=self.device)
        key = ("parts", tag, S, M, N, dtype)
        buf = self._ws.get(key)
        if buf is None:
            buf = torch.empty(S, M, N, dtype=dtype, device=self.device)
            self._ws[key] = buf
        return buf

    def _proj(self, tag, x: torch.Tensor, w: torch.Tensor, is_decode: bool):
        """Plain projection: Parts on the weight-streaming path, else bf16."""
        M, K = x.shape
        if tag in ("o", "down") and not is_decode and overlap.applies(M, x.device):
            return RowPar(x, w)
        if self._pgemm_ok(M, K, w.shape[0], is_decode):
            return ops.pgemm(0, x, w)
        cfg = self._wcfg(M, w.shape[0], K, 0, is_decode)
        if cfg is None:
            return ops.linear(x, w)
        nw, nwaves, S = cfg
        return Parts(self._wgemm(2, x, w, S, nw, nwaves,
                                 out=self._parts(tag, S, M, w.shape[0], self._slab_dtype(nwaves))))

    def add_norm(self, x, residual: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        """residual += x (TP-reduced); returns RMSNorm(residual) * w."""
        eps = self.cfg.rms_eps
        if isinstance(x, RowPar):
            return overlap.rowparallel_add_norm(x.x, x.w, residual, w, eps)
        if isinstance(x, Parts):
            if self.tp == 1:
                return ops.splitk_add_rmsnorm(x.t, residual, w, eps)
            x = ops.splitk_reduce(x.t)
        if self.tp > 1:
            return pstate.tp_all_reduce_add_rmsnorm(x, residual, w, eps)
        ops.fused_add_rmsnorm(x, residual, w, eps)
        return x

    _min_rows = int(os.environ.get("OMNIA_PGEMM_MIN_ROWS", "2049"))  # this forward's threshold (mixed steps: the higher one)

    def _pgemm_ok(self, M: int, K: int, N: int, is_decode: bool, tn: int = 256) -> bool:
        """A prefill-sized projection the hand 256x256 MFMA kernel covers (the
        unfused paths: TP shards, MoE attention, CP): K whole 128-k iterations,
        N whole column tiles, and at least this forward's row threshold."""
        # TP ranks rehearsed on ONE device (ipc transport) keep the library GEMMs:
        # a 256x256 tile's 132 KB of LDS cannot share a CU with the peers'
        # spinning all-reduce blocks, so a rank's GEMM can wait out their spin
        # bound (the comm.hip error flag) -- real TP has one rank per GPU
        return (self.use_pgemm and not is_decode and self.device.type == "cuda"
                and M >= self._min_rows and K % 128 == 0 and N % tn == 0
                and (self.tp == 1 or pstate.ranks_per_device() == 1))

    def mlp(self, layer: dict, h: torch.Tensor, is_decode: bool = False):
        M, K = h.shape
        I2 = layer["gate_up"].shape[0]
        if self._pgemm_ok(M, K, I2 // 2, is_decode, 128):
            # gate_up + SwiGLU in the prefill kernel's epilogue (pgemm EPI 1)
            return self._proj("down", ops.pgemm(1, h, layer["gate_up"]), layer["down"], False)
        cfg = self._wcfg(M, I2 // 2, K, 1, is_decode)
        if cfg is None:
            a = ops.linear_silu(h, layer["gate_up"])  # SwiGLU fused into decode GEMMs
        elif cfg[1] == ops.PGEMM_SPLIT and cfg[2] == 1:
            a = ops.pgemm(1, h, layer["gate_up"])  # mid-size step: the unsplit fused tile
        else:
            nw, nwaves, S = cfg
            if S == 1 and nwaves != ops.PGEMM_SPLIT:
                a = self._wgemm(1, h, layer["gate_up"], 1, nw, nwaves)
            else:
                a = ops.splitk_swiglu(self._wgemm(
                    2, h, layer["gate_up"], S, nw, nwaves,
                    out=self._parts("gu", S, M, I2, self._slab_dtype(nwaves))))
        return self._proj("down", a, layer["down"], is_decode)

    def attention(self, li: int, h: torch.Tensor, fb: ForwardBatch, kv: KVCache):
        T = h.shape[0]
        D = self.cfg.head_dim
        wqkv = self.w["layers"][li]["qkv"]
        if fb.cp is None and D == 128 and (self.hq + 2 * self.hkv) % 2 == 0 and \
                self._pgemm_ok(T, h.shape[1], wqkv.shape[0], fb.is_decode):
            # QKV + RoPE + paged KV write in the prefill kernel's epilogue (pgemm
            # EPI 3, no row scale: h is already normalised on this path)
            q = ops.pgemm(3, h, wqkv, positions=fb.positions, cos_sin=self.cos_sin,
                          k_cache=kv.k[li], v_cache=kv.v[li], slots=fb.slots, hq=self.hq,
                          hkv=self.hkv, block_size=kv.block_size)
            q3 = q.view(T, self.hq, D)
            if fb.num_decode:
                o = self._mixed_attention(li, q3, fb, kv)
            else:
                o = ops.prefill_attention(q3, kv.k[li], kv.v[li], fb.block_tables,
                                          fb.q_start_loc, fb.seq_lens, self.scale, fb.tile_seq,
                                          fb.tile_q0)
            return self._proj("o", o.view(T, self.hq * D), self.w["layers"][li]["o"], False)
        qkv = self._proj("qkv", h, wqkv, fb.is_decode)
        if fb.cp is not None:
            cp = fb.cp
            q = qkv[:, : self.hq * D]
            ops.rope_kv(q, qkv[:, self.hq * D: (self.hq + self.hkv) * D],
                        qkv[:, (self.hq + self.hkv) * D:], fb.positions, self.cos_sin,
                        cp.scratch[0], cp.scratch[1], fb.slots, self.hq, self.hkv, cp.bs)
            o = cp.attention(kv.k[li], kv.v[li], q.view(T, self.hq, D), self.scale)
            return self._proj("o", o.view(T, self.hq * D), self.w["layers"][li]["o"], False)
        if isinstance(qkv, Parts):
            q = ops.splitk_rope_kv(qkv.t, fb.positions, self.cos_sin, kv.k[li], kv.v[li],
                                   fb.slots, self.hq, self.hkv, kv.block_size)
        else:
            q = qkv[:, : self.hq * D]
            k = qkv[:, self.hq * D: (self.hq + self.hkv) * D]
            v = qkv[:, (self.hq + self.hkv) * D:]
            ops.rope_kv(q, k, v, fb.positions, self.cos_sin, kv.k[li], kv.v[li], fb.slots,
                        self.hq, self.hkv, kv.block_size)
        q3 = q.view(T, self.hq, D)
        if fb.is_decode:
            part, splits = self.decode_part(T, fb.block_tables.shape[1] * kv.block_size)
            ws = self._decode_ws(T, fb.block_tables.shape[1], kv.block_size, h.device, part,
                                 splits)
            o = ops.decode_attention(q3, kv.k[li], kv.v[li], fb.block_tables, fb.seq_lens,
                                     self.scale, part_size=part, workspace=ws, splits=splits)
        elif fb.num_decode:
            o = self._mixed_attention(li, q3, fb, kv)
        else:
            o = ops.prefill_attention(q3, kv.k[li], kv.v[li], fb.block_tables, fb.q_start_loc,
                                      fb.seq_lens, self.scale, fb.tile_seq, fb.tile_q0)
        return self._proj("o", o.view(T, self.hq * D), self.w["layers"][li]["o"], fb.is_decode)

    def _mixed_attention(self, li: int, q3: torch.Tensor, fb: ForwardBatch, kv: KVCache):
        """Mixed step: decode rows (the first ``num_decode``) on the split-K decode
        kernel (K/V read once per GQA group), prefill chunks on the flash prefill
        kernel, one output."""
        T, D = q3.shape[0], self.cfg.head_dim
        Bd = fb.num_decode
        o = torch.empty_like(q3) if q3.is_contiguous() else torch.empty(
            T, self.hq, D, dtype=q3.dtype, device=q3.device)
        mb = fb.dec_block_tables.shape[1]
        part, splits = self.decode_part(Bd, mb * kv.block_size)
        ws = self._decode_ws(1 << max(0, Bd - 1).bit_length(), mb, kv.block_size, q3.device,
                             part, splits)  # pow2 rows: few workspace shapes across mixed steps
        ops.decode_attention(q3[:Bd], kv.k[li], kv.v[li], fb.dec_block_tables,
                             fb.dec_seq_lens, self.scale, part_size=part, workspace=ws,
                             out=o[:Bd], splits=splits)
        if T > Bd:
            ops.prefill_attention(q3[Bd:], kv.k[li], kv.v[li], fb.block_tables,
                                  fb.q_start_loc, fb.seq_lens, self.scale, fb.tile_seq,
                                  fb.tile_q0, out=o[Bd:])
        return o

    def decode_part(self, batch: int, max_ctx: int) -> tuple[int, int]:
        """(partition length, splits) of the split-K decode attention.

        With >= DECODE_SPLIT_PAIRS (sequence, kv head) pairs the pairs alone fill
        the chip: partitions as long as possible (fewer partials to merge, no
        merge kernel when one partition covers the context) while keeping
        >= ~2048 workgroups.  With fewer pairs (small batches, one KV head per TP
        rank) every live context is cut on the device into up to ``splits``
        equal partitions (``ops.decode_attention``), so short contexts still
        spread over the CUs; the captured graph needs no host-known length."""
        pairs = batch * self.hkv
        if 0 < pairs < DECODE_SPLIT_PAIRS:
            splits = -(-DECODE_SPLIT_PAIRS // pairs)
            splits = max(1, min(splits, -(-max_ctx // ops.DECODE_SPLIT_MIN)))
            return self.decode_part_size, splits
        part = self.decode_part_size
        while part < 2048 and part < max_ctx and \
                batch * self.hkv * ((max_ctx + 2 * part - 1) // (2 * part)) >= 2048:
            part *= 2
        return part, 0

    def _decode_ws(self, B, max_blocks, bs, device, part, splits=0):
        key = (B, max_blocks, bs, str(device), part, splits)
        ws = self._ws.get(key)
        if ws is None:
            if device.type != "cuda":
                return None
            ws = ops.decode_workspace(B, self.hq, max_blocks, bs, part, device, splits)
            self._ws[key] = ws
        return ws

    def embed(self, ids: torch.Tensor, src: torch.Tensor | None = None,
              tok_slots: torch.Tensor | None = None) -> torch.Tensor:
        h = ops.embedding(ids, self.w["embed"], self.vocab_start, src=src, tok_slots=tok_slots)
        return pstate.tp_all_reduce(h) if self.tp > 1 else h

    # ------------------------------------------------ fused prefill (pgemm.hip)
    use_pgemm = os.environ.get("OMNIA_PGEMM", "1") != "0"
    # prefill chunks take the fused layer from this many rows.  Below it the
    # unsplit 256x256 tile leaves most CUs idle on qkv / o / down; the unfused
    # path runs them split-K on the same tile (ops.midm_config) and is 1.2-2.2x
    # faster per layer at 512-2048 rows (profiles/r6/open/)
    PGEMM_MIN_ROWS = int(os.environ.get("OMNIA_PGEMM_MIN_ROWS", "2049"))
    # mixed steps take the fused layer only from this many rows: at the open-loop
    # trickle (~256 decode rows + a few hundred prompt tokens) pgemm's 256x256
    # tiles leave most CUs idle, and the split decode / library path is 1.5x
    # faster per step (profiles/r5/mixed_open_loop/: p50 TPOT 14.9 vs 22.9 ms)
    PGEMM_MIXED_MIN_ROWS = int(os.environ.get("OMNIA_PGEMM_MIXED_MIN_ROWS", "4096"))

    def _use_fused(self, fb: ForwardBatch) -> bool:
        """Prefill chunks -- and mixed steps, whose decode rows ride the same
        GEMMs -- on one GPU run the fused-epilogue prefill layer: QKV+RoPE+KV-write,
        O+residual, gate_up+SwiGLU, down+residual, with the RMSNorms riding the
        epilogues (no standalone norm / SwiGLU / RoPE launch)."""
        if not (self.use_pgemm and self.device.type == "cuda" and not fb.is_decode
                and fb.cp is None and self.tp == 1):
            return False
        T = fb.input_ids.shape[0]
        if T < (self.PGEMM_MIXED_MIN_ROWS if fb.num_decode else self.PGEMM_MIN_ROWS):
            return False
        cfg, d = self.cfg, self.cfg.hidden_size
        return (cfg.head_dim == 128 and d % 256 == 0 and d % 128 == 0
                and (self.hq + 2 * self.hkv) % 2 == 0
                and self.inter % 128 == 0
                and self.fold_post_norm and not self.cfg.is_moe)

    def _fused_residual(self, fb: ForwardBatch, kv: KVCache) -> torch.Tensor:
        """Residual stream after the last layer (un-normalised) of a prefill chunk."""
        cfg = self.cfg
        T, d, D = fb.input_ids.shape[0], cfg.hidden_size, cfg.head_dim
        inv_d, eps = 1.0 / d, cfg.rms_eps
        h = self.embed(fb.input_ids)
        ss = ops.row_sumsq(h).view(T, 1)
        nsl = d // 256
        ss_mid = torch.empty(T, nsl, dtype=torch.float32, device=h.device)
        ss_out = torch.empty(T, nsl, dtype=torch.float32, device=h.device)
        q = torch.empty(T, self.hq * D, dtype=h.dtype, device=h.device)
        act = torch.empty(T, self.inter, dtype=h.dtype, device=h.device)
        for li, layer in enumerate(self.w["layers"]):
            ops.pgemm(3, h, layer["qkv"], out=q, ss_in=ss, inv_d=inv_d, eps=eps,
                      positions=fb.positions, cos_sin=self.cos_sin, k_cache=kv.k[li],
                      v_cache=kv.v[li], slots=fb.slots, hq=self.hq, hkv=self.hkv,
                      block_size=kv.block_size)
            if fb.num_decode:
                o = self._mixed_attention(li, q.view(T, self.hq, D), fb, kv)
            else:
                o = ops.prefill_attention(q.view(T, self.hq, D), kv.k[li], kv.v[li],
                                          fb.block_tables, fb.q_start_loc, fb.seq_lens,
                                          self.scale, fb.tile_seq, fb.tile_q0)
            ops.pgemm(2, o.view(T, self.hq * D), layer["o"], out=h, ss_out=ss_mid)
            ops.pgemm(1, h, layer["gate_up"], out=act, ss_in=ss_mid, inv_d=inv_d, eps=eps)
            ops.pgemm(2, act, layer["down"], out=h, ss_out=ss_out)
            ss = ss_out  # the next QKV reads it before the next down overwrites it
        return h

    def hidden_states(self, fb: ForwardBatch, kv: KVCache) -> torch.Tensor:
        cfg = self.cfg
        if self._use_fused(fb):
            return ops.rmsnorm(self._fused_residual(fb, kv), self.w["final_norm"], cfg.rms_eps)
        self._min_rows = self.PGEMM_MIXED_MIN_ROWS if fb.num_decode else self.PGEMM_MIN_ROWS
        residual = self.embed(fb.input_ids, fb.ids_src, fb.tok_slots)
        h = ops.rmsnorm(residual, self.w["layers"][0]["in_norm"], cfg.rms_eps)
        m = None
        for li, layer in enumerate(self.w["layers"]):
            if li > 0:
                h = self.add_norm(m, residual, layer["in_norm"])
            a = self.attention(li, h, fb, kv)
            h = self.add_norm(a, residual, layer["post_norm"])
            m = self.mlp(layer, h, fb.is_decode)
        return self.add_norm(m, residual, self.w["final_norm"])

    def logits(self, h: torch.Tensor, gather: bool = True,
               is_decode: bool = False) -> torch.Tensor:
        """LM head.  Under TP the result is this rank's vocab slice unless
        ``gather`` (the distributed sampler, parallel/tp_sampling.py, needs
        only the slice).  Decode batches use the weight-streaming tile kernel
        when the measured table lists an unsplit (bf16-out) config for it."""
        W = self.w["lm_head"]
        cfg = self._wcfg(h.shape[0], W.shape[0], h.shape[1], 0, is_decode)
        if cfg is not None and cfg[2] == 1:
            lg = ops.wgemm(0, h, W, 1, cfg[0], cfg[1])
        else:
            lg = ops.linear(h, W)
        return pstate.tp_all_gather_lastdim(lg) if (self.tp > 1 and gather) else lg

    def forward(self, fb: ForwardBatch, kv: KVCache, gather: bool = True) -> torch.Tensor:
        if self._use_fused(fb):
            h = self._fused_residual(fb, kv).index_select(0, fb.logits_indices)
            return self.logits(ops.rmsnorm(h, self.w["final_norm"], self.cfg.rms_eps), gather,
                               False)
        h = self.hidden_states(fb, kv)
        # decode rows are their own logits rows (logits_indices is the identity)
        sel = h if fb.is_decode and fb.logits_indices.shape[0] == h.shape[0] else \
            h.index_select(0, fb.logits_indices)
        return self.logits(sel, gather, fb.is_decode)
