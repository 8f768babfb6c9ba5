"""Kernel front-end for the in-node engine.

On a GPU tensor every op runs the hand-written gfx950 HIP kernel from
``_omnia_kernels.so`` -- and fails LOUDLY if the extension is missing (a silent
eager fallback would hide a broken build).  On CPU tensors the plain-PyTorch
reference in :mod:`omnia_amd.ops.reference` runs instead (the CPU test-suite and
the mock/CPU engine path).
"""
from __future__ import annotations

import importlib
import os
import threading

import torch
import torch.nn.functional as F

from . import checks
from . import reference as ref

_lock = threading.Lock()
_ext = None
_ext_err: Exception | None = None


def kernels():
    """Return the loaded extension module, building it in-tree on first use if needed."""
    global _ext, _ext_err
    if _ext is not None:
        return _ext
    with _lock:
        if _ext is not None:
            return _ext
        try:
            _ext = importlib.import_module("omnia_amd.ops._omnia_kernels")
        except ImportError as e:  # pragma: no cover - exercised on fresh checkouts
            if os.environ.get("OMNIA_NO_AUTOBUILD"):
                _ext_err = e
                raise RuntimeError(
                    "omnia_amd HIP extension not built; run `python -m omnia_amd.ops.build`"
                ) from e
            from .build import build

            build(verbose=True)
            _ext = importlib.import_module("omnia_amd.ops._omnia_kernels")
        # prefill GEMM main loop: 1 = 4-wave (one wave per SIMD), 0 = 8-wave ping-pong
        sched = os.environ.get("OMNIA_PGEMM_SCHED")
        if sched is not None and hasattr(_ext, "pgemm_set_schedule"):
            _ext.pgemm_set_schedule(int(sched))
    return _ext


def extension_available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False


# --------------------------------------------------------------------- ops
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    if x.is_cuda:
        out = torch.empty_like(x) if out is None else out
        kernels().rmsnorm(out, x, w, eps)
        return out
    r = ref.rmsnorm(x, w, eps)
    if out is not None:
        out.copy_(r)
        return out
    return r


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """In place: residual += x; x = rmsnorm(residual) * w.  Returns (x, residual)."""
    if x.is_cuda:
        kernels().fused_add_rmsnorm(x, residual, w, eps)
        return x, residual
    y, r = ref.fused_add_rmsnorm(x, residual, w, eps)
    x.copy_(y)
    residual.copy_(r)
    return x, residual


def rope_kv(q, k, v, positions, cos_sin, k_cache, v_cache, slots, hq, hkv, block_size):
    """Rotate q/k in place (neox) and write k/v rows into the paged cache at `slots`."""
    if q.is_cuda:
        if checks.active(q):
            checks.slots("rope_kv", slots, k_cache)
        kernels().rope_kv(q, k, v, positions, cos_sin, k_cache, v_cache, slots, hq, hkv,
                          block_size)
        return
    T = q.shape[0]
    D = q.shape[1] // hq
    qr = ref.apply_rope(q.view(T, hq, D), positions, cos_sin)
    kr = ref.apply_rope(k.reshape(T, hkv, D), positions, cos_sin)
    q.copy_(qr.view(T, hq * D))
    k.copy_(kr.reshape(T, hkv * D))
    if slots is not None:
        ref.write_kv(k_cache, v_cache, kr, v.reshape(T, hkv, D), slots)


# ------------------------------------------------------- decode GEMM (K3/K8/K9/K10)
DGEMM_MAX_M = 256
_DGEMM_WS_FLOATS = 16 << 20  # 64 MiB of split-K slabs per device
_DGEMM_CNT = 8192
_dgemm_ws: dict = {}
_dgemm_table: dict | None = None
_dgemm_on = os.environ.get("OMNIA_DGEMM", "1") != "0"
_dgemm_force = os.environ.get("OMNIA_DGEMM", "") == "force"


def dgemm_prepare(device) -> None:
    """Allocate the split-K workspace + zeroed tile counters for ``device``.

    Call eagerly (model init) so nothing is allocated while a hipGraph captures."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _dgemm_ws:
        _dgemm_ws[key] = (torch.empty(_DGEMM_WS_FLOATS, dtype=torch.float32, device=dev),
                          torch.zeros(_DGEMM_CNT, dtype=torch.int32, device=dev))


def _dgemm_tuned() -> dict:
    global _dgemm_table
    if _dgemm_table is None:
        import json

        p = os.path.join(os.path.dirname(__file__), "tuned", "dgemm_mi355x.json")
        tab = {}
        if os.path.exists(p):
            with open(p) as f:
                for k, v in json.load(f).items():
                    tab[k] = tuple(v)
        _dgemm_table = tab
    return _dgemm_table


DGEMM_BUCKETS = (8, 32, 64, 128, 256)


def dgemm_bucket(M: int) -> int:
    for b in DGEMM_BUCKETS:
        if M <= b:
            return b
    return 0


def dgemm_config(M: int, N: int, K: int, mode: int, force: bool | None = None
                 ) -> tuple[int, int, int] | None:
    """(wm, wn, splits) for a decode GEMM, or None to use hipBLASLt.

    Dispatch is measured, not assumed: ``ops/tuned/dgemm_mi355x.json`` (written
    by ``scripts/dgemm_sweep.py`` on an MI355X, keyed ``mode:Mbucket:N:K``) lists
    the shapes where the hand kernel beat the tuned hipBLASLt solution; every
    other shape stays on the library.  ``force`` (or ``OMNIA_DGEMM=force``) uses
    the heuristic config for any covered shape (tests, sweeps)."""
    if M < 1 or M > DGEMM_MAX_M or K % 64:
        return None
    wm = 1 if M <= 64 else 2 if M <= 128 else 4
    hit = _dgemm_tuned().get(f"{mode}:{dgemm_bucket(M)}:{N}:{K}")
    if hit is not None:
        return tuple(hit)
    if not (force if force is not None else _dgemm_force):
        return None
    wn = 2
    cols = 64 * wn if mode == 0 else 32 * wn
    if N % cols:
        wn = 1
        cols = 64 if mode == 0 else 32
        if N % cols:
            return None
    tiles = N // cols
    s = 1
    while (tiles * s < 256 and s < 8 and K % (64 * s * 2) == 0
           and N * (s * 2) * 64 * wm * ((M + 64 * wm - 1) // (64 * wm))
           * (1 if mode == 0 else 2) <= _DGEMM_WS_FLOATS):
        s *= 2
    return wm, wn, s


def _dgemm(mode: int, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None):
    if not (_dgemm_on and x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.is_contiguous()):
        return None
    M, K = x.shape
    N = w.shape[0] if mode == 0 else w.shape[0] // 2
    cfg = dgemm_config(M, N, K, mode)
    if cfg is None:
        return None
    key = x.device.index if x.device.index is not None else torch.cuda.current_device()
    if key not in _dgemm_ws:
        dgemm_prepare(x.device)
    ws, cnt = _dgemm_ws[key]
    x = x.contiguous()
    out = x.new_empty(M, N) if out is None else out
    wm, wn, s = cfg
    kernels().dgemm(mode, out, x, w, ws, cnt, s, wm, wn)
    return out


# ------------------------------------------ weight-streaming decode GEMM (wgemm.hip)
WGEMM_MAX_M = 256


_wgemm_table: dict | None = None
_wgemm_on = os.environ.get("OMNIA_WGEMM", "1") != "0"
WGEMM_BUCKETS = (16, 32, 64, 128, 192, 256)
PGEMM_SPLIT = -64  # table nwaves code: pgemm 256x256 split-K tile, fp16 slabs


def wgemm_config(M: int, N: int, K: int, mode: int) -> tuple[int, int, int] | None:
    """(nw, nwaves, splits) of the weight-streaming kernel for a decode projection
    (nwaves == 0 selects the wide-batch 32x32x16 kernel, wgemm_wide.hip, with nw
    32-column tiles per wave; nwaves < 0 the full-batch tile kernel, tgemm.hip,
    with nw weight rows per block and non-temporal weight loads when -2;
    nwaves == PGEMM_SPLIT the 256x256 split-K tile, pgemm.hip EPI 4),
    or None to keep the library / gemm.hip path.  ``mode`` 0 = plain projection
    (its split-K slabs are reduced by the consumer kernel), 1 = gate_up + SwiGLU.
    Measured dispatch: ``ops/tuned/wgemm_mi355x.json`` (scripts/wgemm_sweep.py +
    scripts/wgemm_table.py) lists only the shapes where it won on an MI355X."""
    global _wgemm_table
    if not _wgemm_on or M < 1 or M > WGEMM_MAX_M:
        return None
    if _wgemm_table is None:
        import json

        p = os.path.join(os.path.dirname(__file__), "tuned", "wgemm_mi355x.json")
        _wgemm_table = {}
        if os.path.exists(p):
            with open(p) as f:
                _wgemm_table = {k: tuple(v) for k, v in json.load(f).items()}
    b = next(x for x in WGEMM_BUCKETS if M <= x)
    cfg = _wgemm_table.get(f"{mode}:{b}:{N}:{K}")
    if cfg is None and b == 192:  # the 192 bucket only lists its own wins
        cfg = _wgemm_table.get(f"{mode}:256:{N}:{K}")
    return cfg


MIDM_BUCKETS = (512, 768, 1024, 1536, 2048, 3072, 4096)
_midm_table: dict | None = None
_midm_on = os.environ.get("OMNIA_MIDM", "1") != "0"


def midm_config(M: int, N: int, K: int, mode: int) -> tuple[int, int, int] | None:
    """Mid-size projections (M = 257..4096 rows: open-loop mixed steps, which
    the unsplit 256x256 prefill tile under-fills): ``(256, PGEMM_SPLIT, S)``
    when ``ops/tuned/midm_mi355x.json`` lists a split-K win of the 256x256 tile
    (+ its slab consumer) over the library path for this shape's M bucket
    (``scripts/midm_sweep.py``), else None (library GEMM)."""
    global _midm_table
    if not (_wgemm_on and _midm_on) or M <= WGEMM_MAX_M or M > MIDM_BUCKETS[-1]:
        return None
    if _midm_table is None:
        import json

        p = os.path.join(os.path.dirname(__file__), "tuned", "midm_mi355x.json")
        _midm_table = {}
        if os.path.exists(p):
            with open(p) as f:
                _midm_table = {k: int(v) for k, v in json.load(f).items()}
    b = next(x for x in MIDM_BUCKETS if M <= x)
    S = _midm_table.get(f"{mode}:{b}:{N}:{K}")
    return (256, PGEMM_SPLIT, S) if S else None


def wgemm(mode: int, x: torch.Tensor, w: torch.Tensor, splits: int = 1, nw: int = 2,
          nwaves: int = 4, out: torch.Tensor | None = None) -> torch.Tensor:
    """Decode GEMM with W streamed HBM -> MFMA registers (``csrc/wgemm.hip``).

    mode 0: bf16 ``x @ w.T``; mode 1: bf16 ``silu(x Wg^T) * (x Wu^T)`` with
    ``w = [Wg; Wu]``; mode 2: fp32 split-K partial slabs ``[splits, M, N]`` whose
    sum is ``x @ w.T`` (reduced by the consumer kernel)."""
    if nwaves == PGEMM_SPLIT:  # table code for the 256x256 split-K tile (pgemm.hip EPI 4)
        if mode not in (2, 3):
            raise ValueError("the pgemm split-K table entry produces fp16 slabs (mode 2/3)")
        return pgemm_splitk(x, w, splits, out)
    if nwaves == 0:  # table code for the wide-batch kernel: nw = 32-col tiles per wave
        return wgemm_wide(mode, x, w, splits, nw, out)
    if nwaves < 0:  # table code for the full-batch tile kernel: nw = weight rows per block,
        # -1 - nwaves = tgemm flags (bit 0 non-temporal W, bit 1 32-k stages)
        return tgemm(mode, x, w, splits, nw, -1 - nwaves, out)
    M, K = x.shape
    N = w.shape[0] // 2 if mode == 1 else w.shape[0]
    if out is None:
        out = (torch.empty(splits, M, N, dtype=torch.float32, device=x.device) if mode == 2
               else x.new_empty(M, N))
    kernels().wgemm(mode, out, x.contiguous(), w, splits, nw, nwaves)
    return out


def wgemm_wide(mode: int, x: torch.Tensor, w: torch.Tensor, splits: int = 1, wt: int = 2,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """Wide-batch (128 < M <= 256) weight-streaming decode GEMM on 32x32x16 MFMA
    (``csrc/wgemm_wide.hip``); same modes and outputs as :func:`wgemm`."""
    M, K = x.shape
    N = w.shape[0] // 2 if mode == 1 else w.shape[0]
    if out is None:
        out = (torch.empty(splits, M, N, dtype=torch.float32, device=x.device) if mode == 2
               else x.new_empty(M, N))
    kernels().wgemm_wide(mode, out, x.contiguous(), w, splits, wt)
    return out


def tgemm(mode: int, x: torch.Tensor, w: torch.Tensor, splits: int = 1, bn: int = 128,
          wnt: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
    """Tile GEMM (``csrc/tgemm.hip``; mode 3 = mode 2's split-K slabs in fp16):
    decode batches (M <= 256, one block owns all
    rows x ``bn`` weight rows) and prefill chunks (256-row tiles), both operands LDS-DMA staged through an
    NS-deep ring with counted waits.  Same modes / outputs as :func:`wgemm`
    (mode 1 = fused SwiGLU needs ``splits == 1``).  ``wnt`` bit 0: non-temporal
    weight loads; bit 1: 32-k ring stages (twice the stages in flight, BN >= 128)."""
    M, K = x.shape
    N = w.shape[0] // 2 if mode == 1 else w.shape[0]
    if out is None:
        out = (torch.empty(splits, M, N, device=x.device,
                           dtype=torch.float32 if mode == 2 else torch.float16) if mode >= 2
               else x.new_empty(M, N))
    if not x.is_cuda:
        r = x.float() @ w.float().t()
        if mode == 1:
            r = ref.silu_mul(r.to(x.dtype)).float()
        if mode >= 2:
            out.zero_()
            out[0].copy_(r)
        else:
            out.copy_(r.to(out.dtype))
        return out
    kernels().tgemm(mode, out, x.contiguous(), w, splits, bn, wnt)
    return out


def tgemm_pack(w: torch.Tensor, bn: int, mode: int) -> torch.Tensor:
    """``w`` [R, K] re-laid for ``tgemm`` (wnt bit 3): [tile][k-stage][bn rows][64],
    the rows of each tile in the kernel's order (mode 1: every wave's gate rows
    then the matching up rows of W = [Wg; Wu]) and each row's eight 16-B chunks
    pre-permuted by the LDS bank swizzle (stored chunk p = chunk p ^ (row & 7)),
    so one k-stage of a tile is one contiguous run the LDS-DMA reads lane by
    lane.  Returned with the original [R, K] shape (same elements, new order)."""
    R, K = w.shape
    BK = 64
    if K % BK:
        raise ValueError("tgemm_pack: K must be a multiple of 64")
    nk = K // BK
    wtn = bn // (4 if bn >= 256 else 2)
    dev = w.device
    rr = torch.arange(bn, device=dev)
    if mode == 1:
        N = R // 2
        ntiles = N // (bn // 2)
        wv, q = rr // wtn, rr % wtn
        f0 = torch.arange(ntiles, device=dev)[:, None] * (bn // 2) + (wv * (wtn // 2))[None, :]
        rows = torch.where((q < wtn // 2)[None, :], f0 + q[None, :], N + f0 + (q - wtn // 2)[None, :])
    else:
        ntiles = R // bn
        rows = torch.arange(ntiles, device=dev)[:, None] * bn + rr[None, :]
    if ntiles * bn != R:
        raise ValueError("tgemm_pack: rows are not a whole number of tiles")
    t = w[rows.reshape(-1)].view(ntiles, bn, nk, 8, 8)
    perm = torch.arange(8, device=dev)[None, :] ^ (rr[:, None] & 7)  # [bn, 8]
    t = torch.gather(t, 3, perm[None, :, None, :, None].expand(ntiles, bn, nk, 8, 8))
    return t.permute(0, 2, 1, 3, 4).contiguous().view(R, K)


def pgemm(epi: int, x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
          ss_in: torch.Tensor | None = None, inv_d: float = 0.0, eps: float = 0.0,
          ss_out: torch.Tensor | None = None, positions=None, cos_sin=None, k_cache=None,
          v_cache=None, slots=None, hq: int = 0, hkv: int = 0, block_size: int = 0):
    """Prefill GEMM ``x @ w.T`` with a fused epilogue (``csrc/pgemm.hip``).

    ``ss_in`` ([M, n] fp32 partial row sums of squares of ``x``) scales row r by
    ``rsqrt(sum(ss_in[r]) * inv_d + eps)`` -- RMSNorm with the norm weight folded
    into ``w``.  epi 0: out = scaled GEMM; 1: out = silu(g) * u with
    ``w = [Wg; Wu]``; 2: ``out`` is the residual, updated in place (out += GEMM)
    with ``ss_out[r, t]`` = sum of squares of its new 256-column slice t;
    3: QKV -> RoPE'd q in ``out`` [M, hq*128], RoPE'd k and v written to the
    paged caches at ``slots``."""
    M, K = x.shape
    N = w.shape[0] // 2 if epi == 1 else w.shape[0]
    if out is None:
        out = x.new_empty(M, hq * 128 if epi == 3 else N)
    if x.is_cuda:
        if epi == 3 and checks.active(x):
            checks.slots("pgemm qkv", slots, k_cache)
        kernels().pgemm(epi, out, x.contiguous(), w, ss_in, inv_d, eps, ss_out, positions,
                        cos_sin, k_cache, v_cache, slots, hq, hkv, block_size)
        return out
    h = x.float() @ w.float().t()
    if ss_in is not None and epi != 2:
        h = h * torch.rsqrt(ss_in.float().sum(1) * inv_d + eps)[:, None]
    if epi == 0:
        out.copy_(h.to(out.dtype))
    elif epi == 1:
        out.copy_((F.silu(h[:, :N]) * h[:, N:]).to(out.dtype))
    elif epi == 2:
        new = (out.float() + h.to(out.dtype).float()).to(out.dtype)
        out.copy_(new)
        ss_out.copy_(new.float().pow(2).view(M, -1, 256).sum(-1))
    else:
        D = 128
        qkv = h.to(out.dtype)
        qq = ref.apply_rope(qkv[:, : hq * D].reshape(M, hq, D), positions, cos_sin)
        kk = ref.apply_rope(qkv[:, hq * D:(hq + hkv) * D].reshape(M, hkv, D), positions, cos_sin)
        vv = qkv[:, (hq + hkv) * D:].reshape(M, hkv, D)
        keep = slots >= 0
        ref.write_kv(k_cache, v_cache, kk[keep], vv[keep], slots[keep])
        out.copy_(qq.reshape(M, hq * D))
    return out


def pgemm_splitk(x: torch.Tensor, w: torch.Tensor, splits: int, out: torch.Tensor | None = None,
                 sched: int = 0) -> torch.Tensor:
    """fp16 split-K slabs ``[splits, M, N]`` of ``x @ w.T`` on the 256x256 MFMA tile
    (``csrc/pgemm.hip`` EPI 4; ``sched`` 0 / 1 = 8-wave / 4-wave main loop).  Each
    slab is one K-slice's fp32 sum saturated to fp16; the splitk consumers reduce
    them.  Decode projections at M <= 256 (one m-tile; the K split fills the chip)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(splits, M, N, dtype=torch.float16, device=x.device)
    if x.is_cuda:
        kernels().pgemm_splitk(out, x.contiguous(), w, sched)
        return out
    ks = K // splits
    for s in range(splits):
        r = x[:, s * ks:(s + 1) * ks].float() @ w[:, s * ks:(s + 1) * ks].float().t()
        out[s].copy_(r.clamp(-65504.0, 65504.0).to(out.dtype))
    return out


def row_sumsq(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 [M] sums of squares of the rows of a bf16 [M, d] matrix."""
    if out is None:
        out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    if x.is_cuda:
        kernels().row_sumsq(out, x)
        return out
    out.copy_(x.float().pow(2).sum(1))
    return out


def splitk_add_rmsnorm(parts: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                       out: torch.Tensor | None = None) -> torch.Tensor:
    """``residual += bf16(sum_s parts[s])`` in place; returns ``RMSNorm(residual) * w``."""
    if parts.is_cuda:
        out = residual.new_empty(residual.shape) if out is None else out
        kernels().splitk_add_rmsnorm(out, parts, residual, w, eps)
        return out
    o, r = ref.fused_add_rmsnorm(parts.sum(0).to(residual.dtype), residual, w, eps)
    residual.copy_(r)
    return o


def splitk_rope_kv(parts, positions, cos_sin, k_cache, v_cache, slots, hq, hkv, block_size,
                   q: torch.Tensor | None = None) -> torch.Tensor:
    """QKV split-K partials -> RoPE'd q ``[T, hq*D]`` (returned); RoPE'd k and v
    written to the paged cache at ``slots``."""
    T = parts.shape[1]
    D = 128
    if parts.is_cuda:
        if checks.active(parts):
            checks.slots("splitk_rope_kv", slots, k_cache)
        q = torch.empty(T, hq * D, dtype=k_cache.dtype, device=parts.device) if q is None else q
        kernels().splitk_rope_kv(q, parts, positions, cos_sin, k_cache, v_cache, slots, hq, hkv,
                                 block_size)
        return q
    qkv = parts.sum(0).to(k_cache.dtype)
    qq = qkv[:, : hq * D].reshape(T, hq, D)
    kk = qkv[:, hq * D:(hq + hkv) * D].reshape(T, hkv, D)
    vv = qkv[:, (hq + hkv) * D:].reshape(T, hkv, D)
    qq = ref.apply_rope(qq, positions, cos_sin)
    kk = ref.apply_rope(kk, positions, cos_sin)
    ref.write_kv(k_cache, v_cache, kk, vv, slots)
    return qq.reshape(T, hq * D)


def splitk_swiglu(parts: torch.Tensor) -> torch.Tensor:
    S, M, N2 = parts.shape
    if parts.is_cuda:
        out = torch.empty(M, N2 // 2, dtype=torch.bfloat16, device=parts.device)
        kernels().splitk_swiglu(out, parts)
        return out
    return ref.silu_mul(parts.sum(0).to(torch.bfloat16))


def splitk_reduce(parts: torch.Tensor) -> torch.Tensor:
    S, M, N = parts.shape
    if parts.is_cuda:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=parts.device)
        kernels().splitk_reduce(out, parts)
        return out
    return parts.sum(0).to(torch.bfloat16)


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``x @ w.T`` (w in [out, in] layout).  Decode-sized GPU batches (M <= 256)
    run the hand MFMA kernel (gemm.hip); larger batches (prefill) hipBLASLt."""
    r = _dgemm(0, x, w, out)
    if r is not None:
        return r
    if out is not None:
        return torch.mm(x, w.t(), out=out)
    return F.linear(x, w)


def linear_silu(x: torch.Tensor, w_gu: torch.Tensor) -> torch.Tensor:
    """``silu(x Wg^T) * (x Wu^T)`` with ``w_gu = [Wg; Wu]``: the SwiGLU MLP's first
    half.  Decode batches fuse the activation into the GEMM epilogue."""
    r = _dgemm(1, x, w_gu, None)
    if r is not None:
        return r
    return silu_mul(F.linear(x, w_gu))


def silu_mul(x: torch.Tensor, out: torch.Tensor | None = None):
    inter = x.shape[-1] // 2
    if x.is_cuda:
        out = x.new_empty(*x.shape[:-1], inter) if out is None else out
        kernels().silu_mul(out, x)
        return out
    r = ref.silu_mul(x)
    if out is not None:
        out.copy_(r)
        return out
    return r


def embedding(ids: torch.Tensor, w: torch.Tensor, vocab_start: int = 0,
              out: torch.Tensor | None = None, src: torch.Tensor | None = None,
              tok_slots: torch.Tensor | None = None):
    """Token embedding gather.  ``src`` / ``tok_slots`` (decode): row t's token
    is ``tok_slots[src[t]]`` where ``src[t] >= 0`` (sampled on the device by an
    earlier step), else ``ids[t]`` -- resolved inside the kernel."""
    if ids.is_cuda:
        out = w.new_empty(ids.numel(), w.shape[1]) if out is None else out
        kernels().embedding(out, ids, w, vocab_start, src, tok_slots)
        return out
    if src is not None:
        ids = torch.where(src >= 0, tok_slots.index_select(0, src.clamp(min=0).long()), ids)
    local = (ids >= vocab_start) & (ids < vocab_start + w.shape[0])
    idx = torch.where(local, ids - vocab_start, torch.zeros_like(ids)).long()
    r = w[idx] * local[:, None].to(w.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


def decode_workspace(batch: int, hq: int, max_blocks: int, block_size: int, part_size: int,
                     device, splits: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    max_parts = max((max_blocks * block_size + part_size - 1) // part_size, splits)
    part_o = torch.empty(batch * hq * max_parts * 128, dtype=torch.float32, device=device)
    part_ml = torch.empty(batch * hq * max_parts * 2, dtype=torch.float32, device=device)
    return part_o, part_ml


DECODE_SPLIT_MIN = int(os.environ.get("OMNIA_DECODE_SPLIT_MIN", "64"))


def decode_attention(q, k_cache, v_cache, block_tables, seq_lens, scale, part_size=512,
                     workspace=None, out=None, splits=0, split_min=None):
    """q: [B, Hq, D] one query per sequence at position seq_len-1.

    ``part_size``: partition length (splits = 0), or the longest partition the
    length-balanced split may use (splits > 0: each context is cut on the device
    into up to ``splits`` equal page-aligned partitions of >= ``split_min`` keys)."""
    if q.is_cuda:
        B, hq, _ = q.shape
        split_min = DECODE_SPLIT_MIN if split_min is None else split_min
        if checks.active(q):
            checks.paged("decode_attention", block_tables, seq_lens, k_cache, B)
        if out is None:
            out = torch.empty(B, hq, q.shape[2], dtype=q.dtype, device=q.device)
        if workspace is None:
            workspace = decode_workspace(B, hq, block_tables.shape[1], k_cache.shape[2],
                                         part_size, q.device, splits)
        kernels().decode_attention(out, q, k_cache, v_cache, block_tables, seq_lens,
                                   workspace[0], workspace[1], part_size, scale, splits,
                                   split_min)
        return out
    B = q.shape[0]
    qsl = torch.arange(B + 1, dtype=torch.int32)
    r = ref.paged_attention(q, k_cache, v_cache, block_tables, qsl, seq_lens, scale)
    if out is not None:
        out.copy_(r)
        return out
    return r


PREFILL_Q_TILE = int(os.environ.get("OMNIA_PREFILL_Q_TILE", "32"))  # 32 (32-row waves) | 64 | 128


def prefill_tiles(q_lens: list[int], tile: int | None = None) -> tuple[list[int], list[int]]:
    tile = tile or PREFILL_Q_TILE
    seqs, q0s = [], []
    for s, n in enumerate(q_lens):
        for q0 in range(0, n, tile):
            seqs.append(s)
            q0s.append(q0)
    return seqs, q0s


def prefill_attention(q, k_cache, v_cache, block_tables, q_start_loc, seq_lens, scale,
                      tile_seq=None, tile_q0=None, out=None, heads_per_wave: int = 0,
                      q_tile: int | None = None, lse=None, kv_lens=None):
    """q: [T, Hq, D] new tokens of several sequences (varlen, causal w/ cached prefix).

    ``lse`` (fp32 [T, Hq], optional) receives each row's natural-log sum of
    exp of the scaled scores -- the statistic ring attention merges blocks
    with.  ``kv_lens`` (int32 [B], optional) caps the visible keys of sequence
    ``s`` at ``kv_lens[s]`` on top of the causal bound, so a K/V block that lies
    wholly before the queries is attended in full: ``seq_lens = kv_len + qlen``
    puts the queries after every key."""
    if q.is_cuda:
        if tile_seq is None:
            qsl = q_start_loc.cpu().tolist()
            s, q0 = prefill_tiles([qsl[i + 1] - qsl[i] for i in range(len(qsl) - 1)], q_tile)
            tile_seq = torch.tensor(s, dtype=torch.int32, device=q.device)
            tile_q0 = torch.tensor(q0, dtype=torch.int32, device=q.device)
        out = torch.empty_like(q) if out is None else out
        if checks.active(q):
            checks.paged("prefill_attention", block_tables, seq_lens, k_cache,
                         q_start_loc.numel() - 1)
        kernels().prefill_attention(out, q, k_cache, v_cache, block_tables, q_start_loc,
                                    seq_lens, tile_seq, tile_q0, scale, heads_per_wave,
                                    q_tile or PREFILL_Q_TILE, lse, kv_lens)
        return out
    if lse is not None or kv_lens is not None:
        r, l = ref.paged_attention_lse(q, k_cache, v_cache, block_tables, q_start_loc, seq_lens,
                                       scale, kv_lens)
        if lse is not None:
            lse[: l.shape[0]].copy_(l)
    else:
        r = ref.paged_attention(q, k_cache, v_cache, block_tables, q_start_loc, seq_lens, scale)
    if out is not None:
        out.copy_(r)
        return out
    return r


def sample(logits, temperature, top_k=None, top_p=None, seeds=None, steps=None, counts=None,
           freq_pen=None, pres_pen=None, rep_pen=None, out=None, out_logprob=None,
           tok_slots=None, dst=None):
    """Fused GPU sampler; returns int32 [B] token ids.  With ``tok_slots`` /
    ``dst`` the kernel also writes row r's token to ``tok_slots[dst[r]]`` (the
    sequence's device token slot: no scatter op after it in a decode graph)."""
    if logits.is_cuda:
        B = logits.shape[0]
        out = torch.empty(B, dtype=torch.int32, device=logits.device) if out is None else out
        kernels().sample(out, out_logprob, logits, temperature, top_k, top_p, seeds, steps,
                         counts, freq_pen, pres_pen, rep_pen, tok_slots, dst)
        return out
    x = ref.apply_penalties(logits, counts, freq_pen, pres_pen, rep_pen)
    g = None
    if seeds is not None:
        g = torch.Generator().manual_seed(int(seeds[0]) + int(steps[0] if steps is not None else 0))
    r = ref.sample(x, temperature, top_k, top_p, generator=g)
    if counts is not None:
        counts[torch.arange(r.numel()), r.long()] += 1
    if tok_slots is not None:
        tok_slots.index_copy_(0, dst, r.to(tok_slots.dtype))
    if out is not None:
        out.copy_(r)
        return out
    return r


def apply_token_mask(logits: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """K13: in place, logits[r, v] = -inf where bit v of int32 ``mask[r]`` is clear."""
    if logits.is_cuda:
        kernels().apply_token_mask(logits, mask.to(device=logits.device, dtype=torch.int32)
                                   .contiguous())
        return logits
    return ref.apply_token_mask(logits, mask)


# ------------------------------------------------------------- memory tier (K17 / K18)
def mean_pool_l2(hidden: torch.Tensor, cu_seqlens: torch.Tensor) -> torch.Tensor:
    """[T, D] bf16 hidden states + [B+1] int32 offsets -> [B, D] fp32 unit vectors."""
    if hidden.is_cuda:
        B = cu_seqlens.numel() - 1
        out = torch.empty(B, hidden.shape[1], dtype=torch.float32, device=hidden.device)
        kernels().mean_pool_l2(out, hidden, cu_seqlens.to(device=hidden.device,
                                                          dtype=torch.int32).contiguous())
        return out
    return ref.mean_pool_l2(hidden, cu_seqlens)


def cosine_topk(q: torch.Tensor, m: torch.Tensor, k: int, valid: torch.Tensor | None = None):
    """Exact top-k of q . m over unit vectors.

    q: [NQ, D] (any float dtype, normalised), m: [N, D] bf16 (normalised rows),
    valid: optional uint8 [N] (0 = tombstoned).  Returns (scores fp32 [NQ, k],
    indices int64 [NQ, k]) sorted by descending score, ties by ascending index."""
    nq, N = q.shape[0], m.shape[0]
    k = min(k, N)
    if k == 0:
        return (torch.empty(nq, 0, dtype=torch.float32, device=m.device),
                torch.empty(nq, 0, dtype=torch.long, device=m.device))
    if m.is_cuda:
        kk = kernels()
        D = m.shape[1]
        vals, idxs = [], []
        # the kernel stages up to 64 KiB of queries in LDS: chunk by 8/4/2/1
        max_nq = max(1, min(8, (64 * 1024) // (4 * D)))
        i = 0
        while i < nq:
            n = min(max_nq, nq - i)
            npad = 1 if n == 1 else 2 if n == 2 else 4 if n <= 4 else 8
            qq = torch.zeros(npad, D, dtype=torch.float32, device=m.device)
            qq[:n] = q[i:i + n].to(device=m.device, dtype=torch.float32)
            scores = torch.empty(npad, N, dtype=torch.float32, device=m.device)
            kk.cosine_scores(scores, qq, m, valid)
            oi = torch.empty(npad, k, dtype=torch.int32, device=m.device)
            ov = torch.empty(npad, k, dtype=torch.float32, device=m.device)
            kk.topk(oi, ov, scores, k)
            vals.append(ov[:n])
            idxs.append(oi[:n].long())
            i += n
        return torch.cat(vals), torch.cat(idxs)
    return ref.cosine_topk(q, m, k, valid)


# ------------------------------------------------------------- MoE (K14)
MOE_LIBRARY_ROWS = 1024  # mean rows/expert above which eager calls use hipBLASLt per expert
# mean rows per local expert from which the grouped GEMMs run on the 256x256
# prefill tile (pgemm.hip EPI 5 / 6, 256-row expert segments); below it the
# 64-row grouped kernels (moe.hip) waste less padding.  Both are graph-safe.
MOE_TILE256_ROWS = int(os.environ.get("OMNIA_MOE_TILE256_ROWS", "512"))


def _moe_grouped(x, w_gu, w_down, ids, wts, k, n_experts, e_lo, e_hi, bm):
    """Grouped expert FFN over device-sorted assignments, no host sync: Y [T*k, d]
    (row t*k + j = slot j of token t, routing weight applied; other experts' rows
    unwritten).  ``bm`` 256: the 256x256 MFMA prefill tile; 64: moe.hip."""
    kk = kernels()
    n = ids.numel()
    mb = kk.moe_max_blocks(n, e_hi - e_lo, bm)
    sorted_ids = torch.empty(mb * bm, dtype=torch.int32, device=x.device)
    blk = torch.empty(mb, dtype=torch.int32, device=x.device)
    nblk = torch.empty(1, dtype=torch.int32, device=x.device)
    kk.moe_align(sorted_ids, blk, nblk, ids, n_experts, e_lo, e_hi)
    act = torch.empty(mb * bm, w_down.shape[2], dtype=x.dtype, device=x.device)
    Y = torch.empty(n, x.shape[1], dtype=x.dtype, device=x.device)
    gemm = kk.pgemm_moe if bm == 256 else kk.moe_gemm
    gemm(0, act, x, w_gu, sorted_ids, blk, nblk, None, k, n, e_lo)
    gemm(1, Y, act, w_down, sorted_ids, blk, nblk, wts.view(-1), k, n, e_lo)
    return Y


def moe_rows(rows: torch.Tensor, eids: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor,
             e_lo: int, n_experts: int) -> torch.Tensor:
    """Expert FFN of each row under its own expert id (the receive side of an
    expert-parallel all-to-all): ``y[r] = down_e(silu(gate_e x) * up_e x)`` with
    ``e = eids[r]`` for local experts ``[e_lo, e_lo + w_gu.shape[0])``; rows whose
    id is outside that range (padding, ``-1``) are left unwritten.  Static shapes
    and no host sync (hipGraph-safe): the grouped MFMA kernels with top-1 routing."""
    R, d = rows.shape
    e_hi = e_lo + w_gu.shape[0]
    if not rows.is_cuda:
        y = rows.new_zeros(R, w_down.shape[1])
        local = (eids.long() - e_lo)
        ok = (local >= 0) & (local < w_gu.shape[0])
        li = local.clamp(0, w_gu.shape[0] - 1)
        h = torch.bmm(w_gu.index_select(0, li).float(), rows.float()[:, :, None])[:, :, 0]
        a = ref.silu_mul(h)
        o = torch.bmm(w_down.index_select(0, li).float(), a[:, :, None])[:, :, 0]
        return torch.where(ok[:, None], o.to(rows.dtype), y)
    kk = kernels()
    ids = eids.to(torch.int32).view(R, 1).contiguous()
    mb = kk.moe_max_blocks(R, e_hi - e_lo)
    sorted_ids = torch.empty(mb * 64, dtype=torch.int32, device=rows.device)
    blk = torch.empty(mb, dtype=torch.int32, device=rows.device)
    nblk = torch.empty(1, dtype=torch.int32, device=rows.device)
    kk.moe_align(sorted_ids, blk, nblk, ids, n_experts, e_lo, e_hi)
    act = torch.empty(mb * 64, w_down.shape[2], dtype=rows.dtype, device=rows.device)
    kk.moe_gemm(0, act, rows, w_gu, sorted_ids, blk, nblk, None, 1, R, e_lo)
    y = torch.empty(R, w_down.shape[1], dtype=rows.dtype, device=rows.device)
    ones = torch.ones(R, dtype=torch.float32, device=rows.device)
    kk.moe_gemm(1, y, act, w_down, sorted_ids, blk, nblk, ones, 1, R, e_lo)
    return y


def moe(x: torch.Tensor, router: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor,
        k: int, n_experts: int, e_lo: int = 0, renorm: bool = True,
        graph_safe: bool = True) -> torch.Tensor:
    """Top-k MoE FFN over the local experts ``[e_lo, e_lo + w_gu.shape[0])``.

    x [T, d] bf16, router [E, d], w_gu [E_loc, 2I, d] (gate ; up), w_down [E_loc, d, I].
    Returns the local experts' weighted contribution [T, d] (all-reduce over the
    EP group to complete it).  ``graph_safe`` keeps every shape static and the
    whole path on device (hipGraph decode); otherwise large batches run each
    expert's GEMMs on hipBLASLt after one host sync on the expert counts."""
    e_hi = e_lo + w_gu.shape[0]
    if not x.is_cuda:
        return ref.moe(x, router, w_gu, w_down, k, e_lo, renorm).to(x.dtype)
    kk = kernels()
    T, d = x.shape
    n = T * k
    ids = torch.empty(T, k, dtype=torch.int32, device=x.device)
    wts = torch.empty(T, k, dtype=torch.float32, device=x.device)
    # router GEMM + softmax top-k in one hand kernel (moe.hip): no logits tensor,
    # no library GEMM
    kk.moe_router_topk(ids, wts, x.contiguous(), router, k, renorm)
    out = torch.empty_like(x)
    d, inter = x.shape[1], w_down.shape[2]
    if n >= MOE_TILE256_ROWS * (e_hi - e_lo) and d % 256 == 0 and inter % 128 == 0:
        # prefill-sized: the 256x256 MFMA tile, grouped by 256-row expert segments
        # (pgemm.hip EPI 5 / 6) -- hand kernels, graph-safe, no per-expert library
        # calls and no host sync
        Y = _moe_grouped(x, w_gu, w_down, ids, wts, k, n_experts, e_lo, e_hi, 256)
        kk.moe_combine(out, Y, ids, k, e_lo, e_hi)
        return out
    if not graph_safe and n >= MOE_LIBRARY_ROWS * (e_hi - e_lo) and \
            os.environ.get("OMNIA_MOE_LIBRARY", "0") == "1":
        # opt-in comparison path: per-expert hipBLASLt after one host sync
        flat = ids.view(-1)
        order = torch.argsort(flat, stable=True)
        counts = torch.bincount(flat, minlength=n_experts).tolist()  # host sync (eager only)
        xs = x.index_select(0, (order // k))
        ys = torch.empty(n, d, dtype=x.dtype, device=x.device)
        o = sum(counts[:e_lo])
        for e in range(e_lo, e_hi):
            c = counts[e]
            if c:
                h = F.linear(xs[o:o + c], w_gu[e - e_lo])
                ys[o:o + c] = F.linear(silu_mul(h), w_down[e - e_lo])
            o += c
        Y = torch.empty(n, d, dtype=x.dtype, device=x.device)
        Y.index_copy_(0, order, ys * wts.view(-1).index_select(0, order)[:, None].to(x.dtype))
        kk.moe_combine(out, Y, ids, k, e_lo, e_hi)
        return out
    Y = _moe_grouped(x, w_gu, w_down, ids, wts, k, n_experts, e_lo, e_hi, 64)
    kk.moe_combine(out, Y, ids, k, e_lo, e_hi)
    return out
