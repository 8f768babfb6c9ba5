"""Row-parallel GEMM + TP all-reduce overlap for prefill.

A Megatron row-parallel projection (attention O, MLP down) produces a partial
sum on every TP rank that must be all-reduced before the residual add + RMSNorm
of the layer boundary.  Done whole, the GEMM and the collective serialise: the
xGMI links idle during the GEMM and the matrix cores idle during the reduce.

Here the projection is split along M (tokens) into chunks of ``rows`` rows:

    main stream:  GEMM(c0)  GEMM(c1)  GEMM(c2)  ...            wait(side)
    side stream:            RED(c0)   RED(c1)   RED(c2) ...

``RED(c)`` = all-reduce of chunk c's partial sums fused with ``residual[c] +=``
and ``RMSNorm(residual[c]) * w`` (the layer boundary).  On the ``ipc``
transport (ranks sharing devices) it is the two-shot IPC kernel with the norm
fused in (``comm.hip``), in row pieces that fit one slot; on ``rccl`` it is the
RCCL all-reduce plus the fused add-norm kernel, both on the side stream.  Each
chunk's reduce starts as soon as its GEMM retires, so all but the last chunk's
collective hides under the following GEMMs.

Bit-exactness: the chunk GEMM is the hand prefill kernel (``pgemm.hip`` plain
epilogue) whenever its shape constraints hold, and with ``rows`` a multiple of
its 256-row tile every output row is computed by exactly the same instruction
sequence whatever the chunking -- so the overlapped result equals the serial
(``overlap=False``) result bit for bit; only the scheduling differs.

Ordering rules that keep it race-free:
  * ``side.wait_stream(main)`` before each reduce: the chunk's GEMM, and every
    earlier producer of ``residual``, completed;
  * the main stream never touches ``residual`` or a chunk already handed to
    the side stream until ``main.wait_stream(side)`` at the end;
  * only one stream issues collectives at a time (the side stream, in chunk
    order), so RCCL / IPC epoch order is identical on every rank.
"""
from __future__ import annotations

import os

import torch

from .. import ops
from . import state as pstate

OVERLAP = os.environ.get("OMNIA_TP_OVERLAP", "1") != "0"
ROWS = int(os.environ.get("OMNIA_TP_OVERLAP_ROWS", "1024"))
MIN_ROWS = int(os.environ.get("OMNIA_TP_OVERLAP_MIN_ROWS", "2048"))

_SIDE: dict = {}


def side_stream(device) -> torch.cuda.Stream:
    s = _SIDE.get(device)
    if s is None:  # high priority: the collective should not queue behind GEMM waves
        s = _SIDE[device] = torch.cuda.Stream(device=device, priority=-1)
    return s


def applies(T: int, device: torch.device) -> bool:
    st = pstate.get_state()
    return (OVERLAP and st.tp_size > 1 and device.type == "cuda" and T >= MIN_ROWS)


def _gemm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor) -> None:
    K, N = x.shape[1], w.shape[0]
    if K % 128 == 0 and N % 256 == 0 and x.dtype == torch.bfloat16:
        ops.pgemm(0, x, w, out=out)
    else:
        torch.mm(x, w.t(), out=out)


def reduce_add_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                    eps: float) -> torch.Tensor:
    """``residual += allreduce(x)``; ``x = RMSNorm(residual) * w`` (in place)."""
    st = pstate.get_state()
    ar = st.custom_ar
    if st.transport == "ipc" and ar is not None and not ar.can_fuse_norm(x):
        # ipc: fused two-shot pieces that fit one slot (4 B per element staged)
        rows = max(1, ar.slot_bytes // (4 * x.shape[1]))
        for r0 in range(0, x.shape[0], rows):
            ar.all_reduce_add_rmsnorm(x[r0:r0 + rows], residual[r0:r0 + rows], w, eps)
        return x
    return pstate.tp_all_reduce_add_rmsnorm(x, residual, w, eps)


def rowparallel_add_norm(inp: torch.Tensor, w: torch.Tensor, residual: torch.Tensor,
                         norm_w: torch.Tensor, eps: float, rows: int = ROWS,
                         overlap: bool = True) -> torch.Tensor:
    """``residual += allreduce(inp @ w.T)``; returns ``RMSNorm(residual) * norm_w``
    -- chunked along M with each chunk's reduce on the side stream."""
    T = inp.shape[0]
    out = torch.empty(T, w.shape[0], dtype=inp.dtype, device=inp.device)
    rows = max(256, rows // 256 * 256)
    main = torch.cuda.current_stream(inp.device)
    side = side_stream(inp.device) if overlap else None
    for r0 in range(0, T, rows):
        r1 = min(T, r0 + rows)
        _gemm(inp[r0:r1], w, out[r0:r1])
        if side is None:
            reduce_add_norm(out[r0:r1], residual[r0:r1], norm_w, eps)
            continue
        side.wait_stream(main)
        with torch.cuda.stream(side):
            reduce_add_norm(out[r0:r1], residual[r0:r1], norm_w, eps)
    if side is not None:
        main.wait_stream(side)
    return out
