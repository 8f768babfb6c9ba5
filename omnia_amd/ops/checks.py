"""Debug bounds checks for the paged-KV kernels (SURVEY §5.2 [design]:
"bounds-checked debug variants of the paged-attention kernels, which assert on
block-table indices").

With ``OMNIA_KERNEL_CHECKS=1``, every paged attention / KV-write launch first
validates, on the device with plain torch ops, the indices it is about to
follow:

* the pages each sequence reads lie in ``[0, num_blocks)``, for the first
  ``ceil(seq_len / block_size)`` entries of its block-table row;
* ``seq_len`` fits that row;
* the KV slots are ``-1`` (a padded row, skipped by the kernels) or lie in
  ``[0, num_blocks * block_size)``.

A violation raises :class:`KernelCheckError`, naming the op and the first bad
row, before anything is launched. This replaces an in-kernel ``assert``: a
device trap takes the GPU down with it, and on a shared node that can reset
every GPU. The checks synchronise the host (``.item()``), so they are skipped
while a stream captures a graph, and they are off by default.
"""
from __future__ import annotations

import os

import torch

ENABLED = os.environ.get("OMNIA_KERNEL_CHECKS", "0") == "1"


class KernelCheckError(ValueError):
    pass


def active(t: torch.Tensor) -> bool:
    if not ENABLED:
        return False
    return not (t.is_cuda and torch.cuda.is_current_stream_capturing())


def paged(op: str, block_tables: torch.Tensor, seq_lens: torch.Tensor, k_cache: torch.Tensor,
          rows: int | None = None) -> None:
    """Pages read by ``rows`` sequences (default: every row of ``seq_lens``)."""
    nb, bs = k_cache.shape[0], k_cache.shape[2]
    B = seq_lens.numel() if rows is None else rows
    if B == 0:
        return
    sl = seq_lens[:B].long()
    width = block_tables.shape[1]
    if bool((sl < 0).any()) or bool((sl > width * bs).any()):
        b = int(((sl < 0) | (sl > width * bs)).nonzero()[0])
        raise KernelCheckError(f"{op}: seq_len {int(sl[b])} of row {b} does not fit its "
                               f"block-table row ({width} pages x {bs})")
    used = torch.arange(width, device=sl.device)[None, :] < ((sl + bs - 1) // bs)[:, None]
    bt = block_tables[:B].long()
    bad = used & ((bt < 0) | (bt >= nb))
    if bool(bad.any()):
        b, j = (int(x) for x in bad.nonzero()[0])
        raise KernelCheckError(f"{op}: row {b} page {j} -> block {int(bt[b, j])} outside "
                               f"[0, {nb})")


def slots(op: str, slot: torch.Tensor, k_cache: torch.Tensor) -> None:
    """KV write slots: -1 (padded row) or inside the cache."""
    if slot is None or slot.numel() == 0:
        return
    cap = k_cache.shape[0] * k_cache.shape[2]
    s = slot.long()
    bad = (s < -1) | (s >= cap)
    if bool(bad.any()):
        i = int(bad.nonzero()[0])
        raise KernelCheckError(f"{op}: KV slot {int(s[i])} of row {i} outside [-1, {cap})")
