"""Capture-time guard for the engine's hipGraphs (verdict r5 item 5).

A captured graph replays the exact kernels, pointers and launch parameters of
its capture.  Two things captured by accident go stale without any error:

  * a framework (ATen) compute op whose hidden state -- a workspace, a launch
    heuristic, an allocation it made itself -- is captured once and reused on
    every replay (the class of bug behind the round-5 TP fault,
    ``profiles/r5/tp_fault.md``); the decode graph must contain only the hand
    kernels and plain copies;
  * a caching-allocator block handed out during capture from a pool OTHER than
    the graph's private one: the allocator may give it to someone else after
    capture while every replay still writes it.

:class:`CaptureGuard` wraps one capture.  A ``TorchDispatchMode`` records every
ATen op dispatched inside it; ops outside :data:`ALLOWED` (views, empty tensors,
copies) are violations.  Memory snapshots before and after list the blocks that
became active during the capture in segments whose pool is not a graph pool.
``OMNIA_CAPTURE_GUARD``: ``strict`` raises :class:`CaptureGuardError`, ``warn``
(default) logs and counts, ``off`` skips the checks.
"""
from __future__ import annotations

import logging
import os

import torch
from torch.utils._python_dispatch import TorchDispatchMode

log = logging.getLogger("omnia.engine.capture_guard")

# ATen ops a decode graph may contain: metadata-only views, allocation, and copies
# (a device-to-device copy is a copyBuffer, not a framework kernel with state)
ALLOWED = {
    "aten::view", "aten::_unsafe_view", "aten::slice", "aten::select", "aten::as_strided",
    "aten::empty", "aten::empty_strided", "aten::empty_like", "aten::new_empty",
    "aten::detach", "aten::alias", "aten::t", "aten::transpose", "aten::unsqueeze",
    "aten::squeeze", "aten::expand", "aten::permute", "aten::reshape", "aten::split",
    "aten::narrow", "aten::lift_fresh", "aten::copy_", "aten::_to_copy", "aten::unbind",
    "aten::split_with_sizes", "aten::view_as", "aten::contiguous", "aten::resize_",
    "aten::set_", "aten::_reshape_alias", "aten::clone",
}


class CaptureGuardError(RuntimeError):
    pass


class _OpRecorder(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops: dict[str, int] = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func._schema.name
        if name not in ALLOWED:
            self.ops[name] = self.ops.get(name, 0) + 1
        return func(*args, **(kwargs or {}))


def _active_default_blocks(device) -> set:
    """(address, size) of the active blocks in segments of the default pool."""
    out = set()
    for seg in torch.cuda.memory_snapshot():
        if seg.get("device") != device.index:
            continue
        pool = tuple(seg.get("segment_pool_id") or (0, 0))
        if pool != (0, 0):
            continue  # a graph's private pool
        addr = seg.get("address", 0)
        for b in seg.get("blocks", []):
            a = b.get("address", addr)
            if b.get("state") == "active_allocated":
                out.add((a, b.get("size", 0)))
            addr = a + b.get("size", 0)
    return out


class CaptureGuard:
    """``with CaptureGuard(device, what):`` around a capture; see module doc."""

    def __init__(self, device, what: str = "graph", mode: str | None = None):
        self.device = torch.device(device)
        self.what = what
        self.mode = (mode or os.environ.get("OMNIA_CAPTURE_GUARD", "warn")).lower()
        self.ops: dict[str, int] = {}
        self.leaked: list = []
        self._rec = None
        self._before = None

    @property
    def enabled(self) -> bool:
        return self.mode != "off"

    def __enter__(self):
        if not self.enabled:
            return self
        if self.device.type == "cuda":
            self._before = _active_default_blocks(self.device)
        self._rec = _OpRecorder()
        self._rec.__enter__()
        return self

    def __exit__(self, et, ev, tb):
        if not self.enabled:
            return False
        self._rec.__exit__(et, ev, tb)
        if et is not None:
            return False
        self.ops = dict(self._rec.ops)
        if self._before is not None:
            self.leaked = sorted(_active_default_blocks(self.device) - self._before)
        self.check()
        return False

    def violations(self) -> list[str]:
        v = [f"framework op {k} x{n}" for k, n in sorted(self.ops.items())]
        v += [f"block {a:#x}+{s} allocated outside the graph pool" for a, s in self.leaked]
        return v

    def check(self) -> None:
        v = self.violations()
        if not v:
            return
        msg = f"{self.what}: {len(v)} capture-guard violation(s): " + "; ".join(v[:8])
        if self.mode == "strict":
            raise CaptureGuardError(msg)
        log.error(msg)
