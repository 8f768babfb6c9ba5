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

import contextlib
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
# library GEMMs (hipBLASLt): pointer-stable under capture (PyTorch sizes their
# workspace per stream up front); allowed, but counted separately so a decode
# step that should be all hand kernels shows them
LIBRARY = {"aten::mm", "aten::addmm", "aten::bmm", "aten::linear", "aten::matmul"}


class CaptureGuardError(RuntimeError):
    pass


class _OpRecorder(TorchDispatchMode):
    def __init__(self, trace: bool = False):
        super().__init__()
        self.ops: dict[str, int] = {}
        self.library: dict[str, int] = {}
        self.where: dict[str, str] = {}  # first call site per op (OMNIA_CAPTURE_GUARD_TRACE=1)
        self.trace = trace

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func._schema.name
        if name in LIBRARY:
            self.library[name] = self.library.get(name, 0) + 1
        elif name not in ALLOWED:
            self.ops[name] = self.ops.get(name, 0) + 1
            if self.trace and name not in self.where:
                import traceback

                self.where[name] = "".join(traceback.format_stack(limit=12)[:-1])
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
        self.library: dict[str, int] = {}
        self.leaked: list = []
        self._rec = None
        self._before = None

    @property
    def enabled(self) -> bool:
        return self.mode != "off"

    def __enter__(self):
        self._mem_enter()
        self._ops_enter()
        return self

    def __exit__(self, et, ev, tb):
        self._ops_exit(et, ev, tb)
        self._mem_exit(et)
        if et is None and self.enabled:
            self.check()
        return False

    # the two halves separately: the op recorder goes INSIDE the capture (so
    # PyTorch's own capture_begin / capture_end work -- e.g. the RNG generator's
    # seed / offset fill_ -- is not counted) and the memory snapshots OUTSIDE it
    # (no allocator query while the stream captures); then check()
    @contextlib.contextmanager
    def ops_scope(self):
        self._ops_enter()
        try:
            yield self
        except BaseException as e:
            self._ops_exit(type(e), e, None)
            raise
        self._ops_exit(None, None, None)

    @contextlib.contextmanager
    def memory_scope(self):
        self._mem_enter()
        try:
            yield self
        except BaseException:
            self._mem_exit(RuntimeError)
            raise
        self._mem_exit(None)

    def _ops_enter(self):
        if not self.enabled:
            return
        self._rec = _OpRecorder(os.environ.get("OMNIA_CAPTURE_GUARD_TRACE") == "1")
        self._rec.__enter__()

    def _ops_exit(self, et, ev, tb):
        if not self.enabled or self._rec is None:
            return
        self._rec.__exit__(et, ev, tb)
        self.ops = dict(self._rec.ops)
        self.library = dict(self._rec.library)
        for name, where in self._rec.where.items():
            log.error("capture guard: %s first dispatched at\n%s", name, where)

    def _mem_enter(self):
        if self.enabled and self.device.type == "cuda":
            self._before = _active_default_blocks(self.device)
            self._hist = os.environ.get("OMNIA_CAPTURE_GUARD_TRACE") == "1"
            if self._hist:  # allocation stacks for the leak report
                torch.cuda.memory._record_memory_history(max_entries=100000)

    def _mem_exit(self, et):
        if self.enabled and et is None and self._before is not None:
            self.leaked = sorted(_active_default_blocks(self.device) - self._before)
        if getattr(self, "_hist", False):
            if self.leaked:
                self._log_leak_stacks()
            torch.cuda.memory._record_memory_history(enabled=None)
            self._hist = False

    def _log_leak_stacks(self):
        want = {a for a, _ in self.leaked}
        for seg in torch.cuda.memory._snapshot().get("segments", []):
            for b in seg.get("blocks", []):
                if b.get("address") in want:
                    frames = b.get("frames") or []
                    where = "\n".join(f"  {f.get('filename')}:{f.get('line')} {f.get('name')}"
                                      for f in frames[:14])
                    log.error("capture guard: block %#x+%d allocated at\n%s",
                              b["address"], b.get("size", 0), where)

    def violations(self) -> list[str]:
        v = [f"framework op {k} x{n}" for k, n in sorted(self.ops.items())]
        if not self.library:
            v += [f"block {a:#x}+{s} allocated outside the graph pool" for a, s in self.leaked]
        return v

    def library_blocks(self) -> list:
        """Out-of-pool blocks of a capture that ran library GEMMs: the library
        handle's per-stream workspace, which PyTorch keeps outside graph pools
        on purpose (held for the handle's life, never freed under a graph) --
        reported, not a violation.  A capture without library GEMMs (the
        serving decode graph) has none."""
        return list(self.leaked) if self.library else []

    def check(self) -> None:
        v = self.violations()
        if not v:
            return
        msg = f"{self.what}: {len(v)} capture-guard violation(s): " + "; ".join(v[:8])
        if self.mode == "strict":
            raise CaptureGuardError(msg)
        log.error(msg)
