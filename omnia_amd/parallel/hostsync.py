"""Host shared-memory agreement for lockstep replicas on one node.

The DP-attention + EP engine (``engine/ep.py``) and the context-parallel
engine (``engine/cp.py``) are groups of independent replicas that must agree,
every step, on a few integers (who is active, the step-global token count, the
graph bucket, who owns a long prompt).  A device collective for that costs a
launch, a device -> host copy (``.tolist()``) and, on RCCL, a stream sync per
step; this is a host-only all-gather over one mmap'd page instead:

* layout: ``[world]`` rows of ``(seq, pid, 2 parity slots x nvals)`` int64;
* ``gather(vals)``: write ``vals`` into parity slot ``seq & 1`` of my row, then
  publish ``seq`` (stored last), then spin until every row's ``seq`` has caught
  up and read every row's slot.  Two parity slots are enough: a rank can write
  slot ``s & 1`` again (call ``s + 2``) only after everyone published ``s + 1``,
  which each does only after it finished reading call ``s``;
* ordering relies on x86-64 total store order (numpy stores land in program
  order; loads are not reordered with older loads), checked at construction;
* liveness: while spinning, every peer's pid is probed once a second, so a
  replica that died makes the others raise instead of spinning forever
  (``timeout_s`` bounds the wait as well).

The page path is created by group rank 0 under ``/dev/shm`` and handed to the
group once over the process group (any backend).
"""
from __future__ import annotations

import mmap
import os
import platform
import time
import uuid

import numpy as np


def check_tso() -> None:
    m = platform.machine().lower()
    if m not in ("x86_64", "amd64"):
        raise RuntimeError(f"host shared-memory rings assume x86-64 store ordering, not {m}")


def _alive(pid: int) -> bool:
    if pid <= 0:
        return True
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


class ShmAgreement:
    def __init__(self, path: str, world: int, rank: int, nvals: int, create: bool):
        check_tso()
        self.path, self.world, self.rank, self.nvals = path, world, rank, nvals
        self.row = 2 + 2 * nvals
        size = max(4096, 8 * world * self.row)
        if create:
            fd = os.open(path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
            os.ftruncate(fd, size)
        else:
            fd = os.open(path, os.O_RDWR)
        self.mm = mmap.mmap(fd, size)
        os.close(fd)
        self.a = np.ndarray((world, self.row), dtype=np.int64, buffer=self.mm)
        if create:
            self.a[:] = 0
        self.seq = 0
        self.a[rank, 1] = os.getpid()
        self.stats = {"calls": 0, "spins": 0}

    @classmethod
    def for_group(cls, group, nvals: int) -> "ShmAgreement":
        """Collective: group rank 0 creates the page, everyone maps it."""
        import torch.distributed as dist

        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        obj = [f"/dev/shm/omnia-agree-{uuid.uuid4().hex}" if rank == 0 else None]
        if rank == 0:
            ag = cls(obj[0], world, rank, nvals, create=True)
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group else 0,
                                   group=group)
        if rank != 0:
            ag = cls(obj[0], world, rank, nvals, create=False)
        dist.barrier(group=group)  # every rank mapped (and wrote its pid)
        if rank == 0:
            try:  # the mapping keeps the page alive; no file left behind
                os.unlink(obj[0])
            except FileNotFoundError:
                pass
        return ag

    def gather(self, vals, timeout_s: float = 3600.0) -> np.ndarray:
        """All ranks' ``vals`` (``[world, nvals]`` int64), host-only."""
        self.seq += 1
        s = self.seq
        off = 2 + (s & 1) * self.nvals
        me = self.a[self.rank]
        me[off:off + len(vals)] = vals
        me[off + len(vals):off + self.nvals] = 0
        me[0] = s  # publish last
        t0 = time.monotonic()
        probe = t0 + 1.0
        spins = 0
        while int(self.a[:, 0].min()) < s:
            spins += 1
            if spins > 64:
                time.sleep(0)
            now = time.monotonic()
            if now > probe:
                probe = now + 1.0
                for r in range(self.world):
                    if int(self.a[r, 0]) < s and not _alive(int(self.a[r, 1])):
                        raise RuntimeError(f"lockstep peer rank {r} (pid {int(self.a[r, 1])}) "
                                           "died")
                if now - t0 > timeout_s:
                    raise TimeoutError("lockstep agreement: a peer never arrived")
        self.stats["calls"] += 1
        self.stats["spins"] += spins
        return self.a[:, off:off + self.nvals].copy()

    def max(self, vals) -> list[int]:
        return [int(v) for v in self.gather(vals).max(axis=0)]

    def close(self):
        try:
            self.a = None
            self.mm.close()
        except (BufferError, ValueError):
            pass
