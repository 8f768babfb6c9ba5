"""Untraced per-wave timeline across the serving tree.

A rocprof trace distorts what it measures (the traced decode span was 12.8 ms
against 9.4 ms of kernel time in round 4), and the wall time of a bench wave
that is NOT in kernels spans four processes: the client, the facade, the
runtime and the engine-core.  This recorder is cheap enough to leave on during
a measured run: each process appends ``(t, event, fields)`` tuples to an
in-memory list -- one ``perf_counter`` read and one append per event -- and
writes them as JSON lines to ``$OMNIA_TIMELINE_DIR/<role>-<pid>.jsonl`` at
exit or on :func:`flush`.  ``time.perf_counter`` is ``CLOCK_MONOTONIC`` on
Linux, so the four processes' clocks are directly comparable.

GPU time comes from timing hipEvents recorded around each engine step
(``engine.py``); :func:`device_anchor` pairs one event with a host timestamp
so the event times map onto the same monotonic clock.
``scripts/wave_timeline.py`` merges the files into a per-wave attribution.
"""
from __future__ import annotations

import atexit
import json
import os
import threading
import time

_DIR = os.environ.get("OMNIA_TIMELINE_DIR", "")
ENABLED = bool(_DIR)
_role = "proc"
_events: list = []
_lock = threading.Lock()
_clock = time.perf_counter


def set_role(role: str) -> None:
    global _role
    _role = role


def mark(event: str, **fields) -> None:
    """Record ``event`` now (no-op unless ``OMNIA_TIMELINE_DIR`` is set)."""
    if ENABLED:
        _events.append((_clock(), event, fields))


def mark_at(t: float, event: str, **fields) -> None:
    if ENABLED:
        _events.append((t, event, fields))


def flush() -> str | None:
    """Append the buffered events to this process's file; returns its path."""
    if not ENABLED:
        return None
    with _lock:
        evs = _events[:]
        del _events[:len(evs)]
    os.makedirs(_DIR, exist_ok=True)
    path = os.path.join(_DIR, f"{_role}-{os.getpid()}.jsonl")
    with open(path, "a") as f:
        for t, ev, fields in evs:
            f.write(json.dumps({"t": round(t, 6), "ev": ev, **fields}) + "\n")
    return path


def device_anchor():
    """(hip event, host time) with the event known complete at ~host time: maps
    ``anchor_event.elapsed_time(e)`` onto the monotonic clock."""
    import torch

    e = torch.cuda.Event(enable_timing=True)
    e.record()
    e.synchronize()
    return e, _clock()


if ENABLED:
    atexit.register(flush)
