"""Env-driven failpoints for fault-injection tests (SURVEY §5.3 [design]).

The reference has no fault-injection framework; its failure handling (breakers,
retries, fail-closed policy, ring-buffered session writes, HasConversation's
UNAVAILABLE state) is exercised only by unit tests.  Here every failure path
that matters for serving can be triggered on a live process:

    OMNIA_FAILPOINT="engine.decode_step:0.01,tool.call:once,session.write:2@5"

Spec per name (comma separated ``name:spec``):
  ``P``      (float in (0, 1])  fail with probability P on each hit (seeded by
             ``OMNIA_FAILPOINT_SEED`` for reproducible runs)
  ``once``   fail the first hit only
  ``N@K``    fail N consecutive hits starting at hit K (1-based)
  ``always`` fail every hit
  ``off``    disabled
Hook points: ``engine.prefill``, ``engine.decode_step`` (engine step, before
launch), ``engine.hang`` (simulated stalled step, trips the watchdog),
``tool.call`` (tool executor dispatch), ``session.write`` (session store
writes), ``provider.stream`` (provider call start), ``runtime.dial`` (facade ->
runtime connect).
"""
from __future__ import annotations

import os
import random
import threading


class FailpointError(RuntimeError):
    """Raised by an armed failpoint."""

    def __init__(self, name: str):
        super().__init__(f"failpoint {name} triggered")
        self.name = name


class _Point:
    def __init__(self, spec: str):
        self.spec = spec.strip()
        self.hits = 0
        self.fired = 0
        s = self.spec.lower()
        self.prob = None
        self.start = self.count = None
        self.mode = "off"
        if s in ("", "off", "0"):
            return
        if s == "always":
            self.mode = "always"
        elif s == "once":
            self.mode, self.start, self.count = "range", 1, 1
        elif "@" in s:
            n, k = s.split("@", 1)
            self.mode, self.count, self.start = "range", int(n), int(k)
        else:
            self.mode, self.prob = "prob", float(s)
            if not 0.0 < self.prob <= 1.0:
                raise ValueError(f"failpoint probability out of range: {spec!r}")

    def should_fire(self, rng: random.Random) -> bool:
        self.hits += 1
        if self.mode == "always":
            fire = True
        elif self.mode == "range":
            fire = self.start <= self.hits < self.start + self.count
        elif self.mode == "prob":
            fire = rng.random() < self.prob
        else:
            fire = False
        self.fired += fire
        return fire


_lock = threading.Lock()
_points: dict[str, _Point] = {}
_rng = random.Random(int(os.environ.get("OMNIA_FAILPOINT_SEED", "0")))


def parse(spec: str) -> dict[str, _Point]:
    out = {}
    for item in (spec or "").split(","):
        item = item.strip()
        if not item:
            continue
        name, _, sp = item.partition(":")
        out[name.strip()] = _Point(sp or "always")
    return out


def configure(spec: str | None = None) -> None:
    """(Re)load from ``spec`` or ``OMNIA_FAILPOINT``."""
    global _points
    with _lock:
        _points = parse(os.environ.get("OMNIA_FAILPOINT", "") if spec is None else spec)


def arm(name: str, spec: str = "always") -> None:
    with _lock:
        _points[name] = _Point(spec)


def clear() -> None:
    with _lock:
        _points.clear()


def active() -> bool:
    return bool(_points)


def triggered(name: str) -> bool:
    """True when the failpoint fires on this hit (for non-raising hooks)."""
    if not _points:
        return False
    with _lock:
        p = _points.get(name)
        return p is not None and p.should_fire(_rng)


def hit(name: str) -> None:
    """Raise :class:`FailpointError` when ``name`` fires on this hit."""
    if _points and triggered(name):
        raise FailpointError(name)


def stats() -> dict:
    with _lock:
        return {k: {"spec": p.spec, "hits": p.hits, "fired": p.fired} for k, p in _points.items()}


configure()
