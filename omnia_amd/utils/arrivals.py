"""Opt-in per-request stage timestamps (host-path latency hunting).

``OMNIA_TRACE_ARRIVALS=<dir>``: :func:`mark` appends ``<unix time> <tag>`` to
``<dir>/<pid>.txt`` (line-buffered) at each instrumented stage of a turn's start:
facade WS message in, runtime Converse message in, runtime engine submit,
engine-core add.  ``scripts/arrival_spread.py`` turns the files into per-stage
arrival spreads for the bench's waves.  With ``OMNIA_TIMELINE_DIR`` set the same stages go to
the buffered timeline instead (monotonic clock, one append per event)."""
from __future__ import annotations

import os
import time

from ..observability import timeline as _tl

_f = None
_dir = os.environ.get("OMNIA_TRACE_ARRIVALS") or ""


def mark(tag: str) -> None:
    global _f
    if _tl.ENABLED:  # the buffered cross-process timeline (observability/timeline.py)
        _tl.mark(tag)
        return
    if not _dir:
        return
    if _f is None:
        os.makedirs(_dir, exist_ok=True)
        _f = open(os.path.join(_dir, f"{os.getpid()}.txt"), "a", buffering=1)
    _f.write(f"{time.time():.6f} {tag}\n")
