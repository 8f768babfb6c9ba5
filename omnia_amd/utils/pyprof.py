"""Opt-in Python profiling of a serving process (host-overhead hunting).

``OMNIA_PYPROFILE=<dir>`` makes :func:`maybe_start` enable ``cProfile`` on the
calling (main / event-loop) thread; ``SIGUSR1`` then writes
``<dir>/<name>-<pid>.prof`` (and keeps profiling), so a benchmark can snapshot
the facade, runtime and engine-core processes of a pod after its timed waves
(bench.py does, when the variable is set).  Read with ``python -m pstats``."""
from __future__ import annotations

import os
import signal


def maybe_start(name: str) -> bool:
    d = os.environ.get("OMNIA_PYPROFILE")
    if not d:
        return False
    import cProfile

    os.makedirs(d, exist_ok=True)
    prof = cProfile.Profile()
    path = os.path.join(d, f"{name}-{os.getpid()}.prof")

    def dump(*_):
        prof.disable()
        try:
            prof.dump_stats(path)
        finally:
            prof.enable()

    signal.signal(signal.SIGUSR1, dump)
    prof.enable()
    return True
