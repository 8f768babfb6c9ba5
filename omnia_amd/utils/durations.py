"""Go ``time.ParseDuration`` plus ``d`` days (``parseExtendedDuration`` in the
reference's policy packages): "720h", "30d", "1d12h", "90m", "1.5s"."""
from __future__ import annotations

import re

_GO_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h|d)")
_UNIT = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0,
         "d": 86400.0}


def parse_duration(s: str) -> float:
    """Seconds; ``ValueError`` on an empty or malformed duration."""
    if not s:
        raise ValueError("empty duration")
    pos, total = 0, 0.0
    for m in _GO_DUR.finditer(s):
        if m.start() != pos:
            break
        total += float(m.group(1)) * _UNIT[m.group(2)]
        pos = m.end()
    if pos != len(s) or pos == 0:
        raise ValueError(f"invalid duration {s!r}")
    return total
