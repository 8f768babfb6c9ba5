"""Standard cron schedules (robfig/cron ``ParseStandard`` semantics, UTC).

Five fields ``minute hour day-of-month month day-of-week`` with ``*``, lists,
ranges, steps (``*/15``, ``1-30/5``) and the descriptors ``@hourly``,
``@daily``/``@midnight``, ``@weekly``, ``@monthly``, ``@yearly``/``@annually``
and ``@every <duration>``.  Like cron, when both day-of-month and day-of-week
are restricted a day matches if EITHER does.  Used by the key-rotation and
retention controllers (reference: ``ee/internal/controller/keyrotation_controller.go``
``calculateNextRotation`` via ``cron.ParseStandard(...).Next``).
"""
from __future__ import annotations

import calendar
import re
import time
from dataclasses import dataclass

_DESCRIPTORS = {"@yearly": "0 0 1 1 *", "@annually": "0 0 1 1 *", "@monthly": "0 0 1 * *",
                "@weekly": "0 0 * * 0", "@daily": "0 0 * * *", "@midnight": "0 0 * * *",
                "@hourly": "0 * * * *"}
_BOUNDS = [(0, 59), (0, 23), (1, 31), (1, 12), (0, 6)]
_UNITS = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


class CronError(ValueError):
    pass


def _field(spec: str, lo: int, hi: int) -> tuple[frozenset, bool]:
    """-> (allowed values, restricted?)"""
    out = set()
    for part in spec.split(","):
        step = 1
        if "/" in part:
            part, s = part.split("/", 1)
            if not s.isdigit() or int(s) == 0:
                raise CronError(f"bad step in {spec!r}")
            step = int(s)
        if part in ("*", "?"):
            a, b = lo, hi
        elif "-" in part:
            x, y = part.split("-", 1)
            if not (x.isdigit() and y.isdigit()):
                raise CronError(f"bad range in {spec!r}")
            a, b = int(x), int(y)
        elif part.isdigit():
            a = int(part)
            b = hi if step > 1 else a
        else:
            raise CronError(f"bad cron field {spec!r}")
        if a < lo or b > hi or a > b:
            raise CronError(f"cron field {spec!r} out of range {lo}-{hi}")
        out.update(range(a, b + 1, step))
    return frozenset(out), spec not in ("*", "?")


def _duration(s: str) -> float:
    total, pos = 0.0, 0
    for m in re.finditer(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)", s):
        if m.start() != pos:
            raise CronError(f"bad duration {s!r}")
        total += float(m.group(1)) * _UNITS[m.group(2)]
        pos = m.end()
    if pos != len(s) or total <= 0:
        raise CronError(f"bad duration {s!r}")
    return total


@dataclass(frozen=True)
class Schedule:
    minute: frozenset = frozenset()
    hour: frozenset = frozenset()
    dom: frozenset = frozenset()
    month: frozenset = frozenset()
    dow: frozenset = frozenset()
    dom_star: bool = True
    dow_star: bool = True
    every_s: float = 0.0

    def _day_ok(self, y: int, mo: int, d: int) -> bool:
        if mo not in self.month:
            return False
        wd = (calendar.weekday(y, mo, d) + 1) % 7  # cron: 0 = Sunday
        if self.dom_star or self.dow_star:
            return d in self.dom and wd in self.dow
        return d in self.dom or wd in self.dow

    def next(self, after: float) -> float:
        """First fire time strictly after ``after`` (epoch seconds, UTC)."""
        if self.every_s:
            return after + self.every_s
        t = int(after // 60) * 60 + 60  # next whole minute
        g = time.gmtime(t)
        y, mo, d, h, mi = g.tm_year, g.tm_mon, g.tm_mday, g.tm_hour, g.tm_min
        for _ in range(366 * 5):  # at most five years of days
            if self._day_ok(y, mo, d):
                for hh in range(h, 24):
                    if hh not in self.hour:
                        continue
                    for mm in range(mi if hh == h else 0, 60):
                        if mm in self.minute:
                            return float(calendar.timegm((y, mo, d, hh, mm, 0)))
            # next day, from midnight
            h, mi = 0, 0
            d += 1
            if d > calendar.monthrange(y, mo)[1]:
                d, mo = 1, mo + 1
                if mo > 12:
                    mo, y = 1, y + 1
        raise CronError("schedule never fires")


def parse(expr: str) -> Schedule:
    e = " ".join((expr or "").split())
    if e.startswith("@every "):
        return Schedule(every_s=_duration(e[len("@every "):].strip()))
    e = _DESCRIPTORS.get(e, e)
    parts = e.split(" ")
    if len(parts) != 5:
        raise CronError(f"expected 5 cron fields, got {len(parts)} in {expr!r}")
    vals = []
    flags = []
    for p, (lo, hi) in zip(parts, _BOUNDS):
        if p == "7" and hi == 6:
            p = "0"
        v, r = _field(p, lo, hi)
        vals.append(v)
        flags.append(r)
    return Schedule(*vals, dom_star=not flags[2], dow_star=not flags[4])


def next_fire(expr: str, after: float) -> float:
    return parse(expr).next(after)
