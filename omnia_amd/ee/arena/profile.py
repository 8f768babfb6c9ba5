"""Load profile (``ee/cmd/arena-worker/load_profile.go``): linear ramp-up to the
target concurrency; ramp-down proportional to remaining work once fewer than
2 x target items are pending."""
from __future__ import annotations

import math


class LoadProfile:
    def __init__(self, concurrency: int, ramp_up_s: float = 0.0, ramp_down_s: float = 0.0):
        self.target = concurrency
        self.ramp_up = ramp_up_s
        self.ramp_down = ramp_down_s

    def allowed(self, elapsed_s: float, pending: int) -> int:
        if self.target <= 0:
            return 0
        if self.ramp_up <= 0 and self.ramp_down <= 0:
            return self.target
        allowed = self.target
        if self.ramp_up > 0 and elapsed_s < self.ramp_up:
            allowed = math.ceil(min(1.0, elapsed_s / self.ramp_up) * self.target)
        if self.ramp_down > 0:
            thr = self.target * 2
            rd = self.target if pending >= thr else max(1, math.ceil(pending / thr * self.target))
            allowed = min(allowed, rd)
        return allowed
