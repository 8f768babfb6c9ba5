"""Token-bucket rate limiter (``pkg/ratelimit/limiter.go``; facade split limits
50 msg/s burst 100 for text and 2 MiB/s burst 16 MiB for media,
``internal/facade/server_config.go:87-94``)."""
from __future__ import annotations

import time


class TokenBucket:
    def __init__(self, rate: float, burst: float, clock=time.monotonic):
        self.rate = float(rate)
        self.burst = float(burst)
        self.tokens = float(burst)
        self.clock = clock
        self.t = clock()

    def allow(self, n: float = 1.0) -> bool:
        now = self.clock()
        self.tokens = min(self.burst, self.tokens + (now - self.t) * self.rate)
        self.t = now
        if self.tokens >= n:
            self.tokens -= n
            return True
        return False


class KeyedLimiter:
    """Per-key buckets (e.g. per client IP for session-api)."""

    def __init__(self, rate: float, burst: float, max_keys: int = 100_000):
        self.rate, self.burst, self.max_keys = rate, burst, max_keys
        self.b: dict[str, TokenBucket] = {}

    def allow(self, key: str, n: float = 1.0) -> bool:
        bk = self.b.get(key)
        if bk is None:
            if len(self.b) >= self.max_keys:
                self.b.clear()
            bk = self.b[key] = TokenBucket(self.rate, self.burst)
        return bk.allow(n)
