"""Tool-call resilience: per-tool circuit breaker and retry with backoff.

Reference: ``internal/runtime/tools/circuit_breaker.go:38-121`` (5 consecutive
failures -> open 30 s -> 1 half-open probe) and ``retry.go:33-153`` +
``retry_classify.go`` (exponential backoff with jitter, Retry-After honoured,
per-attempt timeout, only transient failures retried).
"""
from __future__ import annotations

import asyncio
import random
import time
from dataclasses import dataclass


class CircuitOpen(Exception):
    pass


class CircuitBreaker:
    CLOSED, OPEN, HALF_OPEN = "closed", "open", "half-open"

    def __init__(self, failure_threshold: int = 5, open_seconds: float = 30.0,
                 half_open_max: int = 1, clock=time.monotonic):
        self.failure_threshold = failure_threshold
        self.open_seconds = open_seconds
        self.half_open_max = half_open_max
        self.clock = clock
        self.state = self.CLOSED
        self.failures = 0
        self.opened_at = 0.0
        self.half_open_inflight = 0

    def allow(self) -> bool:
        if self.state == self.OPEN:
            if self.clock() - self.opened_at >= self.open_seconds:
                self.state = self.HALF_OPEN
                self.half_open_inflight = 0
            else:
                return False
        if self.state == self.HALF_OPEN:
            if self.half_open_inflight >= self.half_open_max:
                return False
            self.half_open_inflight += 1
        return True

    def record(self, ok: bool) -> None:
        if ok:
            self.state = self.CLOSED
            self.failures = 0
            self.half_open_inflight = 0
            return
        if self.state == self.HALF_OPEN:
            self._open()
            return
        self.failures += 1
        if self.failures >= self.failure_threshold:
            self._open()

    def _open(self):
        self.state = self.OPEN
        self.opened_at = self.clock()
        self.failures = 0
        self.half_open_inflight = 0


class TransientError(Exception):
    """Retryable failure (network, 5xx, 429, gRPC UNAVAILABLE...)."""

    def __init__(self, msg: str, retry_after: float | None = None):
        super().__init__(msg)
        self.retry_after = retry_after


class PermanentError(Exception):
    pass


@dataclass
class RetryPolicy:
    max_attempts: int = 3
    initial_backoff: float = 0.1
    multiplier: float = 2.0
    max_backoff: float = 5.0
    jitter: float = 0.2
    per_attempt_timeout: float | None = None
    respect_retry_after: bool = True
    retryable_status: tuple = (429, 502, 503, 504)

    @classmethod
    def from_cfg(cls, d: dict | None) -> "RetryPolicy":
        from ..runtime.context_store import parse_ttl

        if not d:
            return cls()

        def dur(v, default):
            if v is None:
                return default
            if isinstance(v, (int, float)):
                return float(v)
            s = str(v)
            if s.endswith("ms"):
                return float(s[:-2]) / 1000
            return float(parse_ttl(s) or default)

        return cls(max_attempts=int(d.get("maxAttempts", 3)),
                   initial_backoff=dur(d.get("initialBackoff"), 0.1),
                   multiplier=float(d.get("backoffMultiplier", 2.0)),
                   max_backoff=dur(d.get("maxBackoff"), 5.0),
                   retryable_status=tuple(int(x) for x in d.get("retryOn", [])
                                          if str(x).isdigit()) or (429, 502, 503, 504))

    def backoff(self, attempt: int) -> float:
        b = min(self.max_backoff, self.initial_backoff * self.multiplier ** attempt)
        return b * (1 + random.uniform(-self.jitter, self.jitter))


async def call_with_retry(fn, policy: RetryPolicy, sleep=asyncio.sleep):
    last = None
    for attempt in range(max(1, policy.max_attempts)):
        try:
            if policy.per_attempt_timeout:
                return await asyncio.wait_for(fn(), policy.per_attempt_timeout)
            return await fn()
        except (TransientError, asyncio.TimeoutError, ConnectionError, OSError) as e:
            last = e
            if attempt + 1 >= policy.max_attempts:
                break
            delay = policy.backoff(attempt)
            ra = getattr(e, "retry_after", None)
            if policy.respect_retry_after and ra:
                delay = min(max(delay, ra), policy.max_backoff * 4)
            await sleep(delay)
    raise last
