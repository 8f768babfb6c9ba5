"""Aggregation + threshold evaluation (``ee/pkg/arena/aggregator``,
``ee/pkg/arena/threshold/evaluator.go:112-209``).

Beyond the reference (which reports percentile metrics as "unavailable"), the
per-item latencies and TTFTs are kept, so p50/p90/p95/p99 are real.
Unavailable metrics and unparseable targets pass, like the reference."""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field


@dataclass
class JobStats:
    total: int = 0
    passed: int = 0
    failed: int = 0
    errors: int = 0
    total_cost: float = 0.0
    tokens: int = 0
    wall_s: float = 0.0
    latencies_ms: list = field(default_factory=list)
    ttfts_ms: list = field(default_factory=list)

    @classmethod
    def from_results(cls, results: list[dict], wall_s: float = 0.0) -> "JobStats":
        s = cls(wall_s=wall_s)
        for r in results:
            s.total += 1
            if r.get("error"):
                s.errors += 1
            if r.get("passed"):
                s.passed += 1
            else:
                s.failed += 1
            s.total_cost += float(r.get("cost") or 0.0)
            s.tokens += int(r.get("output_tokens") or 0)
            if r.get("latency_ms") is not None:
                s.latencies_ms.append(float(r["latency_ms"]))
            if r.get("ttft_ms") is not None:
                s.ttfts_ms.append(float(r["ttft_ms"]))
        return s

    def to_json(self) -> dict:
        out = {"total": self.total, "passed": self.passed, "failed": self.failed,
               "errors": self.errors, "totalCost": round(self.total_cost, 6),
               "outputTokens": self.tokens}
        for m in METRICS:
            v = metric(self, m)
            if v is not None:
                out[m] = round(v, 6)
        return out


def _pct(xs: list, q: float):
    if not xs:
        return None
    s = sorted(xs)
    k = (len(s) - 1) * q
    lo, hi = math.floor(k), math.ceil(k)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


METRICS = ("latency_avg", "latency_p50", "latency_p90", "latency_p95", "latency_p99",
           "ttft_avg", "ttft_p50", "ttft_p90", "ttft_p95", "ttft_p99", "error_rate",
           "pass_rate", "total_cost", "tokens_per_second")


def metric(s: JobStats, name: str):
    """Latency / TTFT metrics in seconds."""
    if name.startswith(("latency_", "ttft_")):
        xs = s.latencies_ms if name.startswith("latency_") else s.ttfts_ms
        if not xs:
            return None
        kind = name.split("_", 1)[1]
        v = sum(xs) / len(xs) if kind == "avg" else _pct(xs, int(kind[1:]) / 100)
        return v / 1000.0
    if name == "error_rate":
        return s.errors / s.total if s.total else None
    if name == "pass_rate":
        return s.passed / s.total if s.total else None
    if name == "total_cost":
        return s.total_cost
    if name == "tokens_per_second":
        return s.tokens / s.wall_s if s.wall_s > 0 else None
    return None


_DUR = re.compile(r"^\s*([\d.]+)\s*(ms|s|m|h)?\s*$")


def parse_target(name: str, value: str) -> float:
    v = str(value)
    if name.startswith(("latency_", "ttft_")):
        m = _DUR.match(v)
        if not m:
            raise ValueError(v)
        x = float(m.group(1))
        return x * {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0, None: 1.0}[m.group(2)]
    return float(v)


@dataclass
class ThresholdResult:
    metric: str
    operator: str
    target: str
    actual: float | None
    passed: bool

    def __str__(self):
        a = "unavailable" if self.actual is None else f"{self.actual:.4g}"
        return f"{self.metric}: {a} {self.operator} {self.target} {'PASS' if self.passed else 'FAIL'}"


def evaluate(thresholds: list[dict], s: JobStats) -> tuple[list[ThresholdResult], bool]:
    """thresholds: [{"metric": m, "max": v} | {"metric": m, "min": v} |
    {"metric": m, "operator": "<", "value": v}]"""
    out, ok = [], True
    ops = {"<": lambda a, b: a < b, "<=": lambda a, b: a <= b, ">": lambda a, b: a > b,
           ">=": lambda a, b: a >= b}
    for t in thresholds or []:
        name = t.get("metric", "")
        if "max" in t:
            op, tv = "<=", t["max"]
        elif "min" in t:
            op, tv = ">=", t["min"]
        else:
            op, tv = t.get("operator", "<="), t.get("value")
        actual = metric(s, name)
        try:
            passed = True if actual is None else ops[op](actual, parse_target(name, tv))
        except (ValueError, KeyError, TypeError):
            passed = True
        out.append(ThresholdResult(name, op, str(tv), actual, passed))
        ok &= passed
    return out, ok
