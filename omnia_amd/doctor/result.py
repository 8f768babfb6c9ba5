"""Doctor result model (``internal/doctor/result.go``): a run is categories of
test results, each pass / fail / skip with a detail, an optional error and its
duration; ``running`` is the in-flight marker streamed before a check ends."""
from __future__ import annotations

import time
from dataclasses import asdict, dataclass, field

RUNNING, PASS, FAIL, SKIP = "running", "pass", "fail", "skip"


@dataclass
class TestResult:
    name: str = ""
    category: str = ""
    status: str = PASS
    duration_ms: float = 0.0
    detail: str = ""
    error: str = ""

    __test__ = False  # not a pytest class

    def to_json(self) -> dict:
        d = asdict(self)
        if not d["error"]:
            d.pop("error")
        return d


def passed(detail: str = "") -> TestResult:
    return TestResult(status=PASS, detail=detail)


def failed(error: str, detail: str = "") -> TestResult:
    return TestResult(status=FAIL, error=error, detail=detail)


def skipped(detail: str) -> TestResult:
    return TestResult(status=SKIP, detail=detail)


@dataclass
class CategoryResult:
    name: str
    tests: list[TestResult] = field(default_factory=list)


@dataclass
class RunResult:
    id: str
    status: str = RUNNING
    started_at: float = field(default_factory=time.time)
    duration_ms: float = 0.0
    categories: list[CategoryResult] = field(default_factory=list)

    @property
    def summary(self) -> dict:
        s = {"total": 0, "passed": 0, "failed": 0, "skipped": 0}
        key = {PASS: "passed", FAIL: "failed", SKIP: "skipped"}
        for c in self.categories:
            for t in c.tests:
                s["total"] += 1
                if t.status in key:
                    s[key[t.status]] += 1
        return s

    def results(self) -> list[TestResult]:
        return [t for c in self.categories for t in c.tests]

    def to_json(self) -> dict:
        return {"id": self.id, "status": self.status, "startedAt": self.started_at,
                "durationMs": self.duration_ms, "summary": self.summary,
                "categories": [{"name": c.name, "tests": [t.to_json() for t in c.tests]}
                               for c in self.categories]}
