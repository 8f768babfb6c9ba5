"""Doctor check runner (``internal/doctor/runner.go``).

Checks are grouped by category in registration order.  Categories run
concurrently; the checks inside one category run in order (later checks may use
state the earlier ones left, e.g. the session the agent check opened), and
categories placed in one *sequential group* run one after another (the memory
and privacy probes share a user and must not interleave).  Every check emits a
``running`` marker and then its result through the optional ``on_result``
callback (the server streams both as SSE)."""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass
from typing import Awaitable, Callable

from .result import FAIL, PASS, RUNNING, CategoryResult, RunResult, TestResult


@dataclass
class Check:
    name: str
    category: str
    run: Callable[[], Awaitable[TestResult]]


class Runner:
    def __init__(self):
        self.checks: list[Check] = []
        self.sequential: dict[str, str] = {}  # category -> group name
        self._seq = 0

    def register(self, *checks: Check) -> "Runner":
        self.checks.extend(checks)
        return self

    def sequential_group(self, group: str, *categories: str) -> "Runner":
        for c in categories:
            self.sequential[c] = group
        return self

    async def _one(self, chk: Check, on_result, timeout_s: float) -> TestResult:
        if on_result:
            await on_result(TestResult(chk.name, chk.category, RUNNING))
        t0 = time.perf_counter()
        try:
            r = await asyncio.wait_for(chk.run(), timeout_s)
        except asyncio.TimeoutError:
            r = TestResult(status=FAIL, error=f"timed out after {timeout_s:.0f}s")
        except Exception as e:  # noqa: BLE001 - a check never takes the run down
            r = TestResult(status=FAIL, error=f"{type(e).__name__}: {e}")
        r.name, r.category = chk.name, chk.category
        r.duration_ms = (time.perf_counter() - t0) * 1e3
        if on_result:
            await on_result(r)
        return r

    async def run(self, on_result=None, timeout_s: float = 120.0) -> RunResult:
        self._seq += 1
        run = RunResult(id=f"{int(time.time() * 1000) % 100000}-{self._seq}")
        order: list[str] = []
        by_cat: dict[str, list[Check]] = {}
        for c in self.checks:
            if c.category not in by_cat:
                order.append(c.category)
                by_cat[c.category] = []
            by_cat[c.category].append(c)
        groups: list[list[str]] = []
        named: dict[str, list[str]] = {}
        for cat in order:
            g = self.sequential.get(cat)
            if g is None:
                groups.append([cat])
            elif g in named:
                named[g].append(cat)
            else:
                named[g] = [cat]
                groups.append(named[g])
        results: dict[str, CategoryResult] = {}

        async def run_group(cats):
            for cat in cats:
                cr = CategoryResult(cat)
                for chk in by_cat[cat]:
                    cr.tests.append(await self._one(chk, on_result, timeout_s))
                results[cat] = cr

        t0 = time.perf_counter()
        await asyncio.gather(*(run_group(g) for g in groups))
        run.categories = [results[c] for c in order]
        run.duration_ms = (time.perf_counter() - t0) * 1e3
        run.status = FAIL if run.summary["failed"] else PASS
        return run
