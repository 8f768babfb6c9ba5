"""Arena worker: a virtual-user pool draining a job's work queue
(``ee/cmd/arena-worker/vu_pool.go:26-242``, ``worker_loop.go``).

Each work item is one scenario x provider run: the scenario's turns are played
over one session, every turn is timed (TTFT + latency) and its assertions are
checked with the runtime's eval assertions.  Providers run either in ``fleet``
mode (WebSocket to a deployed facade) or ``direct`` mode (an in-process
provider object, e.g. the local MI355X engine provider).  Concurrency follows
the :class:`LoadProfile`; a budget caps total spend."""
from __future__ import annotations

import asyncio
import logging
import os
import time
import uuid

from ...runtime.evals import evaluate
from .fleet import FleetSession
from .profile import LoadProfile
from .queue import WorkItem

log = logging.getLogger("omnia.arena.worker")


async def run_fleet(item: WorkItem, scenario: dict, provider: dict) -> dict:
    turns = []
    async with FleetSession(provider["url"], provider.get("agent", ""),
                            provider.get("headers")) as fs:
        for t in scenario.get("turns", []):
            r = await fs.turn(t["user"], t.get("metadata"))
            r["assertions"] = [evaluate(a, t["user"], r["content"])
                               for a in t.get("assertions", [])]
            turns.append(r)
    return _summarise(turns)


async def run_direct(item: WorkItem, scenario: dict, provider: dict) -> dict:
    from ...engine.sampling_params import SamplingParams
    from ...runtime.chat import Message

    prov = provider["object"]
    params = SamplingParams(**(provider.get("params") or {"temperature": 0.0,
                                                         "max_tokens": 128}))
    sid = f"arena-{item.id}"
    msgs = [Message("system", scenario.get("system", "You are a helpful assistant."))]
    turns = []
    for t in scenario.get("turns", []):
        msgs.append(Message("user", t["user"]))
        t0 = time.perf_counter()
        ttft, text, usage = None, [], None
        async for ev in prov.stream(msgs, [], params, session_id=sid,
                                    metadata=t.get("metadata")):
            if ev.type == "text":
                if ttft is None:
                    ttft = time.perf_counter() - t0
                text.append(ev.text)
            elif ev.type == "error":
                raise RuntimeError(ev.text)
            elif ev.type == "done":
                usage = ev.usage
        lat = time.perf_counter() - t0
        content = "".join(text)
        msgs.append(Message("assistant", content))
        turns.append({"content": content, "ttft_ms": (ttft or lat) * 1e3,
                      "latency_ms": lat * 1e3,
                      "usage": {"output_tokens": getattr(usage, "output_tokens", 0),
                                "cost": getattr(usage, "cost", 0.0)} if usage else {},
                      "assertions": [evaluate(a, t["user"], content)
                                     for a in t.get("assertions", [])]})
    return _summarise(turns)


def _summarise(turns: list[dict]) -> dict:
    checks = [a for t in turns for a in t["assertions"] if not a.get("skipped")]
    out_tok = sum(int((t.get("usage") or {}).get("output_tokens") or
                      (t.get("usage") or {}).get("outputTokens") or 0) for t in turns)
    cost = sum(float((t.get("usage") or {}).get("cost") or
                     (t.get("usage") or {}).get("costUsd") or 0.0) for t in turns)
    return {"passed": all(a.get("passed") for a in checks),
            "latency_ms": sum(t["latency_ms"] for t in turns),
            "ttft_ms": turns[0]["ttft_ms"] if turns else None,
            "turns": [{"latency_ms": t["latency_ms"], "ttft_ms": t["ttft_ms"]} for t in turns],
            "output_tokens": out_tok, "cost": cost,
            "assertions": checks}


class ArenaWorker:
    def __init__(self, queue, job_id: str, scenarios: dict, providers: dict,
                 profile: LoadProfile, budget: float | None = None,
                 consumer: str | None = None, visibility_s: float = 300.0):
        self.q = queue
        self.job = job_id
        self.scenarios = scenarios
        self.providers = providers
        self.profile = profile
        self.budget = budget
        self.consumer = consumer or f"worker-{os.getpid()}-{uuid.uuid4().hex[:6]}"
        self.visibility_s = visibility_s
        self.spent = 0.0
        self.active = 0
        self.done = 0

    async def _execute(self, item: WorkItem):
        scen = self.scenarios[item.scenario_id]
        prov = self.providers[item.provider_id]
        try:
            fn = run_fleet if prov.get("mode", "fleet") == "fleet" else run_direct
            res = await fn(item, scen, prov)
            res.update(scenario=item.scenario_id, provider=item.provider_id,
                       attempt=item.attempt)
            self.spent += res.get("cost") or 0.0
            await self.q.complete(item, res)
        except Exception as e:  # noqa: BLE001
            log.info("item %s failed: %s", item.id, e)
            await self.q.fail(item, str(e))
        finally:
            self.active -= 1
            self.done += 1

    async def run(self, idle_exit_s: float = 1.0):
        """Drain the queue; returns when it stays empty for ``idle_exit_s``."""
        t0 = time.monotonic()
        tasks: set[asyncio.Task] = set()
        idle_since = None
        while True:
            if self.budget is not None and self.spent >= self.budget:
                log.warning("arena budget exhausted (%.4f)", self.spent)
                break
            prog = await self.q.progress(self.job)
            allowed = self.profile.allowed(time.monotonic() - t0, prog["pending"])
            room = allowed - self.active
            items = await self.q.claim(self.job, self.consumer, room) if room > 0 else []
            for it in items:
                self.active += 1
                tk = asyncio.create_task(self._execute(it))
                tasks.add(tk)
                tk.add_done_callback(tasks.discard)
            if not items and self.active == 0:
                await self.q.reclaim(self.job, self.visibility_s)
                if (await self.q.progress(self.job))["pending"] == 0:
                    idle_since = idle_since or time.monotonic()
                    if time.monotonic() - idle_since >= idle_exit_s:
                        break
            else:
                idle_since = None
            await asyncio.sleep(0.005 if items else 0.02)
        if tasks:
            await asyncio.gather(*tasks, return_exceptions=True)
