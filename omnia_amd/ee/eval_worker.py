"""Eval worker (``ee/cmd/arena-eval-worker``, ``ee/pkg/evals``).

Consumes ``omnia:eval-events:<namespace>`` (consumer group ``eval-workers``)
published by session-api on every message append.  For each assistant message of
a sampled session it fetches the turn from session-api, runs the agent's eval
definitions and posts the results back (``POST /api/v1/eval-results``).

* sampling: deterministic per-session FNV-1a over ``"<session>:<tier>"`` % 100
  against a rate (lightweight tier default 100 %, extended/LLM-judge tier 10 %)
  (``sampling.go:27-95``);
* lightweight evals = the runtime's deterministic assertions; extended evals =
  LLM judge through any provider (the in-node engine by default), graded 1-5
  from a rubric prompt;
* token-bucket rate limit on judge calls and a spend budget
  (``rate_limiter.go``, ``budget_tracker.go``).
"""
from __future__ import annotations

import asyncio
import json
import logging
import re
import time

from ..runtime.evals import evaluate
from ..utils.ratelimit import TokenBucket

log = logging.getLogger("omnia.eval_worker")

DEFAULT_RATE = 100
DEFAULT_EXTENDED_RATE = 10
TIER_LIGHT, TIER_EXTENDED = "lightweight", "extended"
GROUP = "eval-workers"


def fnv1a32(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode():
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def should_sample(session_id: str, tier: str, rate: int) -> bool:
    if rate <= 0:
        return False
    if rate >= 100:
        return True
    return fnv1a32(f"{session_id}:{tier}") % 100 < rate


class Budget:
    def __init__(self, limit: float | None):
        self.limit, self.spent = limit, 0.0

    def allow(self) -> bool:
        return self.limit is None or self.spent < self.limit

    def add(self, cost: float):
        self.spent += cost or 0.0


JUDGE_PROMPT = ("You are grading an AI assistant's reply.\nCriteria: {criteria}\n"
                "User message: {user}\nAssistant reply: {output}\n"
                "Answer with a single line 'SCORE: <1-5>' followed by a short reason.")


async def llm_judge(provider, spec: dict, user: str, output: str) -> dict:
    from ..engine.sampling_params import SamplingParams
    from ..runtime.chat import Message

    p = spec.get("params") or {}
    prompt = JUDGE_PROMPT.format(criteria=p.get("criteria", "helpful, correct and safe"),
                                 user=user, output=output)
    text, cost = [], 0.0
    async for ev in provider.stream([Message("user", prompt)], [],
                                    SamplingParams(temperature=0.0, max_tokens=64)):
        if ev.type == "text":
            text.append(ev.text)
        elif ev.type == "done" and ev.usage is not None:
            cost = getattr(ev.usage, "cost", 0.0) or 0.0
    reply = "".join(text)
    m = re.search(r"SCORE:\s*([1-5])", reply)
    score = int(m.group(1)) / 5.0 if m else 0.0
    thr = float(p.get("pass_threshold", 0.6))
    return {"id": spec.get("id", "llm_judge"), "type": "llm_judge", "passed": score >= thr,
            "score": score, "details": {"reply": reply[:500]}, "cost": cost}


class EvalWorker:
    def __init__(self, redis, session_client, namespaces: list[str], eval_defs,
                 judge_provider=None, default_rate: int = DEFAULT_RATE,
                 extended_rate: int = DEFAULT_EXTENDED_RATE, judge_rps: float = 5.0,
                 budget: float | None = None, consumer: str = "eval-worker-0"):
        self.r = redis
        self.sessions = session_client  # async get_messages(session_id) -> list[dict]
        self.namespaces = namespaces
        self.eval_defs = eval_defs  # callable(agent, namespace) -> list[spec]
        self.judge = judge_provider
        self.rate, self.ext_rate = default_rate, extended_rate
        self.bucket = TokenBucket(judge_rps, max(1.0, judge_rps))
        self.budget = Budget(budget)
        self.consumer = consumer
        self.stats = {"events": 0, "evaluated": 0, "skipped": 0, "judge_calls": 0,
                      "rate_limited": 0, "budget_exhausted": 0}

    async def setup(self):
        for ns in self.namespaces:
            await self.r.xgroup_create(f"omnia:eval-events:{ns}", GROUP, "0")

    async def handle(self, ev: dict) -> list[dict]:
        self.stats["events"] += 1
        if ev.get("type") != "message.appended" or ev.get("role") != "assistant":
            self.stats["skipped"] += 1
            return []
        sid = ev.get("sessionId", "")
        tiers = [t for t, rate in ((TIER_LIGHT, self.rate), (TIER_EXTENDED, self.ext_rate))
                 if should_sample(sid, t, rate)]
        if not tiers:
            self.stats["skipped"] += 1
            return []
        msgs = await self.sessions.get_messages(sid)
        idx = next((i for i, m in enumerate(msgs) if m.get("id") == ev.get("messageId")),
                   len(msgs) - 1)
        output = msgs[idx].get("content", "") if msgs else ""
        user = next((m.get("content", "") for m in reversed(msgs[:idx])
                     if m.get("role") == "user"), "")
        results = []
        for spec in self.eval_defs(ev.get("agentName", ""), ev.get("namespace", "")):
            is_judge = spec.get("type") == "llm_judge"
            if is_judge:
                if TIER_EXTENDED not in tiers or self.judge is None:
                    continue
                if not self.budget.allow():
                    self.stats["budget_exhausted"] += 1
                    continue
                if not self.bucket.allow():
                    self.stats["rate_limited"] += 1
                    continue
                self.stats["judge_calls"] += 1
                r = await llm_judge(self.judge, spec, user, output)
                self.budget.add(r.pop("cost", 0.0))
            else:
                if TIER_LIGHT not in tiers:
                    continue
                r = evaluate(spec, user, output)
                if r.get("skipped"):
                    continue
            results.append({"sessionId": sid, "messageId": ev.get("messageId", ""),
                            "evalId": r["id"], "evalType": r["type"], "passed": r["passed"],
                            "score": r.get("score", 0.0), "details": r.get("details", {}),
                            "source": "worker", "agentName": ev.get("agentName", ""),
                            "namespace": ev.get("namespace", "")})
        if results:
            await self.sessions.post_eval_results(results)
            self.stats["evaluated"] += len(results)
        return results

    async def poll_once(self, count: int = 50) -> int:
        n = 0
        for ns in self.namespaces:
            stream = f"omnia:eval-events:{ns}"
            resp = await self.r.xreadgroup(GROUP, self.consumer, {stream: ">"}, count=count)
            for _s, entries in resp or []:
                for eid, fields in entries:
                    f = dict(zip(fields[::2], fields[1::2]))
                    raw = f.get(b"event") or f.get("event")
                    try:
                        await self.handle(json.loads(raw))
                    except Exception as e:  # noqa: BLE001 - never wedge the stream
                        log.warning("eval event failed: %s", e)
                    await self.r.xack(stream, GROUP, eid)
                    n += 1
        return n

    async def run(self, idle_sleep: float = 0.5):
        await self.setup()
        while True:
            if await self.poll_once() == 0:
                await asyncio.sleep(idle_sleep)


class SessionAPIClient:
    """The two session-api calls the worker needs."""

    def __init__(self, base_url: str):
        self.base = base_url.rstrip("/")

    async def get_messages(self, sid: str) -> list[dict]:
        import aiohttp

        async with aiohttp.ClientSession() as s:
            async with s.get(f"{self.base}/api/v1/sessions/{sid}/messages") as r:
                d = await r.json()
        return d.get("messages", d if isinstance(d, list) else [])

    async def post_eval_results(self, results: list[dict]):
        import aiohttp

        async with aiohttp.ClientSession() as s:
            async with s.post(f"{self.base}/api/v1/eval-results",
                              json={"results": results}) as r:
                if r.status >= 400:
                    raise RuntimeError(f"eval-results POST {r.status}")


def _now():
    return time.time()
