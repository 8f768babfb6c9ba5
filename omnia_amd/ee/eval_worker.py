"""Eval worker (``ee/cmd/arena-eval-worker``, ``ee/pkg/evals``).

Consumes the session event streams ``omnia:eval-events:<namespace>`` (consumer
group ``eval-workers``) that session-api publishes and runs the agent's
PromptPack evals out of band, writing results back to session-api
(``POST /api/v1/eval-results``).  Triggers (``worker_triggers.go``):

* ``message.assistant`` (legacy ``message.appended`` with role assistant) --
  per-turn evals (``every_turn`` / ``sample_turns``) on the new reply; the
  session is recorded as active in the completion tracker;
* ``session.completed`` -- session-level evals (``on_session_complete`` /
  ``sample_sessions``) over the whole transcript; sessions that simply go
  quiet for ``inactivity_timeout_s`` complete too (``completion_tracker.go``:
  each session completes once, tracker entries are evicted after 2x timeout);
* ``session.evaluate`` -- on-demand evaluation of a session (``POST
  /api/v1/sessions/{id}/evaluate``), results tagged ``source: manual``.

Where the evals come from (``promptpack_loader.go``): the session's PromptPack
(name + version carried by the event) loaded through a pack source -- the
PromptPack CR's ConfigMap via the kube API in a cluster -- and cached per
(namespace, pack) until the version changes.  Only evals of the WORKER groups
run here (``AgentRuntime.spec.evals.worker.groups``, default
``long-running`` + ``external``); deterministic ``fast-running`` evals run
inline in the runtime, so no eval runs on both paths.

Judges: an ``llm_judge`` eval's ``params.provider`` names one of the agent's
providers, resolved from its Provider CRs (``provider_resolver.go:33-54``,
cached 5 min), falling back to the worker's default judge (the in-node engine).

Sampling (``sampling.go``): deterministic per-session FNV-1a over
``"<session>:<tier>"`` % 100 against the agent's ``spec.evals.sampling`` rates
(lightweight default 100 %, extended/LLM-judge 10 %), plus a per-eval
``sample_percentage`` for the ``sample_*`` triggers.  Judge calls pass a token
bucket and a spend budget (``rate_limiter.go``, ``budget_tracker.go``).

Alerts (``webhook_dispatcher.go:45-366``): after results are written each eval's
recent window is checked against every configured webhook -- pass rate below
``threshold`` over the last ``windowSize`` results, or ``consecutiveFails`` in a
row -- and fired (JSON payload, retries with backoff, 1-minute rate limit per
(eval, url), absolute http(s) URLs only).

Delivery (``worker_consume.go``): an event is acked only after its results are
written; a failure leaves it pending, and pending entries idle longer than
``reclaim_min_idle_s`` are re-claimed (XAUTOCLAIM) and retried, up to
``max_deliveries`` attempts (then dead-lettered: acked and counted).
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging
import os
import re
import time
import urllib.parse

from ..runtime.evals import JUDGE_TYPES, EvalContext, evaluate, groups_of
from ..utils.ratelimit import TokenBucket

log = logging.getLogger("omnia.eval_worker")

DEFAULT_RATE = 100
DEFAULT_EXTENDED_RATE = 10
TIER_LIGHT, TIER_EXTENDED = "lightweight", "extended"
GROUP = "eval-workers"
EV_MESSAGE, EV_MESSAGE_LEGACY = "message.assistant", "message.appended"
EV_SESSION_DONE, EV_EVALUATE = "session.completed", "session.evaluate"
TURN_TRIGGERS = ("every_turn", "per_turn", "sample_turns")
SESSION_TRIGGERS = ("on_session_complete", "sample_sessions")
GROUP_FAST, GROUP_LONG, GROUP_EXTERNAL = "fast-running", "long-running", "external"
DEFAULT_WORKER_GROUPS = (GROUP_LONG, GROUP_EXTERNAL)
# JUDGE_TYPES (llm_judge, llm_judge_turn, llm_judge_session, ...) and every
# deterministic type come from the one registry in runtime/evals.py


def fnv1a32(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode():
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def should_sample(session_id: str, tier: str, rate: float) -> bool:
    if rate <= 0:
        return False
    if rate >= 100:
        return True
    return fnv1a32(f"{session_id}:{tier}") % 100 < rate


def eval_groups(spec: dict) -> list[str]:
    """An eval's groups: ``params.groups`` when set, else its registered type's
    (judges call a model: long-running + external; deterministic assertions:
    fast-running)."""
    return groups_of(spec)


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
    prompt = (p.get("judge_prompt") or JUDGE_PROMPT).format(
        criteria=p.get("criteria", "helpful, correct and safe"), user=user, output=output)
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
    thr = float(p.get("pass_threshold", p.get("passing_score", 3) / 5.0
                      if "passing_score" in p else 0.6))
    return {"id": spec.get("id", "llm_judge"), "type": spec.get("type", "llm_judge"),
            "passed": score >= thr, "score": score, "details": {"reply": reply[:500]},
            "cost": cost}


# ------------------------------------------------------------------ completion
class CompletionTracker:
    """Sessions complete on an explicit ``session.completed`` event or after
    ``timeout_s`` without activity -- exactly once each (``completion_tracker.go``)."""

    def __init__(self, timeout_s: float, on_complete=None, now=time.monotonic):
        self.timeout_s = timeout_s
        self.on_complete = on_complete  # async (session_id) -> None
        self.now = now
        self.last_seen: dict[str, float] = {}
        self.completed: set = set()

    def record_activity(self, sid: str):
        if sid not in self.completed:
            self.last_seen[sid] = self.now()

    async def mark_completed(self, sid: str):
        """Explicit ``session.completed``: run the session evals now.  Unlike the
        inactivity path, a failure PROPAGATES and the session is not marked
        completed, so the stream entry stays un-acked (XAUTOCLAIM retries it,
        then dead-letters) instead of the evals being lost."""
        if sid in self.completed:
            return
        self.completed.add(sid)
        self.last_seen.setdefault(sid, self.now())
        if self.on_complete is None:
            return
        try:
            await self.on_complete(sid)
        except BaseException:
            self.completed.discard(sid)  # a redelivery runs the evals again
            raise

    def _expired(self) -> list[str]:
        now = self.now()
        out = []
        for sid, t in list(self.last_seen.items()):
            age = now - t
            if sid in self.completed:
                if age >= 2 * self.timeout_s:  # evict finished entries
                    self.last_seen.pop(sid, None)
                    self.completed.discard(sid)
                continue
            if age >= self.timeout_s:
                self.completed.add(sid)
                out.append(sid)
        return out

    async def check_inactive(self) -> list[str]:
        expired = self._expired()
        for sid in expired:
            await self._fire(sid)
        return expired

    async def _fire(self, sid: str):
        if self.on_complete is None:
            return
        try:
            await self.on_complete(sid)
        except Exception as e:  # noqa: BLE001
            log.error("completion callback failed for %s: %s", sid, e)

    def cleanup(self, sid: str):
        self.last_seen.pop(sid, None)
        self.completed.discard(sid)

    @property
    def tracked(self) -> int:
        return len(self.last_seen)


# ------------------------------------------------------------------ webhooks
def validate_webhook_url(url: str) -> None:
    p = urllib.parse.urlparse(url)
    if not p.scheme or not p.netloc:
        raise ValueError("URL must be absolute")
    if p.scheme not in ("http", "https"):
        raise ValueError(f"unsupported scheme {p.scheme!r}")
    if not p.hostname:
        raise ValueError("URL must include hostname")


class WebhookDispatcher:
    """Eval alert webhooks (``webhook_dispatcher.go``).  ``configs``: dicts with
    ``url``, ``threshold`` (pass-rate floor), ``windowSize``, ``consecutiveFails``,
    ``headers``."""

    RATE_LIMIT_S = 60.0
    MAX_RETRIES = 3

    def __init__(self, configs: list[dict], post=None, backoff_s: float = 1.0):
        self.configs = list(configs or [])
        self.post = post or self._http_post  # async (url, body, headers) -> status
        self.backoff_s = backoff_s
        self.last_fired: dict[str, float] = {}
        self.sent: list[dict] = []
        self.stats = {"fired": 0, "rate_limited": 0, "failed": 0, "invalid_url": 0}
        self._session = None

    async def _http_post(self, url: str, body: bytes, headers: dict) -> int:
        import aiohttp

        if self._session is None:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=10))
        async with self._session.post(url, data=body, headers=headers) as r:
            return r.status

    async def close(self):
        if self._session is not None:
            await self._session.close()
            self._session = None

    @staticmethod
    def pass_rate(results: list[dict]) -> float:
        return sum(1 for r in results if r.get("passed")) / len(results) if results else 1.0

    @staticmethod
    def consecutive_fails(results: list[dict]) -> int:
        n = 0
        for r in reversed(results):
            if r.get("passed"):
                break
            n += 1
        return n

    def should_fire(self, cfg: dict, window: list[dict]) -> bool:
        if not window:
            return False
        if self.pass_rate(window) < float(cfg.get("threshold", 0.0)):
            return True
        cf = int(cfg.get("consecutiveFails", 0) or 0)
        return cf > 0 and self.consecutive_fails(window) >= cf

    async def check_and_fire(self, eval_id: str, agent: str, namespace: str,
                             recent: list[dict]) -> int:
        fired = 0
        mine = [r for r in recent if r.get("evalId") == eval_id]
        now = time.time()
        for k in [k for k, t in self.last_fired.items() if now - t >= 3600]:
            self.last_fired.pop(k, None)  # lastFiredMaxAge
        for cfg in self.configs:
            ws = int(cfg.get("windowSize", 0) or 0)
            window = mine[-ws:] if 0 < ws < len(mine) else mine
            if not self.should_fire(cfg, window):
                continue
            key = f"{eval_id}|{cfg['url']}"
            if now - self.last_fired.get(key, float("-inf")) < self.RATE_LIMIT_S:
                self.stats["rate_limited"] += 1
                continue
            try:
                validate_webhook_url(cfg["url"])
            except ValueError as e:
                self.stats["invalid_url"] += 1
                log.error("invalid webhook URL %s: %s", cfg.get("url"), e)
                continue
            payload = {"agentName": agent, "namespace": namespace, "evalId": eval_id,
                       "currentPassRate": self.pass_rate(window),
                       "threshold": float(cfg.get("threshold", 0.0)),
                       "windowSize": len(window),
                       "triggeredAt": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
                       "recentFailures": [{"sessionId": r.get("sessionId", ""),
                                           "messageId": r.get("messageId", ""),
                                           "createdAt": r.get("createdAt", "")}
                                          for r in window if not r.get("passed")]}
            body = json.dumps(payload).encode()
            hdrs = {"Content-Type": "application/json", **(cfg.get("headers") or {})}
            backoff, ok = self.backoff_s, False
            for attempt in range(self.MAX_RETRIES):
                if attempt:
                    await asyncio.sleep(backoff)
                    backoff *= 2
                try:
                    st = await self.post(cfg["url"], body, hdrs)
                    ok = st < 400
                except Exception as e:  # noqa: BLE001
                    log.warning("webhook attempt %d to %s failed: %s", attempt + 1, cfg["url"], e)
                if ok:
                    break
            if ok:
                self.last_fired[key] = now
                self.stats["fired"] += 1
                self.sent.append(payload)
                fired += 1
            else:
                self.stats["failed"] += 1
        return fired


# ------------------------------------------------------------------ pack evals
class PackEvalLoader:
    """PromptPack evals by (namespace, pack), cached until the version moves
    (``promptpack_loader.go``).  ``source``: async (namespace, name, version) ->
    pack dict (or None)."""

    def __init__(self, source):
        self.source = source
        self.cache: dict[tuple, tuple[str, dict]] = {}
        self.loads = 0

    async def load(self, namespace: str, name: str, version: str = "") -> dict | None:
        if not name:
            return None
        hit = self.cache.get((namespace, name))
        if hit is not None and (not version or hit[0] == version):
            return hit[1]
        pack = await self.source(namespace, name, version)
        self.loads += 1
        if not pack:
            return None
        evals = list(pack.get("evals") or [])
        for p in (pack.get("prompts") or {}).values():
            evals.extend(p.get("evals") or [])
        out = {"packName": pack.get("id") or name, "packVersion": pack.get("version", version),
               "evals": [e for e in evals if e.get("enabled", True)]}
        self.cache[(namespace, name)] = (out["packVersion"], out)
        return out


class KubePackSource:
    """The PromptPack CR's ConfigMap (``pack.json``) through the kube API."""

    def __init__(self, kube):
        self.kube = kube

    async def __call__(self, namespace: str, name: str, version: str = ""):
        loop = asyncio.get_running_loop()

        def get():
            pp = self.kube.get("PromptPack", name, namespace)
            src = (pp.get("spec") or {}).get("source") or {}
            cm_name = (src.get("configMapRef") or {}).get("name") or f"{name}-pack"
            cm = self.kube.get("ConfigMap", cm_name, namespace)
            data = (cm.get("data") or {})
            raw = data.get("pack.json") or next(iter(data.values()), None)
            return json.loads(raw) if raw else None

        try:
            return await loop.run_in_executor(None, get)
        except Exception as e:  # noqa: BLE001
            log.warning("pack %s/%s unavailable: %s", namespace, name, e)
            return None


class ProviderResolver:
    """Judge providers, sampling and worker groups of an agent from its
    AgentRuntime / Provider CRs (``provider_resolver.go``), cached ``ttl_s``."""

    def __init__(self, kube, ttl_s: float = 300.0, build=None, now=time.monotonic):
        self.kube = kube
        self.ttl_s = ttl_s
        self.now = now
        if build is None:
            from ..runtime.providers import build_provider as build
        self.build = build
        self.cache: dict[str, tuple[float, dict]] = {}

    def _agent(self, agent: str, ns: str) -> dict | None:
        try:
            return self.kube.get("AgentRuntime", agent, ns)
        except Exception:  # noqa: BLE001
            return None

    def providers(self, agent: str, ns: str) -> dict:
        key = f"{ns}/{agent}"
        hit = self.cache.get(key)
        if hit is not None and self.now() < hit[0]:
            return hit[1]
        ar = self._agent(agent, ns)
        out = {}
        for np in ((ar or {}).get("spec") or {}).get("providers") or []:
            ref = np.get("providerRef") or {}
            try:
                pr = self.kube.get("Provider", ref.get("name", np.get("name", "")),
                                   ref.get("namespace") or ns)
                out[np.get("name") or ref.get("name")] = self.build(pr.get("spec") or {})
            except Exception as e:  # noqa: BLE001
                log.warning("provider %s of %s/%s unresolved: %s", np.get("name"), ns, agent, e)
        self.cache[key] = (self.now() + self.ttl_s, out)
        return out

    def sampling(self, agent: str, ns: str) -> dict:
        ar = self._agent(agent, ns) or {}
        return ((ar.get("spec") or {}).get("evals") or {}).get("sampling") or {}

    def worker_groups(self, agent: str, ns: str) -> list[str] | None:
        """None when the agent is unknown (no filtering); default groups when the
        agent sets none."""
        ar = self._agent(agent, ns)
        if ar is None:
            return None
        w = ((ar.get("spec") or {}).get("evals") or {}).get("worker") or {}
        return list(w.get("groups") or DEFAULT_WORKER_GROUPS)


# ------------------------------------------------------------------ worker
class EvalWorker:
    def __init__(self, redis, session_client, namespaces: list[str], eval_defs=None,
                 judge_provider=None, default_rate: int = DEFAULT_RATE,
                 extended_rate: int = DEFAULT_EXTENDED_RATE, judge_rps: float = 5.0,
                 budget: float | None = None, consumer: str = "eval-worker-0",
                 pack_loader: PackEvalLoader | None = None, resolver=None,
                 webhooks: WebhookDispatcher | None = None,
                 inactivity_timeout_s: float = 300.0, reclaim_min_idle_s: float = 120.0,
                 reclaim_interval_s: float = 30.0, max_deliveries: int = 5):
        self.r = redis
        self.sessions = session_client
        self.namespaces = namespaces
        self.eval_defs = eval_defs  # legacy: callable(agent, namespace) -> list[spec]
        self.judge = judge_provider
        self.rate, self.ext_rate = default_rate, extended_rate
        self.bucket = TokenBucket(judge_rps, max(1.0, judge_rps))
        self.budget = Budget(budget)
        self.consumer = consumer
        self.packs = pack_loader
        self.resolver = resolver
        self.webhooks = webhooks
        self.tracker = CompletionTracker(inactivity_timeout_s, self._on_session_complete)
        self.reclaim_min_idle_s = reclaim_min_idle_s
        self.reclaim_interval_s = reclaim_interval_s
        self._last_reclaim = float("-inf")
        self.max_deliveries = max_deliveries
        self.deliveries: dict[str, int] = {}
        self.recent: dict[tuple, collections.deque] = {}
        self._done_events: dict[str, dict] = {}
        self.stats = {"events": 0, "evaluated": 0, "skipped": 0, "judge_calls": 0,
                      "rate_limited": 0, "budget_exhausted": 0, "failed": 0, "retried": 0,
                      "dead_lettered": 0, "session_completions": 0, "manual": 0,
                      "reclaimed": 0}

    async def setup(self):
        for ns in self.namespaces:
            await self.r.xgroup_create(f"omnia:eval-events:{ns}", GROUP, "0")

    # ---------------------------------------------------------- eval sources
    async def _evals(self, ev: dict, triggers) -> tuple[list[dict], dict]:
        """(eval specs for these triggers, pack info) -- pack evals when a pack
        loader is configured and the session has a pack, else the legacy
        ``eval_defs`` callable; filtered to this worker's eval groups."""
        agent, ns = ev.get("agentName", ""), ev.get("namespace", "")
        info = {"packName": ev.get("promptPackName", ""),
                "packVersion": ev.get("promptPackVersion", "")}
        specs: list[dict] = []
        if self.packs is not None and info["packName"]:
            pack = await self.packs.load(ns, info["packName"], info["packVersion"])
            if pack is None:
                return [], info
            info = {"packName": pack["packName"], "packVersion": pack["packVersion"]}
            specs = [e for e in pack["evals"] if e.get("trigger", "every_turn") in triggers]
        elif self.eval_defs is not None:
            specs = [e for e in self.eval_defs(agent, ns)
                     if e.get("trigger", "every_turn") in triggers]
        groups = self.resolver.worker_groups(agent, ns) if self.resolver is not None else None
        if groups is not None:
            specs = [e for e in specs if set(eval_groups(e)) & set(groups)]
        return specs, info

    def _rates(self, agent: str, ns: str) -> tuple[float, float]:
        if self.resolver is not None:
            s = self.resolver.sampling(agent, ns)
            return (float(s.get("defaultRate", self.rate)),
                    float(s.get("extendedRate", self.ext_rate)))
        return self.rate, self.ext_rate

    def _judge_for(self, spec: dict, agent: str, ns: str):
        name = (spec.get("params") or {}).get("provider")
        if name and self.resolver is not None:
            p = self.resolver.providers(agent, ns).get(name)
            if p is not None:
                return p
        return self.judge

    # ---------------------------------------------------------- running evals
    async def _tool_calls(self, sid: str, since: float | None = None,
                          until: float | None = None) -> list[dict]:
        """The session's tool calls (session-api ``tool_calls`` rows, one per call
        id, final status wins) in call order, optionally within [since, until]."""
        get = getattr(self.sessions, "get_tool_calls", None)
        if get is None:
            return []
        rows = await get(sid)
        by_id: dict = {}
        for r in sorted(rows, key=lambda r: r.get("createdAt", r.get("created_at", 0)) or 0):
            t = r.get("createdAt", r.get("created_at", 0)) or 0
            if since is not None and isinstance(t, (int, float)) and t < since:
                continue
            if until is not None and isinstance(t, (int, float)) and t > until:
                continue
            key = r.get("callId") or r.get("call_id") or r.get("id")
            st = r.get("status", "success")
            prev = by_id.get(key)
            if prev is None or st != "pending":
                by_id[key] = {"name": r.get("name", ""), "arguments": r.get("arguments") or {},
                              "error": st == "error", "status": st}
        return list(by_id.values())

    async def _run_specs(self, specs, ev: dict, user: str, output: str, message_id: str,
                         sampling_key: str, manual: bool = False,
                         ctx: EvalContext | None = None) -> list[dict]:
        agent, ns, sid = ev.get("agentName", ""), ev.get("namespace", ""), ev.get("sessionId", "")
        light_rate, ext_rate = self._rates(agent, ns)
        results = []
        for spec in specs:
            is_judge = spec.get("type") in JUDGE_TYPES
            if not manual:
                tier = TIER_EXTENDED if is_judge else TIER_LIGHT
                if not should_sample(sampling_key, tier, ext_rate if is_judge else light_rate):
                    continue
                trig = spec.get("trigger", "every_turn")
                if trig in ("sample_turns", "sample_sessions") and not should_sample(
                        f"{sampling_key}:{spec.get('id')}", "pct",
                        float(spec.get("sample_percentage", 5))):
                    continue
            if is_judge:
                judge = self._judge_for(spec, agent, ns)
                if judge is None:
                    continue
                if not self.budget.allow():
                    self.stats["budget_exhausted"] += 1
                    continue
                if not self.bucket.allow():
                    self.stats["rate_limited"] += 1
                    continue
                self.stats["judge_calls"] += 1
                r = await llm_judge(judge, spec, user, output)
                self.budget.add(r.pop("cost", 0.0))
            else:
                r = evaluate(spec, ctx or EvalContext(output=output, user=user))
                if r.get("skipped"):
                    continue
                if r.get("error"):  # unknown type / bad params: an error row, not a drop
                    r.setdefault("details", {})["error"] = r["error"]
            results.append({"sessionId": sid, "messageId": message_id, "evalId": r["id"],
                            "evalType": r["type"], "passed": r["passed"],
                            "score": r.get("score", 0.0), "details": r.get("details", {}),
                            "trigger": spec.get("trigger", "every_turn"),
                            "source": "manual" if manual else "worker", "agentName": agent,
                            "namespace": ns, "promptPackName": ev.get("promptPackName", ""),
                            "promptPackVersion": ev.get("promptPackVersion", ""),
                            "createdAt": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())})
        return results

    async def _write(self, results: list[dict]):
        if not results:
            return
        await self.sessions.post_eval_results(results)  # raises -> event stays pending
        self.stats["evaluated"] += len(results)
        for r in results:
            key = (r["namespace"], r["agentName"], r["evalId"])
            self.recent.setdefault(key, collections.deque(maxlen=200)).append(r)
        if self.webhooks is not None:
            for key in {(r["namespace"], r["agentName"], r["evalId"]) for r in results}:
                await self.webhooks.check_and_fire(key[2], key[1], key[0],
                                                   list(self.recent[key]))

    async def _session_meta(self, ev: dict) -> dict:
        if ev.get("agentName") and ev.get("promptPackName") is not None:
            return ev
        get = getattr(self.sessions, "get_session", None)
        if get is None:
            return ev
        s = await get(ev["sessionId"]) or {}
        return {**ev, "agentName": ev.get("agentName") or s.get("agentName", ""),
                "namespace": ev.get("namespace") or s.get("namespace", ""),
                "promptPackName": ev.get("promptPackName") or s.get("promptPackName", ""),
                "promptPackVersion": ev.get("promptPackVersion") or
                s.get("promptPackVersion", "")}

    async def process_turn(self, ev: dict) -> list[dict]:
        sid = ev.get("sessionId", "")
        self.tracker.record_activity(sid)
        specs, info = await self._evals(ev, TURN_TRIGGERS)
        if not specs:
            self.stats["skipped"] += 1
            return []
        msgs = await self.sessions.get_messages(sid)
        idx = next((i for i, m in enumerate(msgs) if m.get("id") == ev.get("messageId")),
                   len(msgs) - 1)
        output = msgs[idx].get("content", "") if msgs else ""
        user = next((m.get("content", "") for m in reversed(msgs[:idx])
                     if m.get("role") == "user"), "")
        ev = {**ev, **{k: v for k, v in (("promptPackName", info["packName"]),
                                         ("promptPackVersion", info["packVersion"])) if v}}
        ctx = None
        if any(not e.get("type") in JUDGE_TYPES for e in specs):
            # the turn's tool calls: those recorded after its user message
            t_user = next((m.get("timestamp") for m in reversed(msgs[:idx])
                           if m.get("role") == "user"), None)
            t_out = msgs[idx].get("timestamp") if msgs else None
            ctx = EvalContext(output=output, user=user,
                              tool_calls=await self._tool_calls(sid, t_user, t_out))
        results = await self._run_specs(specs, ev, user, output, ev.get("messageId", ""), sid,
                                        ctx=ctx)
        await self._write(results)
        return results

    async def _session_evals(self, ev: dict, manual: bool) -> list[dict]:
        ev = await self._session_meta(ev)
        sid = ev["sessionId"]
        triggers = SESSION_TRIGGERS + (TURN_TRIGGERS if manual else ())
        specs, info = await self._evals(ev, triggers)
        if not specs:
            return []
        msgs = await self.sessions.get_messages(sid)
        user = "\n".join(m.get("content", "") for m in msgs if m.get("role") == "user")
        output = next((m.get("content", "") for m in reversed(msgs)
                       if m.get("role") == "assistant"), "")
        ev = {**ev, "promptPackName": info["packName"] or ev.get("promptPackName", ""),
              "promptPackVersion": info["packVersion"] or ev.get("promptPackVersion", "")}
        last_id = next((m.get("id", "") for m in reversed(msgs) if m.get("role") == "assistant"),
                       "")
        ctx = EvalContext(output=output, user=user, messages=msgs,
                          tool_calls=await self._tool_calls(sid))
        results = await self._run_specs(specs, ev, user, output, last_id, f"{sid}:session",
                                        manual=manual, ctx=ctx)
        await self._write(results)
        return results

    async def _on_session_complete(self, sid: str):
        """Completion callback: an explicit ``session.completed`` (its event in
        ``_done_events``) or the inactivity timeout (metadata from session-api)."""
        self.stats["session_completions"] += 1
        ev = self._done_events.pop(sid, None) or {"sessionId": sid}
        await self._session_evals(ev, manual=False)

    async def handle(self, ev: dict) -> list[dict]:
        self.stats["events"] += 1
        t = ev.get("type") or ev.get("eventType")
        role = ev.get("role") or ev.get("messageRole")
        if t == EV_SESSION_DONE:
            sid = ev.get("sessionId", "")
            self._done_events[sid] = ev
            await self.tracker.mark_completed(sid)
            return []
        if t == EV_EVALUATE:
            self.stats["manual"] += 1
            return await self._session_evals(ev, manual=True)
        if t in (EV_MESSAGE, EV_MESSAGE_LEGACY) and role == "assistant":
            return await self.process_turn(ev)
        self.stats["skipped"] += 1
        return []

    # ---------------------------------------------------------- consumption
    async def _handle_entry(self, stream: str, eid, fields) -> bool:
        f = dict(zip(fields[::2], fields[1::2]))
        raw = f.get(b"event") or f.get("event") or f.get(b"payload") or f.get("payload")
        key = eid.decode() if isinstance(eid, bytes) else str(eid)
        try:
            ev = json.loads(raw)
        except (TypeError, ValueError):
            await self.r.xack(stream, GROUP, eid)  # unparsable: never retryable
            self.stats["failed"] += 1
            return True
        try:
            await self.handle(ev)
        except Exception as e:  # noqa: BLE001 - keep it pending for a retry
            n = self.deliveries[key] = self.deliveries.get(key, 0) + 1
            self.stats["failed"] += 1
            if n >= self.max_deliveries:
                log.error("eval event %s dead-lettered after %d attempts: %s", key, n, e)
                self.stats["dead_lettered"] += 1
                self.deliveries.pop(key, None)
                await self.r.xack(stream, GROUP, eid)
                return True
            log.warning("eval event %s failed (attempt %d), left pending: %s", key, n, e)
            return False
        self.deliveries.pop(key, None)
        await self.r.xack(stream, GROUP, eid)
        return True

    async def poll_once(self, count: int = 50) -> int:
        n = 0
        for ns in self.namespaces:
            stream = f"omnia:eval-events:{ns}"
            resp = await self.r.xreadgroup(GROUP, self.consumer, {stream: ">"}, count=count)
            for _s, entries in resp or []:
                for eid, fields in entries:
                    await self._handle_entry(stream, eid, fields)
                    n += 1
        await self.reclaim()
        await self.tracker.check_inactive()
        return n

    async def reclaim(self, force: bool = False) -> int:
        """Retry pending entries idle longer than ``reclaim_min_idle_s``
        (XAUTOCLAIM to this consumer), at most every ``reclaim_interval_s``."""
        now = time.monotonic()
        if not force and now - self._last_reclaim < self.reclaim_interval_s:
            return 0
        self._last_reclaim = now
        n = 0
        for ns in self.namespaces:
            stream = f"omnia:eval-events:{ns}"
            try:
                res = await self.r.execute("XAUTOCLAIM", stream, GROUP, self.consumer,
                                           int(self.reclaim_min_idle_s * 1000), "0-0",
                                           "COUNT", 25)
            except Exception as e:  # noqa: BLE001
                log.debug("XAUTOCLAIM failed on %s: %s", stream, e)
                continue
            for eid, fields in (res[1] if res else []) or []:
                self.stats["reclaimed"] += 1
                self.stats["retried"] += 1
                await self._handle_entry(stream, eid, fields)
                n += 1
        return n

    async def run(self, idle_sleep: float = 0.5):
        await self.setup()
        while True:
            if await self.poll_once() == 0:
                await asyncio.sleep(idle_sleep)


class SessionAPIClient:
    """The session-api calls the worker needs, over ONE shared HTTP session."""

    def __init__(self, base_url: str):
        self.base = base_url.rstrip("/")
        self._s = None

    async def _session(self):
        import aiohttp

        if self._s is None or self._s.closed:
            self._s = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30))
        return self._s

    async def get_messages(self, sid: str) -> list[dict]:
        s = await self._session()
        async with s.get(f"{self.base}/api/v1/sessions/{sid}/messages") as r:
            if r.status >= 400:
                raise RuntimeError(f"messages GET {r.status}")
            d = await r.json()
        return d.get("messages", d if isinstance(d, list) else [])

    async def get_session(self, sid: str) -> dict:
        s = await self._session()
        async with s.get(f"{self.base}/api/v1/sessions/{sid}") as r:
            if r.status >= 400:
                raise RuntimeError(f"session GET {r.status}")
            d = await r.json()
        return d.get("session", d)

    async def get_tool_calls(self, sid: str) -> list[dict]:
        s = await self._session()
        async with s.get(f"{self.base}/api/v1/sessions/{sid}/tool-calls") as r:
            if r.status >= 400:
                raise RuntimeError(f"tool-calls GET {r.status}")
            d = await r.json()
        if isinstance(d, list):
            return d
        return d.get("tool-calls") or d.get("toolCalls") or d.get("tool_calls") or []

    async def post_eval_results(self, results: list[dict]):
        s = await self._session()
        async with s.post(f"{self.base}/api/v1/eval-results", json={"results": results}) as r:
            if r.status >= 400:
                raise RuntimeError(f"eval-results POST {r.status}")

    async def close(self):
        if self._s is not None:
            await self._s.close()


def main():  # pragma: no cover - container entrypoint (operator subresources.py)
    from ..observability.logging import configure as configure_logging
    from ..utils.resp import RedisClient

    configure_logging()
    env = os.environ
    nss = [n for n in (env.get("NAMESPACES") or env.get("NAMESPACE", "default")).split(",") if n]
    session_url = env.get("SESSION_API_URL") or env.get("OMNIA_SESSION_API_URL", "")
    kube = None
    try:
        from ..operator.kube import KubeClient

        kube = KubeClient.from_env()
    except Exception as e:  # noqa: BLE001
        log.warning("no kube API (pack evals / provider resolution off): %s", e)
    hooks = json.loads(env.get("OMNIA_EVAL_WEBHOOKS", "[]") or "[]")
    worker = EvalWorker(
        RedisClient(env.get("REDIS_URL", "redis://127.0.0.1:6379/0")),
        SessionAPIClient(session_url), nss,
        pack_loader=PackEvalLoader(KubePackSource(kube)) if kube is not None else None,
        resolver=ProviderResolver(kube) if kube is not None else None,
        webhooks=WebhookDispatcher(hooks) if hooks else None,
        consumer=env.get("HOSTNAME", "eval-worker-0"),
        inactivity_timeout_s=float(env.get("OMNIA_EVAL_INACTIVITY_S", "300")))
    asyncio.run(worker.run())


if __name__ == "__main__":  # pragma: no cover
    main()
