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
            r["user"] = t["user"]
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
        turns.append({"user": t["user"], "content": content, "ttft_ms": (ttft or lat) * 1e3,
                      "latency_ms": lat * 1e3,
                      "usage": {"output_tokens": getattr(usage, "output_tokens", 0),
                                "cost": getattr(usage, "cost", 0.0)} if usage else {},
                      "assertions": [evaluate(a, t["user"], content)
                                     for a in t.get("assertions", [])]})
    return _summarise(turns)


async def _complete(prov, msgs, params, sid, source: str, calls: list) -> tuple[str, float, float]:
    """One provider call -> (text, ttft_s, latency_s), recorded in ``calls``."""
    t0 = time.perf_counter()
    ttft, text, usage = None, [], None
    async for ev in prov.stream(msgs, [], params, session_id=sid):
        if ev.type == "text":
            if ttft is None:
                ttft = time.perf_counter() - t0
            text.append(ev.text)
        elif ev.type == "error":
            raise RuntimeError(ev.text)
        elif ev.type == "done":
            usage = ev.usage
    lat = time.perf_counter() - t0
    calls.append({"source": source, "provider": getattr(prov, "name", ""),
                  "model": getattr(prov, "model", ""), "latency_ms": lat * 1e3,
                  "output_tokens": getattr(usage, "output_tokens", 0) if usage else 0})
    return "".join(text), (ttft or lat), lat


async def run_selfplay(item: WorkItem, scenario: dict, provider: dict) -> dict:
    """Self-play (reference ``selfplay_capture.go`` + PromptKit personas): a
    persona model plays the USER -- it sees the conversation with roles swapped
    and its persona prompt (goals, constraints, style) as system -- against the
    agent under test, for ``max_turns`` exchanges or until the persona emits
    ``[DONE]``.  Provider calls are tagged ``agent`` / ``selfplay``."""
    from ...engine.sampling_params import SamplingParams
    from ...runtime.chat import Message

    sp = scenario.get("self_play") or {}
    agent, persona = provider["object"], provider["persona_object"]
    params = SamplingParams(**(provider.get("params") or {"temperature": 0.0,
                                                         "max_tokens": 128}))
    pp = sp.get("persona") or {}
    persona_sys = pp.get("system_prompt") or (
        f"You are role-playing a user. {pp.get('description', '')} Goals: "
        f"{'; '.join(pp.get('goals') or [])}. Constraints: "
        f"{'; '.join(pp.get('constraints') or [])}. Style: {pp.get('style', 'concise')}. "
        "Reply with only the user's next message, or [DONE] when the goals are met.")
    sid = f"arena-sp-{item.id}"
    agent_msgs = [Message("system", scenario.get("system", "You are a helpful assistant."))]
    persona_msgs = [Message("system", persona_sys)]
    opener = sp.get("opening_message") or (scenario.get("turns") or [{}])[0].get("user")
    calls, turns = [], []
    user = opener
    for i in range(int(sp.get("max_turns", 4))):
        if user is None:
            user, _, _ = await _complete(persona, persona_msgs, params, sid + "-u",
                                         "selfplay", calls)
        user = user.strip()
        if not user or "[DONE]" in user:
            break
        agent_msgs.append(Message("user", user))
        persona_msgs.append(Message("assistant", user))
        reply, ttft, lat = await _complete(agent, agent_msgs, params, sid, "agent", calls)
        agent_msgs.append(Message("assistant", reply))
        persona_msgs.append(Message("user", reply))  # roles swapped for the persona
        turns.append({"user": user, "content": reply, "ttft_ms": ttft * 1e3,
                      "latency_ms": lat * 1e3, "usage": {},
                      "assertions": [evaluate(a, user, reply)
                                     for a in sp.get("assertions", [])]})
        user = None
    out = _summarise(turns)
    out["transcript"] = [{"user": t["user"], "assistant": t["content"]} for t in turns]
    out["provider_calls"] = calls
    return out


def _render(template: str, variables: dict) -> str:
    for k, v in variables.items():
        template = template.replace("{{" + k + "}}", str(v)).replace("{{ " + k + " }}", str(v))
    return template


async def run_datagen(item: WorkItem, scenario: dict, provider: dict) -> dict:
    """Data generation (ArenaJob type ``datagen``): render the scenario's prompt
    template with variables sampled deterministically per item, run it through
    the provider, return the (input, output) record."""
    import random

    from ...engine.sampling_params import SamplingParams
    from ...runtime.chat import Message

    rng = random.Random(f"{item.job_id}:{item.id}")
    choices = scenario.get("variables") or {}
    variables = {k: (rng.choice(v) if isinstance(v, list) and v else v)
                 for k, v in choices.items()}
    prompt = _render(scenario.get("prompt") or (scenario.get("turns") or [{}])[0].get(
        "user", ""), variables)
    params = SamplingParams(**(provider.get("params") or {"temperature": 0.7,
                                                         "max_tokens": 128}))
    msgs = [Message("system", scenario.get("system", "You generate training data.")),
            Message("user", prompt)]
    calls: list = []
    text, ttft, lat = await _complete(provider["object"], msgs, params, f"dg-{item.id}",
                                      "datagen", calls)
    return {"passed": True, "latency_ms": lat * 1e3, "ttft_ms": ttft * 1e3,
            "turns": [{"latency_ms": lat * 1e3, "ttft_ms": ttft * 1e3}],
            "output_tokens": calls[0]["output_tokens"], "cost": 0.0, "assertions": [],
            "record": {"id": item.id, "scenario": item.scenario_id, "variables": variables,
                       "input": prompt, "output": text}}


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
                 consumer: str | None = None, visibility_s: float = 300.0,
                 job_type: str = "evaluation", recorder=None):
        self.q = queue
        self.job = job_id
        self.scenarios = scenarios
        self.providers = providers
        self.profile = profile
        self.budget = budget
        self.consumer = consumer or f"worker-{os.getpid()}-{uuid.uuid4().hex[:6]}"
        self.visibility_s = visibility_s
        self.job_type = job_type
        self.recorder = recorder  # ArenaSessionRecorder: played runs -> session-api
        self.spent = 0.0
        self.active = 0
        self.done = 0

    async def _execute(self, item: WorkItem):
        scen = self.scenarios[item.scenario_id]
        prov = self.providers[item.provider_id]
        try:
            if self.job_type == "datagen":
                fn = run_datagen
            elif scen.get("self_play"):
                fn = run_selfplay
            else:
                fn = run_fleet if prov.get("mode", "fleet") == "fleet" else run_direct
            res = await fn(item, scen, prov)
            res.update(scenario=item.scenario_id, provider=item.provider_id,
                       attempt=item.attempt, item_id=item.id)
            self.spent += res.get("cost") or 0.0
            if self.recorder is not None and res.get("turns"):
                try:
                    res["session_id"] = await self.recorder.record(item, res)
                except Exception as e:  # noqa: BLE001 -- recording never fails a run
                    log.warning("recording item %s failed: %s", item.id, e)
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
