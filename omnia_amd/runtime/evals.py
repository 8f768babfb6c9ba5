"""Inline (real-time) evals run after each turn (``internal/runtime/evals.go:40-157``).

Deterministic assertion evals from the PromptPack ``evals`` list run in-process;
results are recorded to session-api through the event sink.  LLM-judge evals are
queued to the eval worker via the session event stream instead (EE eval worker).
"""
from __future__ import annotations

import json
import re


def evaluate(spec: dict, user: str, output: str) -> dict:
    t = spec.get("type", "")
    p = spec.get("params", {}) or {}
    ok, score = True, 1.0
    if t in ("contains", "content_includes"):
        pats = p.get("patterns") or [p.get("value", "")]
        ok = all(x.lower() in output.lower() for x in pats if x)
    elif t in ("not_contains", "content_excludes"):
        pats = p.get("patterns") or [p.get("value", "")]
        ok = not any(x.lower() in output.lower() for x in pats if x)
    elif t == "regex":
        ok = re.search(p.get("pattern", ""), output) is not None
    elif t == "max_length":
        ok = len(output) <= int(p.get("max", 10**9))
    elif t == "min_length":
        ok = len(output) >= int(p.get("min", 0))
    elif t == "json_valid":
        try:
            json.loads(output)
        except json.JSONDecodeError:
            ok = False
    else:
        return {"id": spec.get("id", t), "type": t, "skipped": True}
    if not ok:
        score = 0.0
    return {"id": spec.get("id", t), "type": t, "passed": ok, "score": score}


class InlineEvaluator:
    def __init__(self, sink=None):
        self.sink = sink
        self.results: list[dict] = []

    async def on_turn(self, session_id, user, res, prompt):
        for spec in prompt.evals or []:
            if spec.get("trigger", "every_turn") not in ("every_turn", "per_turn"):
                continue
            r = evaluate(spec, user, res.content)
            r["session_id"] = session_id
            self.results.append(r)
            if self.sink is not None and not r.get("skipped"):
                try:
                    await self.sink.record(session_id, "eval_result", r)
                except Exception:  # noqa: BLE001
                    pass
