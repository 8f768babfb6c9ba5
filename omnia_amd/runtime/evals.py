"""Eval type registry and the inline (real-time) eval path.

Reference: ``internal/runtime/evals.go`` (``LoadAllEvalDefs``, ``ValidateEvalDefs``,
``DefaultInlineEvalGroups``, ``buildEvalOptions``), whose handlers come from the
PromptKit eval registry; the types a pack may name are the ones its shipped
sample uses (``config/samples/omnia_v1alpha1_promptpack.yaml:135-303``) and the
realtime-evals docs list (``docs/.../configure-realtime-evals.md:105-141``).

Every type is registered with its groups:
  * ``fast-running`` -- deterministic, in-process: content / regex / length /
    JSON / PII assertions over the turn's output and tool-call assertions over
    the turn's (or the session's) recorded tool calls;
  * ``long-running`` + ``external`` -- LLM judges (``llm_judge``,
    ``llm_judge_turn``, ...): run by the eval worker (``ee/eval_worker.py``).
The runtime's inline path runs the evals whose groups meet its filter (default
``fast-running``); the worker runs the complement.  A type nobody registered is
never silently dropped: :func:`validate_eval_defs` lists it at startup and
:func:`evaluate` returns an error row for it.
"""
from __future__ import annotations

import json
import logging
import re
from dataclasses import dataclass, field
from typing import Callable

log = logging.getLogger("omnia.runtime.evals")

GROUP_FAST, GROUP_LONG, GROUP_EXTERNAL = "fast-running", "long-running", "external"
DEFAULT_INLINE_GROUPS = (GROUP_FAST,)
TURN_TRIGGERS = ("every_turn", "per_turn", "sample_turns")
SESSION_TRIGGERS = ("on_session_complete", "sample_sessions")


@dataclass
class EvalContext:
    """What an eval sees.  ``tool_calls``: ``{"name", "arguments", "error"}``
    dicts in call order (the turn's for turn triggers, the session's for
    session triggers); ``violations``: validator types that fired."""

    output: str = ""
    user: str = ""
    tool_calls: list = field(default_factory=list)
    violations: list = field(default_factory=list)
    messages: list = field(default_factory=list)


@dataclass
class EvalType:
    fn: Callable | None  # (params, ctx) -> (passed, score, details); None = judge (worker)
    groups: tuple


REGISTRY: dict[str, EvalType] = {}


def register(name: str, groups=(GROUP_FAST,)):
    def deco(fn):
        REGISTRY[name] = EvalType(fn, tuple(groups))
        return fn
    return deco


def register_judge(name: str) -> None:
    REGISTRY[name] = EvalType(None, (GROUP_LONG, GROUP_EXTERNAL))


for _j in ("llm_judge", "llm_judge_turn", "llm_judge_session", "llm_judge_conversation",
           "judge", "rubric"):
    register_judge(_j)

JUDGE_TYPES = tuple(k for k, v in REGISTRY.items() if v.fn is None)


def groups_of(spec: dict) -> list[str]:
    """An eval's groups: ``params.groups`` / ``groups`` when set, else its type's."""
    g = (spec.get("params") or {}).get("groups") or spec.get("groups")
    if g:
        return list(g)
    t = REGISTRY.get(spec.get("type", ""))
    return list(t.groups) if t else [GROUP_FAST]


def is_judge(spec: dict) -> bool:
    t = REGISTRY.get(spec.get("type", ""))
    return t is not None and t.fn is None


def validate_eval_defs(defs) -> list[str]:
    """Eval types in ``defs`` with no registered handler (``ValidateEvalDefs``)."""
    missing, seen = [], set()
    for d in defs or []:
        t = d.get("type", "")
        if t in seen:
            continue
        seen.add(t)
        if t not in REGISTRY:
            missing.append(t)
    return missing


# --------------------------------------------------------------- helpers
def _patterns(p: dict) -> list[str]:
    if p.get("patterns"):
        return [x for x in p["patterns"] if x]
    v = p.get("pattern", p.get("value", ""))
    return [v] if v else []


def _should(p: dict, key: str = "should_match", default: bool = True) -> bool:
    v = p.get(key, p.get("expect_match", default) if key == "should_match" else default)
    return v if isinstance(v, bool) else str(v).lower() not in ("false", "0", "no")


def _int(p: dict, keys, default: int) -> int:
    for k in keys:
        if k in p:
            return int(p[k])
    return default


def _search(pat: str, text: str) -> bool:
    try:
        return re.search(pat, text, re.I) is not None
    except re.error:
        return pat.lower() in text.lower()


def _names(p: dict) -> list[str]:
    v = p.get("tool_names") or p.get("tools") or p.get("names") or []
    return [v] if isinstance(v, str) else list(v)


def _called(ctx: EvalContext) -> list[str]:
    return [c.get("name", "") for c in ctx.tool_calls]


# ------------------------------------------------------- content assertions
@register("content_includes")
@register("contains")
def _includes(p, ctx):
    pats = _patterns(p)
    if p.get("regex") or ("pattern" in p and "patterns" not in p and "value" not in p):
        hit = _search(pats[0], ctx.output) if pats else False  # regex form
    else:
        hit = bool(pats) and all(x.lower() in ctx.output.lower() for x in pats)
    return hit == _should(p), None


@register("content_excludes")
@register("not_contains")
def _excludes(p, ctx):
    hit = any(x.lower() in ctx.output.lower() for x in _patterns(p))
    return not hit, None


@register("regex_match")
@register("regex")
def _regex(p, ctx):
    pat = p.get("pattern", "")
    try:
        hit = re.search(pat, ctx.output) is not None
    except re.error as e:
        raise ValueError(f"bad pattern: {e}") from None
    return hit == _should(p), None


@register("banned_words")
def _banned(p, ctx):
    words = p.get("words") or []
    found = [w for w in words if re.search(r"\b" + re.escape(w) + r"\b", ctx.output, re.I)]
    return not found, {"found": found} if found else None


@register("max_length")
def _max_len(p, ctx):
    lim = _int(p, ("max_characters", "maxLength", "max_length", "max"), 10**9)
    return len(ctx.output) <= lim, {"length": len(ctx.output)}


@register("min_length")
def _min_len(p, ctx):
    lim = _int(p, ("min_characters", "minLength", "min_length", "min"), 0)
    return len(ctx.output) >= lim, {"length": len(ctx.output)}


@register("json_valid")
def _json_valid(p, ctx):
    try:
        json.loads(ctx.output)
    except (json.JSONDecodeError, TypeError):
        return False, None
    return True, None


PII_PATTERNS = {
    "credit_card": r"\b(?:\d[ -]?){13,16}\b",
    "ssn": r"\b\d{3}-\d{2}-\d{4}\b",
    "email": r"\b[\w.+-]+@[\w-]+\.[\w.-]+\b",
    "phone": r"(?:\+\d{1,2}\s?)?\(?\d{3}\)?[\s.-]\d{3}[\s.-]\d{4}\b",
    "ip_address": r"\b(?:\d{1,3}\.){3}\d{1,3}\b",
}


def _luhn(digits: str) -> bool:
    s, alt = 0, False
    for ch in reversed(digits):
        d = ord(ch) - 48
        if alt:
            d *= 2
            if d > 9:
                d -= 9
        s += d
        alt = not alt
    return s % 10 == 0


@register("pii_detection")
def _pii(p, ctx):
    types = p.get("types") or list(PII_PATTERNS)
    found = []
    for t in types:
        pat = PII_PATTERNS.get(t)
        if pat is None:
            raise ValueError(f"unknown PII type {t!r}")
        for m in re.finditer(pat, ctx.output):
            if t == "credit_card":
                digits = re.sub(r"\D", "", m.group(0))
                if not (13 <= len(digits) <= 16 and _luhn(digits)):
                    continue
            found.append(t)
            break
    return not found, {"found": found} if found else None


@register("guardrail_triggered")
def _guardrail(p, ctx):
    want = p.get("validator") or p.get("guardrail") or p.get("type")
    fired = [v for v in ctx.violations if not want or v == want]
    return bool(fired) == _should(p, "should_trigger", True), {"fired": fired}


# ------------------------------------------------------ tool-call assertions
@register("tools_called")
def _tools_called(p, ctx):
    names, called = _names(p), set(_called(ctx))
    missing = [n for n in names if n not in called]
    if str(p.get("mode", "all")).lower() == "any":
        return bool(set(names) & called), {"called": sorted(called)}
    return not missing, {"missing": missing} if missing else None


@register("tools_not_called")
def _tools_not_called(p, ctx):
    hit = sorted(set(_names(p)) & set(_called(ctx)))
    return not hit, {"called": hit} if hit else None


@register("tool_call_chain")
def _chain(p, ctx):
    chain = list(p.get("chain") or p.get("tool_names") or [])
    i = 0
    for n in _called(ctx):  # the chain must appear in order (a subsequence)
        if i < len(chain) and n == chain[i]:
            i += 1
    return i == len(chain), {"matched": i, "chain": chain}


@register("no_tool_errors")
def _no_errors(p, ctx):
    errs = [c.get("name", "") for c in ctx.tool_calls if c.get("error")]
    return not errs, {"errors": errs} if errs else None


@register("tool_efficiency")
def _efficiency(p, ctx):
    n = len(ctx.tool_calls)
    errs = sum(1 for c in ctx.tool_calls if c.get("error"))
    rate = errs / n if n else 0.0
    ok = True
    if "max_calls" in p:
        ok &= n <= int(p["max_calls"])
    if "max_error_rate" in p:
        ok &= rate <= float(p["max_error_rate"])
    return ok, {"calls": n, "error_rate": round(rate, 4)}


# ------------------------------------------------------------------- run
def evaluate(spec: dict, ctx: EvalContext | str, output: str | None = None) -> dict:
    """Run one deterministic eval.  Returns ``{"id", "type", "passed", "score"}``
    (+ ``details``); a judge type returns ``skipped`` (the worker runs it); an
    unregistered type or a bad parameter returns ``passed: False`` with
    ``error`` -- a result row, never a silent drop.

    ``evaluate(spec, user, output)`` (two strings) is the old call form."""
    if not isinstance(ctx, EvalContext):
        ctx = EvalContext(output=output or "", user=ctx or "")
    t = spec.get("type", "")
    rid = spec.get("id", t)
    et = REGISTRY.get(t)
    if et is None:
        log.warning("eval %r: unknown eval type %r", rid, t)
        return {"id": rid, "type": t, "passed": False, "score": 0.0,
                "error": f"unknown eval type {t!r}"}
    if et.fn is None:
        return {"id": rid, "type": t, "skipped": True}
    try:
        ok, details = et.fn(spec.get("params") or {}, ctx)
    except (ValueError, TypeError, KeyError) as e:
        return {"id": rid, "type": t, "passed": False, "score": 0.0, "error": str(e)}
    r = {"id": rid, "type": t, "passed": bool(ok), "score": 1.0 if ok else 0.0}
    if details:
        r["details"] = details
    return r


class InlineEvaluator:
    """The runtime's inline eval path: after each turn, the pack's turn-trigger
    evals whose groups meet ``groups`` (``spec.evals.inline.groups``, default
    fast-running) run over the turn; when the conversation stream closes, its
    session-trigger evals run over the session's accumulated tool calls.
    Results go to session-api through the event sink (source runtime-inline)."""

    def __init__(self, sink=None, groups=None, pack_evals=None):
        self.sink = sink
        self.groups = set(groups or DEFAULT_INLINE_GROUPS)
        self.results: list[dict] = []
        self._sessions: dict[str, dict] = {}  # sid -> {"tools", "prompt", "last"}
        missing = validate_eval_defs(pack_evals or [])
        if missing:
            log.warning("PromptPack names eval types with no registered handler: %s "
                        "(they will record error results)", ", ".join(missing))
        self.missing = missing

    def _specs(self, prompt, triggers):
        for spec in (getattr(prompt, "evals", None) or []):
            if spec.get("enabled", True) is False:
                continue
            if spec.get("trigger", "every_turn") not in triggers:
                continue
            if spec.get("type") in REGISTRY and not (set(groups_of(spec)) & self.groups):
                continue  # the worker's half
            yield spec

    async def _emit(self, session_id, r, trigger):
        r["session_id"] = session_id
        r["trigger"] = trigger
        r["source"] = "runtime-inline"
        self.results.append(r)
        if self.sink is not None:
            try:
                await self.sink.record(session_id, "eval_result", r)
            except Exception:  # noqa: BLE001
                pass

    async def on_turn(self, session_id, user, res, prompt):
        tools = list(getattr(res, "tool_records", None) or [])
        st = self._sessions.setdefault(session_id, {"tools": [], "prompt": prompt, "last": ""})
        st["tools"].extend(tools)
        st["prompt"], st["last"] = prompt, res.content
        ctx = EvalContext(output=res.content, user=user, tool_calls=tools,
                          violations=[str(v).split(":", 1)[0] for v in
                                      (getattr(res, "violations", None) or [])])
        for spec in self._specs(prompt, TURN_TRIGGERS):
            r = evaluate(spec, ctx)
            if not r.get("skipped"):
                await self._emit(session_id, r, spec.get("trigger", "every_turn"))

    async def on_session_complete(self, session_id):
        st = self._sessions.pop(session_id, None)
        if st is None:
            return
        ctx = EvalContext(output=st["last"], tool_calls=st["tools"])
        for spec in self._specs(st["prompt"], SESSION_TRIGGERS):
            r = evaluate(spec, ctx)
            if not r.get("skipped"):
                await self._emit(session_id, r, spec.get("trigger"))
