"""Declarative compositions: step graphs run by a workflow state with
``orchestration: composition``.

Reference shape: the compiled packs ``config/samples/
omnia_v1alpha1_promptpack_doc_analysis.yaml`` and ``charts/omnia-demos/
templates/composition-demo.yaml`` (PromptKit RFC 0010), which exercise the five
v1 step kinds:

* ``prompt``   -- one model call: the ``prompt_task``'s system prompt plus the
  templated ``input`` as the user message, no tools.  The output is the reply,
  parsed as JSON when it is a JSON document (so later steps can address
  ``${classify.output.type}``);
* ``tool``     -- one tool call with templated ``args`` through the agent's
  executor (server-side handlers, or CLIENT tools round-tripped to the caller);
* ``parallel`` -- its ``branches`` run concurrently; ``reduce: {strategy:
  barrier, into: X}`` waits for all and publishes ``{branch id: output}`` as
  ``${X.output...}`` (and under the parallel step's own id);
* ``branch``   -- evaluates ``predicate {path, op, value}`` and enables
  ``then`` or ``else``; the step it did not choose is skipped;
* ``agent``    -- a bounded tool loop of the ``prompt_task`` with only the
  listed ``tools``, at most ``termination.max_steps`` rounds.

Steps run in declared order.  A step is skipped when a branch routed around it
or when anything it ``depends_on`` was skipped.  Templates are ``${input.text}``
(the turn's user text), ``${<step id>.output[.field...]}``; a string that is a
single expression yields the raw value (objects stay objects).  The
composition's result is the output of the last step that ran.
``modifiers.eval`` names are recorded on the step's trace entry.
"""
from __future__ import annotations

import asyncio
import dataclasses
import json
import re
import time
import uuid

from .chat import Message, ToolCallReq

_EXPR = re.compile(r"\$\{\s*([A-Za-z_][\w\-]*(?:\.[\w\-]+)*)\s*\}")


class CompositionError(RuntimeError):
    pass


def lookup(env: dict, path: str):
    cur = env
    for part in path.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        elif isinstance(cur, list) and part.isdigit() and int(part) < len(cur):
            cur = cur[int(part)]
        else:
            return None
    return cur


def template(value, env: dict):
    if isinstance(value, str):
        m = _EXPR.fullmatch(value.strip())
        if m:
            return lookup(env, m.group(1))

        def rep(mm):
            v = lookup(env, mm.group(1))
            return "" if v is None else v if isinstance(v, str) else json.dumps(v)

        return _EXPR.sub(rep, value)
    if isinstance(value, dict):
        return {k: template(v, env) for k, v in value.items()}
    if isinstance(value, list):
        return [template(v, env) for v in value]
    return value


def _num(x):
    try:
        return float(x)
    except (TypeError, ValueError):
        return None


def evaluate(pred: dict, env: dict) -> bool:
    v = template(pred["path"], env)
    op, want = pred["op"], pred.get("value")
    if op == "exists":
        return v is not None
    if op == "equals":
        return v == want or (v is not None and str(v) == str(want))
    if op == "not_equals":
        return not (v == want or (v is not None and str(v) == str(want)))
    if op == "contains":
        return v is not None and want is not None and (
            str(want) in v if isinstance(v, str) else want in v if isinstance(v, (list, dict))
            else False)
    if op == "in":
        return isinstance(want, (list, str)) and v in want
    a, b = _num(v), _num(want)
    if a is None or b is None:
        return False
    return {"gt": a > b, "gte": a >= b, "lt": a < b, "lte": a <= b}[op]


def parse_output(text: str):
    t = text.strip()
    if t.startswith("```"):
        t = t.strip("`")
        t = t[t.find("\n") + 1:] if "\n" in t else t
    for cand in (t, t[t.find("{"):t.rfind("}") + 1] if "{" in t else ""):
        if cand:
            try:
                return json.loads(cand)
            except ValueError:
                pass
    return text


class CompositionRunner:
    """Runs one composition for one turn of ``agent`` (a runtime :class:`Agent`)."""

    def __init__(self, agent, name: str, session_id: str, io, ctx, metadata: dict, res):
        self.agent = agent
        self.name = name
        self.comp = agent.pack.compositions[name]
        self.sid = session_id
        self.io, self.ctx, self.md, self.res = io, ctx, metadata, res
        self.trace: list[dict] = []

    async def run(self, input_text: str):
        env = {"input": {"text": input_text}}
        enabled: dict[str, bool] = {}   # branch targets: id -> chosen?
        skipped: set[str] = set()
        last = None
        for step in self.comp["steps"]:
            sid = step["id"]
            if enabled.get(sid) is False or any(d in skipped for d in step.get("depends_on")
                                                 or []):
                skipped.add(sid)
                self.trace.append({"id": sid, "kind": step["kind"], "status": "skipped"})
                continue
            if step["kind"] == "branch":
                chosen = evaluate(step["predicate"], env)
                tgt, other = (step["then"], step.get("else")) if chosen else \
                    (step.get("else"), step["then"])
                if tgt:
                    enabled[tgt] = True
                if other and other != tgt:
                    enabled[other] = False
                env[sid] = {"output": {"taken": "then" if chosen else "else", "target": tgt}}
                self.trace.append({"id": sid, "kind": "branch", "status": "ok",
                                   "taken": "then" if chosen else "else"})
                continue
            out = await self._step(step, env)
            env[sid] = {"output": out}
            red = step.get("reduce") or {}
            if red.get("into"):
                env[red["into"]] = {"output": out}
            last = out
        return last, env

    async def _step(self, step: dict, env: dict):
        t0 = time.perf_counter()
        entry = {"id": step["id"], "kind": step["kind"], "status": "ok"}
        if (step.get("modifiers") or {}).get("eval"):
            entry["evals"] = list(step["modifiers"]["eval"])
        try:
            k = step["kind"]
            if k == "prompt":
                out = await self._prompt(step, env)
            elif k == "tool":
                out = await self._tool(step, env)
            elif k == "agent":
                out = await self._agent(step, env)
            elif k == "parallel":
                outs = await asyncio.gather(*(self._step(b, env) for b in step["branches"]))
                out = {b["id"]: o for b, o in zip(step["branches"], outs)}
                for b, o in zip(step["branches"], outs):
                    env[b["id"]] = {"output": o}
            else:
                raise CompositionError(f"step {step['id']!r}: kind {k!r} cannot run here")
        except Exception as e:
            entry["status"] = "error"
            entry["error"] = str(e)
            self.trace.append(entry)
            raise CompositionError(f"composition {self.name!r} step {step['id']!r}: {e}") from e
        entry["ms"] = round((time.perf_counter() - t0) * 1000, 3)
        self.trace.append(entry)
        return out

    async def _prompt(self, step, env):
        a = self.agent
        prompt = a.pack.prompts[step["prompt_task"]]
        msgs = [a._system_message(None, prompt),
                Message("user", _as_text(template(step.get("input", "${input.text}"), env)))]
        text, _, usage = await a.provider.complete(msgs, None, a.params(prompt=prompt),
                                                   self.sid, self.md)
        self.res.usage += usage
        return parse_output(text)

    async def _tool(self, step, env):
        call = ToolCallReq(id="call_" + uuid.uuid4().hex[:12], name=step["tool"],
                           arguments=template(step.get("args") or {}, env))
        got = await self.agent._run_tools([call], self.io, self.ctx, self.md)
        r = got.get(call.id) or {}
        if r.get("is_error"):
            raise CompositionError(f"tool {step['tool']!r} failed: {r.get('result_json')}")
        try:
            return json.loads(r.get("result_json", "null"))
        except ValueError:
            return r.get("result_json")

    async def _agent(self, step, env):
        from .agent import Agent, _CollectIO

        a = self.agent
        base = a.pack.prompts[step["prompt_task"]]
        prompt = dataclasses.replace(base, tools=list(step.get("tools") or base.tools),
                                     tool_policy=dataclasses.replace(
                                         base.tool_policy,
                                         max_rounds=int((step.get("termination") or {}).get(
                                             "max_steps", base.tool_policy.max_rounds))))
        sub = Agent(a.pack, a.provider, a.store, a.executor, a.cfg, a.extra, a.memory,
                    a.event_sink, None, a.tokenizer, graph=False)
        sub.prompt = prompt
        sid = f"{self.sid}/composition/{self.name}/{step['id']}"
        r = await sub.run_turn(sid, _as_text(template(step.get("input", "${input.text}"), env)),
                               _CollectIO(), ctx=dataclasses.replace(self.ctx, session_id=sid),
                               persist=False)
        self.res.usage += r.usage
        return parse_output(r.content)


def _as_text(v) -> str:
    return v if isinstance(v, str) else json.dumps(v)


def result_text(out) -> str:
    return out if isinstance(out, str) else json.dumps(out)


__all__ = ["CompositionRunner", "CompositionError", "evaluate", "template", "lookup",
           "parse_output", "result_text"]
