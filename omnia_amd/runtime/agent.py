"""The agent loop: one conversation turn = render -> LLM stream -> tools -> ... -> Done.

Reference behaviour (``internal/runtime/message.go:40-431``, PromptKit pipeline):
  * the conversation is resumed from the context store or opened fresh with the
    PromptPack system prompt (``conversation.go:260-276``);
  * text deltas stream as Chunk frames; server-side tool calls run inside the
    runtime (policy broker, retry, circuit breaker) and are NOT sent to the
    facade; client-side tools are emitted as ``ToolCall{execution: CLIENT}`` and
    the loop blocks for their ``ClientToolResult`` (``message.go:268-357``);
  * ``tool_policy.max_rounds`` (default 5) and ``max_tool_calls_per_turn``
    (default 10) bound the loop; ``tool_choice: none`` hides tools;
  * the turn ends with Done{final_content, usage{input, output, cost}}.
  * workflow / multi-agent packs (:mod:`.workflow`): the active prompt follows
    the conversation's workflow state; transitions and member-agent calls are
    runtime-internal server-side tools.
  * context window: ``ProviderDefaults.contextWindow`` + ``truncationStrategy``
    (sliding = drop oldest, summarize = fold oldest turns into a summary,
    custom = warn and fall back to sliding) (``agentruntime_types.go:417-476``).
"""
from __future__ import annotations

import dataclasses

import asyncio
import json
import logging
import time
import uuid
from dataclasses import dataclass, field

from ..engine.sampling_params import SamplingParams
from ..observability import metrics as M
from ..utils import failpoints
from ..observability import tracing
from ..tools.executor import CallContext, OmniaExecutor
from ..observability import logging as logctx
from .chat import Message, ToolCallReq
from .context_store import StoreUnavailable
from .promptpack import Prompt, PromptPack, run_validators
from .providers import Provider, ProviderError, ProviderEvent, Usage
from .workflow import (AGENT_TOOL_PREFIX, ARTIFACT_TOOL, TRANSITION_TOOL, Workflow, WorkflowError,
                       member_tool_specs, scope_skill_specs, scoped_skill_names)

log = logging.getLogger("omnia.runtime.agent")


@dataclass
class TurnResult:
    content: str = ""
    usage: Usage = field(default_factory=Usage)
    cost: float = 0.0
    tool_calls: int = 0
    tool_records: list = field(default_factory=list)  # {"name", "arguments", "error"} per call
    rounds: int = 0
    violations: list = field(default_factory=list)
    ttft: float | None = None
    finish_reason: str = ""
    workflow: dict | None = None  # the conversation's workflow snapshot after the turn
    transitions: list = field(default_factory=list)
    composition: list | None = None  # step trace when a composition state ran


@dataclass
class AgentConfig:
    prompt_name: str | None = None
    variables: dict = field(default_factory=dict)
    context_window: int = 0  # tokens; 0 = unlimited
    truncation: str = "sliding"
    defaults: dict = field(default_factory=dict)  # ProviderDefaults
    response_format: str = ""  # "" | text | json | json_schema (function mode)
    response_schema: dict | None = None
    max_rounds: int | None = None


class _CollectIO:
    """TurnIO of a member-agent sub-turn: text is collected, client tools refused."""

    async def chunk(self, text: str) -> None:
        pass

    async def client_tool_calls(self, calls, meta):
        raise RuntimeError("client tools are not available to member agents")


class TurnIO:
    """Transport hooks for one turn (implemented by the gRPC Converse handler)."""

    async def chunk(self, text: str) -> None:  # pragma: no cover - interface
        pass

    async def client_tool_calls(self, calls: list[ToolCallReq], meta: dict) -> dict[str, dict]:
        """Emit CLIENT tool calls and wait for results {call_id: {result_json, is_rejected...}}."""
        raise RuntimeError("client tools unsupported on this transport")


def _approx_tokens(text: str) -> int:
    return max(1, len(text) // 4)


class Agent:
    def __init__(self, pack: PromptPack, provider: Provider, store, executor: OmniaExecutor | None,
                 cfg: AgentConfig | None = None, extra_providers: dict | None = None,
                 memory=None, event_sink=None, evaluator=None, tokenizer=None,
                 graph: bool = True):
        self.pack = pack
        self.provider = provider
        self.store = store
        self.executor = executor
        self.cfg = cfg or AgentConfig()
        self.extra = extra_providers or {}
        self.memory = memory  # retriever with async retrieve(session, query, ctx) -> str
        self.event_sink = event_sink  # async record(kind, session_id, payload)
        self.evaluator = evaluator
        self.tokenizer = tokenizer
        # workflow / multi-agent packs open at their declared entry
        # (pack_entry.go:54-86); ``graph=False`` is a member agent's view
        self.workflow = Workflow(pack.workflow) if graph and pack.workflow else None
        self.multi_agent = bool(graph and pack.agents)
        if graph and (pack.workflow or pack.agents):
            self.prompt = pack.prompts[pack.entry()]
        else:
            self.prompt = pack.prompt(self.cfg.prompt_name)
        self._members: dict[str, Agent] = {}

    # ------------------------------------------------------------ state
    def _skills(self):
        h = self.executor.handlers.get("skills") if self.executor is not None else None
        return h if getattr(h, "type", "") == "skills" else None

    def _system_message(self, variables: dict | None, prompt: Prompt | None = None) -> Message:
        from .skills import preloaded_instructions

        vs = {**self.cfg.variables, **(variables or {})}
        return Message("system", self.pack.render_system(prompt or self.prompt, vs)
                       + preloaded_instructions(self._skills()))

    def _active_prompt(self, snap: dict | None) -> Prompt:
        if self.workflow is not None and snap is not None:
            key = self.workflow.prompt_key(snap)  # None in a composition state
            return self.pack.prompts[key] if key else self.prompt
        return self.prompt

    def _tools(self, prompt: Prompt, snap: dict | None) -> list[dict]:
        if prompt.tool_policy.tool_choice == "none":
            return []
        if snap is not None and snap.get("exhausted") == "max_tool_calls":
            return []  # the workflow's tool-call budget is spent
        tools = []
        if self.executor is not None:
            tools = self.pack.tool_specs(prompt, self.executor.specs())
            if self.workflow is not None and snap is not None:
                sk = self._skills()
                tools = scope_skill_specs(tools, self.workflow.skill_scope(snap),
                                          sk.skills if sk else {})
        if self.workflow is not None and snap is not None:
            if self.workflow.model_can_fire(snap):
                tools.append(self.workflow.tool_spec(snap))
            art = self.workflow.artifact_spec(snap)
            if art is not None:
                tools.append(art)
        if self.multi_agent and self.pack.key_of(prompt) == self.pack.agents["entry"]:
            tools += member_tool_specs(self.pack)
        return tools

    async def _enter_state(self, session_id: str, snap: dict, rec: dict, msgs: list[Message],
                           variables: dict | None, user: Message | None) -> list[Message]:
        """Switch the context to the state just entered (``rec``)."""
        if rec.get("budget_exhausted"):  # stopped where it stands
            await self._completed(session_id, snap)
            return msgs
        system = self._system_message(variables, self._active_prompt(snap))
        if self.workflow.persistence(rec["to_state"]) == "transient":
            msgs = [system] + ([user] if user is not None else [])
        else:
            if msgs and msgs[0].role == "system":
                msgs[0] = system
            else:
                msgs.insert(0, system)
        span = tracing.start_span("omnia.workflow.transition", {
            "workflow.from_state": rec["from_state"], "workflow.to_state": rec["to_state"],
            "workflow.event": rec["event"], "workflow.prompt_task": rec["prompt_task"]})
        tracing.end_span(span)
        await self._emit(session_id, "workflow.transitioned", rec)
        if snap["completed"]:
            await self._completed(session_id, snap)
        return msgs

    async def _completed(self, session_id: str, snap: dict):
        ev = {"final_state": snap["state"], "transition_count": snap["transitions"]}
        if snap.get("exhausted"):
            ev["budget_exhausted"] = snap["exhausted"]
        await self._emit(session_id, "workflow.completed", ev)

    async def _run_composition(self, name: str, session_id: str, content: str, io, ctx,
                               metadata: dict, res: TurnResult) -> str:
        from .composition import CompositionRunner, result_text

        runner = CompositionRunner(self, name, session_id, io, ctx, metadata, res)
        span = tracing.start_span("omnia.workflow.composition", {"composition.name": name})
        try:
            out, _ = await runner.run(content)
        finally:
            res.composition = runner.trace
            tracing.end_span(span, {"composition.steps": len(runner.trace)})
            await self._emit(session_id, "workflow.composition",
                             {"composition": name, "steps": runner.trace})
        return result_text(out)

    async def _emit(self, session_id: str, kind: str, payload: dict):
        if self.event_sink is None:
            return
        try:
            await self.event_sink.record(session_id, kind, payload)
        except Exception as e:  # noqa: BLE001
            log.debug("event sink failed: %s", e)

    async def load_state(self, session_id: str) -> dict | None:
        return await self.store.load(session_id)

    async def new_state(self, variables=None) -> dict:
        st = {"messages": [self._system_message(variables).to_dict()], "turn": 0,
              "created": time.time()}
        if self.workflow is not None:
            st["workflow"] = self.workflow.initial()
        return st

    def params(self, overrides: dict | None = None, guided: bool = False,
               prompt: Prompt | None = None) -> SamplingParams:
        """Sampling params for a turn.  ``guided``: enforce the function-mode response
        format in the engine (K13 grammar masks; ignored by remote/mock providers) --
        only on tool-free turns, where the whole answer is the JSON document."""
        d = {}
        dd = self.cfg.defaults or {}
        for k_src, k in (("temperature", "temperature"), ("topP", "top_p"),
                         ("maxTokens", "max_tokens")):
            if dd.get(k_src) is not None:
                # Provider CRD carries temperature / topP as decimal strings
                v = dd[k_src]
                d[k] = int(v) if k == "max_tokens" else float(v)
        d.update((prompt or self.prompt).parameters or {})
        d.update(overrides or {})
        if guided and self.cfg.response_format in ("json", "json_schema"):
            if self.cfg.response_format == "json_schema" and self.cfg.response_schema:
                d.setdefault("json_schema", self.cfg.response_schema)
            else:
                d.setdefault("json_object", True)
        return SamplingParams.from_dict(d)

    def _count(self, m: Message) -> int:
        if self.tokenizer is not None:
            return len(self.tokenizer.encode(m.content)) + 4
        return _approx_tokens(m.content) + 4

    async def _truncate(self, msgs: list[Message], budget: int) -> list[Message]:
        if budget <= 0:
            return msgs
        total = sum(self._count(m) for m in msgs)
        if total <= budget:
            return msgs
        system = [m for m in msgs if m.role == "system"][:1]
        rest = [m for m in msgs if not (m.role == "system" and system and m is system[0])]
        strategy = self.cfg.truncation or "sliding"
        if strategy == "custom":
            log.warning("custom truncation strategy not supported; falling back to sliding")
            strategy = "sliding"
        pinned = []  # a summary of dropped turns stays, like the system prompt
        if strategy == "summarize" and len(rest) > 2:
            cut = len(rest) // 2
            while cut < len(rest) and rest[cut].role == "tool":
                cut += 1  # never separate a tool call from its results
            old, keep = rest[:cut], rest[cut:]
            convo = "\n".join(f"{m.role}: {m.content}" for m in old)
            try:
                summary, _, _ = await self.provider.complete(
                    [Message("system", "Summarize the conversation so far in a few sentences."),
                     Message("user", convo)],
                    params=SamplingParams(temperature=0.0, max_tokens=128))
            except Exception:  # noqa: BLE001
                summary = ""
            pinned = [Message("system", f"Summary of earlier conversation: {summary}")]
            rest = keep
            msgs = system + pinned + rest
            if sum(self._count(m) for m in msgs) <= budget:
                return msgs
        # sliding: drop oldest non-system messages; a tool result never survives
        # without the assistant message that called it
        while rest and sum(self._count(m) for m in system + pinned + rest) > budget:
            rest.pop(0)
            while rest and rest[0].role == "tool":
                rest.pop(0)
        return system + pinned + rest

    # ------------------------------------------------------------ the turn
    async def run_turn(self, session_id: str, content: str, io: TurnIO, parts: list | None = None,
                       metadata: dict | None = None, ctx: CallContext | None = None,
                       variables: dict | None = None, persist: bool = True) -> TurnResult:
        t_start = time.perf_counter()
        logctx.bind(session_id=session_id, agent=getattr(ctx, "agent", "") or "")
        M.PIPELINES_ACTIVE.inc()
        ctx = ctx or CallContext(session_id=session_id)
        res = TurnResult()
        span = tracing.start_span("omnia.runtime.conversation.turn",
                                  {"session.id": session_id})
        try:
            state = await self.load_state(session_id) if persist else None
            if state is None:
                state = await self.new_state(variables)
            msgs = [Message.from_dict(d) for d in state["messages"]]
            user = Message("user", content, parts=parts or [])
            snap = None
            if self.workflow is not None:
                snap = state.setdefault("workflow", self.workflow.initial())
                if self.workflow.check_time(snap):
                    await self._completed(session_id, snap)
                ev = (metadata or {}).get("workflow_event")
                if ev:  # caller-driven transition (orchestration external / hybrid)
                    if not self.workflow.caller_can_fire(snap):
                        raise WorkflowError(f"state {snap['state']!r} does not accept "
                                            f"caller events")
                    rec = self.workflow.fire(snap, ev)
                    res.transitions.append(rec)
                    msgs = await self._enter_state(session_id, snap, rec, msgs, variables, None)
            prompt = self._active_prompt(snap)
            if self.memory is not None:
                try:
                    mem = await self.memory.retrieve(session_id, content, ctx)
                except Exception as e:  # noqa: BLE001
                    log.warning("memory retrieval failed: %s", e)
                    mem = ""
                if mem:
                    msgs.append(Message("system", f"Relevant memories:\n{mem}"))
            msgs.append(user)
            overrides = (metadata or {}).get("parameters") \
                if isinstance((metadata or {}).get("parameters"), dict) else None
            policy = prompt.tool_policy
            tools = self._tools(prompt, snap)
            params = self.params(overrides, guided=not tools, prompt=prompt)
            max_rounds = self.cfg.max_rounds or policy.max_rounds
            text_acc: list[str] = []
            calls_total = 0
            while True:
                comp = self.workflow.composition(snap) if snap is not None else None
                if comp:  # a composition state answers the turn with its step graph
                    text = await self._run_composition(comp, session_id, content, io, ctx,
                                                       metadata or {}, res)
                    await io.chunk(text)
                    text_acc.append(text)
                    msgs.append(Message("assistant", text))
                    res.rounds += 1
                    break
                window = await self._truncate(msgs, self.cfg.context_window)
                if tools and getattr(self.provider, "type", "") == "local" \
                        and policy.tool_choice in ("auto", "required"):
                    # the in-node engine enforces tool calls with a grammar.  "required"
                    # forces a valid call of an offered tool on every round until
                    # max_rounds tool rounds have run; the round after that is free
                    # ("auto") so the agent answers instead of hitting the round cap
                    params = dataclasses.replace(
                        params, tool_grammar=[{"name": t["name"],
                                               "parameters": t.get("parameters")
                                               or {"type": "object"}} for t in tools],
                        tool_choice=policy.tool_choice if res.rounds < max_rounds
                        else "auto")
                round_text: list[str] = []
                round_calls: list[ToolCallReq] = []
                span_llm = tracing.start_span("genai.chat", {
                    "gen_ai.system": self.provider.type, "gen_ai.request.model": self.provider.model})
                t_llm = time.perf_counter()
                status = "ok"
                try:
                    failpoints.hit("provider.stream")
                    async for ev in self.provider.stream(window, tools, params, session_id,
                                                         metadata):
                        if ev.type == "text" and ev.text:
                            round_text.append(ev.text)
                            text_acc.append(ev.text)
                            await io.chunk(ev.text)
                        elif ev.type == "tool_calls":
                            round_calls.extend(ev.tool_calls)
                        elif ev.type == "error":
                            raise ProviderError(ev.text or "provider error",
                                                ev.code or "PROVIDER_ERROR")
                        elif ev.type == "done":
                            if ev.usage:
                                res.usage += ev.usage
                            if res.ttft is None and ev.ttft is not None:
                                res.ttft = ev.ttft
                            res.finish_reason = ev.finish_reason
                except Exception:
                    status = "error"
                    raise
                finally:
                    M.child(M.PROVIDER_REQUESTS, self.provider.type, self.provider.model,
                            status).inc()
                    M.child(M.PROVIDER_DURATION, self.provider.type, self.provider.model).observe(
                        time.perf_counter() - t_llm)
                    tracing.end_span(span_llm, {"gen_ai.usage.input_tokens": res.usage.input_tokens,
                                                "gen_ai.usage.output_tokens":
                                                    res.usage.output_tokens})
                res.rounds += 1
                msgs.append(Message("assistant", "".join(round_text), tool_calls=round_calls))
                if not round_calls:
                    break
                if res.rounds > max_rounds:
                    log.warning("max_rounds %d reached; ending turn", max_rounds)
                    msgs[-1].tool_calls = []
                    break
                budget = policy.max_tool_calls_per_turn - calls_total
                allowed = round_calls[:max(0, budget)]
                calls_total += len(round_calls)
                results = await self._run_tools(allowed, io, ctx, metadata or {}, snap, res)
                for c in round_calls:
                    r = results.get(c.id) or {"result_json": json.dumps(
                        {"error": "max_tool_calls_per_turn exceeded"}), "is_error": True}
                    msgs.append(Message("tool", r["result_json"], tool_call_id=c.id, name=c.name))
                    res.tool_records.append({"name": c.name, "arguments": c.arguments or {},
                                             "error": bool(r.get("is_error"))})
                res.tool_calls = calls_total
                if snap is not None and self.workflow.count_tool_calls(snap, len(allowed)):
                    await self._completed(session_id, snap)
                    tools = []
                    params = self.params(overrides, guided=True, prompt=prompt)
                rec = results.get("__transition__")
                if rec is not None:  # the model moved the workflow: new prompt from here on
                    msgs = await self._enter_state(session_id, snap, rec, msgs, variables, user)
                    prompt = self._active_prompt(snap)
                    policy = prompt.tool_policy
                    tools = self._tools(prompt, snap)
                    params = self.params(overrides, guided=not tools, prompt=prompt)
            res.content = "".join(text_acc) if not msgs[-1].content else msgs[-1].content
            if res.rounds > 1:
                res.content = msgs[-1].content or "".join(text_acc)
            res.violations = run_validators(prompt, res.content)
            res.workflow = json.loads(json.dumps(snap)) if snap is not None else None
            for v in res.violations:
                M.VALIDATIONS.labels(v.split(":")[0], "fail").inc()
            res.cost = self.provider.pricing.cost(res.usage)
            M.child(M.PROVIDER_INPUT_TOKENS, self.provider.type, self.provider.model).inc(
                res.usage.input_tokens)
            M.child(M.PROVIDER_OUTPUT_TOKENS, self.provider.type, self.provider.model).inc(
                res.usage.output_tokens)
            M.child(M.PROVIDER_COST, self.provider.type, self.provider.model).inc(res.cost)
            if persist:
                state["messages"] = [m.to_dict() for m in msgs
                                     if not (m.role == "system" and m.content.startswith(
                                         "Relevant memories:"))]
                state["turn"] = state.get("turn", 0) + 1
                try:
                    await self.store.save(session_id, state)
                except StoreUnavailable as e:
                    log.warning("context store save failed: %s", e)
            if self.event_sink is not None:
                await self._record(session_id, content, res)
            if self.evaluator is not None:
                asyncio.get_running_loop().create_task(
                    self.evaluator.on_turn(session_id, content, res, prompt))
            return res
        finally:
            M.PIPELINES_ACTIVE.dec()
            M.PIPELINE_DURATION.observe(time.perf_counter() - t_start)
            tracing.end_span(span, {"gen_ai.usage.input_tokens": res.usage.input_tokens,
                                    "gen_ai.usage.output_tokens": res.usage.output_tokens,
                                    "gen_ai.usage.cost": res.cost})

    async def _run_tools(self, calls: list[ToolCallReq], io: TurnIO, ctx: CallContext,
                         metadata: dict, snap: dict | None = None,
                         res: TurnResult | None = None) -> dict[str, dict]:
        out: dict[str, dict] = {}
        internal = [c for c in calls if c.name in (TRANSITION_TOOL, ARTIFACT_TOOL)
                    or (self.multi_agent and c.name.startswith(AGENT_TOOL_PREFIX))]
        calls = [c for c in calls if all(c is not i for i in internal)]
        for c in internal:
            out[c.id] = await self._run_internal(c, ctx, snap, res, out)
        if self.executor is None:
            for c in calls:
                out[c.id] = {"result_json": json.dumps({"error": f"unknown tool {c.name}"}),
                             "is_error": True}
            return out
        if snap is not None and self.workflow is not None and self.workflow.skill_scope(snap):
            sk = self._skills()
            allowed = scoped_skill_names(self.workflow.skill_scope(snap), sk.skills if sk else {})
            for c in calls:
                if c.name.startswith("skill__") and (c.arguments or {}).get("name") not in allowed:
                    out[c.id] = {"result_json": json.dumps(
                        {"error": f"skill not available in state {snap['state']!r}"}),
                        "is_error": True}
            calls = [c for c in calls if c.id not in out]
        server = [c for c in calls if not self.executor.is_client_tool(c.name)]
        client = [c for c in calls if self.executor.is_client_tool(c.name)]

        async def run(c):
            span = tracing.start_span("omnia.tool.call", {"tool.name": c.name})
            sid = getattr(ctx, "session_id", "") or ""
            # session-api tool_calls rows (runtime/event_store.go:498-568): a pending
            # row when the call starts, a success / error row linked by call id
            await self._emit(sid, "tool_call", {"call_id": c.id, "name": c.name,
                                                "arguments": c.arguments or {},
                                                "status": "pending"})
            t0 = time.perf_counter()
            r, err = await self.executor.execute(c.name, c.arguments, ctx)
            tracing.end_span(span, {"tool.error": err})
            out[c.id] = {"result_json": r, "is_error": err}
            await self._emit(sid, "tool_call", {
                "call_id": c.id, "name": c.name, "status": "error" if err else "success",
                "duration_ms": int((time.perf_counter() - t0) * 1000),
                "result": r if not err else None, "error": r if err else ""})

        if server:
            await asyncio.gather(*(run(c) for c in server))
        if client:
            meta = {c.id: self.executor.tools[c.name].meta for c in client}
            got = await io.client_tool_calls(client, meta)
            for c in client:
                r = got.get(c.id)
                if r is None:
                    out[c.id] = {"result_json": json.dumps({"error": "no result"}),
                                 "is_error": True}
                elif r.get("is_rejected"):
                    out[c.id] = {"result_json": json.dumps(
                        {"rejected": True, "reason": r.get("rejection_reason", "")}),
                        "is_error": True}
                else:
                    out[c.id] = {"result_json": r.get("result_json", "null"), "is_error": False}
        return out

    async def _run_internal(self, c: ToolCallReq, ctx: CallContext, snap: dict | None,
                            res: TurnResult | None, out: dict) -> dict:
        args = c.arguments if isinstance(c.arguments, dict) else {}
        if c.name == ARTIFACT_TOOL:
            if self.workflow is None or snap is None:
                return {"result_json": json.dumps({"error": "no workflow"}), "is_error": True}
            try:
                r = self.workflow.put_artifact(snap, str(args.get("name", "")),
                                               args.get("content", ""))
            except WorkflowError as e:
                return {"result_json": json.dumps({"error": str(e)}), "is_error": True}
            return {"result_json": json.dumps(r), "is_error": False}
        if c.name == TRANSITION_TOOL:
            if self.workflow is None or snap is None:
                return {"result_json": json.dumps({"error": "no workflow"}), "is_error": True}
            if "__transition__" in out:
                return {"result_json": json.dumps(
                    {"error": "one transition per round; already moved to "
                              f"{snap['state']!r}"}), "is_error": True}
            if not self.workflow.model_can_fire(snap):
                return {"result_json": json.dumps(
                    {"error": f"state {snap['state']!r} is not model-orchestrated"}),
                    "is_error": True}
            try:
                rec = self.workflow.fire(snap, str(args.get("event", "")))
            except WorkflowError as e:
                return {"result_json": json.dumps({"error": str(e)}), "is_error": True}
            out["__transition__"] = rec
            if res is not None:
                res.transitions.append(rec)
            return {"result_json": json.dumps({"transitioned": True, **rec,
                                               "completed": snap["completed"]}),
                    "is_error": False}
        member = c.name[len(AGENT_TOOL_PREFIX):]
        if member not in (self.pack.agents or {}).get("members", {}) or \
                member == self.pack.agents["entry"]:
            return {"result_json": json.dumps({"error": f"unknown agent {member!r}"}),
                    "is_error": True}
        sub = self._members.get(member)
        if sub is None:
            sub = Agent(self.pack, self.provider, self.store, self.executor,
                        dataclasses.replace(self.cfg, prompt_name=member), self.extra,
                        self.memory, self.event_sink, None, self.tokenizer, graph=False)
            sub.prompt = self.pack.prompts[member]
            self._members[member] = sub
        sid = f"{ctx.session_id or ''}/agent/{member}"
        span = tracing.start_span("omnia.agent.delegate", {"agent.member": member})
        try:
            r = await sub.run_turn(sid, str(args.get("message", "")), _CollectIO(),
                                   ctx=dataclasses.replace(ctx, session_id=sid))
        except Exception as e:  # noqa: BLE001 - a failing member is a tool error
            tracing.end_span(span, error=True)
            return {"result_json": json.dumps({"agent": member, "error": str(e)}),
                    "is_error": True}
        tracing.end_span(span)
        if res is not None:
            res.usage += r.usage
        return {"result_json": json.dumps({"agent": member, "content": r.content}),
                "is_error": False}

    async def _record(self, session_id: str, user: str, res: TurnResult):
        try:
            await self.event_sink.record(session_id, "provider_call", {
                "provider": self.provider.type, "model": self.provider.model,
                "input_tokens": res.usage.input_tokens, "output_tokens": res.usage.output_tokens,
                "cached_tokens": res.usage.cached_tokens, "cost_usd": res.cost,
                "rounds": res.rounds, "tool_calls": res.tool_calls})
        except Exception as e:  # noqa: BLE001
            log.debug("event sink failed: %s", e)
