"""PromptPack workflows and multi-agent packs in the runtime.

Reference surface: ``internal/schema/promptpack.schema.json:200-216`` and the
``WorkflowConfig`` / ``WorkflowState`` / ``AgentsConfig`` / ``AgentDef`` defs
(``:1211-1343``); entry resolution ``internal/runtime/pack_entry.go:54-86``;
session events ``workflow.transitioned`` / ``workflow.completed``
(``internal/runtime/event_store.go:279-282``) with the span attributes of
``internal/session/otlp/attributes.go:97-104``.  The reference runtime delegates
the state machine to the PromptKit SDK; this module is the in-repo engine.

Workflow
    A conversation sits in one state at a time; the state's ``prompt_task``
    is the prompt the agent runs (system prompt, tools, parameters,
    validators).  The per-conversation snapshot ``{"state", "transitions",
    "completed", "history"}`` is stored with the conversation, so it survives
    runtime restarts through the context store like the messages do.

    Events fire from two sides, by the state's ``orchestration``:

    * ``internal`` (default): the model fires them through the server-side
      tool ``workflow__transition(event)`` whose ``event`` enum is the current
      state's ``on_event`` keys;
    * ``external``: only the caller fires them, with the message metadata key
      ``workflow_event`` (applied before the turn runs);
    * ``hybrid``: both.

    Entering a state with ``persistence: transient`` resets the context to the
    new system prompt (plus the in-flight user message); ``persistent`` (the
    default) keeps the history and swaps the system prompt.  A state with no
    ``on_event`` entries is terminal: entering it completes the workflow.
    A state's ``skills`` scopes the skill tools: ``"none"`` hides them, a path
    keeps only skills mounted under it.

    Loops and budgets (the compiled-pack fields of the reference's
    ``deep_research`` sample): a state with ``max_visits`` that would be
    entered once more is replaced by its ``on_max_visits`` state;
    ``engine.budget`` caps ``max_total_visits`` (state entries),
    ``max_tool_calls`` (over the whole workflow) and ``max_wall_time_sec``
    (since the workflow started) -- exhausting one completes the workflow where
    it stands (``snap["exhausted"]`` names the cap) and withdraws the
    transition tool (and, for the tool-call cap, every tool).  A state's
    ``artifacts`` ({name: {type, mode: append|replace}}) are written by the
    model through ``workflow__artifact`` and kept in the snapshot.  A state
    with ``orchestration: composition`` runs a declarative step graph
    (:mod:`.composition`) instead of a chat round.

Multi-agent
    The ``agents.entry`` prompt is the agent the conversation talks to; every
    other member is offered to it as a server-side tool ``agent__<member>``
    (``{"message": str}``).  A call runs one turn of the member's prompt on the
    same provider/engine, in the member's own persistent thread
    ``<session>/agent/<member>``, and returns its answer.  Members do not see
    other members (no recursion).  The A2A agent card lists the members as
    skills (:func:`card_skills`).
"""
from __future__ import annotations

import json

from .providers import ProviderError

TRANSITION_TOOL = "workflow__transition"
ARTIFACT_TOOL = "workflow__artifact"
AGENT_TOOL_PREFIX = "agent__"


class WorkflowError(ProviderError):
    def __init__(self, msg: str):
        super().__init__(msg, "INVALID_WORKFLOW_EVENT")


class Workflow:
    def __init__(self, cfg: dict):
        self.cfg = cfg
        self.entry: str = cfg["entry"]
        self.states: dict[str, dict] = cfg["states"]
        self.budget: dict = dict(((cfg.get("engine") or {}).get("budget")) or {})

    # ------------------------------------------------------------ snapshot
    def initial(self, now: float | None = None) -> dict:
        import time

        return {"state": self.entry, "transitions": 0,
                "completed": self.is_terminal(self.entry), "history": [],
                "visits": {self.entry: 1}, "tool_calls": 0,
                "started": time.time() if now is None else now, "artifacts": {}}

    def state(self, snap: dict) -> dict:
        return self.states[snap["state"]]

    def prompt_key(self, snap: dict) -> str | None:
        return self.state(snap).get("prompt_task")

    def composition(self, snap: dict) -> str | None:
        st = self.state(snap)
        return st.get("composition") if st.get("orchestration") == "composition" else None

    def events(self, snap: dict) -> dict[str, str]:
        return dict(self.state(snap).get("on_event") or {})

    def is_terminal(self, name: str) -> bool:
        st = self.states[name]
        return bool(st.get("terminal")) or not (st.get("on_event") or {})

    def orchestration(self, snap: dict) -> str:
        return self.state(snap).get("orchestration") or "internal"

    def persistence(self, name: str) -> str:
        return self.states[name].get("persistence") or "persistent"

    def model_can_fire(self, snap: dict) -> bool:
        return not snap["completed"] and self.orchestration(snap) in ("internal", "hybrid")

    def caller_can_fire(self, snap: dict) -> bool:
        return not snap["completed"] and self.orchestration(snap) in ("external", "hybrid")

    def skill_scope(self, snap: dict) -> str:
        """"" = every skill, "none" = no skills, else a mount-path prefix."""
        return self.state(snap).get("skills") or ""

    # ------------------------------------------------------------ budget
    def exhaust(self, snap: dict, cap: str):
        snap["completed"] = True
        snap["exhausted"] = cap

    def check_time(self, snap: dict, now: float | None = None) -> bool:
        """Complete the workflow if its wall-time budget ran out; True if it did."""
        import time

        lim = self.budget.get("max_wall_time_sec")
        if lim and not snap["completed"] and \
                (time.time() if now is None else now) - snap.get("started", 0) > lim:
            self.exhaust(snap, "max_wall_time_sec")
            return True
        return False

    def count_tool_calls(self, snap: dict, n: int) -> bool:
        """Account ``n`` tool calls; True if that exhausted the budget."""
        snap["tool_calls"] = snap.get("tool_calls", 0) + n
        lim = self.budget.get("max_tool_calls")
        if lim and snap["tool_calls"] >= lim and snap.get("exhausted") != "max_tool_calls":
            self.exhaust(snap, "max_tool_calls")
            return True
        return False

    # ------------------------------------------------------------ events
    def fire(self, snap: dict, event: str) -> dict:
        """Apply ``event`` to ``snap`` in place; returns the transition record
        ``{from_state, to_state, event, prompt_task}`` (plus ``redirected_from``
        when a ``max_visits`` loop bound rerouted it, or ``budget_exhausted``
        when the visit budget stopped it where it was)."""
        if snap["completed"]:
            raise WorkflowError(f"workflow already completed in state {snap['state']!r}")
        evs = self.events(snap)
        if event not in evs:
            raise WorkflowError(f"state {snap['state']!r} has no event {event!r} "
                                f"(events: {sorted(evs)})")
        src, dst = snap["state"], evs[event]
        visits = snap.setdefault("visits", {})
        redirected = None
        seen = set()
        while True:  # follow on_max_visits while the target is at its bound
            st = self.states[dst]
            mv = st.get("max_visits")
            if not mv or visits.get(dst, 0) < mv or dst in seen:
                break
            if not st.get("on_max_visits"):
                raise WorkflowError(f"state {dst!r} reached max_visits {mv}")
            seen.add(dst)
            redirected = redirected or dst
            dst = st["on_max_visits"]
        lim = self.budget.get("max_total_visits")
        if lim and sum(visits.values()) >= lim:
            self.exhaust(snap, "max_total_visits")
            return {"from_state": src, "to_state": src, "event": event,
                    "prompt_task": self.states[src].get("prompt_task"),
                    "budget_exhausted": "max_total_visits"}
        rec = {"from_state": src, "to_state": dst, "event": event,
               "prompt_task": self.states[dst].get("prompt_task")}
        if redirected:
            rec["redirected_from"] = redirected
        snap["state"] = dst
        snap["transitions"] += 1
        visits[dst] = visits.get(dst, 0) + 1
        snap["history"].append(rec)
        snap["completed"] = self.is_terminal(dst)
        return rec

    # ------------------------------------------------------------ artifacts
    def artifact_spec(self, snap: dict) -> dict | None:
        arts = self.state(snap).get("artifacts") or {}
        if not arts:
            return None
        lines = [f"- {n} ({a.get('type', 'text/plain')}, {a.get('mode', 'replace')}): "
                 f"{a.get('description', '')}" for n, a in sorted(arts.items())]
        return {"name": ARTIFACT_TOOL,
                "description": "Record a workflow artifact of the current state:\n"
                               + "\n".join(lines),
                "parameters": {"type": "object",
                               "properties": {"name": {"type": "string", "enum": sorted(arts)},
                                              "content": {"type": "string"}},
                               "required": ["name", "content"]}}

    def put_artifact(self, snap: dict, name: str, content) -> dict:
        arts = self.state(snap).get("artifacts") or {}
        if name not in arts:
            raise WorkflowError(f"state {snap['state']!r} declares no artifact {name!r}")
        store = snap.setdefault("artifacts", {})
        if arts[name].get("mode", "replace") == "append":
            store.setdefault(name, []).append(content)
        else:
            store[name] = content
        return {"artifact": name, "mode": arts[name].get("mode", "replace"),
                "state": snap["state"]}

    def tool_spec(self, snap: dict) -> dict:
        evs = self.events(snap)
        lines = []
        for ev, target in sorted(evs.items()):
            desc = self.states[target].get("description", "")
            lines.append(f"- {ev} -> {target}" + (f": {desc}" if desc else ""))
        here = self.state(snap).get("description", "")
        return {"name": TRANSITION_TOOL,
                "description": (f"Move the conversation to the next workflow state. Current "
                                 f"state: {snap['state']}" + (f" ({here})" if here else "")
                                 + ". Events:\n" + "\n".join(lines)),
                "parameters": {"type": "object",
                               "properties": {"event": {"type": "string", "enum": sorted(evs)},
                                              "reason": {"type": "string"}},
                               "required": ["event"]}}


# ---------------------------------------------------------------- multi-agent
def member_tool_specs(pack) -> list[dict]:
    ag = pack.agents or {}
    out = []
    for key, d in (ag.get("members") or {}).items():
        if key == ag.get("entry"):
            continue
        p = pack.prompts[key]
        desc = (d or {}).get("description") or p.raw.get("description") or \
            f"Delegate to the {p.name} agent"
        out.append({"name": AGENT_TOOL_PREFIX + key,
                    "description": desc,
                    "parameters": {"type": "object",
                                   "properties": {"message": {
                                       "type": "string",
                                       "description": "the request for this agent"}},
                                   "required": ["message"]}})
    return out


def card_skills(pack) -> list[dict]:
    """A2A agent-card skills of a multi-agent pack (one per member)."""
    ag = pack.agents or {}
    out = []
    for key, d in (ag.get("members") or {}).items():
        d = d or {}
        p = pack.prompts[key]
        out.append({"id": key, "name": p.name,
                    "description": d.get("description") or p.raw.get("description", ""),
                    "tags": list(d.get("tags") or []),
                    "inputModes": list(d.get("input_modes") or ["text/plain"]),
                    "outputModes": list(d.get("output_modes") or ["text/plain"])})
    return out


def scoped_skill_names(scope: str, skills: dict) -> set[str]:
    """Skills visible under a workflow state's ``skills`` filter ("" = all)."""
    if not scope:
        return set(skills)
    if scope == "none":
        return set()
    prefix = (scope[2:] if scope.startswith("./") else scope).strip("/")
    return {n for n, s in skills.items()
            if s.mount_as.removeprefix("./").strip("/").startswith(prefix)}


def scope_skill_specs(specs: list[dict], scope: str, skills: dict) -> list[dict]:
    """Apply a workflow state's ``skills`` filter to the offered tool specs.
    ``skills``: name -> object with ``mount_as`` (the skills handler's table)."""
    if not scope:
        return specs
    allowed = sorted(scoped_skill_names(scope, skills))
    out = []
    for s in specs:
        if s["name"].startswith("skill__"):
            if not allowed:
                continue
            s = json.loads(json.dumps(s))
            s["parameters"]["properties"]["name"]["enum"] = allowed
        out.append(s)
    return out
