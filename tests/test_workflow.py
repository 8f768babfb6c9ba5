"""PromptPack ``workflow`` / ``agents`` / ``skills`` sections
(``internal/schema/promptpack.schema.json:200-216, 1211-1404``), entry
resolution (``internal/runtime/pack_entry.go:54-86``, cases mirrored from
``pack_entry_test.go``), and their execution in the agent loop: model- and
caller-driven transitions, persistence, terminal states, per-state skill
scoping, member-agent delegation, and the A2A card."""
import asyncio
import json

import pytest

from omnia_amd.runtime.agent import Agent, AgentConfig, TurnIO
from omnia_amd.runtime.context_store import MemoryContextStore
from omnia_amd.runtime.promptpack import PackError, PromptPack
from omnia_amd.runtime.providers import MockProvider
from omnia_amd.runtime.workflow import (TRANSITION_TOOL, WorkflowError, card_skills,
                                        scoped_skill_names)
from omnia_amd.tools.executor import OmniaExecutor


def _prompt(key, system, **kw):
    return {"id": key, "name": key, "version": "1.0.0", "system_template": system, **kw}


def _pack(**extra):
    return {"id": "support", "name": "support", "version": "1.0.0",
            "template_engine": {"version": "v1", "syntax": "{{variable}}"},
            "prompts": {"triage": _prompt("triage", "You triage."),
                        "billing": _prompt("billing", "You handle billing for {{company}}.",
                                           parameters={"temperature": 0.1}),
                        "closing": _prompt("closing", "You close the conversation.")},
            **extra}


WORKFLOW = {"version": 1, "entry": "triage",
            "states": {"triage": {"prompt_task": "triage", "description": "find the topic",
                                  "on_event": {"billing_issue": "billing", "done": "closing"}},
                       "billing": {"prompt_task": "billing", "on_event": {"resolved": "closing"},
                                   "persistence": "persistent"},
                       "closing": {"prompt_task": "closing", "on_event": {}}}}


class _IO(TurnIO):
    def __init__(self):
        self.text = []

    async def chunk(self, text):
        self.text.append(text)


class _Sink:
    def __init__(self):
        self.events = []

    async def record(self, sid, kind, payload):
        self.events.append((sid, kind, payload))


def _run(coro):
    return asyncio.run(coro)


# ------------------------------------------------------------------ schema
def test_workflow_agents_skills_sections_load():
    p = PromptPack(_pack(workflow=WORKFLOW,
                         agents={"entry": "triage",
                                 "members": {"triage": {"description": "router"},
                                             "billing": {"tags": ["billing"]}}},
                         skills=["./skills", {"path": "./more", "preload": True},
                                 {"name": "refunds", "description": "refund policy",
                                  "instructions": "Refund within 30 days."}]))
    assert p.workflow["entry"] == "triage" and p.agents["entry"] == "triage"
    assert len(p.skill_sources) == 3


@pytest.mark.parametrize("bad,msg", [
    ({"workflow": {"version": 1, "entry": "nope", "states": WORKFLOW["states"]}},
     "workflow.entry"),
    ({"workflow": {"version": 1, "entry": "a",
                   "states": {"a": {"prompt_task": "ghost", "on_event": {}}}}}, "prompt_task"),
    ({"workflow": {"version": 1, "entry": "a",
                   "states": {"a": {"prompt_task": "triage", "on_event": {"x": "zz"}}}}},
     "unknown state"),
    ({"workflow": {"version": 0, "entry": "a",
                   "states": {"a": {"prompt_task": "triage", "on_event": {}}}}}, "invalid"),
    ({"workflow": {"version": 1, "entry": "a", "states": {}}}, "invalid"),
    ({"workflow": {"version": 1, "entry": "a",
                   "states": {"a": {"on_event": {}}}}}, "prompt_task"),
    ({"workflow": {"version": 1, "entry": "a", "states": {
        "a": {"orchestration": "composition", "composition": "nope"}}}}, "composition"),
    ({"workflow": {"version": 1, "entry": "a", "states": {
        "a": {"prompt_task": "triage", "max_visits": 2, "on_max_visits": "zz"}}}},
     "on_max_visits"),
    ({"compositions": {"c": {"steps": [{"id": "x", "kind": "prompt", "prompt_task": "ghost"}]}}},
     "not a prompt"),
    ({"compositions": {"c": {"steps": [{"id": "x", "kind": "branch", "then": "y",
                                        "predicate": {"path": "${a}", "op": "equals"}}]}}},
     "branch target"),
    ({"compositions": {"c": {"steps": [
        {"id": "x", "kind": "tool", "tool": "t"}, {"id": "x", "kind": "tool", "tool": "t"}]}}},
     "duplicate"),
    ({"compositions": {"c": {"steps": [{"id": "x", "kind": "loop"}]}}}, "invalid"),
    ({"workflow": {"version": 1, "entry": "a", "states": {
        "a": {"prompt_task": "triage", "on_event": {}, "persistence": "forever"}}}}, "invalid"),
    ({"workflow": {"version": 1, "entry": "a", "extra": 1, "states": {
        "a": {"prompt_task": "triage", "on_event": {}}}}}, "invalid"),
    ({"agents": {"entry": "boss", "members": {"triage": {}}}}, "agents.entry"),
    ({"agents": {"entry": "ghost", "members": {"ghost": {}}}}, "not a prompt"),
    ({"agents": {"entry": "triage", "members": {}}}, "invalid"),
    ({"agents": {"entry": "triage", "members": {"triage": {"colour": "red"}}}}, "invalid"),
    ({"skills": [{"name": "x", "description": "", "instructions": "y"}]}, "invalid"),
    ({"skills": [{"path": "./s", "preload": "yes"}]}, "invalid"),
    ({"skills": [42]}, "invalid"),
])
def test_graph_sections_rejected(bad, msg):
    with pytest.raises(PackError, match=msg):
        PromptPack(_pack(**bad))


def test_entry_resolution_order():
    # workflow.entry wins over agents.entry; resolves to the entry state's prompt
    p = PromptPack(_pack(workflow={**WORKFLOW, "entry": "billing"},
                         agents={"entry": "triage", "members": {"triage": {}}}))
    assert p.entry() == "billing" and p.prompt().id == "billing"
    p = PromptPack(_pack(agents={"entry": "closing", "members": {"closing": {}}}))
    assert p.entry() == "closing"
    one = _pack()
    one["prompts"] = {"solo": _prompt("solo", "only")}
    assert PromptPack(one).entry("default") == "solo"
    assert PromptPack(_pack()).entry("default") == "default"  # multi-prompt plain pack


def test_pack_load_keeps_base_dir(tmp_path):
    (tmp_path / "pack.json").write_text(json.dumps(_pack(workflow=WORKFLOW)))
    p = PromptPack.load(tmp_path)
    assert p.base_dir == tmp_path and p.workflow["entry"] == "triage"


# ------------------------------------------------------------------ execution
def _agent(pack_data, scenarios, executor=None, sink=None, store=None):
    pack = PromptPack(pack_data)
    prov = MockProvider(scenarios={"scenarios": scenarios})
    return Agent(pack, prov, store or MemoryContextStore(), executor,
                 AgentConfig(variables={"company": "Acme"}), event_sink=sink), prov


def test_model_driven_transition_switches_prompt_and_completes():
    sink = _Sink()
    agent, prov = _agent(_pack(workflow=WORKFLOW), {"s": {"turns": [
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "billing_issue"}}]},
        {"response": "Billing here: what is the invoice number?"},
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "resolved"}}]},
        {"response": "Glad it is resolved. Bye!"}]}}, sink=sink)
    md = {"mock_scenario": "s"}
    r1 = _run(agent.run_turn("c1", "my invoice is wrong", _IO(), metadata=md))
    assert r1.content == "Billing here: what is the invoice number?"
    assert r1.workflow["state"] == "billing" and not r1.workflow["completed"]
    assert [t["to_state"] for t in r1.transitions] == ["billing"]
    # round 1 ran the triage prompt with the transition tool; round 2 the billing prompt
    c0, c1 = prov.calls[0], prov.calls[1]
    assert c0["messages"][0]["content"] == "You triage."
    assert TRANSITION_TOOL in c0["tools"]
    assert c1["messages"][0]["content"] == "You handle billing for Acme."
    assert c1["messages"][-1]["role"] == "tool"  # persistent: history kept
    ev_tool = json.loads(c1["messages"][-1]["content"])
    assert ev_tool["transitioned"] and ev_tool["to_state"] == "billing"
    r2 = _run(agent.run_turn("c1", "it's fixed now", _IO(), metadata=md))
    assert r2.workflow["state"] == "closing" and r2.workflow["completed"]
    assert r2.workflow["transitions"] == 2
    # the terminal state offers no transition tool
    assert TRANSITION_TOOL not in prov.calls[-1]["tools"]
    kinds = [k for _, k, _ in sink.events if k.startswith("workflow.")]
    assert kinds == ["workflow.transitioned", "workflow.transitioned", "workflow.completed"]
    done = [p for _, k, p in sink.events if k == "workflow.completed"][0]
    assert done == {"final_state": "closing", "transition_count": 2}


def test_workflow_state_survives_restart_through_store():
    store = MemoryContextStore()
    sc = {"s": {"turns": [
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "billing_issue"}}]},
        {"response": "ok"}]}}
    a1, _ = _agent(_pack(workflow=WORKFLOW), sc, store=store)
    _run(a1.run_turn("c9", "hi", _IO(), metadata={"mock_scenario": "s"}))
    a2, prov2 = _agent(_pack(workflow=WORKFLOW), {"d": {"turns": [{"response": "again"}]}},
                       store=store)  # a new runtime process, same context store
    r = _run(a2.run_turn("c9", "still there?", _IO(), metadata={"mock_scenario": "d"}))
    assert r.workflow["state"] == "billing"
    assert prov2.calls[0]["messages"][0]["content"] == "You handle billing for Acme."


def test_invalid_event_is_a_tool_error_not_a_transition():
    agent, prov = _agent(_pack(workflow=WORKFLOW), {"s": {"turns": [
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "teleport"}}]},
        {"response": "sorry"}]}})
    r = _run(agent.run_turn("c2", "x", _IO(), metadata={"mock_scenario": "s"}))
    assert r.workflow["state"] == "triage" and r.transitions == []
    err = json.loads(prov.calls[1]["messages"][-1]["content"])
    assert "no event 'teleport'" in err["error"]


def test_transient_state_resets_context():
    wf = json.loads(json.dumps(WORKFLOW))
    wf["states"]["billing"]["persistence"] = "transient"
    agent, prov = _agent(_pack(workflow=wf), {"s": {"turns": [
        {"response": "hello, what's up?"},
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "billing_issue"}}]},
        {"response": "billing"}]}})
    md = {"mock_scenario": "s"}
    _run(agent.run_turn("c3", "hi", _IO(), metadata=md))
    _run(agent.run_turn("c3", "my bill", _IO(), metadata=md))
    msgs = prov.calls[-1]["messages"]
    assert [m["role"] for m in msgs] == ["system", "user"]
    assert msgs[0]["content"].startswith("You handle billing") and msgs[1]["content"] == "my bill"


def test_caller_driven_transitions_by_orchestration():
    wf = json.loads(json.dumps(WORKFLOW))
    wf["states"]["triage"]["orchestration"] = "external"
    agent, prov = _agent(_pack(workflow=wf), {"s": {"turns": [{"response": "r"}]}})
    # external state: the model is not offered the transition tool
    _run(agent.run_turn("c4", "hi", _IO(), metadata={"mock_scenario": "s"}))
    assert TRANSITION_TOOL not in prov.calls[-1]["tools"]
    r = _run(agent.run_turn("c4", "bill", _IO(),
                            metadata={"mock_scenario": "s", "workflow_event": "billing_issue"}))
    assert r.workflow["state"] == "billing"
    assert prov.calls[-1]["messages"][0]["content"].startswith("You handle billing")
    # billing is internal-only: a caller event is refused with a coded error
    with pytest.raises(WorkflowError):
        _run(agent.run_turn("c4", "x", _IO(),
                            metadata={"mock_scenario": "s", "workflow_event": "resolved"}))


def test_state_skill_scoping(tmp_path):
    for name, mount in (("billing-faq", "billing"), ("chit-chat", "general")):
        d = tmp_path / "skills" / mount / name
        d.mkdir(parents=True)
        (d / "SKILL.md").write_text(f"---\nname: {name}\ndescription: {name} d\n---\nDo {name}.")
    data = _pack(workflow=json.loads(json.dumps(WORKFLOW)),
                 skills=["./skills/billing", "./skills/general"])
    data["workflow"]["states"]["billing"]["skills"] = "./skills/billing"
    data["workflow"]["states"]["triage"]["skills"] = "none"
    (tmp_path / "pack.json").write_text(json.dumps(data))
    pack = PromptPack.load(tmp_path)
    ex = OmniaExecutor({})
    from omnia_amd.runtime.skills import attach_skills

    h = attach_skills(ex, manifest_path="", pack=pack)
    assert set(h.skills) == {"billing-faq", "chit-chat"}
    assert scoped_skill_names("./skills/billing", h.skills) == {"billing-faq"}
    _run(ex.discover())
    prov = MockProvider(scenarios={"scenarios": {"s": {"turns": [
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "billing_issue"}}]},
        {"tool_calls": [{"name": "skill__activate", "arguments": {"name": "chit-chat"}},
                        {"name": "skill__activate", "arguments": {"name": "billing-faq"}}]},
        {"response": "done"}]}}})
    agent = Agent(pack, prov, MemoryContextStore(), ex, AgentConfig())
    _run(agent.run_turn("c5", "hi", _IO(), metadata={"mock_scenario": "s"}))
    assert not any(t.startswith("skill__") for t in prov.calls[0]["tools"])  # triage: none
    assert "skill__activate" in prov.calls[1]["tools"]
    tool_msgs = [m for m in prov.calls[2]["messages"] if m["role"] == "tool"]
    denied, ok = json.loads(tool_msgs[-2]["content"]), json.loads(tool_msgs[-1]["content"])
    assert "not available" in denied["error"]
    assert ok["instructions"] == "Do billing-faq."


def test_inline_preloaded_skill_is_in_system_prompt():
    pack = PromptPack(_pack(skills=[{"name": "refunds", "description": "refund policy",
                                     "instructions": "Refund within 30 days."}]))
    ex = OmniaExecutor({})
    from omnia_amd.runtime.skills import attach_skills

    attach_skills(ex, manifest_path="", pack=pack)
    _run(ex.discover())
    prov = MockProvider(scenarios={"default_response": "ok"})
    agent = Agent(pack, prov, MemoryContextStore(), ex, AgentConfig(prompt_name="triage"))
    _run(agent.run_turn("c6", "hi", _IO()))
    sys_msg = prov.calls[0]["messages"][0]["content"]
    assert sys_msg.startswith("You triage.") and "Refund within 30 days." in sys_msg


AGENTS = {"entry": "triage",
          "members": {"triage": {"description": "front desk"},
                      "billing": {"description": "billing specialist", "tags": ["billing"],
                                  "input_modes": ["text/plain", "application/json"]}}}


def test_multi_agent_delegation():
    sink = _Sink()
    agent, prov = _agent(_pack(agents=AGENTS), {
        "s": {"turns": [
            {"tool_calls": [{"name": "agent__billing",
                             "arguments": {"message": "invoice 42 is wrong"}}]},
            {"response": "Billing says: corrected."}]},
        "default": {"turns": [{"response": "Invoice 42 corrected."}]}}, sink=sink)
    r = _run(agent.run_turn("c7", "fix my invoice", _IO(), metadata={"mock_scenario": "s"}))
    assert r.content == "Billing says: corrected."
    assert prov.calls[0]["tools"] == ["agent__billing"]  # the entry sees members, not itself
    sub = prov.calls[1]
    assert sub["messages"][0]["content"] == "You handle billing for Acme."
    assert sub["messages"][-1] == {"role": "user", "content": "invoice 42 is wrong"} or \
        sub["messages"][-1]["content"] == "invoice 42 is wrong"
    assert sub["tools"] == []  # members don't delegate further
    res = json.loads(prov.calls[2]["messages"][-1]["content"])
    assert res == {"agent": "billing", "content": "Invoice 42 corrected."}
    # the member keeps its own thread per parent conversation
    st = _run(agent.store.load("c7/agent/billing"))
    assert [m["role"] for m in st["messages"]] == ["system", "user", "assistant"]


def test_card_skills_from_agents():
    pack = PromptPack(_pack(agents=AGENTS))
    cs = card_skills(pack)
    assert [c["id"] for c in cs] == ["triage", "billing"]
    assert cs[1]["tags"] == ["billing"] and cs[1]["inputModes"] == ["text/plain",
                                                                    "application/json"]
    assert cs[0]["outputModes"] == ["text/plain"]


def test_a2a_card_lists_members(tmp_path, monkeypatch):
    from aiohttp.test_utils import TestClient, TestServer
    from aiohttp import web

    from omnia_amd.facade.a2a import mount_a2a

    (tmp_path / "pack.json").write_text(json.dumps(_pack(agents=AGENTS)))
    monkeypatch.setenv("OMNIA_PROMPTPACK_PATH", str(tmp_path / "pack.json"))

    class _Fac:
        class cfg:
            agent = "support"
        app = web.Application()

    mount_a2a(_Fac, runtime_client=None)

    async def go():
        async with TestClient(TestServer(_Fac.app)) as c:
            r = await c.get("/.well-known/agent.json")
            return await r.json()

    card = _run(go())
    assert [s["id"] for s in card["skills"]] == ["triage", "billing"]


# ------------------------------------------------------------------ compiled reference packs
def _reference_pack(path):
    """pack.json embedded in a reference sample's ConfigMap (yaml.safe_load)."""
    import os

    import yaml

    full = os.path.join("/root/reference", path)
    if not os.path.exists(full):
        pytest.skip("reference samples not available")
    with open(full) as f:
        for doc in yaml.safe_load_all(f):
            if doc and doc.get("kind") == "ConfigMap" and "pack.json" in (doc.get("data") or {}):
                return json.loads(doc["data"]["pack.json"])
    raise AssertionError("no pack.json in " + path)


@pytest.mark.parametrize("path", [
    "config/samples/omnia_v1alpha1_promptpack.yaml",
    "config/samples/omnia_v1alpha1_promptpack_deep_research.yaml",
    "config/samples/omnia_v1alpha1_promptpack_doc_analysis.yaml",
    "config/samples/dev/deep-research-function.yaml",
])
def test_reference_sample_packs_load(path):
    p = PromptPack(_reference_pack(path))
    assert p.workflow and p.entry() in p.prompts


def _deep_research():
    data = _reference_pack("config/samples/omnia_v1alpha1_promptpack_deep_research.yaml")
    return data


def test_max_visits_redirects_and_budget_completes():
    from omnia_amd.runtime.workflow import Workflow

    wf = Workflow(_deep_research()["workflow"])
    snap = wf.initial(now=0.0)
    wf.fire(snap, "start")                       # plan -> gather (visit 1)
    for _ in range(3):                           # gather <-> assess loop: gather visits 2..4
        wf.fire(snap, "assess")
        wf.fire(snap, "need_more")
    assert snap["state"] == "gather" and snap["visits"]["gather"] == 4
    wf.fire(snap, "assess")
    rec = wf.fire(snap, "need_more")             # 5th gather visit -> on_max_visits
    assert rec["to_state"] == "synthesize" and rec["redirected_from"] == "gather"
    assert sum(snap["visits"].values()) == 10
    wf.fire(snap, "done")                        # review: 11th visit
    wf.fire(snap, "revise")                      # synthesize: 12th (= max_total_visits)
    rec = wf.fire(snap, "done")                  # a 13th entry exceeds the budget
    assert rec["budget_exhausted"] == "max_total_visits"
    assert snap["completed"] and snap["state"] == "synthesize"
    with pytest.raises(WorkflowError):
        wf.fire(snap, "approve")


def test_wall_time_and_tool_call_budgets():
    from omnia_amd.runtime.workflow import Workflow

    wf = Workflow(_deep_research()["workflow"])
    snap = wf.initial(now=100.0)
    assert not wf.check_time(snap, now=150.0)
    assert wf.check_time(snap, now=191.0) and snap["exhausted"] == "max_wall_time_sec"
    snap = wf.initial(now=0.0)
    assert not wf.count_tool_calls(snap, 29)
    assert wf.count_tool_calls(snap, 1) and snap["exhausted"] == "max_tool_calls"


def test_tool_budget_withdraws_tools_in_the_agent_loop():
    data = _pack(workflow=json.loads(json.dumps(WORKFLOW)))
    data["workflow"]["engine"] = {"budget": {"max_tool_calls": 1}}
    sink = _Sink()
    agent, prov = _agent(data, {"s": {"turns": [
        {"tool_calls": [{"name": TRANSITION_TOOL, "arguments": {"event": "billing_issue"}}]},
        {"response": "answering without tools"}]}}, sink=sink)
    r = _run(agent.run_turn("b1", "x", _IO(), metadata={"mock_scenario": "s"}))
    assert r.workflow["exhausted"] == "max_tool_calls" and r.workflow["completed"]
    assert prov.calls[-1]["tools"] == []
    assert ("b1", "workflow.completed", {"final_state": "billing", "transition_count": 1,
                                         "budget_exhausted": "max_tool_calls"}) in sink.events


def test_artifacts_append_and_replace():
    data = _pack(workflow=json.loads(json.dumps(WORKFLOW)))
    data["workflow"]["states"]["triage"]["artifacts"] = {
        "notes": {"type": "application/json", "mode": "append"},
        "summary": {"type": "text/markdown", "mode": "replace"}}
    agent, prov = _agent(data, {"s": {"turns": [
        {"tool_calls": [{"name": "workflow__artifact", "arguments": {"name": "notes",
                                                                     "content": "a"}},
                        {"name": "workflow__artifact", "arguments": {"name": "notes",
                                                                     "content": "b"}},
                        {"name": "workflow__artifact", "arguments": {"name": "summary",
                                                                     "content": "v1"}},
                        {"name": "workflow__artifact", "arguments": {"name": "summary",
                                                                     "content": "v2"}},
                        {"name": "workflow__artifact", "arguments": {"name": "nope",
                                                                     "content": "x"}}]},
        {"response": "noted"}]}})
    r = _run(agent.run_turn("a1", "x", _IO(), metadata={"mock_scenario": "s"}))
    assert r.workflow["artifacts"] == {"notes": ["a", "b"], "summary": "v2"}
    assert "workflow__artifact" in prov.calls[0]["tools"]
    assert "no artifact 'nope'" in prov.calls[1]["messages"][-1]["content"]


# ------------------------------------------------------------------ compositions
def test_composition_state_runs_the_step_graph():
    """The reference's doc-analysis pack: intake -> (proceed) -> analyze, a
    composition with prompt / parallel(prompt + tool) / branch / agent steps."""
    from omnia_amd.tools.executor import InProcessHandler

    data = _reference_pack("config/samples/omnia_v1alpha1_promptpack_doc_analysis.yaml")
    ex = OmniaExecutor({})
    seen = {}

    async def parse(args, ctx):
        seen["parse"] = args
        return {"sections": ["Abstract", "Methods"]}

    async def lookup(args, ctx):
        return {"text": "methods text"}

    async def refs(args, ctx):
        return {"hits": 3}

    ex.add_handler(InProcessHandler("docs", {
        "doc_parse_structure": ("parse", {"type": "object"}, parse),
        "doc_section_lookup": ("lookup", {"type": "object"}, lookup),
        "ref_search": ("refs", {"type": "object"}, refs)}))
    _run(ex.discover())
    pack = PromptPack(data)
    systems = {k: pack.render_system(p) for k, p in pack.prompts.items()}

    class Scripted(MockProvider):
        """Answers by which prompt is speaking (the system message)."""
        script = {"triage": [[(TRANSITION_TOOL, {"event": "proceed"})]],
                  "classifier": ['{"type": "research_paper", "confidence": 0.9}'],
                  "title_extractor": ['{"title": "On Things"}'],
                  "paper_analyzer": [[("doc_section_lookup", {"section": "Methods"})],
                                     "The paper's methods are sound."],
                  "summarizer": ["a summary"]}

        async def stream(self, messages, tools, params, session_id=None, metadata=None):
            from omnia_amd.runtime.chat import ToolCallReq
            from omnia_amd.runtime.providers import ProviderEvent, Usage

            who = next(k for k, v in systems.items() if messages[0].content.startswith(v))
            self.calls.append({"who": who, "tools": [t["name"] for t in tools or []],
                               "messages": [m.to_dict() for m in messages]})
            nxt = self.script[who].pop(0)
            if isinstance(nxt, list):
                yield ProviderEvent("tool_calls", tool_calls=[
                    ToolCallReq(id=f"c{i}", name=n, arguments=a) for i, (n, a) in enumerate(nxt)])
            else:
                yield ProviderEvent("text", text=nxt)
            yield ProviderEvent("done", usage=Usage(1, 1))

    prov = Scripted()
    agent = Agent(pack, prov, MemoryContextStore(), ex, AgentConfig())
    io = _IO()
    r = _run(agent.run_turn("d1", "A study of things. Abstract... Methods...", io,
                            metadata={"mock_scenario": "s"}))
    assert r.workflow["state"] == "analyze" and r.workflow["completed"]
    trace = {t["id"]: t for t in r.composition}
    assert trace["classify"]["status"] == "ok"
    assert trace["route"]["taken"] == "then"
    assert trace["analyze_paper"]["status"] == "ok" and trace["analyze_paper"]["evals"] == \
        ["analysis_quality"]
    assert trace["summarize"]["status"] == "skipped"
    assert seen["parse"] == {"content": "A study of things. Abstract... Methods..."}
    assert r.content == "The paper's methods are sound."
    # the agent step offered only its listed tools, bounded by termination.max_steps
    agent_call = [c for c in prov.calls if c["who"] == "paper_analyzer"][0]
    assert sorted(agent_call["tools"]) == ["doc_section_lookup", "ref_search"]
    assert [c["who"] for c in prov.calls].count("summarizer") == 0  # routed around
    assert r.usage.input_tokens == 5  # triage + classify + title + 2 agent rounds


def test_composition_primitives():
    from omnia_amd.runtime.composition import evaluate, parse_output, template

    env = {"input": {"text": "hi"}, "a": {"output": {"type": "x", "n": 3, "tags": ["k"]}}}
    assert template("${input.text}", env) == "hi"
    assert template("${a.output}", env) == {"type": "x", "n": 3, "tags": ["k"]}
    assert template("say ${input.text} / ${a.output.n}", env) == "say hi / 3"
    assert template({"q": ["${a.output.type}"]}, env) == {"q": ["x"]}
    assert evaluate({"path": "${a.output.type}", "op": "equals", "value": "x"}, env)
    assert evaluate({"path": "${a.output.n}", "op": "gt", "value": 2}, env)
    assert not evaluate({"path": "${a.output.n}", "op": "lt", "value": "2"}, env)
    assert evaluate({"path": "${a.output.tags}", "op": "contains", "value": "k"}, env)
    assert evaluate({"path": "${a.output.type}", "op": "in", "value": ["x", "y"]}, env)
    assert not evaluate({"path": "${a.output.missing}", "op": "exists"}, env)
    assert parse_output('```json\n{"a": 1}\n```') == {"a": 1}
    assert parse_output('Sure: {"a": 2} done') == {"a": 2}
    assert parse_output("plain") == "plain"
