"""Eval-type registry parity (verdict r5 item 3): every eval type of the
reference's shipped sample PromptPack (``config/samples/omnia_v1alpha1_promptpack.yaml``,
its definitions in ``fixtures/sample_pack_evals.json``) and the realtime-evals
doc's ``llm_judge_turn`` is registered; scripted tool turns drive every eval of
the pack to a pass AND a fail, inline (runtime) and in the eval worker; unknown
types produce error rows, never a silent skip."""
import asyncio
import json
import os
from dataclasses import dataclass, field

import pytest

from omnia_amd.runtime import evals as E

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "sample_pack_evals.json")
REF = "/root/reference/config/samples/omnia_v1alpha1_promptpack.yaml"


def _pack():
    with open(FIX) as f:
        return json.load(f)


def _all_evals(pack):
    out = list(pack["pack_evals"])
    for p in pack["prompts"].values():
        out.extend(p["evals"])
    return out


def test_fixture_matches_reference_sample():
    if not os.path.exists(REF):
        pytest.skip("reference tree not present")
    import yaml

    docs = [d for d in yaml.safe_load_all(open(REF)) if d and d.get("kind") == "ConfigMap"]
    ref = json.loads(docs[0]["data"]["pack.json"])
    want = {(e["id"], e["type"]) for e in ref.get("evals", [])}
    for p in ref["prompts"].values():
        want |= {(e["id"], e["type"]) for e in p.get("evals", [])}
    assert want == {(e["id"], e["type"]) for e in _all_evals(_pack())}


def test_every_sample_and_doc_type_is_registered():
    defs = _all_evals(_pack()) + [{"type": "llm_judge_turn"}, {"type": "pii_detection"},
                                  {"type": "guardrail_triggered"},
                                  {"type": "content_includes"}, {"type": "banned_words"}]
    assert E.validate_eval_defs(defs) == []
    assert E.validate_eval_defs([{"type": "sentiment_magic"}]) == ["sentiment_magic"]
    assert "llm_judge_turn" in E.JUDGE_TYPES
    assert E.groups_of({"type": "llm_judge_turn"}) == [E.GROUP_LONG, E.GROUP_EXTERNAL]
    assert E.groups_of({"type": "tools_called"}) == [E.GROUP_FAST]


def test_unknown_type_is_an_error_row_not_a_skip():
    r = E.evaluate({"id": "x", "type": "sentiment_magic"}, E.EvalContext(output="hi"))
    assert r["passed"] is False and "unknown eval type" in r["error"]
    assert not r.get("skipped")


# scripted sessions per prompt of the pack: a good one and two bad ones (tool
# calls + final output); the pack-level evals apply to every prompt
GOOD = {
    "triage": ("This is a billing request: the customer was charged twice.", []),
    "billing": ("Your order 7 is on its way and the subscription renews monthly.",
                [{"name": "lookup_order", "arguments": {"id": 7}, "error": False},
                 {"name": "lookup_subscription", "arguments": {}, "error": False}]),
    "technical": ("I searched the knowledge base and filed ticket 42 for the crash.",
                  [{"name": "search_knowledge_base", "arguments": {"q": "crash"}, "error": False},
                   {"name": "create_ticket", "arguments": {"t": "bug"}, "error": False}]),
    "closing": ("Thanks for contacting us, have a great day!", []),
}
BAD_TOOLS = [{"name": "create_ticket", "arguments": {}, "error": True},
             {"name": "search_knowledge_base", "arguments": {}, "error": True}] + \
            [{"name": "lookup_order", "arguments": {"i": i}, "error": False} for i in range(8)]
BAD_OUT = ("I don't know. Card 4111 1111 1111 1111, see https://example.com " + "x" * 3000)
SHORT_OUT = "ok"  # too short for min_length, names no triage category


def _scenarios(pack):
    """(session id, prompt evals, output, tool calls) for every prompt."""
    for pid, p in pack["prompts"].items():
        specs = list(pack["pack_evals"]) + p["evals"]
        out, tools = GOOD.get(pid, GOOD["closing"])
        yield f"{pid}:good", specs, out, tools
        yield f"{pid}:bad", specs, BAD_OUT, BAD_TOOLS
        yield f"{pid}:short", specs, SHORT_OUT, []


def _check(got, pack):
    """Every deterministic eval of every prompt ran in all three sessions,
    passed the good one and failed at least one bad one."""
    for pid, p in pack["prompts"].items():
        for e in list(pack["pack_evals"]) + p["evals"]:
            if e["type"] in E.JUDGE_TYPES:
                continue
            g = {k.split(":")[1]: v for k, v in got.get(e["id"], {}).items()
                 if k.startswith(pid + ":")}
            assert set(g) == {"good", "bad", "short"}, (pid, e["id"], g)
            assert g["good"] is True and False in (g["bad"], g["short"]), (pid, e["id"], g)


@dataclass
class _Res:
    content: str
    tool_records: list = field(default_factory=list)
    violations: list = field(default_factory=list)


class _Prompt:
    def __init__(self, evals):
        self.evals = evals


def test_inline_path_passes_and_fails_every_deterministic_eval():
    pack = _pack()
    ev = E.InlineEvaluator(sink=None, pack_evals=_all_evals(pack))
    assert ev.missing == []

    async def drive():
        for sid, specs, out, tools in _scenarios(pack):
            await ev.on_turn(sid, "help me", _Res(out, tools), _Prompt(specs))
            await ev.on_session_complete(sid)

    asyncio.run(drive())
    got = {}
    for r in ev.results:
        assert "error" not in r, r
        assert r["source"] == "runtime-inline"
        got.setdefault(r["id"], {})[r["session_id"]] = r["passed"]
    _check(got, pack)
    # judges are the worker's half: none ran inline
    assert not set(got) & {e["id"] for e in _all_evals(pack) if e["type"] in E.JUDGE_TYPES}


class _Judge:
    def __init__(self, score):
        self.score = score

    async def stream(self, msgs, tools, params, session_id=None, metadata=None):
        from omnia_amd.runtime.providers import ProviderEvent, Usage

        yield ProviderEvent("text", text=f"SCORE: {self.score}\nok")
        yield ProviderEvent("done", usage=Usage(input_tokens=1, output_tokens=1))


class _Sessions:
    """session-api stand-in: messages + tool_calls rows (pending + final)."""

    def __init__(self):
        self.msgs, self.calls, self.posted = {}, {}, []

    def add(self, sid, out, tools, t0=100.0):
        self.msgs[sid] = [{"id": "u1", "role": "user", "content": "help", "timestamp": t0},
                          {"id": "a1", "role": "assistant", "content": out,
                           "timestamp": t0 + 10}]
        rows = []
        for i, c in enumerate(tools):
            t = t0 + 1 + i * 0.1
            rows.append({"callId": f"c{i}", "name": c["name"], "arguments": c["arguments"],
                         "status": "pending", "createdAt": t})
            rows.append({"callId": f"c{i}", "name": c["name"], "arguments": c["arguments"],
                         "status": "error" if c["error"] else "success", "createdAt": t + 0.05})
        self.calls[sid] = rows

    async def get_messages(self, sid):
        return self.msgs[sid]

    async def get_session(self, sid):
        return {"agentName": "a", "namespace": "ns1"}

    async def get_tool_calls(self, sid):
        return self.calls[sid]

    async def post_eval_results(self, results):
        self.posted.extend(results)


@pytest.mark.parametrize("judge_score", [5, 1])
def test_worker_path_runs_every_eval_of_the_pack(judge_score):
    from omnia_amd.ee.eval_worker import EvalWorker

    pack = _pack()
    extra = [{"id": "turn-judge", "type": "llm_judge_turn", "trigger": "every_turn",
              "params": {"criteria": "helpful"}},
             {"id": "mystery", "type": "sentiment_magic", "trigger": "every_turn"}]
    ses = _Sessions()
    by_sid = {}
    for sid, specs, out, tools in _scenarios(pack):
        ses.add(sid, out, tools)
        by_sid[sid] = specs + extra
    current = {}
    w = EvalWorker(None, ses, ["ns1"], eval_defs=lambda a, n: by_sid[current["sid"]],
                   judge_provider=_Judge(judge_score), default_rate=100, extended_rate=100,
                   judge_rps=1e6)

    async def go():
        for sid in by_sid:
            current["sid"] = sid
            await w.handle({"type": "session.evaluate", "sessionId": sid, "agentName": "a",
                            "namespace": "ns1"})
    asyncio.run(go())
    got = {}
    for r in ses.posted:
        got.setdefault(r["evalId"], {})[r["sessionId"]] = r["passed"]
    _check(got, pack)
    for e in _all_evals(pack):  # judges: pass / fail by the judge's score
        if e["type"] in E.JUDGE_TYPES:
            thr = (e.get("params") or {}).get("passing_score", 3)
            assert set(got[e["id"]].values()) == {judge_score >= thr}, (e["id"], got[e["id"]])
    # llm_judge_turn runs as a judge; the unknown type leaves an error row
    assert set(got["turn-judge"].values()) == {judge_score >= 3}
    mystery = [r for r in ses.posted if r["evalId"] == "mystery"]
    assert mystery and all(not r["passed"] and "unknown eval type" in r["details"]["error"]
                           for r in mystery)


def test_worker_turn_window_counts_only_that_turns_tool_calls():
    from omnia_amd.ee.eval_worker import EvalWorker

    ses = _Sessions()
    ses.add("s", *GOOD["billing"], t0=100.0)
    # an earlier turn's erroring call, before this turn's user message
    ses.calls["s"].insert(0, {"callId": "old", "name": "create_ticket", "status": "error",
                              "createdAt": 50.0})
    spec = [{"id": "turn-no-errors", "type": "no_tool_errors", "trigger": "every_turn"}]
    w = EvalWorker(None, ses, ["ns1"], eval_defs=lambda a, n: spec, default_rate=100)
    asyncio.run(w.handle({"type": "message.assistant", "role": "assistant", "sessionId": "s",
                          "messageId": "a1", "agentName": "a", "namespace": "ns1"}))
    assert [r["passed"] for r in ses.posted] == [True]


def test_promptpack_status_names_unknown_eval_types():
    """The PromptPack reconciler surfaces unregistered eval types as a status
    condition (EvalTypesRegistered=False, reason UnknownEvalType)."""
    from omnia_amd.operator.apistore import get_condition
    from omnia_amd.operator.controllers import PromptPackReconciler
    from omnia_amd.operator.manager import new_store

    store = new_store()
    pack = {"id": "p", "name": "p", "version": "1.0.0",
            "template_engine": {"version": "v1", "syntax": "{{variable}}"}, "prompts": {"main": {
        "id": "main", "name": "m", "version": "1.0.0", "system_template": "hi",
        "evals": [{"id": "a", "type": "tools_called", "params": {"tool_names": ["x"]}},
                  {"id": "b", "type": "sentiment_magic"}]}}}
    store.apply({"apiVersion": "v1", "kind": "ConfigMap",
                 "metadata": {"name": "cm", "namespace": "default"},
                 "data": {"pack.json": json.dumps(pack)}})
    store.apply({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "PromptPack",
                 "metadata": {"name": "pp", "namespace": "default"},
                 "spec": {"packName": "p", "version": "1.0.0",
                          "source": {"type": "configmap", "configMapRef": {"name": "cm"}}}})
    PromptPackReconciler().reconcile(store, "default", "pp")
    pp = store.get("PromptPack", "pp")
    c = get_condition(pp, "EvalTypesRegistered")
    assert c["status"] == "False" and c["reason"] == "UnknownEvalType"
    assert "sentiment_magic" in c["message"] and "tools_called" not in c["message"]
    assert get_condition(pp, "PackContentValid")["status"] == "True"
