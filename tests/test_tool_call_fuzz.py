"""Fuzz test of the Llama-3 tool-call parser (runtime/chat.py
``parse_tool_calls``): a random-init or badly behaved model emits arbitrary
text, so the parser must never raise, every call it returns names a declared
tool with a JSON-serialisable object of arguments, and text without a call
comes back unchanged.  The reference parses provider tool calls in its
runtime (``internal/runtime``); this pins the contract over random inputs.

It found two crashes that ended the agent turn: a ``"name"`` that was not a
string (``unhashable type``) and deeply nested output (``RecursionError``)."""
import json

from hypothesis import given, settings
from hypothesis import strategies as st

from omnia_amd.runtime.chat import parse_tool_calls

TOOLS = {"get_weather", "search", "calc"}

JSON = st.recursive(st.none() | st.booleans() | st.integers() | st.text(max_size=6)
                    | st.floats(allow_nan=False, allow_infinity=False),
                    lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=6), c,
                                                                         max_size=3),
                    max_leaves=10)
NAME = st.one_of(st.sampled_from(sorted(TOOLS)), st.text(max_size=6), JSON)
CALL = st.fixed_dictionaries(
    {"name": NAME},
    optional={"parameters": st.one_of(JSON, JSON.map(json.dumps), st.text(max_size=8)),
              "arguments": st.one_of(JSON, JSON.map(json.dumps))}).map(json.dumps)
PIECE = st.one_of(CALL, st.text(max_size=12), st.sampled_from(
    ["{", "}", ";", "\n", "<|python_tag|>", "[" * 3000, "{\"a\":" * 3000, "{\"name\": ",
     "{\"name\": \"calc\", \"parameters\": " + "[" * 3000]))


def _check(text, names):
    rest, calls = parse_tool_calls(text, names)
    assert isinstance(rest, str)
    for c in calls:
        assert c.name in names
        assert isinstance(c.arguments, dict)
        json.dumps(c.arguments)
    if not calls:
        assert rest == text
    return calls


@given(st.lists(PIECE, max_size=5).map("".join), st.sampled_from([set(), TOOLS, {"calc"}]))
@settings(max_examples=400, deadline=None)
def test_parse_tool_calls_never_raises(text, names):
    _check(text, names)


@given(st.lists(st.tuples(st.sampled_from(sorted(TOOLS)),
                          st.dictionaries(st.text(max_size=5), JSON, max_size=3)),
                min_size=1, max_size=3),
       st.sampled_from(["", ";", "\n", "; "]), st.booleans())
@settings(max_examples=200, deadline=None)
def test_well_formed_calls_round_trip(calls, sep, tag):
    text = ("<|python_tag|>" if tag else "") + sep.join(
        json.dumps({"name": n, "parameters": a}) for n, a in calls)
    got = _check(text, TOOLS)
    assert [(c.name, c.arguments) for c in got] == calls
