"""K13 guided decoding: schema compiler, C++ grammar automaton, token masks and
engine integration (CPU; the GPU mask kernel is in test_kernels_gpu.py)."""
import json
import random

import numpy as np
import pytest
import torch

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.guided import (GuidedRegistry, SchemaError, _bytes_unicode_inverse,
                                     compile_schema, masks_for)
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.engine.tokenizer import SyntheticTokenizer
from omnia_amd.ops import reference as ref
from omnia_amd.utils import jsonschema as js

TOK = SyntheticTokenizer(1024, 1000, (1001, 1004))

SCHEMAS = [
    {"type": "object", "properties": {
        "name": {"type": "string", "maxLength": 10}, "age": {"type": "integer"},
        "tags": {"type": "array", "items": {"enum": ["a", "bb", "c"]}, "maxItems": 3},
        "ok": {"type": "boolean"}, "score": {"type": ["number", "null"]},
        "meta": {"type": "object"}}, "required": ["name", "age", "ok"]},
    {"type": "array", "items": {"type": "integer"}, "minItems": 1, "maxItems": 4},
    {"$defs": {"pt": {"type": "object", "properties": {"x": {"type": "number"},
                                                        "y": {"type": "number"}},
                      "required": ["x", "y"]}},
     "type": "object", "properties": {"pts": {"type": "array", "items": {"$ref": "#/$defs/pt"}},
                                      "label": {"const": "poly"}},
     "required": ["pts", "label"]},
    {"anyOf": [{"type": "string", "minLength": 2}, {"type": "integer"}]},
]


@pytest.fixture(scope="module")
def reg():
    return GuidedRegistry(TOK)


def _walk(reg, schema, rng, json_object=False, max_steps=4000):
    class P:
        pass

    P.json_schema = schema
    P.json_object = json_object
    g = reg.matcher(P)
    out = []
    for _ in range(max_steps):
        m = masks_for([g], reg.words)[0].view(np.uint32)
        allowed = [i for i in range(TOK.vocab_size) if (m[i >> 5] >> (i & 31)) & 1]
        assert allowed, "grammar dead end"
        if any(e in allowed for e in TOK.eos_ids) and (rng.random() < 0.7 or len(allowed) <= 2):
            assert g.accept(1004)
            break
        cand = [a for a in allowed if a not in TOK.eos_ids]
        struct = [a for a in cand if a < 256 and chr(a) in '"}],0123456789tfn']
        c = rng.choice(struct) if struct and rng.random() < 0.4 else rng.choice(cand)
        assert g.accept(c)
        out.append(c)
    else:
        pytest.fail("document never completed")
    return TOK.decode(out)


@pytest.mark.parametrize("si", range(len(SCHEMAS)))
def test_random_walks_stay_valid(reg, si):
    rng = random.Random(si)
    for _ in range(12):
        text = _walk(reg, SCHEMAS[si], rng)
        js.validate(json.loads(text), SCHEMAS[si])  # syntactically valid and schema-valid


def test_json_object_mode(reg):
    rng = random.Random(7)
    for _ in range(10):
        obj = json.loads(_walk(reg, None, rng, json_object=True))
        assert isinstance(obj, dict)


def test_matcher_rejects_and_eos_rules(reg):
    class P:
        json_schema = {"type": "object", "properties": {"a": {"type": "integer"}},
                       "required": ["a"]}
        json_object = False

    g = reg.matcher(P)
    assert not g.accept(ord("["))  # wrong container
    for ch in b'{"a":1':
        assert g.accept(ch)
    assert not g.complete  # '}' still missing
    assert not g.accept(ord(","))  # no more properties
    assert g.accept(ord("2")) and g.accept(ord("}"))
    assert g.complete
    m = masks_for([g], reg.words)[0].view(np.uint32)
    allowed = [i for i in range(TOK.vocab_size) if (m[i >> 5] >> (i & 31)) & 1]
    assert sorted(allowed) == sorted(TOK.eos_ids)  # only EOS after the document


def test_mask_cache_hits(reg):
    g = reg.grammar({"type": "string"})
    h0 = g.cache_hits
    rng = random.Random(3)
    for _ in range(3):
        _walk(reg, {"type": "string"}, rng)
    assert g.cache_hits > h0


def test_schema_errors():
    with pytest.raises(SchemaError):
        compile_schema({"type": "object", "properties": {"a": {"$ref": "#/$defs/missing"}}})
    with pytest.raises(SchemaError):
        compile_schema({"type": "tuple"})
    nodes, root = compile_schema(None)
    assert nodes[0]["kind"] == 0 and nodes[root]["kind"] == 1


def test_mask_reference_unpacks_bits():
    V = 70
    logits = torch.zeros(2, V)
    mask = torch.zeros(2, 3, dtype=torch.int32)
    mask[0, 0] = 0b101
    mask[1, 2] = 1 << 5  # token 69
    ref.apply_token_mask(logits, mask)
    assert torch.isfinite(logits[0]).nonzero().flatten().tolist() == [0, 2]
    assert torch.isfinite(logits[1]).nonzero().flatten().tolist() == [69]


def test_byte_level_alphabet_roundtrip():
    inv = _bytes_unicode_inverse()
    assert len(inv) == 256 and sorted(inv.values()) == list(range(256))
    assert inv["Ġ"] == 32  # GPT-2 space


def test_engine_generates_schema_valid_json():
    e = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=256, block_size=32,
                               max_batch=8, max_model_len=1024))
    schema = {"type": "object", "properties": {"city": {"type": "string", "maxLength": 8},
                                               "unit": {"enum": ["C", "F"]}},
              "required": ["city", "unit"]}
    guided = [e.add_request(list(range(10, 40 + i)), SamplingParams(
        temperature=t, seed=i, max_tokens=300, json_schema=schema))
        for i, t in enumerate([0.0, 0.8, 1.2])]
    obj_mode = e.add_request(list(range(10, 50)), SamplingParams(
        temperature=1.0, seed=9, max_tokens=300, json_object=True))
    free = e.add_request(list(range(10, 30)), SamplingParams(temperature=0, max_tokens=8,
                                                             ignore_eos=True))
    e.run_until_done()
    for s in guided:
        assert s.finish_reason.value == "stop"
        js.validate(json.loads(e.tokenizer.decode(s.output)), schema)
    if obj_mode.finish_reason.value == "stop":  # a random model may run out of tokens
        assert isinstance(json.loads(e.tokenizer.decode(obj_mode.output)), dict)
    else:
        assert obj_mode.finish_reason.value == "length"
        assert e.tokenizer.decode(obj_mode.output).startswith("{")
    assert len(free.output) == 8  # unconstrained neighbours are unaffected


def test_response_format_mapping():
    p = SamplingParams.from_dict({"response_format": {
        "type": "json_schema", "json_schema": {"name": "x", "schema": {"type": "integer"}}}})
    assert p.json_schema == {"type": "integer"} and p.guided
    assert SamplingParams.from_dict({"response_format": {"type": "json_object"}}).json_object


TOOLS = [
    {"name": "get_weather", "parameters": {"type": "object", "properties": {
        "city": {"type": "string", "maxLength": 12}, "unit": {"enum": ["C", "F"]}},
        "required": ["city"]}},
    {"name": "get_time", "parameters": {"type": "object", "properties": {
        "tz": {"type": "integer"}}, "required": ["tz"]}},
    {"name": "ping", "parameters": {"type": "object"}},
]


def _tool_schema_of(name):
    return next(t["parameters"] for t in TOOLS if t["name"] == name)


def test_tool_union_random_walks_are_valid_calls(reg):
    """The tagged tool-call grammar: every completed document is a call of a
    declared tool whose parameters validate against THAT tool's schema."""
    rng = random.Random(5)
    seen = set()
    for _ in range(30):
        text = _walk(reg, {"x-omnia-tool-union": TOOLS}, rng)
        call = json.loads(text)
        assert set(call) == {"name", "parameters"}
        js.validate(call["parameters"], _tool_schema_of(call["name"]))
        seen.add(call["name"])
    assert len(seen) >= 2


def test_tool_union_rejects_wrong_parameters(reg):
    class P:
        json_schema = {"x-omnia-tool-union": TOOLS}
        json_object = False

    ok = b'{"name":"get_time","parameters":{"tz":3}}'
    bad = b'{"name":"get_time","parameters":{"city":"x"}}'
    assert reg.matcher(P).m.accept_bytes(ok)
    assert not reg.matcher(P).m.accept_bytes(bad)
    assert not reg.matcher(P).m.accept_bytes(b'{"name":"nope"')


def test_engine_forced_tool_call_and_auto_trigger():
    """tool_choice=required on the local engine always yields a parseable call of
    an offered tool; "auto" leaves text answers free."""
    from omnia_amd.runtime.chat import parse_tool_calls

    e = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=256, block_size=32,
                               max_batch=8, max_model_len=1024))
    req = [e.add_request(list(range(10, 40 + i)), SamplingParams(
        temperature=t, seed=i, max_tokens=400, tool_grammar=TOOLS, tool_choice="required"))
        for i, t in enumerate([0.0, 0.9, 1.3])]
    auto = e.add_request(list(range(10, 30)), SamplingParams(
        temperature=0.0, max_tokens=6, ignore_eos=True, tool_grammar=TOOLS, tool_choice="auto"))
    e.run_until_done()
    names = {t["name"] for t in TOOLS}
    for s in req:
        text = e.tokenizer.decode(s.output)
        rest, calls = parse_tool_calls(text, names)
        assert s.finish_reason.value == "stop" and len(calls) == 1, text
        js.validate(calls[0].arguments, _tool_schema_of(calls[0].name))
    assert len(auto.output) == 6
