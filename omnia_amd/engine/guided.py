"""Guided (constrained) decoding -- K13.

``SamplingParams.json_schema`` (JSON-schema-constrained) or
``SamplingParams.json_object`` (any JSON object) turn on a per-sequence
:class:`JsonMatcher` (C++, ``omnia_amd/native/csrc/json_grammar.cpp``): before
each sampling step the engine asks every constrained sequence for its allowed
next-token bitmask ([ceil(V/32)] uint32), uploads the masks once and the GPU
kernel ``omnia_apply_token_mask`` sets disallowed logits to -inf ahead of the
fused sampler; the sampled token is then fed back into the matcher.

This module compiles a JSON schema into the automaton's node table.  Supported:
``type`` (object / array / string / number / integer / boolean / null, or a list
of them), ``properties`` + ``required`` (keys emitted in declaration order),
``additionalProperties`` (as the value schema of free-form objects),
``items`` / ``minItems`` / ``maxItems``, ``minLength`` / ``maxLength``,
``enum`` / ``const``, ``anyOf`` / ``oneOf`` (dispatched on the first byte), local
``$ref`` into ``$defs`` / ``definitions``.  Unknown keywords are ignored (the
output stays valid JSON of the declared shape).

Reference parity: function-mode ``json_schema`` response format
(``internal/runtime/response_format.go``) -- the reference can only instruct a
remote provider; the in-node engine enforces it token by token.
"""
from __future__ import annotations

import json

import numpy as np

ANY, OBJECT, ARRAY, STRING, NUMBER, INTEGER, LITERALS, UNION = range(8)
_ANY_LITS = ["true", "false", "null"]


class SchemaError(ValueError):
    pass


def _lit(v) -> str:
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False)


def compile_schema(schema: dict | None) -> tuple[list[dict], int]:
    """schema (None = any JSON object) -> (node table, root index).  Node 0 is ANY."""
    nodes: list[dict] = [{"kind": ANY, "literals": list(_ANY_LITS)}]
    root_schema = schema if isinstance(schema, dict) else None
    defs = {}
    if root_schema:
        defs = dict(root_schema.get("$defs") or {})
        defs.update(root_schema.get("definitions") or {})
    memo: dict[str, int] = {}

    def add(n: dict) -> int:
        nodes.append(n)
        return len(nodes) - 1

    def build(s, depth=0) -> int:
        if depth > 24:
            raise SchemaError("schema nesting too deep")
        if s is True or s is None or s == {}:
            return 0
        if s is False:
            raise SchemaError("false schema cannot be generated")
        if not isinstance(s, dict):
            raise SchemaError(f"bad schema node {s!r}")
        ref = s.get("$ref")
        if ref:
            if ref in memo:
                return memo[ref]
            name = ref.rsplit("/", 1)[-1]
            if not ref.startswith("#/") or name not in defs:
                raise SchemaError(f"unresolvable $ref {ref!r}")
            idx = add({"kind": ANY})  # placeholder (supports recursion)
            memo[ref] = idx
            nodes[idx] = nodes[build(defs[name], depth + 1)].copy()
            return idx
        if "x-omnia-tool-union" in s:
            # Llama-3 tool call {"name": <tool>, "parameters": <that tool's schema>}:
            # a tagged object, the matched name selects the parameters grammar
            tools = s["x-omnia-tool-union"]
            if not tools:
                raise SchemaError("tool union needs at least one tool")
            name_node = add({"kind": LITERALS, "literals": [_lit(t["name"]) for t in tools]})
            params = [build(t.get("parameters") or {"type": "object"}, depth + 1)
                      for t in tools]
            return add({"kind": OBJECT, "props": [(_lit("name"), name_node, True),
                                                  (_lit("parameters"), params[0], True)],
                        "tag_children": params})
        if "const" in s:
            return add({"kind": LITERALS, "literals": [_lit(s["const"])]})
        if "enum" in s:
            lits = [_lit(v) for v in s["enum"]]
            if not lits:
                raise SchemaError("empty enum")
            return add({"kind": LITERALS, "literals": lits})
        alts = s.get("anyOf") or s.get("oneOf")
        if alts:
            return add({"kind": UNION, "children": [build(a, depth + 1) for a in alts]})
        t = s.get("type")
        if isinstance(t, list):
            return add({"kind": UNION, "children": [build({**s, "type": x}, depth + 1)
                                                     for x in t]})
        if t is None:
            if "properties" in s:
                t = "object"
            elif "items" in s:
                t = "array"
            else:
                return 0
        if t == "object":
            props = s.get("properties") or {}
            req = set(s.get("required") or [])
            if props:
                plist = [(_lit(k), build(v, depth + 1), k in req) for k, v in props.items()]
                return add({"kind": OBJECT, "props": plist})
            ap = s.get("additionalProperties", True)
            return add({"kind": OBJECT, "props": [],
                        "items": build(ap if isinstance(ap, dict) else True, depth + 1)})
        if t == "array":
            n = {"kind": ARRAY, "items": build(s.get("items", True), depth + 1),
                 "min_items": int(s.get("minItems", 0))}
            if "maxItems" in s:
                n["max_items"] = int(s["maxItems"])
            return add(n)
        if t == "string":
            n = {"kind": STRING, "min_len": int(s.get("minLength", 0))}
            if "maxLength" in s:
                n["max_len"] = int(s["maxLength"])
            return add(n)
        if t == "number":
            return add({"kind": NUMBER})
        if t == "integer":
            return add({"kind": INTEGER})
        if t == "boolean":
            return add({"kind": LITERALS, "literals": ["true", "false"]})
        if t == "null":
            return add({"kind": LITERALS, "literals": ["null"]})
        raise SchemaError(f"unsupported type {t!r}")

    if root_schema is None:
        root = add({"kind": OBJECT, "props": [], "items": 0})  # json_object mode
    else:
        root = build(root_schema)
    return nodes, root


def _bytes_unicode_inverse() -> dict[str, int]:
    """GPT-2 / tiktoken byte-level alphabet: printable char -> raw byte."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


def token_byte_table(tok) -> list[bytes]:
    """Raw bytes of every vocabulary id (b"" for specials)."""
    n = tok.vocab_size
    if hasattr(tok, "tk"):  # HF tokenizers: byte-level BPE or sentencepiece pieces
        inv = _bytes_unicode_inverse()
        special = set(getattr(tok, "special", {}).values())
        out = []
        for i in range(n):
            piece = tok.tk.id_to_token(i)
            if piece is None or i in special:
                out.append(b"")
            elif all(ch in inv for ch in piece):
                out.append(bytes(inv[ch] for ch in piece))
            elif piece.startswith("<0x") and piece.endswith(">") and len(piece) == 6:
                out.append(bytes([int(piece[3:5], 16)]))
            else:
                out.append(piece.replace("▁", " ").encode("utf-8"))
        return out
    return [tok.token_bytes(i) for i in range(n)]


class GuidedRegistry:
    """Per-tokenizer vocabulary trie + compiled grammars (mask caches live in them)."""

    def __init__(self, tokenizer):
        from ..native import native

        self.nat = native()
        self.tok = tokenizer
        self.table = token_byte_table(tokenizer)
        self.vocab = self.nat.GrammarVocab(self.table, list(tokenizer.eos_token_ids))
        self.words = self.vocab.words
        self.grammars: dict[str, object] = {}

    def grammar(self, schema: dict | None):
        key = json.dumps(schema, sort_keys=True) if schema is not None else "<json_object>"
        g = self.grammars.get(key)
        if g is None:
            table, root = compile_schema(schema)
            g = self.nat.JsonGrammar(self.vocab, table, root)
            self.grammars[key] = g
        return g

    def matcher(self, params) -> "Guide":
        if getattr(params, "tool_grammar", None) is not None:
            g = Guide(self, self.nat.JsonMatcher(self.grammar(
                {"x-omnia-tool-union": params.tool_grammar})))
            return g if params.tool_choice == "required" else TriggeredGuide(g)
        schema = params.json_schema if params.json_schema is not None else None
        return Guide(self, self.nat.JsonMatcher(self.grammar(schema)))


class Guide:
    """One sequence's matcher + its token-bytes view."""

    __slots__ = ("reg", "m")

    def __init__(self, reg: GuidedRegistry, m):
        self.reg = reg
        self.m = m

    def fill(self, row: np.ndarray) -> None:
        self.m.fill_mask(row)

    def accept(self, tid: int) -> bool:
        return self.m.accept_token(int(tid), self.reg.table[tid] if tid < len(self.reg.table)
                                   else b"")

    @property
    def complete(self) -> bool:
        return self.m.is_complete()


class TriggeredGuide:
    """tool_choice "auto" on the local engine: the model is free until it opens
    a JSON object (its first non-space bytes are ``{``); from then on the
    tool-call grammar holds, so a call it starts is always a valid call of a
    declared tool with schema-valid arguments.  Text answers stay unconstrained."""

    __slots__ = ("g", "active", "off", "seen")

    def __init__(self, g: Guide):
        self.g = g
        self.active = False
        self.off = False
        self.seen = b""

    @property
    def m(self):
        return self.g.m if self.active else _Unfinished

    def fill(self, row: np.ndarray) -> None:
        if self.active:
            self.g.fill(row)
        else:
            row[:] = np.uint32(0xFFFFFFFF)

    def accept(self, tid: int) -> bool:
        if self.active:
            return self.g.accept(tid)
        if self.off:
            return True
        b = self.g.reg.table[tid] if tid < len(self.g.reg.table) else b""
        lead = (self.seen + b).lstrip()
        if not lead:
            self.seen += b
            return True
        if lead[:1] == b"{":
            self.active = True
            return self.g.m.accept_bytes(lead)
        self.off = True  # a text answer: never constrain this turn
        return True

    @property
    def complete(self) -> bool:
        return self.g.complete if self.active else False


class _Unfinished:
    finished = False


def masks_for(guides: list, words: int) -> np.ndarray:
    """[len(guides), words] int32 mask rows (all-allowed for ``None`` guides)."""
    out = np.full((len(guides), words), -1, dtype=np.int32)
    for i, g in enumerate(guides):
        if g is not None:
            g.fill(out[i].view(np.uint32))
    return out
