"""Compact JSON-Schema (draft 2020-12 subset) validator.

The reference validates PromptPacks (``internal/schema/validator.go``) and
function-mode input/output bodies (``internal/schemautil``) with a full
draft-2020-12 implementation; ``jsonschema`` is not installed here, so this
implements the keywords those schemas use: type, enum, const, properties,
required, additionalProperties, patternProperties, items/prefixItems,
min/maxItems, uniqueItems, min/maxLength, pattern, minimum/maximum (+exclusive),
multipleOf, allOf/anyOf/oneOf/not, if/then/else, $ref (local JSON pointers,
$defs/definitions), dependentRequired, min/maxProperties, format (date-time,
email, uri: lenient).
"""
from __future__ import annotations

import re
from dataclasses import dataclass


@dataclass
class SchemaError:
    path: str
    message: str

    def __str__(self) -> str:
        return f"{self.path or '$'}: {self.message}"


class ValidationError(ValueError):
    def __init__(self, errors: list[SchemaError]):
        self.errors = errors
        super().__init__("; ".join(str(e) for e in errors[:5]))


_TYPES = {
    "object": lambda v: isinstance(v, dict),
    "array": lambda v: isinstance(v, list),
    "string": lambda v: isinstance(v, str),
    "boolean": lambda v: isinstance(v, bool),
    "null": lambda v: v is None,
    "integer": lambda v: (isinstance(v, int) and not isinstance(v, bool))
    or (isinstance(v, float) and v.is_integer()),
    "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
}


class Validator:
    def __init__(self, schema: dict | bool):
        self.root = schema
        self._re: dict[str, re.Pattern] = {}

    def _resolve(self, ref: str):
        if not ref.startswith("#"):
            raise ValueError(f"only local $ref supported: {ref}")
        node = self.root
        for part in ref[1:].split("/"):
            if not part:
                continue
            part = part.replace("~1", "/").replace("~0", "~")
            node = node[int(part)] if isinstance(node, list) else node[part]
        return node

    def _pattern(self, p: str) -> re.Pattern:
        r = self._re.get(p)
        if r is None:
            r = self._re[p] = re.compile(p)
        return r

    def errors(self, inst, schema=None, path: str = "") -> list[SchemaError]:
        schema = self.root if schema is None else schema
        if schema is True or schema == {}:
            return []
        if schema is False:
            return [SchemaError(path, "not allowed")]
        errs: list[SchemaError] = []
        add = errs.append
        if "$ref" in schema:
            errs += self.errors(inst, self._resolve(schema["$ref"]), path)
        t = schema.get("type")
        if t is not None:
            types = t if isinstance(t, list) else [t]
            if not any(_TYPES[x](inst) for x in types if x in _TYPES):
                add(SchemaError(path, f"expected {t}, got {type(inst).__name__}"))
                return errs
        if "enum" in schema and inst not in schema["enum"]:
            add(SchemaError(path, f"{inst!r} not in enum {schema['enum']}"))
        if "const" in schema and inst != schema["const"]:
            add(SchemaError(path, f"{inst!r} != const {schema['const']!r}"))
        if isinstance(inst, dict):
            props = schema.get("properties", {})
            for r in schema.get("required", []):
                if r not in inst:
                    add(SchemaError(path, f"missing required property {r!r}"))
            pp = schema.get("patternProperties", {})
            for k, v in inst.items():
                sub = f"{path}.{k}" if path else k
                matched = False
                if k in props:
                    matched = True
                    errs += self.errors(v, props[k], sub)
                for pat, ps in pp.items():
                    if self._pattern(pat).search(k):
                        matched = True
                        errs += self.errors(v, ps, sub)
                if not matched and "additionalProperties" in schema:
                    ap = schema["additionalProperties"]
                    if ap is False:
                        add(SchemaError(sub, "additional property not allowed"))
                    elif isinstance(ap, dict):
                        errs += self.errors(v, ap, sub)
            if "minProperties" in schema and len(inst) < schema["minProperties"]:
                add(SchemaError(path, "too few properties"))
            if "maxProperties" in schema and len(inst) > schema["maxProperties"]:
                add(SchemaError(path, "too many properties"))
            for k, deps in schema.get("dependentRequired", {}).items():
                if k in inst:
                    for d in deps:
                        if d not in inst:
                            add(SchemaError(path, f"{k!r} requires {d!r}"))
        if isinstance(inst, list):
            pre = schema.get("prefixItems", [])
            for i, v in enumerate(inst):
                if i < len(pre):
                    errs += self.errors(v, pre[i], f"{path}[{i}]")
                elif "items" in schema and isinstance(schema["items"], (dict, bool)):
                    errs += self.errors(v, schema["items"], f"{path}[{i}]")
            if "minItems" in schema and len(inst) < schema["minItems"]:
                add(SchemaError(path, f"fewer than {schema['minItems']} items"))
            if "maxItems" in schema and len(inst) > schema["maxItems"]:
                add(SchemaError(path, f"more than {schema['maxItems']} items"))
            if schema.get("uniqueItems"):
                seen = []
                for v in inst:
                    if v in seen:
                        add(SchemaError(path, "items not unique"))
                        break
                    seen.append(v)
        if isinstance(inst, str):
            if "minLength" in schema and len(inst) < schema["minLength"]:
                add(SchemaError(path, f"shorter than {schema['minLength']}"))
            if "maxLength" in schema and len(inst) > schema["maxLength"]:
                add(SchemaError(path, f"longer than {schema['maxLength']}"))
            if "pattern" in schema and not self._pattern(schema["pattern"]).search(inst):
                add(SchemaError(path, f"does not match {schema['pattern']!r}"))
            fmt = schema.get("format")
            if fmt == "email" and "@" not in inst:
                add(SchemaError(path, "not an email"))
        if _TYPES["number"](inst):
            if "minimum" in schema and inst < schema["minimum"]:
                add(SchemaError(path, f"< minimum {schema['minimum']}"))
            if "maximum" in schema and inst > schema["maximum"]:
                add(SchemaError(path, f"> maximum {schema['maximum']}"))
            if "exclusiveMinimum" in schema and inst <= schema["exclusiveMinimum"]:
                add(SchemaError(path, f"<= exclusiveMinimum {schema['exclusiveMinimum']}"))
            if "exclusiveMaximum" in schema and inst >= schema["exclusiveMaximum"]:
                add(SchemaError(path, f">= exclusiveMaximum {schema['exclusiveMaximum']}"))
            mo = schema.get("multipleOf")
            if mo and abs(inst / mo - round(inst / mo)) > 1e-9:
                add(SchemaError(path, f"not a multiple of {mo}"))
        for sub in schema.get("allOf", []):
            errs += self.errors(inst, sub, path)
        if "anyOf" in schema and not any(not self.errors(inst, s, path) for s in schema["anyOf"]):
            add(SchemaError(path, "matches none of anyOf"))
        if "oneOf" in schema:
            n = sum(1 for s in schema["oneOf"] if not self.errors(inst, s, path))
            if n != 1:
                add(SchemaError(path, f"matches {n} of oneOf (need exactly 1)"))
        if "not" in schema and not self.errors(inst, schema["not"], path):
            add(SchemaError(path, "must not match 'not' schema"))
        if "if" in schema:
            if not self.errors(inst, schema["if"], path):
                if "then" in schema:
                    errs += self.errors(inst, schema["then"], path)
            elif "else" in schema:
                errs += self.errors(inst, schema["else"], path)
        return errs

    def validate(self, inst) -> None:
        e = self.errors(inst)
        if e:
            raise ValidationError(e)

    def is_valid(self, inst) -> bool:
        return not self.errors(inst)


def validate(inst, schema) -> None:
    Validator(schema).validate(inst)


def check_schema(schema) -> None:
    """Light meta-check: the schema must be an object/bool and refs resolvable."""
    if not isinstance(schema, (dict, bool)):
        raise ValueError("schema must be an object or boolean")
    v = Validator(schema)

    def walk(node):
        if isinstance(node, dict):
            if "$ref" in node:
                v._resolve(node["$ref"])
            if "type" in node:
                ts = node["type"] if isinstance(node["type"], list) else [node["type"]]
                for t in ts:
                    if t not in _TYPES:
                        raise ValueError(f"unknown type {t!r}")
            if "pattern" in node:
                re.compile(node["pattern"])
            for val in node.values():
                walk(val)
        elif isinstance(node, list):
            for val in node:
                walk(val)

    walk(schema)
