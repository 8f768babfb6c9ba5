"""Structural (OpenAPI v3) CRD schemas: a small authoring DSL and the
admission-time validator the API store runs on every create/update.

The validator implements what the kube-apiserver does for a structural CRD
schema, in order, at every node:

1. **defaulting** -- ``default`` of an absent property is filled in before
   anything is validated (``apiextensions`` defaulting happens on read/write);
2. **strict field validation** -- a property the schema does not declare is an
   error (``kubectl``'s default ``--validate=strict`` /
   ``fieldValidation=Strict``) unless the node carries
   ``x-kubernetes-preserve-unknown-fields`` or is a map
   (``additionalProperties``);
3. **OpenAPI value checks** -- type, enum, pattern, min/maxLength,
   minimum/maximum, min/maxItems, required, ``x-kubernetes-int-or-string``;
4. **CEL rules** -- every ``x-kubernetes-validations`` ``{rule, message}`` is
   evaluated with ``self`` bound to the node (and ``oldSelf`` on updates --
   transition rules are skipped on create, as in Kubernetes) by the in-repo CEL
   interpreter (``omnia_amd/utils/cel.py``).  A rule that evaluates to false or
   errors reports its message.

Errors are ``"spec.a.b[2].c: message"`` strings, the apiserver's field-path
style.
"""
from __future__ import annotations

import copy
import re

from ..utils import cel

PRESERVE = "x-kubernetes-preserve-unknown-fields"
RULES = "x-kubernetes-validations"
INT_OR_STRING = "x-kubernetes-int-or-string"


# ------------------------------------------------------------------ DSL
def Str(default=None, pattern=None, min_len=None, max_len=None, fmt=None) -> dict:
    s = {"type": "string"}
    if default is not None:
        s["default"] = default
    if pattern is not None:
        s["pattern"] = pattern
    if min_len is not None:
        s["minLength"] = min_len
    if max_len is not None:
        s["maxLength"] = max_len
    if fmt is not None:
        s["format"] = fmt
    return s


def Int(default=None, minimum=None, maximum=None, fmt="int32") -> dict:
    s = {"type": "integer", "format": fmt}
    if default is not None:
        s["default"] = default
    if minimum is not None:
        s["minimum"] = minimum
    if maximum is not None:
        s["maximum"] = maximum
    return s


def Num(default=None, minimum=None, maximum=None) -> dict:
    s = {"type": "number"}
    if default is not None:
        s["default"] = default
    if minimum is not None:
        s["minimum"] = minimum
    if maximum is not None:
        s["maximum"] = maximum
    return s


def Bool(default=None) -> dict:
    s = {"type": "boolean"}
    if default is not None:
        s["default"] = default
    return s


def Enum(*vals, default=None) -> dict:
    s = {"type": "string", "enum": list(vals)}
    if default is not None:
        s["default"] = default
    return s


def Arr(items: dict, min_items=None, max_items=None, default=None) -> dict:
    s = {"type": "array", "items": items}
    if min_items is not None:
        s["minItems"] = min_items
    if max_items is not None:
        s["maxItems"] = max_items
    if default is not None:
        s["default"] = default
    return s


def Map(values: dict | None = None) -> dict:
    return {"type": "object", "additionalProperties": values or {"type": "string"}}


def Obj(props: dict, required=(), rules=(), preserve: bool = False, default=None) -> dict:
    s = {"type": "object", "properties": props}
    if required:
        s["required"] = list(required)
    if rules:
        s[RULES] = [{"rule": r, "message": m} for r, m in rules]
    if preserve:
        s[PRESERVE] = True
    if default is not None:
        s["default"] = default
    return s


def Rules(schema: dict, *rules) -> dict:
    """Attach CEL rules to an existing schema node (returns a copy)."""
    s = copy.deepcopy(schema)
    s.setdefault(RULES, []).extend({"rule": r, "message": m} for r, m in rules)
    return s


def With(schema: dict, **props) -> dict:
    """Copy of an object schema with extra properties."""
    s = copy.deepcopy(schema)
    s["properties"].update(props)
    return s


JSON_ANY = {PRESERVE: True}                      # apiextensionsv1.JSON / RawExtension
OPEN_OBJ = {"type": "object", PRESERVE: True}    # embedded core types kept opaque
INT_OR_STR = {INT_OR_STRING: True}
DURATION = Str()                                  # metav1.Duration ("30s", "1h5m")
TIME = Str(fmt="date-time")                       # metav1.Time


# ------------------------------------------------------------------ validator
_TYPES = {"string": (str,), "boolean": (bool,), "object": (dict,), "array": (list,)}


def _type_ok(t: str, v) -> bool:
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool)
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return isinstance(v, _TYPES.get(t, (object,)))


_RE_CACHE: dict = {}


def _re(p: str):
    r = _RE_CACHE.get(p)
    if r is None:
        r = _RE_CACHE[p] = re.compile(p)
    return r


_CEL_CACHE: dict = {}


def _prog(rule: str):
    p = _CEL_CACHE.get(rule)
    if p is None:
        p = _CEL_CACHE[rule] = cel.compile(rule)
    return p


def apply_defaults(schema: dict, v):
    """Fill absent defaulted properties (recursively, through arrays and maps)."""
    if not isinstance(schema, dict):
        return v
    if isinstance(v, dict) and schema.get("type") == "object":
        for k, sub in (schema.get("properties") or {}).items():
            if k not in v and "default" in sub:
                v[k] = copy.deepcopy(sub["default"])
            if k in v:
                apply_defaults(sub, v[k])
        ap = schema.get("additionalProperties")
        if isinstance(ap, dict):
            for k in v:
                if k not in (schema.get("properties") or {}):
                    apply_defaults(ap, v[k])
    elif isinstance(v, list) and isinstance(schema.get("items"), dict):
        for it in v:
            apply_defaults(schema["items"], it)
    return v


def validate(schema: dict, v, path: str = "spec", old=None, errs: list | None = None,
             field_validation: str = "Strict", warnings: list | None = None) -> list:
    """Structural validation of ``v`` (defaults must already be applied).

    ``field_validation`` is the apiserver's ``fieldValidation`` mode for fields
    the schema does not declare: ``Strict`` rejects them (what ``kubectl``
    sends), ``Warn`` prunes them and records a warning (the server default for
    other clients), ``Ignore`` prunes silently."""
    errs = [] if errs is None else errs
    fv = field_validation
    if not isinstance(schema, dict) or not schema:
        return errs
    if schema.get(INT_OR_STRING):
        if not (isinstance(v, str) or (isinstance(v, int) and not isinstance(v, bool))):
            errs.append(f"{path}: must be an integer or a string")
        return errs
    t = schema.get("type")
    if t is None:
        return errs  # untyped preserve-unknown node (JSON)
    if v is None:
        errs.append(f"{path}: must not be null")
        return errs
    if not _type_ok(t, v):
        errs.append(f"{path}: must be of type {t}")
        return errs
    if "enum" in schema and v not in schema["enum"]:
        errs.append(f"{path}: Unsupported value: {v!r}: supported values: "
                    + ", ".join(repr(e) for e in schema["enum"]))
    if t == "string":
        if "pattern" in schema and not _re(schema["pattern"]).search(v):
            errs.append(f"{path}: should match '{schema['pattern']}'")
        if "minLength" in schema and len(v) < schema["minLength"]:
            errs.append(f"{path}: should be at least {schema['minLength']} chars long")
        if "maxLength" in schema and len(v) > schema["maxLength"]:
            errs.append(f"{path}: may not be more than {schema['maxLength']} bytes")
    elif t in ("integer", "number"):
        if "minimum" in schema and v < schema["minimum"]:
            errs.append(f"{path}: should be greater than or equal to {schema['minimum']}")
        if "maximum" in schema and v > schema["maximum"]:
            errs.append(f"{path}: should be less than or equal to {schema['maximum']}")
    elif t == "array":
        if "minItems" in schema and len(v) < schema["minItems"]:
            errs.append(f"{path}: should have at least {schema['minItems']} items")
        if "maxItems" in schema and len(v) > schema["maxItems"]:
            errs.append(f"{path}: must have at most {schema['maxItems']} items")
        items = schema.get("items")
        if isinstance(items, dict):
            olds = old if isinstance(old, list) and len(old) == len(v) else None
            for i, it in enumerate(v):
                validate(items, it, f"{path}[{i}]", olds[i] if olds else None, errs, fv,
                         warnings)
    elif t == "object":
        props = schema.get("properties") or {}
        for r in schema.get("required") or []:
            if r not in v:
                errs.append(f"{path}.{r}: Required value")
        ap = schema.get("additionalProperties")
        for k, sub_v in list(v.items()):
            sub = props.get(k)
            sub_old = old.get(k) if isinstance(old, dict) else None
            if sub is not None:
                validate(sub, sub_v, f"{path}.{k}", sub_old, errs, fv, warnings)
            elif isinstance(ap, dict):
                validate(ap, sub_v, f"{path}.{k}", sub_old, errs, fv, warnings)
            elif ap is True or schema.get(PRESERVE):
                continue
            elif fv == "Strict":
                errs.append(f"{path}.{k}: field not declared in schema")
            else:  # structural pruning
                del v[k]
                if fv == "Warn" and warnings is not None:
                    warnings.append(f'unknown field "{path}.{k}"')
    for rule in schema.get(RULES) or []:
        expr = rule["rule"]
        if "oldSelf" in expr and old is None:
            continue  # transition rule: not evaluated on create
        env = {"self": v}
        if old is not None:
            env["oldSelf"] = old
        try:
            ok = _prog(expr).eval(env)
        except cel.CELError as e:
            ok = False
            rule = {**rule, "message": f"{rule.get('message', expr)} (rule error: {e})"}
        if ok is not True:
            errs.append(f"{path}: Invalid value: {rule.get('message') or expr}")
    return errs


def schema_size(schema) -> int:
    """Number of schema nodes (a size diagnostic for the generated CRDs)."""
    if isinstance(schema, dict):
        return 1 + sum(schema_size(v) for v in schema.values())
    if isinstance(schema, list):
        return sum(schema_size(v) for v in schema)
    return 0
