"""JMESPath subset for ToolRegistry ``bodyMapping`` / ``responseMapping``
(``api/v1alpha1/toolregistry_types.go:307-320``); the ``jmespath`` package is
not installed.  Supported: identifiers ("quoted" too), ``a.b``, ``[n]``,
``[a:b:c]``, ``[*]``/``.*`` projections, ``[]`` flatten, ``[?expr]`` filters
with comparators / ``&&`` / ``||`` / ``!``, multiselect ``[a, b]`` and
``{k: expr}``, pipes ``|``, ```literal``` JSON, ``'raw'`` strings, ``@``, and
the functions length, keys, values, to_string, to_number, contains, join,
sort, max, min, sum, type, not_null, starts_with, ends_with.
"""
from __future__ import annotations

import json
import re

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>-?\d+)
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<qid>"(?:[^"\\]|\\.)*")
  | (?P<raw>'(?:[^'\\]|\\.)*')
  | (?P<lit>`(?:[^`\\]|\\.)*`)
  | (?P<op>\|\||&&|==|!=|<=|>=|\[\?|\[\]|[.\[\]{}(),:*|@<>!&])
""", re.X)


class JMESPathError(ValueError):
    pass


def _tokens(s: str):
    pos = 0
    out = []
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise JMESPathError(f"bad expression at {pos}: {s[pos:pos + 10]!r}")
        pos = m.end()
        k = m.lastgroup
        v = m.group(k)
        if k == "ws":
            continue
        if k == "qid":
            out.append(("id", json.loads(v)))
        elif k == "raw":
            out.append(("lit", v[1:-1].replace("\\'", "'")))
        elif k == "lit":
            out.append(("lit", json.loads(v[1:-1])))
        elif k == "num":
            out.append(("num", int(v)))
        else:
            out.append((k if k != "op" else v, v))
    out.append(("eof", None))
    return out


class _Parser:
    # binding powers
    BP = {"eof": 0, "|": 1, "||": 2, "&&": 3, "==": 5, "!=": 5, "<": 5, ">": 5, "<=": 5,
          ">=": 5, ".": 40, "[": 55, "[?": 55, "[]": 55, "(": 60, "*": 20, "]": 0, ")": 0,
          ",": 0, "}": 0, ":": 0}

    def __init__(self, s):
        self.t = _tokens(s)
        self.i = 0

    def peek(self):
        return self.t[self.i][0]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, k):
        tok = self.next()
        if tok[0] != k:
            raise JMESPathError(f"expected {k}, got {tok[0]}")
        return tok

    def parse(self):
        e = self.expr(0)
        if self.peek() != "eof":
            raise JMESPathError(f"trailing tokens at {self.peek()}")
        return e

    def expr(self, rbp):
        left = self.nud(self.next())
        while rbp < self.BP.get(self.peek(), 0):
            left = self.led(self.next(), left)
        return left

    def nud(self, tok):
        k, v = tok
        if k == "id":
            if self.peek() == "(":
                self.next()
                args = []
                while self.peek() != ")":
                    args.append(self.expr(0))
                    if self.peek() == ",":
                        self.next()
                self.expect(")")
                return ("func", v, args)
            return ("field", v)
        if k == "lit":
            return ("lit", v)
        if k == "num":
            return ("lit", v)
        if k == "@":
            return ("cur",)
        if k == "*":
            return ("vproj", ("cur",), self.proj_rhs(20))
        if k == "!":
            return ("not", self.expr(45))
        if k == "(":
            e = self.expr(0)
            self.expect(")")
            return e
        if k == "[]":
            return ("flatten", ("cur",), self.proj_rhs(55))
        if k == "[?":
            cond = self.expr(0)
            self.expect("]")
            return ("filter", ("cur",), cond, self.proj_rhs(55))
        if k == "[":
            return self.bracket(("cur",))
        if k == "{":
            items = []
            while True:
                key = self.next()[1]
                self.expect(":")
                items.append((key, self.expr(0)))
                if self.peek() == ",":
                    self.next()
                    continue
                self.expect("}")
                return ("mhash", items)
        raise JMESPathError(f"unexpected token {k}")

    def bracket(self, left):
        if self.peek() == "*":
            self.next()
            self.expect("]")
            return ("proj", left, self.proj_rhs(55))
        if self.peek() in ("num", ":"):
            parts = [None, None, None]
            idx = 0
            is_slice = False
            while self.peek() != "]":
                if self.peek() == ":":
                    self.next()
                    idx += 1
                    is_slice = True
                else:
                    parts[idx] = self.next()[1]
            self.expect("]")
            if is_slice:
                return ("proj", ("slice", left, parts), self.proj_rhs(55))
            return ("index", left, parts[0])
        # multiselect list
        items = []
        while True:
            items.append(self.expr(0))
            if self.peek() == ",":
                self.next()
                continue
            self.expect("]")
            return ("pipe", left, ("mlist", items))

    def proj_rhs(self, bp):
        if self.BP.get(self.peek(), 0) < 10:
            return ("cur",)
        if self.peek() == ".":
            self.next()
            return self.dot_rhs()
        if self.peek() in ("[", "[?", "[]"):
            return self.expr(bp - 1) if False else self._chain(bp)
        raise JMESPathError("bad projection")

    def _chain(self, bp):
        left = ("cur",)
        while self.peek() in ("[", "[?", "[]", "."):
            left = self.led(self.next(), left)
        return left

    def dot_rhs(self):
        k = self.peek()
        if k == "*":
            self.next()
            return ("vproj", ("cur",), self.proj_rhs(20))
        if k == "[":
            self.next()
            items = []
            while True:
                items.append(self.expr(0))
                if self.peek() == ",":
                    self.next()
                    continue
                self.expect("]")
                return ("mlist", items)
        if k == "{":
            return self.nud(self.next())
        return self.nud(self.next())

    def led(self, tok, left):
        k = tok[0]
        if k == ".":
            return ("pipe", left, self.dot_rhs())
        if k == "|":
            return ("pipe", left, self.expr(1))
        if k in ("||", "&&"):
            return (k, left, self.expr(self.BP[k]))
        if k in ("==", "!=", "<", ">", "<=", ">="):
            return ("cmp", k, left, self.expr(self.BP[k]))
        if k == "[":
            return self.bracket(left)
        if k == "[]":
            return ("flatten", left, self.proj_rhs(55))
        if k == "[?":
            cond = self.expr(0)
            self.expect("]")
            return ("filter", left, cond, self.proj_rhs(55))
        if k == "*":
            return ("vproj", left, self.proj_rhs(20))
        raise JMESPathError(f"unexpected {k}")


def _truthy(v):
    return not (v is None or v is False or v == "" or v == [] or v == {})


def _ev(node, data):
    t = node[0]
    if t == "cur":
        return data
    if t == "lit":
        return node[1]
    if t == "field":
        return data.get(node[1]) if isinstance(data, dict) else None
    if t == "pipe":
        return _ev(node[2], _ev(node[1], data))
    if t == "index":
        v = _ev(node[1], data)
        if not isinstance(v, list):
            return None
        try:
            return v[node[2]]
        except IndexError:
            return None
    if t == "slice":
        v = _ev(node[1], data)
        if not isinstance(v, list):
            return None
        a, b, c = node[2]
        return v[slice(a, b, c)]
    if t == "proj":
        v = _ev(node[1], data)
        if not isinstance(v, list):
            return None
        out = [_ev(node[2], x) for x in v]
        return [x for x in out if x is not None]
    if t == "vproj":
        v = _ev(node[1], data)
        if not isinstance(v, dict):
            return None
        out = [_ev(node[2], x) for x in v.values()]
        return [x for x in out if x is not None]
    if t == "flatten":
        v = _ev(node[1], data)
        if not isinstance(v, list):
            return None
        flat = []
        for x in v:
            flat.extend(x if isinstance(x, list) else [x])
        out = [_ev(node[2], x) for x in flat]
        return [x for x in out if x is not None]
    if t == "filter":
        v = _ev(node[1], data)
        if not isinstance(v, list):
            return None
        out = [_ev(node[3], x) for x in v if _truthy(_ev(node[2], x))]
        return [x for x in out if x is not None]
    if t == "mlist":
        return None if data is None else [_ev(n, data) for n in node[1]]
    if t == "mhash":
        return None if data is None else {k: _ev(n, data) for k, n in node[1]}
    if t == "||":
        a = _ev(node[1], data)
        return a if _truthy(a) else _ev(node[2], data)
    if t == "&&":
        a = _ev(node[1], data)
        return _ev(node[2], data) if _truthy(a) else a
    if t == "not":
        return not _truthy(_ev(node[1], data))
    if t == "cmp":
        op, a, b = node[1], _ev(node[2], data), _ev(node[3], data)
        if op == "==":
            return a == b
        if op == "!=":
            return a != b
        if not (isinstance(a, (int, float)) and isinstance(b, (int, float))):
            return None
        return {"<": a < b, ">": a > b, "<=": a <= b, ">=": a >= b}[op]
    if t == "func":
        args = [_ev(a, data) for a in node[2]]
        return _FUNCS[node[1]](*args)
    raise JMESPathError(f"bad node {t}")


_FUNCS = {
    "length": lambda v: len(v) if v is not None else None,
    "keys": lambda v: list(v.keys()),
    "values": lambda v: list(v.values()),
    "to_string": lambda v: v if isinstance(v, str) else json.dumps(v, separators=(",", ":")),
    "to_number": lambda v: float(v) if not isinstance(v, (int, float)) else v,
    "contains": lambda a, b: b in a if a is not None else False,
    "join": lambda sep, arr: sep.join(arr),
    "sort": lambda arr: sorted(arr),
    "max": lambda arr: max(arr) if arr else None,
    "min": lambda arr: min(arr) if arr else None,
    "sum": lambda arr: sum(arr),
    "type": lambda v: {dict: "object", list: "array", str: "string", bool: "boolean",
                       type(None): "null"}.get(type(v), "number"),
    "not_null": lambda *a: next((x for x in a if x is not None), None),
    "starts_with": lambda s, p: isinstance(s, str) and s.startswith(p),
    "ends_with": lambda s, p: isinstance(s, str) and s.endswith(p),
}

_cache: dict[str, tuple] = {}


def compile(expr: str):
    node = _cache.get(expr)
    if node is None:
        node = _cache[expr] = _Parser(expr).parse()
    return node


def search(expr: str, data):
    return _ev(compile(expr), data)
