"""A self-contained interpreter for the CEL subset Omnia's policies use.

The reference compiles Common Expression Language with cel-go in three places:
memory access deny-filters over ``metadata`` (``internal/memory/access/filter.go:43-80``),
the EE policy broker over ``headers`` / ``body`` / ``identity``
(``ee/pkg/policy/evaluator.go:108-111``) and kubebuilder CRD rules.  cel-go is
not available here, so this module implements the language core directly:

* literals: int, uint (``1u``), double, string (single/double/triple quoted,
  raw ``r''``), bytes (``b''``), bool, null, lists, maps;
* operators with CEL precedence: ``?:``, ``||``, ``&&``, relations
  (``== != < <= > >= in``), ``+ -``, ``* / %``, unary ``! -``;
* member / index access, field-presence macro ``has(a.b)``;
* macros ``all exists exists_one map filter``;
* functions ``size startsWith endsWith contains matches lowerAscii upperAscii
  trim split join replace indexOf int uint double string bool type`` and
  ``timestamp``/``duration`` comparisons over RFC3339 / Go-style durations.

Semantics follow the spec where it matters for policies: missing map keys and
type mismatches are *errors*; ``&&``/``||`` absorb an error when the other side
decides the result (commutative short-circuit); callers decide what an error
means (the memory deny-filter treats it as "deny", the broker as "fail closed").
"""
from __future__ import annotations

import datetime as _dt
import re
from dataclasses import dataclass


class CELError(Exception):
    pass


class CELSyntaxError(CELError):
    pass


# ------------------------------------------------------------------ lexer
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|//[^\n]*)
  | (?P<num>0x[0-9a-fA-F]+u?|\d+\.\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?|\d+[eE][+-]?\d+|\d+u?)
  | (?P<str>[rRbB]{0,2}(?:\"\"\"[\s\S]*?\"\"\"|'''[\s\S]*?'''|"(?:\\.|[^"\\\n])*"|'(?:\\.|[^'\\\n])*'))
  | (?P<op>\|\||&&|==|!=|<=|>=|[-+*/%!<>?:.,\[\](){}])
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)

_ESC = {"n": "\n", "t": "\t", "r": "\r", "\\": "\\", "'": "'", '"': '"', "a": "\a", "b": "\b",
        "f": "\f", "v": "\v", "`": "`", "?": "?"}


@dataclass
class Tok:
    kind: str
    val: object
    pos: int


def _unescape(body: str) -> str:
    out, i = [], 0
    while i < len(body):
        c = body[i]
        if c == "\\" and i + 1 < len(body):
            n = body[i + 1]
            if n in _ESC:
                out.append(_ESC[n])
                i += 2
                continue
            if n in "xX":
                out.append(chr(int(body[i + 2:i + 4], 16)))
                i += 4
                continue
            if n == "u":
                out.append(chr(int(body[i + 2:i + 6], 16)))
                i += 6
                continue
            if n == "U":
                out.append(chr(int(body[i + 2:i + 10], 16)))
                i += 10
                continue
            if n.isdigit():
                out.append(chr(int(body[i + 1:i + 4], 8)))
                i += 4
                continue
        out.append(c)
        i += 1
    return "".join(out)


def tokenize(src: str) -> list[Tok]:
    toks, pos = [], 0
    while pos < len(src):
        m = _TOKEN_RE.match(src, pos)
        if not m:
            raise CELSyntaxError(f"unexpected character {src[pos]!r} at {pos}")
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "num":
            if text.endswith("u"):
                toks.append(Tok("uint", int(text[:-1], 0), pos))
            elif text.startswith(("0x", "0X")):
                toks.append(Tok("int", int(text, 16), pos))
            elif any(c in text for c in ".eE"):
                toks.append(Tok("double", float(text), pos))
            else:
                toks.append(Tok("int", int(text), pos))
        elif kind == "str":
            prefix = ""
            while text[0] in "rRbB":
                prefix += text[0].lower()
                text = text[1:]
            q = 3 if text[:3] in ('"""', "'''") else 1
            body = text[q:-q]
            s = body if "r" in prefix else _unescape(body)
            toks.append(Tok("bytes" if "b" in prefix else "string",
                            s.encode() if "b" in prefix else s, pos))
        elif kind == "op":
            toks.append(Tok("op", text, pos))
        elif kind == "id":
            if text in ("true", "false"):
                toks.append(Tok("bool", text == "true", pos))
            elif text == "null":
                toks.append(Tok("null", None, pos))
            elif text == "in":
                toks.append(Tok("op", "in", pos))
            else:
                toks.append(Tok("id", text, pos))
        pos = m.end()
    toks.append(Tok("eof", None, pos))
    return toks


# ------------------------------------------------------------------ AST
# nodes are tuples: (kind, ...)
_REL = {"==", "!=", "<", "<=", ">", ">=", "in"}
_MACROS = {"all", "exists", "exists_one", "map", "filter"}


class _Parser:
    def __init__(self, src: str):
        self.t = tokenize(src)
        self.i = 0

    def peek(self, v=None):
        tok = self.t[self.i]
        if v is None:
            return tok
        return tok.kind == "op" and tok.val == v

    def eat(self, v=None) -> Tok:
        tok = self.t[self.i]
        if v is not None and not (tok.kind == "op" and tok.val == v):
            raise CELSyntaxError(f"expected {v!r} at {tok.pos}, got {tok.val!r}")
        self.i += 1
        return tok

    def parse(self):
        e = self.expr()
        if self.peek().kind != "eof":
            raise CELSyntaxError(f"unexpected {self.peek().val!r} at {self.peek().pos}")
        return e

    def expr(self):
        c = self.or_()
        if self.peek("?"):
            self.eat("?")
            a = self.or_()
            self.eat(":")
            b = self.expr()
            return ("cond", c, a, b)
        return c

    def or_(self):
        e = self.and_()
        while self.peek("||"):
            self.eat()
            e = ("or", e, self.and_())
        return e

    def and_(self):
        e = self.rel()
        while self.peek("&&"):
            self.eat()
            e = ("and", e, self.rel())
        return e

    def rel(self):
        e = self.add()
        while self.peek().kind == "op" and self.peek().val in _REL:
            op = self.eat().val
            e = ("bin", op, e, self.add())
        return e

    def add(self):
        e = self.mul()
        while self.peek("+") or self.peek("-"):
            op = self.eat().val
            e = ("bin", op, e, self.mul())
        return e

    def mul(self):
        e = self.unary()
        while self.peek("*") or self.peek("/") or self.peek("%"):
            op = self.eat().val
            e = ("bin", op, e, self.unary())
        return e

    def unary(self):
        if self.peek("!"):
            self.eat()
            return ("not", self.unary())
        if self.peek("-"):
            self.eat()
            nxt = self.peek()
            if nxt.kind in ("int", "double") and not self._followed_by_member(1):
                self.eat()
                return ("lit", -nxt.val)
            return ("neg", self.unary())
        return self.member()

    def _followed_by_member(self, off):
        t = self.t[self.i + off]
        return t.kind == "op" and t.val in (".", "[")

    def args(self):
        out = []
        if not self.peek(")"):
            out.append(self.expr())
            while self.peek(","):
                self.eat()
                out.append(self.expr())
        self.eat(")")
        return out

    def member(self):
        e = self.primary()
        while True:
            if self.peek("."):
                self.eat()
                name = self.eat()
                if name.kind != "id":
                    raise CELSyntaxError(f"expected field name at {name.pos}")
                if self.peek("("):
                    self.eat("(")
                    if name.val in _MACROS:
                        var = self.eat()
                        if var.kind != "id":
                            raise CELSyntaxError("macro variable must be an identifier")
                        self.eat(",")
                        body = self.expr()
                        extra = None
                        if name.val == "map" and self.peek(","):
                            self.eat()
                            extra = self.expr()
                        self.eat(")")
                        e = ("macro", name.val, e, var.val, body, extra)
                    else:
                        e = ("call", name.val, e, self.args())
                else:
                    e = ("sel", e, name.val)
            elif self.peek("["):
                self.eat()
                idx = self.expr()
                self.eat("]")
                e = ("index", e, idx)
            else:
                return e

    def primary(self):
        tok = self.eat()
        if tok.kind in ("int", "uint", "double", "string", "bytes", "bool", "null"):
            return ("lit", tok.val)
        if tok.kind == "op" and tok.val == "(":
            e = self.expr()
            self.eat(")")
            return e
        if tok.kind == "op" and tok.val == "[":
            items = []
            if not self.peek("]"):
                items.append(self.expr())
                while self.peek(","):
                    self.eat()
                    if self.peek("]"):
                        break
                    items.append(self.expr())
            self.eat("]")
            return ("list", items)
        if tok.kind == "op" and tok.val == "{":
            items = []
            if not self.peek("}"):
                while True:
                    k = self.expr()
                    self.eat(":")
                    items.append((k, self.expr()))
                    if not self.peek(","):
                        break
                    self.eat()
                    if self.peek("}"):
                        break
            self.eat("}")
            return ("map", items)
        if tok.kind == "op" and tok.val == ".":
            return self.primary()
        if tok.kind == "id":
            if self.peek("("):
                self.eat("(")
                if tok.val == "has":
                    arg = self.expr()
                    self.eat(")")
                    if arg[0] != "sel":
                        raise CELSyntaxError("has() requires a field selection")
                    return ("has", arg[1], arg[2])
                return ("call", tok.val, None, self.args())
            return ("id", tok.val)
        raise CELSyntaxError(f"unexpected {tok.val!r} at {tok.pos}")


# ------------------------------------------------------------------ values
class _Err:
    """An error value (CEL errors propagate as values through && / ||)."""

    __slots__ = ("msg",)

    def __init__(self, msg):
        self.msg = msg


_DUR_RE = re.compile(r"(-?\d+(?:\.\d+)?)(h|ms|us|µs|ns|m|s)")
_DUR_UNIT = {"h": 3600.0, "m": 60.0, "s": 1.0, "ms": 1e-3, "us": 1e-6, "µs": 1e-6, "ns": 1e-9}


def _duration(s: str) -> _dt.timedelta:
    if not isinstance(s, str) or not s:
        raise CELError("duration() requires a string")
    total, pos = 0.0, 0
    for m in _DUR_RE.finditer(s):
        if m.start() != pos:
            raise CELError(f"bad duration {s!r}")
        total += float(m.group(1)) * _DUR_UNIT[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise CELError(f"bad duration {s!r}")
    return _dt.timedelta(seconds=total)


def _timestamp(s: str) -> _dt.datetime:
    if not isinstance(s, str):
        raise CELError("timestamp() requires a string")
    try:
        return _dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
    except ValueError as e:
        raise CELError(f"bad timestamp {s!r}") from e


def _is_num(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _type_name(v) -> str:
    if v is None:
        return "null_type"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "double"
    if isinstance(v, str):
        return "string"
    if isinstance(v, bytes):
        return "bytes"
    if isinstance(v, (list, tuple)):
        return "list"
    if isinstance(v, dict):
        return "map"
    if isinstance(v, _dt.datetime):
        return "google.protobuf.Timestamp"
    if isinstance(v, _dt.timedelta):
        return "google.protobuf.Duration"
    return type(v).__name__


def _eq(a, b) -> bool:
    if _is_num(a) and _is_num(b):
        return a == b
    if type(a) is not type(b) and not (isinstance(a, (list, tuple)) and isinstance(b, (list, tuple))):
        if a is None or b is None:
            return False
        if isinstance(a, bool) or isinstance(b, bool):
            return False
        raise CELError(f"no such overload: {_type_name(a)} == {_type_name(b)}")
    if isinstance(a, (list, tuple)):
        return len(a) == len(b) and all(_eq(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_eq(a[k], b[k]) for k in a)
    return a == b


def _cmp(op, a, b) -> bool:
    ok = (_is_num(a) and _is_num(b)) or (type(a) is type(b) and isinstance(
        a, (str, bytes, bool, _dt.datetime, _dt.timedelta)))
    if not ok:
        raise CELError(f"no such overload: {_type_name(a)} {op} {_type_name(b)}")
    return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]


def _arith(op, a, b):
    if op == "+":
        if isinstance(a, str) and isinstance(b, str):
            return a + b
        if isinstance(a, bytes) and isinstance(b, bytes):
            return a + b
        if isinstance(a, list) and isinstance(b, list):
            return a + b
        if isinstance(a, (_dt.datetime, _dt.timedelta)) and isinstance(b, _dt.timedelta):
            return a + b
    if op == "-" and isinstance(a, (_dt.datetime, _dt.timedelta)) and isinstance(
            b, (_dt.datetime, _dt.timedelta)):
        return a - b
    if not (_is_num(a) and _is_num(b)):
        raise CELError(f"no such overload: {_type_name(a)} {op} {_type_name(b)}")
    if isinstance(a, float) != isinstance(b, float):
        raise CELError(f"no such overload: {_type_name(a)} {op} {_type_name(b)}")
    if op == "+":
        return a + b
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if op == "/":
        if isinstance(a, int):
            if b == 0:
                raise CELError("division by zero")
            q = abs(a) // abs(b)
            return q if (a >= 0) == (b >= 0) else -q
        return a / b if b else (float("inf") if a > 0 else float("-inf") if a < 0 else float("nan"))
    if op == "%":
        if not isinstance(a, int):
            raise CELError("no such overload: double % double")
        if b == 0:
            raise CELError("modulus by zero")
        r = abs(a) % abs(b)
        return r if a >= 0 else -r
    raise CELError(f"unknown operator {op}")


def _size(v):
    if isinstance(v, (str, bytes, list, tuple, dict)):
        return len(v)
    raise CELError(f"no such overload: size({_type_name(v)})")


def _str_method(name, target, args):
    if not isinstance(target, str):
        raise CELError(f"no such overload: {_type_name(target)}.{name}")
    if name == "startsWith":
        return target.startswith(args[0])
    if name == "endsWith":
        return target.endswith(args[0])
    if name == "contains":
        return args[0] in target
    if name == "matches":
        return re.search(args[0], target) is not None
    if name == "lowerAscii":
        return target.lower()
    if name == "upperAscii":
        return target.upper()
    if name == "trim":
        return target.strip()
    if name == "split":
        return target.split(args[0]) if len(args) == 1 else target.split(args[0], args[1] - 1)
    if name == "replace":
        return target.replace(args[0], args[1]) if len(args) == 2 else \
            target.replace(args[0], args[1], args[2])
    if name == "indexOf":
        return target.find(args[0])
    if name == "lastIndexOf":
        return target.rfind(args[0])
    if name == "substring":
        return target[args[0]:args[1]] if len(args) == 2 else target[args[0]:]
    if name == "charAt":
        return target[args[0]] if args[0] < len(target) else ""
    raise CELError(f"unknown function {name}")


def _convert(name, v):
    if name == "int":
        if isinstance(v, bool):
            raise CELError("no such overload: int(bool)")
        if isinstance(v, (int, float)):
            return int(v)
        if isinstance(v, str):
            try:
                return int(v)
            except ValueError as e:
                raise CELError(f"int({v!r})") from e
        if isinstance(v, _dt.datetime):
            return int(v.timestamp())
    if name == "uint":
        r = _convert("int", v)
        if r < 0:
            raise CELError("uint overflow")
        return r
    if name == "double":
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return float(v)
        if isinstance(v, str):
            try:
                return float(v)
            except ValueError as e:
                raise CELError(f"double({v!r})") from e
    if name == "string":
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, (int, float, str)):
            return str(v)
        if isinstance(v, bytes):
            return v.decode()
        if isinstance(v, _dt.datetime):
            return v.isoformat().replace("+00:00", "Z")
        if isinstance(v, _dt.timedelta):
            return f"{v.total_seconds():g}s"
    if name == "bool":
        if isinstance(v, bool):
            return v
        if v in ("true", "True", "TRUE", "t", "1"):
            return True
        if v in ("false", "False", "FALSE", "f", "0"):
            return False
    if name == "bytes" and isinstance(v, str):
        return v.encode()
    raise CELError(f"no such overload: {name}({_type_name(v)})")


class Program:
    """A compiled expression; ``eval(activation)`` returns the value or raises CELError."""

    def __init__(self, src: str):
        self.src = src
        self.ast = _Parser(src).parse()

    def eval(self, activation: dict | None = None):
        r = self._ev(self.ast, dict(activation or {}))
        if isinstance(r, _Err):
            raise CELError(r.msg)
        return r

    # each node returns a value or an _Err (for error absorption in && / ||)
    def _ev(self, n, env):
        try:
            return self._ev_raise(n, env)
        except CELError as e:
            return _Err(str(e))
        except (TypeError, KeyError, IndexError, ValueError, re.error, AttributeError) as e:
            return _Err(f"{type(e).__name__}: {e}")

    def _val(self, n, env):
        v = self._ev(n, env)
        if isinstance(v, _Err):
            raise CELError(v.msg)
        return v

    def _ev_raise(self, n, env):
        k = n[0]
        if k == "lit":
            return n[1]
        if k == "id":
            if n[1] in env:
                return env[n[1]]
            raise CELError(f"undeclared reference to '{n[1]}'")
        if k == "list":
            return [self._val(x, env) for x in n[1]]
        if k == "map":
            return {self._val(a, env): self._val(b, env) for a, b in n[1]}
        if k == "sel":
            obj = self._val(n[1], env)
            if isinstance(obj, dict):
                if n[2] in obj:
                    return obj[n[2]]
                raise CELError(f"no such key: {n[2]}")
            raise CELError(f"type '{_type_name(obj)}' does not support field selection")
        if k == "has":
            obj = self._val(n[1], env)
            if isinstance(obj, dict):
                return n[2] in obj
            raise CELError(f"invalid type for field selection: {_type_name(obj)}")
        if k == "index":
            obj = self._val(n[1], env)
            idx = self._val(n[2], env)
            if isinstance(obj, dict):
                if idx in obj:
                    return obj[idx]
                raise CELError(f"no such key: {idx}")
            if isinstance(obj, (list, tuple)):
                if not isinstance(idx, int) or isinstance(idx, bool):
                    raise CELError("list index must be int")
                if idx < 0 or idx >= len(obj):
                    raise CELError(f"index out of range: {idx}")
                return obj[idx]
            raise CELError(f"type '{_type_name(obj)}' does not support indexing")
        if k == "not":
            v = self._val(n[1], env)
            if not isinstance(v, bool):
                raise CELError("no such overload: !" + _type_name(v))
            return not v
        if k == "neg":
            v = self._val(n[1], env)
            if not _is_num(v):
                raise CELError("no such overload: -" + _type_name(v))
            return -v
        if k in ("and", "or"):
            decisive = k == "or"  # value that short-circuits
            a = self._ev(n[1], env)
            if a is decisive:
                return decisive
            b = self._ev(n[2], env)
            if b is decisive:
                return decisive
            for v in (a, b):
                if isinstance(v, _Err):
                    raise CELError(v.msg)
                if not isinstance(v, bool):
                    raise CELError(f"no such overload: {_type_name(v)} {k}")
            return not decisive
        if k == "cond":
            c = self._val(n[1], env)
            if not isinstance(c, bool):
                raise CELError("conditional requires bool")
            return self._val(n[2] if c else n[3], env)
        if k == "bin":
            op = n[1]
            a, b = self._val(n[2], env), self._val(n[3], env)
            if op == "==":
                return _eq(a, b)
            if op == "!=":
                return not _eq(a, b)
            if op == "in":
                if isinstance(b, dict):
                    return a in b
                if isinstance(b, (list, tuple)):
                    return any(_safe_eq(a, x) for x in b)
                raise CELError(f"no such overload: in {_type_name(b)}")
            if op in ("<", "<=", ">", ">="):
                return _cmp(op, a, b)
            return _arith(op, a, b)
        if k == "macro":
            _, name, target_n, var, body, extra = n
            target = self._val(target_n, env)
            items = list(target.keys()) if isinstance(target, dict) else target
            if not isinstance(items, (list, tuple)):
                raise CELError(f"macro {name} requires a list or map")
            sub = dict(env)
            if name in ("all", "exists"):
                want = name == "exists"
                err = None
                for it in items:
                    sub[var] = it
                    r = self._ev(body, sub)
                    if r is want:
                        return want
                    if isinstance(r, _Err):
                        err = r
                    elif not isinstance(r, bool):
                        raise CELError(f"{name} predicate must be bool")
                if err is not None:
                    raise CELError(err.msg)
                return not want
            if name == "exists_one":
                cnt = 0
                for it in items:
                    sub[var] = it
                    if self._val(body, sub) is True:
                        cnt += 1
                return cnt == 1
            if name == "filter":
                out = []
                for it in items:
                    sub[var] = it
                    if self._val(body, sub) is True:
                        out.append(it)
                return out
            if name == "map":
                out = []
                for it in items:
                    sub[var] = it
                    if extra is not None:  # map(x, pred, expr)
                        if self._val(body, sub) is not True:
                            continue
                        out.append(self._val(extra, sub))
                    else:
                        out.append(self._val(body, sub))
                return out
        if k == "call":
            _, name, target_n, arg_ns = n
            args = [self._val(a, env) for a in arg_ns]
            if target_n is None:
                if name == "size" and len(args) == 1:
                    return _size(args[0])
                if name in ("int", "uint", "double", "string", "bool", "bytes") and len(args) == 1:
                    return _convert(name, args[0])
                if name == "type":
                    return _type_name(args[0])
                if name == "duration":
                    return _duration(args[0])
                if name == "timestamp":
                    return _timestamp(args[0])
                if name == "matches" and len(args) == 2:
                    return _str_method("matches", args[0], args[1:])
                if name == "dyn":
                    return args[0]
                raise CELError(f"undeclared function '{name}'")
            target = self._val(target_n, env)
            if name == "size":
                return _size(target)
            if name == "join" and isinstance(target, list):
                return (args[0] if args else "").join(str(x) for x in target)
            if isinstance(target, _dt.datetime):
                return _time_accessor(name, target)
            return _str_method(name, target, args)
        raise CELError(f"unknown node {k}")


def _safe_eq(a, b):
    try:
        return _eq(a, b)
    except CELError:
        return False


def _time_accessor(name, t: _dt.datetime):
    table = {"getFullYear": t.year, "getMonth": t.month - 1, "getDate": t.day,
             "getDayOfMonth": t.day - 1, "getDayOfWeek": (t.weekday() + 1) % 7,
             "getHours": t.hour, "getMinutes": t.minute, "getSeconds": t.second}
    if name in table:
        return table[name]
    raise CELError(f"unknown function {name}")


_CACHE: dict[str, Program] = {}


def compile(src: str) -> Program:  # noqa: A001 - mirrors cel-go's env.Compile
    p = _CACHE.get(src)
    if p is None:
        p = Program(src)
        if len(_CACHE) < 4096:
            _CACHE[src] = p
    return p


def evaluate(src: str, activation: dict | None = None):
    return compile(src).eval(activation)


class DenyFilter:
    """``internal/memory/access/filter.go``: an expression over ``metadata`` that
    returns true to DENY.  Empty expression = allow all; errors / non-bool = deny
    (fail closed); a malformed expression fails at construction."""

    def __init__(self, expr: str = ""):
        self.expr = (expr or "").strip()
        self.prog = compile(self.expr) if self.expr else None

    def allowed(self, metadata: dict | None) -> bool:
        if self.prog is None:
            return True
        try:
            out = self.prog.eval({"metadata": dict(metadata or {})})
        except CELError:
            return False
        if not isinstance(out, bool):
            return False
        return not out
