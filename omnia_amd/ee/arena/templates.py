"""Arena project templates (``ee/pkg/arena/template``: discovery, variables,
rendering) used by the ArenaTemplateSource controller and the dev console.

* **Discovery** -- a ``.template-index.yaml`` at the source root (or under the
  templates path) lists the templates; otherwise every ``template.yaml`` under
  ``templates/`` (or the root) is loaded.  A template's ``metadata.name`` is
  required; ``spec.files`` defaults to the directory's entries, rendered when
  their extension is yaml / yml / json / txt / md.
* **Variables** -- typed (string / number / boolean / enum) with required,
  default, pattern, options and min / max; :func:`resolve_variables` applies
  defaults and returns every violation at once.
* **Rendering** -- the Go ``text/template`` subset templates use:
  ``{{ .var }}``, pipelines (``{{ .name | lower | replace " " "-" }}``),
  function calls (``{{ default "x" .v }}``), ``if / else if / else / end``,
  ``range`` over lists (``{{ . }}`` is the element), ``{{-`` / ``-}}`` whitespace
  trimming, and the reference's function map (lower, upper, title, trimSpace,
  trimPrefix, trimSuffix, replace, contains, hasPrefix, hasSuffix, split, join,
  toString, toInt, toFloat, toBool, default, ternary, indent, quote, eq, ne, not,
  and, or).
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import asdict, dataclass, field

import yaml

INDEX_FILE = ".template-index.yaml"
TEMPLATE_FILE = "template.yaml"
DEFAULT_TEMPLATES_PATH = "templates"
RENDER_EXT = (".yaml", ".yml", ".json", ".txt", ".md")


@dataclass
class Template:
    name: str
    version: str = ""
    displayName: str = ""
    description: str = ""
    category: str = ""
    tags: list = field(default_factory=list)
    variables: list = field(default_factory=list)
    files: list = field(default_factory=list)
    path: str = ""

    def to_json(self) -> dict:
        return {k: v for k, v in asdict(self).items() if v not in ("", [], None) or
                k in ("name", "path")}


# ------------------------------------------------------------------ discovery
def _default_files(tdir: str) -> list[dict]:
    out = []
    for name in sorted(os.listdir(tdir)):
        if name == TEMPLATE_FILE or name.startswith("."):
            continue
        isdir = os.path.isdir(os.path.join(tdir, name))
        out.append({"path": name + "/" if isdir else name,
                    "render": name.lower().endswith(RENDER_EXT)})
    return out


def load_template(root: str, tdir: str) -> Template:
    with open(os.path.join(tdir, TEMPLATE_FILE)) as f:
        d = yaml.safe_load(f) or {}
    md, spec = d.get("metadata") or {}, d.get("spec") or {}
    if not md.get("name"):
        raise ValueError("template metadata.name is required")
    t = Template(name=md["name"], version=str(md.get("version") or ""),
                 displayName=spec.get("displayName") or md["name"],
                 description=spec.get("description", ""), category=spec.get("category", ""),
                 tags=list(spec.get("tags") or []), variables=list(spec.get("variables") or []),
                 files=list(spec.get("files") or []),
                 path=os.path.relpath(tdir, root))
    if not t.files:
        t.files = _default_files(tdir)
    return t


def discover(root: str, templates_path: str = DEFAULT_TEMPLATES_PATH) -> list[Template]:
    templates_path = (templates_path or DEFAULT_TEMPLATES_PATH).rstrip("/")
    for idx in (os.path.join(root, INDEX_FILE), os.path.join(root, templates_path, INDEX_FILE)):
        if os.path.exists(idx):
            with open(idx) as f:
                d = yaml.safe_load(f) or {}
            out = []
            for e in d.get("templates") or []:
                t = Template(**{k: v for k, v in e.items() if k in Template.__dataclass_fields__})
                t.displayName = t.displayName or t.name
                out.append(t)
            return out
    base = os.path.join(root, templates_path)
    if not os.path.isdir(base):
        base = root
    out = []
    for d, _dirs, files in sorted(os.walk(base)):
        if TEMPLATE_FILE in files:
            try:
                out.append(load_template(root, d))
            except (ValueError, yaml.YAMLError, OSError):
                continue  # a broken template does not hide the others
    return out


def filter_templates(ts: list[Template], category: str = "", tags: list | None = None,
                     query: str = "") -> list[Template]:
    out = [t for t in ts if not category or t.category == category]
    if tags:
        out = [t for t in out if all(x in t.tags for x in tags)]
    if query:
        q = query.lower()
        out = [t for t in out if q in t.name.lower() or q in t.displayName.lower() or
               q in t.description.lower() or any(q in x.lower() for x in t.tags)]
    return out


# ------------------------------------------------------------------ variables
def resolve_variables(t: Template, values: dict) -> tuple[dict, list[str]]:
    out, errs = {}, []
    for v in t.variables:
        name, typ = v["name"], v.get("type", "string")
        raw = values.get(name)
        if raw in (None, ""):
            if v.get("default") not in (None, ""):
                raw = v["default"]
            elif v.get("required"):
                errs.append(f"{name}: required")
                continue
            else:
                continue
        try:
            if typ == "number":
                val = float(raw)
                val = int(val) if val.is_integer() else val
                if v.get("min") not in (None, "") and val < float(v["min"]):
                    errs.append(f"{name}: must be >= {v['min']}")
                if v.get("max") not in (None, "") and val > float(v["max"]):
                    errs.append(f"{name}: must be <= {v['max']}")
            elif typ == "boolean":
                if isinstance(raw, bool):
                    val = raw
                elif str(raw).lower() in ("true", "1", "yes"):
                    val = True
                elif str(raw).lower() in ("false", "0", "no"):
                    val = False
                else:
                    raise ValueError(f"not a boolean: {raw!r}")
            elif typ == "enum":
                val = str(raw)
                if val not in (v.get("options") or []):
                    errs.append(f"{name}: must be one of {v.get('options')}")
            else:
                val = str(raw)
                if v.get("pattern") and not re.fullmatch(v["pattern"], val):
                    errs.append(f"{name}: does not match {v['pattern']}")
        except ValueError as e:
            errs.append(f"{name}: {e}")
            continue
        out[name] = val
    for k, val in values.items():
        out.setdefault(k, val)
    return out, errs


# ------------------------------------------------------------------ rendering
class TemplateError(ValueError):
    pass


def _truthy(v) -> bool:
    return bool(v) and v != 0


def _to_int(v):
    try:
        return int(float(v))
    except (TypeError, ValueError):
        return 0


FUNCS = {
    "lower": lambda s: str(s).lower(), "upper": lambda s: str(s).upper(),
    "title": lambda s: " ".join(w[:1].upper() + w[1:] for w in str(s).split(" ")),
    "trimSpace": lambda s: str(s).strip(),
    "trimPrefix": lambda p, s: str(s)[len(p):] if str(s).startswith(p) else str(s),
    "trimSuffix": lambda p, s: str(s)[:-len(p)] if p and str(s).endswith(p) else str(s),
    "replace": lambda old, new, s: str(s).replace(old, new),
    "contains": lambda s, sub: sub in str(s), "hasPrefix": lambda s, p: str(s).startswith(p),
    "hasSuffix": lambda s, p: str(s).endswith(p), "split": lambda s, sep: str(s).split(sep),
    "join": lambda sep, xs: sep.join(str(x) for x in xs), "toString": lambda v: _fmt(v),
    "toInt": _to_int, "toFloat": lambda v: float(v or 0),
    "toBool": lambda v: str(v).lower() in ("true", "1", "yes") if not isinstance(v, bool) else v,
    "default": lambda d, v=None: d if v in (None, "") else v,
    "ternary": lambda a, b, c: a if c else b,
    "indent": lambda n, s: " " * int(n) + str(s).replace("\n", "\n" + " " * int(n)),
    "quote": lambda s: json.dumps(str(s)), "eq": lambda a, b: a == b, "ne": lambda a, b: a != b,
    "not": lambda a: not _truthy(a), "and": lambda *a: all(_truthy(x) for x in a),
    "or": lambda *a: next((x for x in a if _truthy(x)), a[-1] if a else None),
}


def _fmt(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "<no value>"
    return str(v)


_TOK = re.compile(r'"(?:[^"\\]|\\.)*"|`[^`]*`|\||\(|\)|[^\s|()]+')


def _eval_arg(tok: str, dot, data: dict):
    if tok.startswith('"'):
        return json.loads(tok)
    if tok.startswith("`"):
        return tok[1:-1]
    if tok == ".":
        return dot
    if tok.startswith("$."):
        tok = tok[1:]
        dot = data
    if tok.startswith("."):
        cur = dot
        for part in tok[1:].split("."):
            cur = cur.get(part) if isinstance(cur, dict) else getattr(cur, part, None)
        return cur
    if tok in ("true", "false"):
        return tok == "true"
    if re.fullmatch(r"-?\d+(\.\d+)?", tok):
        return float(tok) if "." in tok else int(tok)
    if tok in FUNCS:
        return FUNCS[tok]()
    raise TemplateError(f"unknown identifier {tok!r}")


def _eval(expr: str, dot, data: dict):
    toks = _TOK.findall(expr)
    cmds, cur = [], []
    for t in toks:
        if t == "|":
            cmds.append(cur)
            cur = []
        else:
            cur.append(t)
    cmds.append(cur)
    val, first = None, True
    for cmd in cmds:
        if not cmd:
            raise TemplateError(f"empty command in {expr!r}")
        head, args = cmd[0], [_eval_arg(a, dot, data) for a in cmd[1:]]
        if head in FUNCS:
            if not first:
                args.append(val)
            try:
                val = FUNCS[head](*args)
            except TypeError as e:
                raise TemplateError(f"{head}: {e}") from e
        else:
            if not first or cmd[1:]:
                raise TemplateError(f"{head!r} is not a function")
            val = _eval_arg(head, dot, data)
        first = False
    return val


_ACTION = re.compile(r"{{(-?)\s*(.*?)\s*(-?)}}", re.S)


def _parse(src: str):
    """-> nested node list: str | ("expr", e) | ("if", [(cond, body)...], else_body)
    | ("range", e, body, else_body)."""
    pieces = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        if pieces and isinstance(pieces[-1], tuple) and pieces[-1][0] == "trimnext":
            text = text.lstrip()
            pieces.pop()
        pieces.append(text)
        pieces.append(("act", m.group(2).strip()))
        if m.group(3):
            pieces.append(("trimnext",))
        pos = m.end()
    tail = src[pos:]
    if pieces and isinstance(pieces[-1], tuple) and pieces[-1][0] == "trimnext":
        tail = tail.lstrip()
        pieces.pop()
    pieces.append(tail)
    pieces = [p for p in pieces if not (isinstance(p, tuple) and p[0] == "trimnext")]

    def block(i, stops):
        out = []
        while i < len(pieces):
            p = pieces[i]
            if isinstance(p, str):
                out.append(p)
                i += 1
                continue
            a = p[1]
            word = a.split(None, 1)[0] if a else ""
            if word in stops:
                return out, i
            if a.startswith("/*"):
                i += 1
                continue
            if word == "if":
                branches, els = [], []
                cond = a[2:].strip()
                body, i = block(i + 1, ("else", "end"))
                branches.append((cond, body))
                while pieces[i][1].startswith("else"):
                    rest = pieces[i][1][4:].strip()
                    if rest.startswith("if"):
                        body, i = block(i + 1, ("else", "end"))
                        branches.append((rest[2:].strip(), body))
                    else:
                        els, i = block(i + 1, ("end",))
                        break
                out.append(("if", branches, els))
                i += 1
            elif word == "range":
                body, i = block(i + 1, ("else", "end"))
                els = []
                if pieces[i][1] == "else":
                    els, i = block(i + 1, ("end",))
                out.append(("range", a[5:].strip(), body, els))
                i += 1
            else:
                out.append(("expr", a))
                i += 1
        if stops:
            raise TemplateError(f"unterminated block (expected {stops[-1]})")
        return out, i

    try:
        nodes, _ = block(0, ())
    except IndexError as e:
        raise TemplateError("unterminated block") from e
    return nodes


def _exec(nodes, dot, data, out: list):
    for n in nodes:
        if isinstance(n, str):
            out.append(n)
        elif n[0] == "expr":
            out.append(_fmt(_eval(n[1], dot, data)))
        elif n[0] == "if":
            for cond, body in n[1]:
                if _truthy(_eval(cond, dot, data)):
                    _exec(body, dot, data, out)
                    break
            else:
                _exec(n[2], dot, data, out)
        elif n[0] == "range":
            seq = _eval(n[1], dot, data) or []
            items = list(seq.values()) if isinstance(seq, dict) else list(seq)
            if not items:
                _exec(n[3], dot, data, out)
            for x in items:
                _exec(n[2], x, data, out)


def render_string(src: str, variables: dict) -> str:
    out: list = []
    _exec(_parse(src), variables, variables, out)
    return "".join(out)


def render(root: str, t: Template, values: dict) -> dict[str, str]:
    """Rendered files of template ``t`` (relative path -> content); raises
    TemplateError listing every variable violation."""
    variables, errs = resolve_variables(t, values)
    if errs:
        raise TemplateError("; ".join(errs))
    # template.yaml is untrusted: every path it names (and every file a directory
    # walk reaches, symlinks resolved) must stay inside the template directory,
    # which itself must stay inside the source root
    root_real = os.path.realpath(root)
    tdir = os.path.realpath(os.path.join(root_real, t.path))
    if not _inside(tdir, root_real):
        raise TemplateError(f"template path escapes the source root: {t.path}")
    files: dict[str, str] = {}
    for spec in t.files:
        rel = spec["path"]
        src = os.path.realpath(os.path.join(tdir, rel.rstrip("/")))
        if not _inside(src, tdir):
            raise TemplateError(f"template file escapes the template directory: {rel}")
        if os.path.isdir(src):
            for d, _, fs in os.walk(src):
                for fn in fs:
                    p = os.path.realpath(os.path.join(d, fn))
                    if not _inside(p, tdir):
                        raise TemplateError(f"template file escapes the template directory: "
                                            f"{os.path.join(d, fn)}")
                    r = os.path.relpath(p, tdir)
                    with open(p) as f:
                        body = f.read()
                    files[r] = render_string(body, variables) if (
                        spec.get("render", False) and fn.lower().endswith(RENDER_EXT)) else body
        elif os.path.exists(src):
            with open(src) as f:
                body = f.read()
            files[rel] = render_string(body, variables) if spec.get("render") else body
    return files


def _inside(path: str, base: str) -> bool:
    return path == base or path.startswith(base.rstrip(os.sep) + os.sep)


def write_output(files: dict[str, str], out_dir: str) -> None:
    base = os.path.realpath(out_dir)
    for rel, body in files.items():
        dst = os.path.realpath(os.path.join(base, rel))
        if not dst.startswith(base + os.sep):
            raise TemplateError(f"template file escapes the output directory: {rel}")
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, "w") as f:
            f.write(body)
