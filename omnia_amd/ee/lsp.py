"""PromptKit language server (reference ``ee/cmd/promptkit-lsp``).

LSP over JSON-RPC for the PromptKit/Arena config files (kinds Arena,
PromptConfig, Provider, Tool, Scenario, Persona, Eval), served two ways like
the reference: a WebSocket endpoint (``/lsp``, the dashboard editor proxies to
it) and stdio with ``Content-Length`` framing (editors).  Plus the HTTP helper
API: ``POST /api/validate`` and ``POST /api/compile``.

Capabilities implemented:
* ``textDocument/publishDiagnostics`` on didOpen/didChange: YAML syntax errors
  at their line/column, missing ``apiVersion``/``kind``/``spec``, unknown kind,
  per-kind required ``spec`` fields and unknown fields (warnings), enum values
  (provider ``type``, tool ``mode``), and references (``tools:``, ``providers:``
  ``prompt_configs:`` file refs) that do not resolve in the workspace;
* ``textDocument/completion``: top-level keys, kind values, per-kind spec
  fields, provider types, and reference names found in the workspace;
* ``textDocument/hover``: field documentation and kind / provider-type docs;
* ``textDocument/definition``: jump from a reference to the defining file;
* ``textDocument/semanticTokens/full``: keys, kind values, template variables
  (``{{var}}``) for highlighting.
The workspace is a directory (``--root``); a document's references resolve
against files under it.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import re
import sys
from pathlib import Path

import yaml

API_VERSION = "promptkit.altairalabs.ai/v1alpha1"

KIND_SPECS = {
    "Arena": {
        "required": ["providers", "defaults"],
        "fields": {
            "prompt_configs": "Prompt configurations under test (file refs).",
            "providers": "Providers to run scenarios against (file refs).",
            "judges": "LLM judges for evaluation.", "judge_defaults": "Judge defaults.",
            "scenarios": "Scenario files to execute.", "evals": "Eval definitions.",
            "tools": "Tool definitions (file refs).", "mcp_servers": "MCP servers to mount.",
            "state_store": "Conversation state store.", "defaults": "Run defaults "
            "(temperature, max_tokens, concurrency, output).",
            "self_play": "Self-play (persona-driven user simulation) settings."}},
    "PromptConfig": {
        "required": ["task_type", "version", "description", "system_template"],
        "fields": {
            "task_type": "Task identifier the prompt serves.", "version": "Semver of the prompt.",
            "description": "Human description.", "template_engine": "Template engine config.",
            "fragments": "Reusable template fragments.",
            "system_template": "System prompt template; {{variables}} are substituted.",
            "variables": "Declared template variables.", "model_overrides": "Per-model tweaks.",
            "allowed_tools": "Tool names the prompt may call.", "media": "Media settings.",
            "validators": "Output validators.", "tested_models": "Models it was tested with.",
            "metadata": "Free-form metadata.", "compilation": "Compilation info."}},
    "Provider": {
        "required": ["id", "type", "model"],
        "fields": {
            "id": "Provider id referenced by arenas and scenarios.", "type": "Provider type.",
            "model": "Model name.", "base_url": "Endpoint override.",
            "rate_limit": "Requests/tokens per second.", "defaults": "Sampling defaults.",
            "pricing": "Per-1K token prices.", "pricing_correct_at": "Pricing date.",
            "include_raw_output": "Keep raw provider output.",
            "additional_config": "Provider-specific settings.",
            "credential": "Credential reference.", "platform": "bedrock / vertex / azure.",
            "capabilities": "Capabilities (tools, vision, audio, ...)."}},
    "Tool": {
        "required": ["name", "description", "input_schema", "output_schema", "mode",
                     "timeout_ms"],
        "fields": {
            "name": "Tool name the model calls.", "description": "What the tool does.",
            "input_schema": "JSON Schema of the arguments.",
            "output_schema": "JSON Schema of the result.",
            "mode": "mock | live", "timeout_ms": "Call timeout in milliseconds.",
            "mock_result": "Static mock result.", "mock_template": "Templated mock result.",
            "http": "Live HTTP binding."}},
    "Scenario": {
        "required": ["id", "task_type", "description", "turns"],
        "fields": {
            "id": "Scenario id.", "task_type": "PromptConfig task_type to run.",
            "mode": "Scenario mode.", "description": "What is exercised.",
            "context_metadata": "Metadata passed to the prompt.",
            "turns": "Conversation turns (role/content/assertions).",
            "context": "Context variables.", "constraints": "Run constraints.",
            "tool_policy": "Tool policy override.", "providers": "Providers to run on.",
            "provider_group": "Provider group.", "required_capabilities": "Needed capabilities.",
            "streaming": "Stream responses.", "context_policy": "Context window policy.",
            "conversation_assertions": "Whole-conversation assertions.",
            "duplex": "Duplex (voice) settings."}},
    "Persona": {
        "required": ["id", "description", "goals", "constraints", "style", "defaults"],
        "fields": {
            "id": "Persona id.", "description": "Who the simulated user is.",
            "prompt_activity": "Activity prompt.", "fragments": "Template fragments.",
            "system_template": "Persona system template.", "required_vars": "Required vars.",
            "optional_vars": "Optional vars.", "system_prompt": "Literal system prompt.",
            "goals": "What the persona tries to achieve.", "constraints": "Behaviour limits.",
            "style": "Tone / verbosity.", "defaults": "Sampling defaults."}},
    "Eval": {
        "required": ["id", "description", "recording"],
        "fields": {
            "id": "Eval id.", "description": "What is evaluated.",
            "recording": "Recorded session to replay.", "turns": "Turn assertions.",
            "conversation_assertions": "Conversation assertions.", "tags": "Tags.",
            "mode": "Replay mode.", "speed": "Replay speed."}},
}
ENUMS = {
    ("Provider", "type"): ["claude", "openai", "gemini", "ollama", "vllm", "mock", "local",
                           "voyageai", "azure", "bedrock", "vertex"],
    ("Tool", "mode"): ["mock", "live"],
}
REF_KEYS = {"tools": "Tool", "providers": "Provider", "prompt_configs": "PromptConfig",
            "scenarios": "Scenario", "personas": "Persona", "evals": "Eval"}
TOP_KEYS = {"apiVersion": "Schema version: " + API_VERSION, "kind": "Document kind.",
            "metadata": "name / labels.", "spec": "Kind-specific configuration."}

SEV_ERROR, SEV_WARNING = 1, 2
TOKEN_TYPES = ["property", "type", "variable", "string"]


def _diag(line, col, msg, sev=SEV_ERROR, end=None):
    return {"range": {"start": {"line": line, "character": col},
                      "end": {"line": line, "character": end if end is not None else col + 1}},
            "severity": sev, "source": "promptkit", "message": msg}


def _key_line(text: str, key: str, indent: int | None = None) -> tuple[int, int]:
    pat = re.compile(r"^(\s*)" + re.escape(key) + r"\s*:")
    for i, ln in enumerate(text.splitlines()):
        m = pat.match(ln)
        if m and (indent is None or len(m.group(1)) == indent):
            return i, len(m.group(1))
    return 0, 0


class Workspace:
    def __init__(self, root: str | None):
        self.root = Path(root) if root else None

    def index(self) -> dict[str, dict[str, str]]:
        """kind -> {name/id: path} for every parseable config under root."""
        out: dict[str, dict[str, str]] = {}
        if self.root is None or not self.root.exists():
            return out
        for p in self.root.rglob("*"):
            if p.suffix not in (".yaml", ".yml", ".json") or not p.is_file():
                continue
            try:
                d = yaml.safe_load(p.read_text())
            except Exception:  # noqa: BLE001
                continue
            if not isinstance(d, dict) or "kind" not in d:
                continue
            spec = d.get("spec") or {}
            name = (d.get("metadata") or {}).get("name") or spec.get("id") or spec.get("name")
            out.setdefault(d["kind"], {})
            rel = str(p.relative_to(self.root))
            out[d["kind"]][rel] = rel
            if name:
                out[d["kind"]][str(name)] = rel
        return out


def validate(text: str, ws: Workspace | None = None) -> list[dict]:
    diags: list[dict] = []
    try:
        doc = yaml.safe_load(text)
    except yaml.YAMLError as e:
        mark = getattr(e, "problem_mark", None)
        return [_diag(mark.line if mark else 0, mark.column if mark else 0,
                      f"YAML syntax error: {getattr(e, 'problem', e)}")]
    if doc is None:
        return [_diag(0, 0, "empty document", SEV_WARNING)]
    if not isinstance(doc, dict):
        return [_diag(0, 0, "document must be a mapping")]
    for k in ("apiVersion", "kind", "spec"):
        if k not in doc:
            diags.append(_diag(0, 0, f"missing required field '{k}'"))
    kind = doc.get("kind")
    if kind is not None and kind not in KIND_SPECS:
        ln, col = _key_line(text, "kind", 0)
        diags.append(_diag(ln, col, f"unknown kind '{kind}' (expected one of "
                                    f"{', '.join(KIND_SPECS)})", end=col + 4))
    spec = doc.get("spec")
    if kind in KIND_SPECS and isinstance(spec, dict):
        ks = KIND_SPECS[kind]
        sl, _ = _key_line(text, "spec", 0)
        for req in ks["required"]:
            if req not in spec:
                diags.append(_diag(sl, 0, f"{kind}: missing required spec field '{req}'",
                                   end=4))
        for k, v in spec.items():
            ln, col = _key_line(text, k)
            if k not in ks["fields"]:
                diags.append(_diag(ln, col, f"{kind}: unknown spec field '{k}'", SEV_WARNING,
                                   end=col + len(k)))
            allowed = ENUMS.get((kind, k))
            if allowed and v not in allowed:
                diags.append(_diag(ln, col, f"{kind}.{k}: '{v}' is not one of "
                                            f"{', '.join(allowed)}", end=col + len(k)))
        if ws is not None and ws.root is not None:
            idx = ws.index()
            for key, rkind in REF_KEYS.items():
                refs = spec.get(key)
                if not isinstance(refs, list):
                    continue
                for r in refs:
                    name = r.get("file") or r.get("ref") or r.get("id") if isinstance(r, dict) \
                        else r
                    if isinstance(name, str) and name not in idx.get(rkind, {}):
                        ln, col = _find_value(text, name)
                        diags.append(_diag(ln, col, f"unresolved {rkind} reference '{name}'",
                                           SEV_WARNING, end=col + len(name)))
    return diags


def _find_value(text: str, value: str) -> tuple[int, int]:
    for i, ln in enumerate(text.splitlines()):
        j = ln.find(value)
        if j >= 0:
            return i, j
    return 0, 0


def _doc_kind(text: str) -> str | None:
    m = re.search(r"^kind:\s*(\w+)", text, re.M)
    return m.group(1) if m else None


def _line_context(text: str, line: int) -> tuple[str, int, str | None]:
    """(current line, indentation, enclosing top-level key)."""
    lines = text.splitlines()
    cur = lines[line] if line < len(lines) else ""
    ind = len(cur) - len(cur.lstrip())
    parent = None
    for j in range(min(line, len(lines) - 1), -1, -1):
        m = re.match(r"^(\s*)([A-Za-z_]+)\s*:", lines[j])
        if m and len(m.group(1)) < ind:
            parent = m.group(2)
            break
    return cur, ind, parent


def complete(text: str, line: int, char: int, ws: Workspace | None = None) -> list[dict]:
    cur, ind, parent = _line_context(text, line)
    prefix = cur[:char]
    kind = _doc_kind(text)
    items = []
    if re.match(r"^\s*kind:\s*\w*$", prefix):
        return [{"label": k, "kind": 13, "detail": "PromptKit kind"} for k in KIND_SPECS]
    m = re.match(r"^\s*type:\s*\w*$", prefix)
    if m and kind == "Provider":
        return [{"label": t, "kind": 13} for t in ENUMS[("Provider", "type")]]
    if parent in REF_KEYS and ws is not None:
        idx = ws.index().get(REF_KEYS[parent], {})
        return [{"label": n, "kind": 18, "detail": f"{REF_KEYS[parent]} -> {p}"}
                for n, p in sorted(idx.items())]
    if ind == 0:
        return [{"label": k, "kind": 10, "documentation": d} for k, d in TOP_KEYS.items()]
    if parent == "spec" and kind in KIND_SPECS:
        for k, d in KIND_SPECS[kind]["fields"].items():
            items.append({"label": k, "kind": 10, "documentation": d,
                          "detail": "required" if k in KIND_SPECS[kind]["required"] else ""})
    return items


def hover(text: str, line: int, char: int) -> dict | None:
    lines = text.splitlines()
    if line >= len(lines):
        return None
    ln = lines[line]
    m = re.match(r"^(\s*)([A-Za-z_]+)\s*:\s*(.*)$", ln)
    if not m:
        return None
    key, val = m.group(2), m.group(3).strip()
    kind = _doc_kind(text)
    key_end = len(m.group(1)) + len(key)
    if char > key_end and key == "kind" and val in KIND_SPECS:
        req = ", ".join(KIND_SPECS[val]["required"])
        return {"contents": {"kind": "markdown", "value": f"**{val}** — required spec: {req}"}}
    if char > key_end and key == "type" and kind == "Provider":
        return {"contents": {"kind": "markdown", "value": f"Provider type **{val}**"}}
    doc = TOP_KEYS.get(key) if not m.group(1) else \
        (KIND_SPECS.get(kind, {}).get("fields", {}).get(key))
    if doc is None:
        return None
    return {"contents": {"kind": "markdown", "value": f"**{key}** — {doc}"},
            "range": {"start": {"line": line, "character": len(m.group(1))},
                      "end": {"line": line, "character": key_end}}}


def definition(text: str, line: int, char: int, ws: Workspace | None, uri_base: str = "file://"):
    if ws is None or ws.root is None:
        return None
    _, _, parent = _line_context(text, line)
    if parent not in REF_KEYS:
        return None
    ln = text.splitlines()[line]
    m = re.search(r"(?:-\s*)?(?:(?:file|ref|id):\s*)?([\w./-]+)\s*$", ln)
    if not m:
        return None
    target = ws.index().get(REF_KEYS[parent], {}).get(m.group(1))
    if not target:
        return None
    return {"uri": uri_base + str((ws.root / target).resolve()),
            "range": {"start": {"line": 0, "character": 0}, "end": {"line": 0, "character": 0}}}


def semantic_tokens(text: str) -> list[int]:
    """LSP relative-encoded tokens: [dLine, dStart, len, type, mods]*."""
    toks = []
    for i, ln in enumerate(text.splitlines()):
        m = re.match(r"^(\s*-?\s*)([A-Za-z_][\w]*)\s*:", ln)
        if m:
            toks.append((i, len(m.group(1)), len(m.group(2)), 0))
            km = re.match(r"^kind:\s*(\w+)", ln)
            if km:
                toks.append((i, ln.index(km.group(1), 5), len(km.group(1)), 1))
        for vm in re.finditer(r"\{\{\s*[\w.]+\s*\}\}", ln):
            toks.append((i, vm.start(), vm.end() - vm.start(), 2))
    toks.sort()
    out, pl, ps = [], 0, 0
    for line, start, length, typ in toks:
        dl = line - pl
        out += [dl, start - (ps if dl == 0 else 0), length, typ, 0]
        pl, ps = line, start
    return out


def compile_pack(files: dict[str, str]) -> dict:
    """Compile PromptConfig documents into a pack.json-shaped dict (the
    reference's ``/api/compile``): prompts keyed by task_type, tools merged."""
    pack = {"id": "compiled", "version": "v1.0.0", "prompts": {}, "tools": {}}
    errors = []
    for path, text in files.items():
        diags = [d for d in validate(text) if d["severity"] == SEV_ERROR]
        if diags:
            errors += [{"file": path, **d} for d in diags]
            continue
        d = yaml.safe_load(text)
        spec = d.get("spec") or {}
        if d.get("kind") == "PromptConfig":
            pack["prompts"][spec["task_type"]] = {
                "id": spec["task_type"], "version": spec.get("version"),
                "system_template": spec["system_template"],
                "variables": spec.get("variables", []),
                "tools": spec.get("allowed_tools", []),
                "validators": spec.get("validators", [])}
        elif d.get("kind") == "Tool":
            pack["tools"][spec["name"]] = {"name": spec["name"],
                                           "description": spec["description"],
                                           "parameters": spec.get("input_schema", {})}
    return {"pack": pack, "errors": errors}


# ------------------------------------------------------------------ JSON-RPC session
class LSPSession:
    def __init__(self, ws: Workspace, send):
        self.ws = ws
        self.send = send  # async (dict) -> None
        self.docs: dict[str, str] = {}
        self.shutdown = False

    async def publish(self, uri: str):
        await self.send({"jsonrpc": "2.0", "method": "textDocument/publishDiagnostics",
                         "params": {"uri": uri, "diagnostics": validate(self.docs[uri],
                                                                        self.ws)}})

    async def handle(self, msg: dict) -> None:
        method, mid, p = msg.get("method"), msg.get("id"), msg.get("params") or {}

        async def reply(result=None, error=None):
            if mid is None:
                return
            body = {"jsonrpc": "2.0", "id": mid}
            body["error" if error else "result"] = error or result
            await self.send(body)

        td = p.get("textDocument") or {}
        uri = td.get("uri")
        pos = p.get("position") or {}
        if method == "initialize":
            await reply({"capabilities": {
                "textDocumentSync": 1, "hoverProvider": True, "definitionProvider": True,
                "completionProvider": {"triggerCharacters": [":", " ", "-"]},
                "semanticTokensProvider": {"legend": {"tokenTypes": TOKEN_TYPES,
                                                      "tokenModifiers": []}, "full": True}},
                "serverInfo": {"name": "omnia-promptkit-lsp", "version": "0.1.0"}})
        elif method == "initialized":
            return
        elif method == "shutdown":
            self.shutdown = True
            await reply(None)
        elif method == "textDocument/didOpen":
            self.docs[uri] = td.get("text", "")
            await self.publish(uri)
        elif method == "textDocument/didChange":
            changes = p.get("contentChanges") or []
            if changes:
                self.docs[uri] = changes[-1].get("text", "")  # full sync
            await self.publish(uri)
        elif method == "textDocument/didClose":
            self.docs.pop(uri, None)
            await self.send({"jsonrpc": "2.0", "method": "textDocument/publishDiagnostics",
                             "params": {"uri": uri, "diagnostics": []}})
        elif method == "textDocument/completion":
            await reply({"isIncomplete": False, "items": complete(
                self.docs.get(uri, ""), pos.get("line", 0), pos.get("character", 0), self.ws)})
        elif method == "textDocument/hover":
            await reply(hover(self.docs.get(uri, ""), pos.get("line", 0),
                              pos.get("character", 0)))
        elif method == "textDocument/definition":
            await reply(definition(self.docs.get(uri, ""), pos.get("line", 0),
                                   pos.get("character", 0), self.ws))
        elif method == "textDocument/semanticTokens/full":
            await reply({"data": semantic_tokens(self.docs.get(uri, ""))})
        elif mid is not None:
            await reply(error={"code": -32601, "message": f"method not found: {method}"})


def build_app(root: str | None = None):
    from aiohttp import WSMsgType, web

    ws_root = Workspace(root)
    app = web.Application()

    async def lsp(request):
        sock = web.WebSocketResponse()
        await sock.prepare(request)
        sess = LSPSession(ws_root, lambda m: sock.send_str(json.dumps(m)))
        async for m in sock:
            if m.type != WSMsgType.TEXT:
                break
            try:
                await sess.handle(json.loads(m.data))
            except json.JSONDecodeError:
                await sock.send_str(json.dumps({"jsonrpc": "2.0", "id": None, "error": {
                    "code": -32700, "message": "parse error"}}))
            if sess.shutdown and sock.closed:
                break
        return sock

    async def api_validate(request):
        body = await request.json()
        return web.json_response({"diagnostics": validate(body.get("content", ""), ws_root)})

    async def api_compile(request):
        body = await request.json()
        return web.json_response(compile_pack(body.get("files") or {}))

    async def healthz(_):
        return web.json_response({"status": "ok"})

    app.router.add_get("/lsp", lsp)
    app.router.add_post("/api/validate", api_validate)
    app.router.add_post("/api/compile", api_compile)
    app.router.add_get("/healthz", healthz)
    return app


async def serve_stdio(root: str | None, rfile=None, wfile=None) -> None:
    """``Content-Length``-framed JSON-RPC over stdio (editor integration)."""
    rfile = rfile or sys.stdin.buffer
    wfile = wfile or sys.stdout.buffer

    async def send(m):
        body = json.dumps(m).encode()
        wfile.write(b"Content-Length: %d\r\n\r\n" % len(body) + body)
        wfile.flush()

    sess = LSPSession(Workspace(root), send)
    loop = asyncio.get_running_loop()
    while True:
        hdr = {}
        while True:
            line = await loop.run_in_executor(None, rfile.readline)
            if not line:
                return
            line = line.strip()
            if not line:
                break
            k, _, v = line.decode().partition(":")
            hdr[k.lower()] = v.strip()
        n = int(hdr.get("content-length", 0))
        body = await loop.run_in_executor(None, rfile.read, n)
        msg = json.loads(body)
        await sess.handle(msg)
        if msg.get("method") == "exit":
            return


def main(argv=None):
    ap = argparse.ArgumentParser("promptkit-lsp")
    ap.add_argument("--root", default=os.getcwd())
    ap.add_argument("--port", type=int, default=8085)
    ap.add_argument("--stdio", action="store_true")
    a = ap.parse_args(argv)
    if a.stdio:
        asyncio.run(serve_stdio(a.root))
        return
    from aiohttp import web

    web.run_app(build_app(a.root), port=a.port)


if __name__ == "__main__":
    main()
