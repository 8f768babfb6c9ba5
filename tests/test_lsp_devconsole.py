"""PromptKit LSP (diagnostics, completion, hover, definition, semantic tokens,
WebSocket + stdio JSON-RPC, /api/validate + /api/compile) and the arena dev
console (hot-reloaded agent over WebSocket)."""
import asyncio
import io
import json

import pytest

from omnia_amd.ee import lsp

PROVIDER = """apiVersion: promptkit.altairalabs.ai/v1alpha1
kind: Provider
metadata:
  name: fast
spec:
  id: fast
  type: openai
  model: gpt-4o-mini
"""

ARENA = """apiVersion: promptkit.altairalabs.ai/v1alpha1
kind: Arena
metadata:
  name: smoke
spec:
  providers:
    - file: providers/fast.yaml
    - file: providers/missing.yaml
  defaults:
    temperature: 0.2
"""

PROMPT = """apiVersion: promptkit.altairalabs.ai/v1alpha1
kind: PromptConfig
spec:
  task_type: support
  version: v1.0.0
  description: Support bot
  system_template: "You help {{customer}} politely."
  bogus_field: 1
"""


@pytest.fixture()
def ws(tmp_path):
    (tmp_path / "providers").mkdir()
    (tmp_path / "providers" / "fast.yaml").write_text(PROVIDER)
    return lsp.Workspace(str(tmp_path))


def test_diagnostics(ws):
    assert lsp.validate(PROVIDER, ws) == []
    d = lsp.validate(ARENA, ws)
    assert [x["message"] for x in d] == ["unresolved Provider reference 'providers/missing.yaml'"]
    assert d[0]["range"]["start"]["line"] == 7
    d = lsp.validate(PROMPT, ws)
    assert any("unknown spec field 'bogus_field'" in x["message"] and x["severity"] == 2
               for x in d)
    d = lsp.validate("kind: Provider\nspec:\n  id: x\n  type: nope\n  model: m\n", ws)
    msgs = " ".join(x["message"] for x in d)
    assert "missing required field 'apiVersion'" in msgs and "'nope' is not one of" in msgs
    d = lsp.validate("kind: [unclosed\n")
    assert d[0]["message"].startswith("YAML syntax error")
    assert "unknown kind" in lsp.validate("apiVersion: x\nkind: Widget\nspec: {}\n")[0]["message"]


def test_completion_hover_definition_tokens(ws):
    items = lsp.complete("kind: ", 0, 6, ws)
    assert {"Arena", "Provider", "Tool"} <= {i["label"] for i in items}
    items = lsp.complete(PROMPT + "  \n", 8, 2, ws)
    assert "system_template" in {i["label"] for i in items}
    items = lsp.complete("kind: Provider\nspec:\n  type: ", 2, 8, ws)
    assert "openai" in {i["label"] for i in items}
    items = lsp.complete(ARENA, 6, 6, ws)
    assert "fast" in {i["label"] for i in items}
    h = lsp.hover(PROMPT, 6, 4)
    assert "System prompt template" in h["contents"]["value"]
    assert "required spec" in lsp.hover(PROVIDER, 1, 8)["contents"]["value"]
    loc = lsp.definition(ARENA, 6, 12, ws)
    assert loc["uri"].endswith("providers/fast.yaml")
    toks = lsp.semantic_tokens(PROMPT)
    assert len(toks) % 5 == 0 and 2 in toks[3::5]  # a {{variable}} token


def test_compile_pack():
    tool = ("apiVersion: x\nkind: Tool\nspec:\n  name: lookup\n  description: d\n"
            "  input_schema: {type: object}\n  output_schema: {type: object}\n  mode: mock\n"
            "  timeout_ms: 100\n")
    out = lsp.compile_pack({"p.yaml": PROMPT, "t.yaml": tool, "bad.yaml": "kind: [\n"})
    assert out["pack"]["prompts"]["support"]["system_template"].startswith("You help")
    assert out["pack"]["tools"]["lookup"]["parameters"] == {"type": "object"}
    assert [e["file"] for e in out["errors"]] == ["bad.yaml"]


def test_websocket_session(ws):
    from aiohttp.test_utils import TestClient, TestServer

    async def run():
        c = TestClient(TestServer(lsp.build_app(str(ws.root))))
        await c.start_server()
        try:
            sock = await c.ws_connect("/lsp")
            await sock.send_json({"jsonrpc": "2.0", "id": 1, "method": "initialize",
                                  "params": {}})
            init = await sock.receive_json()
            assert init["result"]["capabilities"]["hoverProvider"]
            await sock.send_json({"jsonrpc": "2.0", "method": "textDocument/didOpen", "params": {
                "textDocument": {"uri": "file:///a.yaml", "text": ARENA}}})
            diag = await sock.receive_json()
            assert diag["method"] == "textDocument/publishDiagnostics"
            assert len(diag["params"]["diagnostics"]) == 1
            await sock.send_json({"jsonrpc": "2.0", "id": 2, "method": "nope"})
            assert (await sock.receive_json())["error"]["code"] == -32601
            r = await c.post("/api/validate", json={"content": PROMPT})
            assert (await r.json())["diagnostics"]
            await sock.close()
        finally:
            await c.close()

    asyncio.run(run())


def test_stdio_framing(ws):
    def frame(m):
        b = json.dumps(m).encode()
        return b"Content-Length: %d\r\n\r\n" % len(b) + b

    inp = io.BytesIO(frame({"jsonrpc": "2.0", "id": 1, "method": "initialize", "params": {}})
                     + frame({"jsonrpc": "2.0", "method": "textDocument/didOpen", "params": {
                         "textDocument": {"uri": "u", "text": PROVIDER}}})
                     + frame({"jsonrpc": "2.0", "method": "exit"}))
    out = io.BytesIO()
    asyncio.run(lsp.serve_stdio(str(ws.root), inp, out))
    raw = out.getvalue()
    assert raw.count(b"Content-Length:") == 2 and b"publishDiagnostics" in raw


def test_dev_console_hot_reload():
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.ee.dev_console import DevConsole, build_app

    con = DevConsole()

    async def run():
        c = TestClient(TestServer(build_app(con)))
        await c.start_server()
        try:
            sock = await c.ws_connect("/ws")
            await sock.send_json({"type": "config", "provider": {
                "type": "mock", "mock": {"scenarios": {"default_response": "first version"}}}})
            assert (await sock.receive_json())["type"] == "configured"
            await sock.send_json({"type": "message", "content": "hi", "session_id": "d1"})
            frames = []
            while True:
                f = await sock.receive_json()
                frames.append(f)
                if f["type"] in ("done", "error"):
                    break
            assert frames[-1]["content"] == "first version"
            await sock.send_json({"type": "reload", "provider": {
                "type": "mock", "mock": {"scenarios": {"default_response": "second version"}}}})
            assert (await sock.receive_json())["type"] == "configured"
            await sock.send_json({"type": "message", "content": "again", "session_id": "d1"})
            while True:
                f = await sock.receive_json()
                if f["type"] in ("done", "error"):
                    break
            assert f["type"] == "done" and f["content"] == "second version"
            await sock.send_json({"type": "wat"})
            assert (await sock.receive_json())["type"] == "error"
            await sock.close()
        finally:
            await c.close()

    asyncio.run(run())
    assert con.reloads == 1
    hist = asyncio.run(con.store.load("d1"))
    roles = [m["role"] for m in hist["messages"]]
    assert roles.count("user") == 2 and roles.count("assistant") == 2  # kept across reload
