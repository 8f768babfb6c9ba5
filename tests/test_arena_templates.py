"""Arena project templates (``ee/pkg/arena/template/*_test.go``,
``arenatemplatesource_controller_test.go``): discovery from template.yaml /
the index file, variable validation and defaults, the Go text/template subset
renderer, path confinement, and the ArenaTemplateSource reconciler publishing
the template index."""
import json
import os

import pytest

from omnia_amd.ee.arena import templates as T
from omnia_amd.operator.apistore import APIStore, get_condition
from omnia_amd.operator.sourcesync import SourceReconciler

TEMPLATE = """apiVersion: arena.omnia.altairalabs.ai/v1alpha1
kind: ArenaTemplate
metadata:
  name: chatbot
  version: 1.2.0
spec:
  displayName: Chat bot
  description: A customer support bot
  category: support
  tags: [chat, starter]
  variables:
    - {name: projectName, type: string, required: true, pattern: "[a-z][a-z0-9-]*"}
    - {name: temperature, type: number, default: "0.7", min: "0", max: "2"}
    - {name: streaming, type: boolean, default: "true"}
    - {name: tier, type: enum, options: [basic, pro], default: basic}
"""


def _tree(root):
    t = root / "templates" / "chatbot"
    (t / "prompts").mkdir(parents=True)
    (t / "template.yaml").write_text(TEMPLATE)
    (t / "config.arena.yaml").write_text(
        "name: {{ .projectName }}\n"
        "title: {{ .projectName | replace \"-\" \" \" | title }}\n"
        "temperature: {{ .temperature }}\n"
        "{{- if .streaming }}\nstreaming: true{{ else }}\nstreaming: false{{ end }}\n"
        "{{ if eq .tier \"pro\" }}tier: PRO{{ else if eq .tier \"basic\" }}tier: basic"
        "{{ end }}\n"
        "tags:{{ range .tags }}\n  - {{ . | upper }}{{ else }} []{{ end }}\n"
        "owner: {{ default \"nobody\" .owner }}\n")
    (t / "prompts" / "system.md").write_text("You help {{ .projectName }} users.\n")
    (t / "logo.png").write_text("{{ not rendered }}")
    bad = root / "templates" / "broken"
    bad.mkdir()
    (bad / "template.yaml").write_text("metadata: {}\n")
    return root


def test_discover_and_defaults(tmp_path):
    ts = T.discover(str(_tree(tmp_path)))
    assert [t.name for t in ts] == ["chatbot"]  # the broken one is skipped
    t = ts[0]
    assert t.version == "1.2.0" and t.category == "support" and t.path == "templates/chatbot"
    files = {f["path"]: f["render"] for f in t.files}
    assert files == {"config.arena.yaml": True, "logo.png": False, "prompts/": False}
    assert T.filter_templates(ts, category="support", tags=["chat"], query="SUPPORT") == ts
    assert T.filter_templates(ts, category="other") == []


def test_index_file_takes_precedence(tmp_path):
    (tmp_path / ".template-index.yaml").write_text(
        "templates:\n  - {name: a, path: x, category: c}\n  - {name: b, displayName: B}\n")
    ts = T.discover(str(tmp_path))
    assert [(t.name, t.displayName) for t in ts] == [("a", "a"), ("b", "B")]


def test_variables_validate_and_default(tmp_path):
    t = T.discover(str(_tree(tmp_path)))[0]
    vals, errs = T.resolve_variables(t, {"projectName": "my-bot"})
    assert not errs and vals["temperature"] == 0.7 and vals["streaming"] is True
    assert vals["tier"] == "basic"
    _, errs = T.resolve_variables(t, {"temperature": "3", "streaming": "maybe",
                                      "tier": "gold", "projectName": "Bad Name"})
    joined = "; ".join(errs)
    for needle in ("temperature: must be <= 2", "streaming: not a boolean",
                   "tier: must be one of", "projectName: does not match"):
        assert needle in joined, joined
    _, errs = T.resolve_variables(t, {})
    assert errs == ["projectName: required"]


def test_render_go_template_subset(tmp_path):
    root = _tree(tmp_path)
    t = T.discover(str(root))[0]
    files = T.render(str(root), t, {"projectName": "acme-help", "tier": "pro",
                                    "tags": ["a", "b"]})
    cfg = files["config.arena.yaml"]
    assert "name: acme-help\n" in cfg and "title: Acme Help\n" in cfg
    assert "temperature: 0.7\nstreaming: true\n" in cfg and "tier: PRO" in cfg
    assert "tags:\n  - A\n  - B\n" in cfg and "owner: nobody" in cfg
    assert files["logo.png"] == "{{ not rendered }}"
    # directories are copied unrendered unless marked render
    assert files["prompts/system.md"] == "You help {{ .projectName }} users.\n"
    out = tmp_path / "out"
    T.write_output(files, str(out))
    assert (out / "prompts" / "system.md").exists()
    with pytest.raises(T.TemplateError):
        T.write_output({"../escape.txt": "x"}, str(out))
    with pytest.raises(T.TemplateError, match="required"):
        T.render(str(root), t, {})


def test_render_confines_reads_to_the_template(tmp_path):
    """template.yaml is untrusted: absolute / '..' file paths, a template path
    outside the source root, and symlinks out of the template are refused."""
    import dataclasses

    root = _tree(tmp_path / "src")
    secret = tmp_path / "secret.txt"
    secret.write_text("top secret")
    t = T.discover(str(root))[0]
    ok = {"projectName": "x"}
    for bad in ("../../../secret.txt", str(secret)):
        evil = dataclasses.replace(t, files=[{"path": bad, "render": False}])
        with pytest.raises(T.TemplateError, match="escapes"):
            T.render(str(root), evil, ok)
    with pytest.raises(T.TemplateError, match="escapes"):
        T.render(str(root), dataclasses.replace(t, path="../.."), ok)
    (root / "templates" / "chatbot" / "prompts" / "leak.md").symlink_to(secret)
    with pytest.raises(T.TemplateError, match="escapes"):
        T.render(str(root), t, ok)


def test_render_string_edge_cases():
    r = T.render_string
    assert r("{{ .a.b }}", {"a": {"b": 3}}) == "3"
    assert r("{{ if and .x .y }}both{{ end }}", {"x": 1, "y": 0}) == ""
    assert r("{{ ternary \"y\" \"n\" .f }}", {"f": True}) == "y"
    assert r("{{ .s | trimSpace | quote }}", {"s": "  hi "}) == '"hi"'
    assert r("a {{- /* c */ -}} b", {}) == "ab"
    assert r("{{ join \",\" .xs }}", {"xs": [1, 2]}) == "1,2"
    with pytest.raises(T.TemplateError):
        r("{{ if .x }}open", {"x": 1})
    with pytest.raises(T.TemplateError):
        r("{{ nosuchfn .x }}", {"x": 1})


def test_arena_template_source_reconciler_publishes_index(tmp_path):
    root = _tree(tmp_path / "src")
    store = APIStore()
    # a local-path source (single-node mode); the CRD admits git / oci / configmap
    store.objs[store.key("ArenaTemplateSource", "default", "starter")] = {
        "apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "ArenaTemplateSource",
        "metadata": {"name": "starter", "namespace": "default", "generation": 1,
                     "resourceVersion": "1", "uid": "u"},
        "spec": {"type": "workspace", "workspace": {"path": str(root)},
                 "syncInterval": "10m", "templatesPath": "templates/"}}
    rec = SourceReconciler("ArenaTemplateSource", root=str(tmp_path / "content"))
    assert rec.reconcile(store, "default", "starter") == 600.0
    st = store.get("ArenaTemplateSource", "starter", "default")["status"]
    assert st["phase"] == "Ready" and st["templateCount"] == 1
    obj = {"status": st}
    assert get_condition(obj, "TemplatesScanned")["status"] == "True"
    assert get_condition(obj, "ArtifactAvailable")["status"] == "True"
    idx = json.loads(open(st["templateIndex"]).read())
    assert idx[0]["name"] == "chatbot" and idx[0]["tags"] == ["chat", "starter"]
    assert os.path.dirname(st["templateIndex"]).endswith(".arena/template-index")
