"""PromptPack skills in the runtime (reference internal/runtime/skills): manifest
parsing (empty / missing / malformed), SKILL.md front matter, activation with
max_active eviction, confined resource reads, and the executor path."""
import asyncio
import json

import pytest

from omnia_amd.runtime import skills as S
from omnia_amd.tools.executor import OmniaExecutor


def _skill(root, name, desc, body, files=None):
    d = root / name
    d.mkdir(parents=True)
    (d / "SKILL.md").write_text(f"---\nname: {name}\ndescription: {desc}\n---\n{body}\n")
    for k, v in (files or {}).items():
        (d / k).write_text(v)
    return d


def test_manifest_edge_cases(tmp_path):
    assert S.read_manifest("").skills == []
    assert S.read_manifest(str(tmp_path / "missing.json")).skills == []
    bad = tmp_path / "bad.json"
    bad.write_text("{not json")
    with pytest.raises(ValueError):
        S.read_manifest(str(bad))


def test_skills_activate_evict_and_resources(tmp_path):
    a = _skill(tmp_path, "refunds", "Process refunds", "Step 1: verify order.",
               {"policy.txt": "30 days"})
    b = _skill(tmp_path, "billing", "Explain invoices", "Read the invoice.")
    c = _skill(tmp_path, "shipping", "Track parcels", "Ask for tracking id.")
    (tmp_path / "secret.txt").write_text("nope")
    man = tmp_path / "manifest.json"
    man.write_text(json.dumps({"version": "1", "config": {"max_active": 2}, "skills": [
        {"mount_as": "billing/refund-processing", "content_path": str(a), "name": "refunds"},
        {"mount_as": "billing/invoices", "content_path": str(b), "name": "billing"},
        {"mount_as": "logistics/shipping", "content_path": str(c), "name": "shipping"}]}))

    async def run():
        ex = OmniaExecutor()
        h = S.attach_skills(ex, str(man))
        await ex.discover()
        assert set(ex.tools) == {"skill__activate", "skill__deactivate", "skill__read_resource"}
        assert "refunds (billing/refund-processing): Process refunds" in \
            ex.tools["skill__activate"].description
        r, err = await ex.execute("skill__activate", {"name": "refunds"})
        assert not err and json.loads(r)["instructions"].startswith("Step 1")
        await ex.execute("skill__activate", {"name": "billing"})
        r, _ = await ex.execute("skill__activate", {"name": "shipping"})
        out = json.loads(r)
        assert out["deactivated"] == ["refunds"] and out["active"] == ["billing", "shipping"]
        r, err = await ex.execute("skill__read_resource", {"name": "refunds",
                                                           "path": "policy.txt"})
        assert not err and json.loads(r)["content"] == "30 days"
        r, err = await ex.execute("skill__read_resource", {"name": "refunds",
                                                           "path": "../secret.txt"})
        assert err and "PermissionError" in r
        r, err = await ex.execute("skill__activate", {"name": "nope"})
        assert err
        assert not ex.is_client_tool("skill__activate")
        assert h.max_active == 2

    asyncio.run(run())


def test_workflow_scoping(tmp_path):
    a = _skill(tmp_path, "refunds", "r", "x")
    b = _skill(tmp_path, "shipping", "s", "y")
    m = S.Manifest(skills=[S.ManifestEntry("billing/refunds", str(a)),
                           S.ManifestEntry("logistics/shipping", str(b))])
    h = S.SkillsHandler(m, workflow_prefix="billing/")
    assert list(h.skills) == ["refunds"]


def test_active_sets_are_per_session(tmp_path):
    """Two conversations activating skills do not evict each other."""
    from omnia_amd.tools.executor import CallContext

    dirs = [_skill(tmp_path, n, n, n) for n in ("a", "b", "c")]
    m = S.Manifest(max_active=1, skills=[S.ManifestEntry(f"x/{d.name}", str(d)) for d in dirs])

    async def run():
        ex = OmniaExecutor()
        ex.add_handler(S.SkillsHandler(m))
        await ex.discover()
        s1, s2 = CallContext(session_id="s1"), CallContext(session_id="s2")
        r, _ = await ex.execute("skill__activate", {"name": "a"}, s1)
        r, _ = await ex.execute("skill__activate", {"name": "b"}, s2)
        assert json.loads(r)["active"] == ["b"] and json.loads(r)["deactivated"] == []
        r, _ = await ex.execute("skill__deactivate", {"name": "c"}, s1)
        assert json.loads(r)["active"] == ["a"]

    asyncio.run(run())


def test_bad_and_duplicate_skills_are_skipped(tmp_path):
    good = _skill(tmp_path, "good", "g", "ok")
    dup = tmp_path / "dup"
    dup.mkdir()
    (dup / "SKILL.md").write_text("---\nname: good\n---\nsecond\n")
    bad = tmp_path / "bad"
    bad.mkdir()
    (bad / "SKILL.md").write_text("---\nname: [unclosed\n---\nx\n")
    lst = tmp_path / "lst"
    lst.mkdir()
    (lst / "SKILL.md").write_text("---\n- a\n- b\n---\nx\n")
    m = S.Manifest(skills=[S.ManifestEntry(f"m/{d.name}", str(d))
                           for d in (good, dup, bad, lst, tmp_path / "missing")])
    h = S.SkillsHandler(m)
    assert list(h.skills) == ["good"] and h.skills["good"].instructions.startswith("ok")
    assert len(h.load_errors) == 4
