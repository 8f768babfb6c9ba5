"""Source sync: git (local repo via the git CLI, branch + commit pinning + sub-path),
ConfigMap and workspace sources, atomic `current` link, history GC, reconciler
status, PromptPackSource publishing."""
import subprocess

import pytest

from omnia_amd.operator.apistore import APIStore
from omnia_amd.operator.sourcesync import SourceReconciler, SourceSyncer, parse_duration


def _git(*a, cwd):
    subprocess.run(["git", *a], cwd=cwd, check=True, capture_output=True,
                   env={"GIT_AUTHOR_NAME": "t", "GIT_AUTHOR_EMAIL": "t@x", "GIT_COMMITTER_NAME": "t",
                        "GIT_COMMITTER_EMAIL": "t@x", "PATH": "/usr/bin:/bin"})


@pytest.fixture
def repo(tmp_path):
    r = tmp_path / "src"
    (r / "skills" / "greet").mkdir(parents=True)
    (r / "skills" / "greet" / "SKILL.md").write_text("# greet\n")
    (r / "README.md").write_text("root")
    _git("init", "-q", "-b", "main", cwd=r)
    _git("add", "-A", cwd=r)
    _git("commit", "-q", "-m", "one", cwd=r)
    return r


def test_parse_duration():
    assert parse_duration("1h30m") == 5400 and parse_duration("45s") == 45
    assert parse_duration(None, 7) == 7


def test_git_skillsource_reconcile_and_revisions(tmp_path, repo):
    store = APIStore()
    store.create({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "SkillSource",
                  "metadata": {"name": "sk", "namespace": "default"},
                  "spec": {"type": "git", "interval": "5m",
                           "git": {"url": "file://" + str(repo), "ref": {"branch": "main"},
                                   "path": "skills"}}})
    rec = SourceReconciler("SkillSource", str(tmp_path / "content"))
    assert rec.reconcile(store, "default", "sk") == 300
    st = store.get("SkillSource", "sk", "default")["status"]
    assert st["phase"] == "Ready" and st["skillCount"] == 1
    rev1 = st["artifact"]["revision"]
    (repo / "skills" / "bye").mkdir()
    (repo / "skills" / "bye" / "SKILL.md").write_text("# bye\n")
    _git("add", "-A", cwd=repo)
    _git("commit", "-q", "-m", "two", cwd=repo)
    rec.reconcile(store, "default", "sk")
    st = store.get("SkillSource", "sk", "default")["status"]
    assert st["artifact"]["revision"] != rev1 and st["skillCount"] == 2
    cur = tmp_path / "content" / "default" / "skillsource" / "sk" / "current"
    assert cur.is_symlink() and (cur / "skills").exists() is False  # path applied
    # pin the first commit
    o = store.get("SkillSource", "sk", "default")
    o["spec"]["git"]["ref"] = {"commit": rev1}
    store.update(o)
    rec.reconcile(store, "default", "sk")
    assert store.get("SkillSource", "sk", "default")["status"]["skillCount"] == 1


def test_configmap_and_bad_git(tmp_path):
    store = APIStore()
    store.create({"apiVersion": "v1", "kind": "ConfigMap",
                  "metadata": {"name": "cfg", "namespace": "default"},
                  "data": {"config.arena.yaml": "scenarios: []\n"}})
    for name, spec in (("a", {"type": "configmap", "interval": "1m",
                              "configMap": {"name": "cfg"}}),
                       ("b", {"type": "git", "interval": "1m",
                              "git": {"url": "file://" + str(tmp_path / "missing")}})):
        store.create({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "ArenaSource",
                      "metadata": {"name": name, "namespace": "default"}, "spec": spec})
    rec = SourceReconciler("ArenaSource", str(tmp_path / "c"))
    rec.reconcile(store, "default", "a")
    rec.reconcile(store, "default", "b")
    a = store.get("ArenaSource", "a", "default")["status"]
    b = store.get("ArenaSource", "b", "default")["status"]
    assert a["phase"] == "Ready" and a["artifact"]["files"] == 1
    assert b["phase"] == "Failed"
    assert b["conditions"][0]["reason"] == "SyncFailed"


def test_syncer_history_gc(tmp_path):
    store = APIStore()
    s = SourceSyncer(str(tmp_path), history_limit=2)
    for i in range(4):
        store.create({"apiVersion": "v1", "kind": "ConfigMap",
                      "metadata": {"name": f"c{i}", "namespace": "default"},
                      "data": {"f": str(i)}})
        s.sync(store, {"kind": "ArenaSource", "metadata": {"name": "x", "namespace": "default"},
                       "spec": {"type": "configmap", "configMap": {"name": f"c{i}"}}})
    revs = [d for d in (tmp_path / "default" / "arenasource" / "x").iterdir()
            if d.is_dir() and not d.is_symlink()]
    assert len(revs) == 2


def test_symlinks_escaping_the_tree_are_dropped(tmp_path):
    """A synced tree keeps in-tree links as links and drops links to host files
    (copytree followed symlinks and copied e.g. SA tokens in)."""
    secret = tmp_path / "host-secret"
    secret.write_text("TOKEN")
    ws = tmp_path / "ws"
    (ws / "skills").mkdir(parents=True)
    (ws / "skills" / "SKILL.md").write_text("# s\n")
    (ws / "leak.txt").symlink_to(secret)
    (ws / "ok.md").symlink_to("skills/SKILL.md")
    s = SourceSyncer(str(tmp_path / "content"))
    out = s.sync(APIStore(), {"kind": "SkillSource",
                              "metadata": {"name": "w", "namespace": "default"},
                              "spec": {"type": "workspace", "workspace": {"path": str(ws)}}})
    from pathlib import Path

    dest = Path(out["path"])
    assert not (dest / "leak.txt").exists() and not (dest / "leak.txt").is_symlink()
    assert (dest / "ok.md").is_symlink() and (dest / "ok.md").read_text() == "# s\n"


def test_git_path_traversal_rejected(tmp_path, repo):
    store = APIStore()
    store.create({"apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "SkillSource",
                  "metadata": {"name": "t", "namespace": "default"},
                  "spec": {"type": "git", "interval": "1m",
                           "git": {"url": "file://" + str(repo), "path": "../../.."}}})
    rec = SourceReconciler("SkillSource", str(tmp_path / "content"))
    rec.reconcile(store, "default", "t")
    st = store.get("SkillSource", "t", "default")["status"]
    assert st["phase"] == "Failed" and "escapes" in st["conditions"][0]["message"]


def test_promptpack_source_publishes_and_gcs_versions(tmp_path):
    """Every new revision of a PromptPackSource becomes a pack-version ConfigMap;
    versions beyond historyLimit are deleted unless a PromptPack still uses
    them (``promptpacksource_gc_test.go``)."""
    from omnia_amd.operator.sourcesync import SourceReconciler

    ws = tmp_path / "pack"
    ws.mkdir()
    store = APIStore()
    store.objs[store.key("PromptPackSource", "default", "pps")] = {
        "apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "PromptPackSource",
        "metadata": {"name": "pps", "namespace": "default", "generation": 1,
                     "resourceVersion": "1", "uid": "u"},
        "spec": {"type": "workspace", "workspace": {"path": str(ws)}, "packName": "support",
                 "interval": "1m", "historyLimit": 2}}
    rec = SourceReconciler("PromptPackSource", root=str(tmp_path / "content"))
    names = []
    for i in range(5):
        (ws / "pack.json").write_text('{"id": "support", "version": "1.0.%d"}' % i)
        rec.reconcile(store, "default", "pps")
        cms = [c["metadata"]["name"] for c in store.list("ConfigMap", "default")]
        names.append(sorted(cms))
        if i == 1:
            # a PromptPack pins the second version: it must survive GC
            pinned = [n for n in cms if n not in names[0]][0]
            store.objs[store.key("PromptPack", "default", "support")] = {
                "apiVersion": "omnia.altairalabs.ai/v1alpha1", "kind": "PromptPack",
                "metadata": {"name": "support", "namespace": "default"},
                "spec": {"source": {"type": "configmap", "configMapRef": {"name": pinned}}}}
    final = {c["metadata"]["name"] for c in store.list("ConfigMap", "default")}
    assert pinned in final and len(final) == 3  # 2 newest + the pinned one
    st = store.get("PromptPackSource", "pps", "default")["status"]
    assert st["versionsDeleted"] == 2
