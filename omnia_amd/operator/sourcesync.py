"""Source sync: materialise PromptKit bundles / skills / arena configs from git,
ConfigMaps, OCI artifacts or a workspace path into the workspace content tree
(``internal/sourcesync/{git,oci,configmap,syncer}.go``, ``SyncToFilesystem``
``syncer.go:92``).

Layout: ``<root>/<namespace>/<kind>/<name>/<revision>/`` with a ``current``
symlink swapped atomically after a successful sync, so readers never see a
half-written tree.  Revisions: git commit sha, ConfigMap content hash, OCI
manifest digest.  ``historyLimit`` old revisions are kept.

* git: ``git`` CLI (clone --depth 1 of a branch/tag, or fetch + checkout of a
  commit), optional sub-``path``; credentials from a Secret's ``username`` /
  ``password`` (HTTPS) via ``GIT_ASKPASS``;
* oci: OCI distribution API over HTTP(S) -- manifest, then each layer blob
  (tar / tar+gzip) unpacked; anonymous bearer-token challenge supported;
* configmap: every data key becomes a file.

:class:`SourceReconciler` drives ArenaSource / SkillSource / PromptPackSource
objects: sync every ``spec.interval`` (unless ``suspend``), write
``status.artifact {path, revision}``, ``phase`` and a Ready condition.
"""
from __future__ import annotations

import hashlib
import io
import logging
import os
import shutil
import subprocess
import tarfile
import tempfile
import time
from pathlib import Path

from .apistore import APIStore, set_condition

log = logging.getLogger("omnia.sourcesync")


class SyncError(RuntimeError):
    pass


def parse_duration(s: str | None, default: float = 300.0) -> float:
    if not s:
        return default
    total, num = 0.0, ""
    units = {"h": 3600, "m": 60, "s": 1}
    for ch in s.strip():
        if ch.isdigit() or ch == ".":
            num += ch
        elif ch in units and num:
            total += float(num) * units[ch]
            num = ""
        else:
            raise ValueError(f"bad duration {s!r}")
    return total + (float(num) if num else 0.0)


def _confined_copytree(src: Path, dest: Path) -> None:
    """Copy ``src`` to ``dest`` keeping symlinks as links (never following them,
    as ``internal/sourcesync/dir.go`` does with Readlink/Symlink), then drop every
    link whose target resolves outside the copied tree, so a synced repo cannot
    smuggle operator-host files (service-account tokens, ...) into the content
    tree that skills and packs later read."""
    shutil.copytree(src, dest, symlinks=True)
    root = dest.resolve()
    for p in sorted(dest.rglob("*"), key=lambda q: len(q.parts), reverse=True):
        if p.is_symlink():
            try:
                tgt = (p.parent / os.readlink(p)).resolve()
            except OSError:
                tgt = None
            if tgt is None or not (tgt == root or str(tgt).startswith(str(root) + os.sep)):
                log.warning("source sync: dropping symlink %s escaping the tree", p)
                p.unlink()


def _workspace_files(p: Path) -> dict[str, bytes]:
    """Content map for hashing a workspace tree; symlinks contribute their link
    text, never the bytes of what they point at."""
    out: dict[str, bytes] = {}
    for f in p.rglob("*"):
        rel = str(f.relative_to(p))
        if f.is_symlink():
            out[rel] = b"link:" + os.readlink(f).encode()
        elif f.is_file():
            out[rel] = f.read_bytes()
    return out


def _hash_tree(files: dict[str, bytes]) -> str:
    h = hashlib.sha256()
    for k in sorted(files):
        h.update(k.encode() + b"\0" + files[k] + b"\0")
    return "sha256:" + h.hexdigest()[:16]


class SourceSyncer:
    def __init__(self, root: str, history_limit: int = 5):
        self.root = Path(root)
        self.history = history_limit

    def target(self, ns, kind, name) -> Path:
        return self.root / ns / kind.lower() / name

    # -------------------------------------------------------------- fetchers
    def _git(self, spec: dict, secret: dict | None, timeout: float) -> tuple[str, Path, Path]:
        g = spec["git"]
        ref = g.get("ref") or {}
        tmp = Path(tempfile.mkdtemp(prefix="omnia-git-"))
        env = dict(os.environ, GIT_TERMINAL_PROMPT="0")
        if secret and secret.get("password"):
            ask = tmp.parent / (tmp.name + "-askpass.sh")
            ask.write_text("#!/bin/sh\ncase \"$1\" in Username*) echo \"$GIT_USER\";; "
                           "*) echo \"$GIT_PASS\";; esac\n")
            ask.chmod(0o700)
            env.update(GIT_ASKPASS=str(ask), GIT_USER=secret.get("username", "git"),
                       GIT_PASS=secret["password"])

        def git(*args, cwd=None):
            r = subprocess.run(["git", *args], cwd=cwd, env=env, capture_output=True,
                               text=True, timeout=timeout)
            if r.returncode != 0:
                raise SyncError(f"git {args[0]} failed: {r.stderr.strip()[:300]}")
            return r.stdout.strip()

        repo = tmp / "repo"
        if ref.get("commit"):
            git("init", "-q", str(repo))
            git("remote", "add", "origin", g["url"], cwd=repo)
            git("fetch", "-q", "--depth", "1", "origin", ref["commit"], cwd=repo)
            git("checkout", "-q", "FETCH_HEAD", cwd=repo)
        else:
            br = ref.get("tag") or ref.get("branch")
            args = ["clone", "-q", "--depth", "1"] + (["--branch", br] if br else [])
            git(*args, g["url"], str(repo))
        rev = git("rev-parse", "HEAD", cwd=repo)
        src = (repo / g["path"]).resolve() if g.get("path") else repo
        rr = repo.resolve()
        if src != rr and not str(src).startswith(str(rr) + os.sep):
            raise SyncError(f"path {g.get('path')!r} escapes the repository")
        if not src.exists():
            raise SyncError(f"path {g.get('path')!r} not found in repository")
        shutil.rmtree(repo / ".git", ignore_errors=True)
        return rev, src, tmp

    def _configmap(self, store: APIStore, ns: str, spec: dict) -> tuple[str, dict]:
        cm = store.try_get("ConfigMap", spec["configMap"]["name"], ns)
        if cm is None:
            raise SyncError(f"ConfigMap {spec['configMap']['name']} not found")
        # every key becomes a file (Data wins over BinaryData); "__" in a key is a
        # path separator, the dashboard deploy route's encoding of nested files
        # (internal/sourcesync/configmap.go:124-199)
        import base64

        data = {k: base64.b64decode(v) for k, v in (cm.get("binaryData") or {}).items()}
        data.update({k: v.encode() if isinstance(v, str) else v for k, v in
                     (cm.get("data") or {}).items()})
        data = {k.replace("__", "/"): v for k, v in sorted(data.items())
                if ".." not in k.replace("__", "/").split("/")}
        return _hash_tree(data), data

    def _oci(self, spec: dict, secret: dict | None, timeout: float) -> tuple[str, dict]:
        import requests

        url = spec["oci"]["url"].removeprefix("oci://")
        host, _, rest = url.partition("/")
        repo, _, tag = rest.partition(":")
        tag = tag or "latest"
        scheme = "http" if spec["oci"].get("insecure") else "https"
        base = f"{scheme}://{host}/v2/{repo}"
        headers = {"Accept": "application/vnd.oci.image.manifest.v1+json"}
        auth = (secret.get("username"), secret.get("password")) if secret else None
        r = requests.get(f"{base}/manifests/{tag}", headers=headers, auth=auth, timeout=timeout)
        if r.status_code == 401 and "Bearer" in r.headers.get("WWW-Authenticate", ""):
            chal = dict(kv.split("=", 1) for kv in r.headers["WWW-Authenticate"][7:]
                        .replace('"', "").split(","))
            tok = requests.get(chal["realm"], params={"service": chal.get("service"),
                                                      "scope": chal.get("scope")},
                               auth=auth, timeout=timeout).json()
            headers["Authorization"] = "Bearer " + (tok.get("token") or tok.get("access_token"))
            r = requests.get(f"{base}/manifests/{tag}", headers=headers, timeout=timeout)
        if r.status_code >= 400:
            raise SyncError(f"OCI manifest HTTP {r.status_code}")
        digest = r.headers.get("Docker-Content-Digest") or \
            "sha256:" + hashlib.sha256(r.content).hexdigest()
        files: dict[str, bytes] = {}
        for layer in r.json().get("layers", []):
            b = requests.get(f"{base}/blobs/{layer['digest']}", headers=headers,
                             timeout=timeout)
            if b.status_code >= 400:
                raise SyncError(f"OCI blob HTTP {b.status_code}")
            mode = "r:gz" if "gzip" in layer.get("mediaType", "") else "r:*"
            with tarfile.open(fileobj=io.BytesIO(b.content), mode=mode) as tf:
                for m in tf.getmembers():
                    if m.isfile() and not m.name.startswith("/") and ".." not in m.name:
                        files[m.name] = tf.extractfile(m).read()
        return digest, files

    # -------------------------------------------------------------- sync
    def sync(self, store: APIStore, obj: dict) -> dict:
        md, spec = obj["metadata"], obj["spec"]
        ns, kind, name = md.get("namespace", "default"), obj["kind"], md["name"]
        timeout = parse_duration(spec.get("timeout"), 60.0)
        secret = None
        sref = ((spec.get("git") or spec.get("oci") or {}).get("secretRef") or {}).get("name")
        if sref:
            s = store.try_get("Secret", sref, ns)
            if s is not None:
                import base64

                secret = {k: base64.b64decode(v).decode() for k, v in
                          (s.get("data") or {}).items()}
                secret.update(s.get("stringData") or {})
        t = spec.get("type")
        dest_root = self.target(ns, kind, name)
        dest_root.mkdir(parents=True, exist_ok=True)
        if t == "git":
            rev, src, tmp = self._git(spec, secret, timeout)
            short = rev[:12]
            dest = dest_root / short
            try:
                if not dest.exists():
                    _confined_copytree(src, dest)
            finally:
                shutil.rmtree(tmp, ignore_errors=True)
                Path(str(tmp) + "-askpass.sh").unlink(missing_ok=True)
        elif t in ("configmap", "oci"):
            rev, files = (self._configmap(store, ns, spec) if t == "configmap"
                          else self._oci(spec, secret, timeout))
            short = rev.split(":")[-1][:12]
            dest = dest_root / short
            if not dest.exists():
                tmp = dest_root / (short + ".tmp")
                shutil.rmtree(tmp, ignore_errors=True)
                for rel, data in files.items():
                    p = (tmp / rel).resolve()
                    if not str(p).startswith(str(tmp.resolve())):
                        raise SyncError(f"path escapes artifact root: {rel}")
                    p.parent.mkdir(parents=True, exist_ok=True)
                    p.write_bytes(data)
                tmp.mkdir(parents=True, exist_ok=True)
                tmp.rename(dest)
        elif t == "workspace":
            p = Path(spec.get("workspace", {}).get("path", ""))
            if not p.is_dir():
                raise SyncError(f"workspace path {p} not found")
            rev = _hash_tree(_workspace_files(p))
            short = rev.split(":")[-1][:12]
            dest = dest_root / short
            if not dest.exists():
                _confined_copytree(p, dest)
        else:
            raise SyncError(f"unsupported source type {t!r}")
        target = dest / spec["targetPath"] if spec.get("targetPath") else dest
        cur = dest_root / "current"
        tmp_link = dest_root / ".current.tmp"
        if tmp_link.is_symlink() or tmp_link.exists():
            tmp_link.unlink()
        tmp_link.symlink_to(dest.name)
        os.replace(tmp_link, cur)
        self._gc(dest_root, keep=dest.name, limit=int(spec.get("historyLimit") or self.history))
        return {"path": str(target), "revision": rev,
                "files": sum(1 for f in dest.rglob("*") if f.is_file())}

    @staticmethod
    def _gc(root: Path, keep: str, limit: int):
        revs = sorted((d for d in root.iterdir() if d.is_dir() and not d.is_symlink()
                       and not d.name.endswith(".tmp")), key=lambda d: d.stat().st_mtime)
        for d in revs[:-max(1, limit)]:
            if d.name != keep:
                shutil.rmtree(d, ignore_errors=True)


class SourceReconciler:
    """ArenaSource / SkillSource / PromptPackSource reconciler."""

    def __init__(self, kind: str, root: str | None = None):
        self.kind = kind
        self.syncer = SourceSyncer(root or os.environ.get("OMNIA_CONTENT_ROOT",
                                                          tempfile.gettempdir() +
                                                          "/omnia-content"))

    def reconcile(self, store: APIStore, ns, name):
        o = store.try_get(self.kind, name, ns)
        if o is None:
            return None
        spec = o["spec"]
        st = dict(o.get("status") or {})
        interval = parse_duration(spec.get("interval") or spec.get("syncInterval"), 300.0)
        if spec.get("suspend"):
            st["phase"] = "Suspended"
            set_condition(st, "Ready", False, "Suspended", "", o["metadata"]["generation"])
        else:
            try:
                art = self.syncer.sync(store, o)
                changed = (st.get("artifact") or {}).get("revision") != art["revision"]
                st.update(phase="Ready", artifact=art, revision=art["revision"],
                          lastSyncTime=time.time())
                if self.kind == "SkillSource":
                    st["skillCount"] = sum(1 for _ in Path(art["path"]).rglob("SKILL.md"))
                if self.kind == "PromptPackSource" and changed:
                    self._publish_pack(store, o, art)
                if self.kind == "PromptPackSource":
                    st["versionsDeleted"] = int(st.get("versionsDeleted", 0)) + \
                        self._gc_pack_versions(store, o)
                if self.kind == "ArenaTemplateSource":
                    self._scan_templates(o, art, st)
                set_condition(st, "Ready", True, "Synced", f"revision {art['revision']}",
                              o["metadata"]["generation"])
            except (SyncError, subprocess.TimeoutExpired, OSError, ValueError, KeyError) as e:
                st["phase"] = "Failed"
                set_condition(st, "Ready", False, "SyncFailed", str(e)[:300],
                              o["metadata"]["generation"])
        st["observedGeneration"] = o["metadata"]["generation"]
        o["status"] = st
        store.update_status(o)
        return interval

    def _scan_templates(self, src: dict, art: dict, st: dict):
        """ArenaTemplateSource: discover the templates of the synced revision and
        publish their index as ``<content root>/<ns>/.arena/template-index/<name>.json``
        (``arenatemplatesource_controller.go`` ``writeTemplateIndex``)."""
        import json as _json

        from ..ee.arena.templates import discover

        gen = src["metadata"]["generation"]
        ts = discover(art["path"], (src.get("spec") or {}).get("templatesPath") or "templates")
        ns = src["metadata"].get("namespace") or "default"
        idx_dir = Path(self.syncer.root) / ns / ".arena" / "template-index"
        idx_dir.mkdir(parents=True, exist_ok=True)
        tmp = idx_dir / (src["metadata"]["name"] + ".json.tmp")
        tmp.write_text(_json.dumps([t.to_json() for t in ts], indent=2))
        os.replace(tmp, idx_dir / (src["metadata"]["name"] + ".json"))
        st.update(templateCount=len(ts), headVersion=art["revision"],
                  templateIndex=str(idx_dir / (src["metadata"]["name"] + ".json")),
                  nextFetchTime=time.time() + parse_duration(
                      (src.get("spec") or {}).get("interval") or
                      (src.get("spec") or {}).get("syncInterval"), 300.0))
        set_condition(st, "TemplatesScanned", True, "ScanComplete",
                      f"Discovered {len(ts)} templates", gen)
        set_condition(st, "ArtifactAvailable", True, "ArtifactStored",
                      f"revision {art['revision']}", gen)

    MIN_RETENTION_S = float(os.environ.get("OMNIA_PACK_MIN_RETENTION_S", "0"))

    def _gc_pack_versions(self, store: APIStore, src: dict) -> int:
        """Keep the newest ``historyLimit`` published versions of the pack; older
        ones go unless a PromptPack still points at them (``configMapRef``) or
        they are younger than the minimum retention age
        (``ee/internal/controller/promptpacksource_gc.go``)."""
        ns = src["metadata"].get("namespace", "default")
        pack = src["spec"]["packName"]
        limit = max(0, int(src["spec"].get("historyLimit", 10)))
        versions = [c for c in store.list("ConfigMap", ns)
                    if (c["metadata"].get("labels") or {}).get(
                        "omnia.altairalabs.ai/pack") == pack]
        if len(versions) <= limit:
            return 0
        versions.sort(key=lambda c: (c["metadata"].get("creationTimestamp", ""),
                                     int(c["metadata"].get("resourceVersion") or 0)),
                      reverse=True)
        used = {((pp.get("spec") or {}).get("source") or {}).get("configMapRef", {}).get("name")
                for pp in store.list("PromptPack", ns)}
        now = time.time()
        deleted = 0
        for c in versions[limit:]:
            name = c["metadata"]["name"]
            if name in used:
                continue
            created = c["metadata"].get("creationTimestamp")
            if created and self.MIN_RETENTION_S > 0:
                import calendar

                t = calendar.timegm(time.strptime(created[:19], "%Y-%m-%dT%H:%M:%S"))
                if now - t < self.MIN_RETENTION_S:
                    continue
            store.delete("ConfigMap", name, ns)
            deleted += 1
        return deleted

    @staticmethod
    def _publish_pack(store: APIStore, src: dict, art: dict):
        """PromptPackSource: a new revision becomes a ConfigMap the PromptPack
        reconciler versions (``createVersionOnSync``)."""
        ns = src["metadata"].get("namespace", "default")
        pack = Path(art["path"])
        data = {f.name: f.read_text() for f in pack.iterdir() if f.is_file() and
                f.suffix in (".json", ".yaml", ".yml", ".md")}
        name = f"{src['spec']['packName']}-{art['revision'].split(':')[-1][:8]}"
        if store.try_get("ConfigMap", name, ns) is None:
            store.create({"apiVersion": "v1", "kind": "ConfigMap",
                          "metadata": {"name": name, "namespace": ns, "labels": {
                              "omnia.altairalabs.ai/pack": src["spec"]["packName"]}},
                          "data": data})

