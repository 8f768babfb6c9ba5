"""PromptPack skills in the runtime (reference
``internal/runtime/skills/manifest.go`` and ``server.go`` ``WithSkillManifest``).

The PromptPack reconciler writes a skill manifest (``OMNIA_PROMPTPACK_MANIFEST_PATH``):
``{"version", "skills": [{"mount_as", "content_path", "name"}], "config":
{"max_active", "selector"}}``. Each entry is a directory that holds a
``SKILL.md`` with YAML front matter (``name``, ``description``) followed by the
skill's instructions. An empty path or a missing file means no skills; a
malformed file is an error.

The agent sees each skill's catalog line (name, mount path, description) in the
server-side tool descriptions. It activates a skill to receive its
instructions and reads the skill's bundled resources on demand:
* ``skill__activate`` returns the instructions. At most ``max_active`` skills
  are active at once; the oldest is dropped first.
* ``skill__deactivate`` removes a skill from the active set.
* ``skill__read_resource`` reads a file inside the skill directory. The path is
  confined to the directory.

These are server-side tools of a :class:`SkillsHandler`, so they go through the
executor's policy, circuit-breaker and metrics path like any other tool. They
are never sent to the facade.

Pack-level ``skills`` (``promptpack.schema.json:210-216``, ``$defs.SkillSource``)
join the manifest's: a string or ``{path, preload}`` names a skill directory
(relative to the pack file) or a directory of skill directories; an inline
``{name, description, instructions}`` is a skill without resources.  Skills
marked ``preload`` are active from the first turn: their instructions are part
of the system prompt (:func:`preloaded_instructions`).
"""
from __future__ import annotations

import json
import logging
import os
from collections import OrderedDict
from dataclasses import dataclass, field

import yaml

from ..tools.executor import CallContext, Handler, ToolDef

log = logging.getLogger("omnia.runtime.skills")

# active-skill sets of this many conversations are kept; the least recently
# used conversation's set is forgotten first
MAX_TRACKED_SESSIONS = 10000


@dataclass
class ManifestEntry:
    mount_as: str
    content_path: str
    name: str = ""


@dataclass
class Manifest:
    version: str = ""
    skills: list = field(default_factory=list)
    max_active: int = 0
    selector: str = ""


def read_manifest(path: str | None) -> Manifest:
    if not path or not os.path.exists(path):
        return Manifest()
    with open(path) as f:
        try:
            raw = json.load(f)
        except json.JSONDecodeError as e:
            raise ValueError(f"parse skill manifest {path}: {e}") from e
    cfg = raw.get("config") or {}
    return Manifest(version=raw.get("version", ""),
                    skills=[ManifestEntry(s.get("mount_as", ""), s.get("content_path", ""),
                                          s.get("name", "")) for s in raw.get("skills") or []],
                    max_active=int(cfg.get("max_active") or 0), selector=cfg.get("selector", ""))


@dataclass
class Skill:
    name: str
    description: str
    mount_as: str
    root: str
    instructions: str
    preload: bool = False


def load_skill(entry: ManifestEntry) -> Skill:
    with open(os.path.join(entry.content_path, "SKILL.md")) as f:
        text = f.read()
    meta, body = {}, text
    if text.startswith("---"):
        end = text.find("\n---", 3)
        if end != -1:
            try:
                meta = yaml.safe_load(text[3:end]) or {}
            except yaml.YAMLError as e:
                raise ValueError(f"skill {entry.content_path}: bad front matter: {e}") from e
            if not isinstance(meta, dict):
                raise ValueError(f"skill {entry.content_path}: front matter is not a mapping")
            body = text[end + 4:].lstrip("\n")
    return Skill(name=str(meta.get("name") or entry.name or os.path.basename(entry.content_path)),
                 description=str(meta.get("description", "")), mount_as=entry.mount_as,
                 root=os.path.realpath(entry.content_path), instructions=body)


class SkillsHandler(Handler):
    type = "skills"

    def __init__(self, manifest: Manifest, workflow_prefix: str = "",
                 extra: list[Skill] | None = None):
        super().__init__({"name": "skills"})
        self.skills: dict[str, Skill] = {}
        self.load_errors: list[str] = []
        for s in extra or []:
            if s.name in self.skills:
                self.load_errors.append(f"duplicate skill {s.name}")
                continue
            self.skills[s.name] = s
        for e in manifest.skills:
            try:
                s = load_skill(e)
            except (OSError, ValueError) as err:
                # one bad skill is logged and skipped; the rest still serve
                log.error("skill %s skipped: %s", e.content_path or e.mount_as, err)
                self.load_errors.append(str(err))
                continue
            if workflow_prefix and not s.mount_as.startswith(workflow_prefix):
                continue  # workflow scoping by mount path
            if s.name in self.skills:
                log.error("duplicate skill name %r (%s and %s): keeping the first",
                          s.name, self.skills[s.name].mount_as, s.mount_as)
                self.load_errors.append(f"duplicate skill {s.name}")
                continue
            self.skills[s.name] = s
        self.max_active = manifest.max_active
        # per-conversation active sets (PromptKit keeps the active set per
        # conversation): session id -> ordered active skill names
        self._active: "OrderedDict[str, OrderedDict[str, None]]" = OrderedDict()

    def active(self, session_id: str) -> "OrderedDict[str, None]":
        cur = self._active.get(session_id)
        if cur is None:
            cur = self._active[session_id] = OrderedDict()
            while len(self._active) > MAX_TRACKED_SESSIONS:
                self._active.popitem(last=False)
        else:
            self._active.move_to_end(session_id)
        return cur

    def catalog(self) -> str:
        return "\n".join(f"- {s.name} ({s.mount_as}): {s.description}"
                         for s in self.skills.values())

    async def discover(self) -> list[ToolDef]:
        if not self.skills:
            return []
        names = sorted(self.skills)
        one = {"type": "object", "properties": {"name": {"type": "string", "enum": names}},
               "required": ["name"]}
        res = {"type": "object", "properties": {"name": {"type": "string", "enum": names},
                                                "path": {"type": "string"}},
               "required": ["name", "path"]}
        cat = self.catalog()
        return [ToolDef("skill__activate", "Activate a skill and receive its instructions. "
                        "Available skills:\n" + cat, one, self.name, self.type),
                ToolDef("skill__deactivate", "Deactivate an active skill.", one, self.name,
                        self.type),
                ToolDef("skill__read_resource", "Read a file bundled with a skill.", res,
                        self.name, self.type)]

    async def call(self, tool: ToolDef, args: dict, ctx: CallContext) -> str:
        s = self.skills.get(args.get("name", ""))
        if s is None:
            raise KeyError(f"unknown skill {args.get('name')!r}")
        active = self.active(ctx.session_id or "")
        if tool.name == "skill__activate":
            active.pop(s.name, None)
            active[s.name] = None
            dropped = []
            while self.max_active and len(active) > self.max_active:
                dropped.append(active.popitem(last=False)[0])
            return json.dumps({"skill": s.name, "instructions": s.instructions,
                               "active": list(active), "deactivated": dropped})
        if tool.name == "skill__deactivate":
            active.pop(s.name, None)
            return json.dumps({"skill": s.name, "active": list(active)})
        if tool.name == "skill__read_resource":
            if not s.root:
                raise PermissionError(f"inline skill {s.name!r} has no resources")
            p = os.path.realpath(os.path.join(s.root, args.get("path", "")))
            if os.path.commonpath([p, s.root]) != s.root or not os.path.isfile(p):
                raise PermissionError("resource outside the skill directory or missing")
            with open(p, errors="replace") as f:
                return json.dumps({"skill": s.name, "path": args["path"],
                                   "content": f.read(256 * 1024)})
        raise KeyError(tool.name)


def pack_skills(pack) -> list[Skill]:
    """Skills declared in the pack's own ``skills`` list."""
    out: list[Skill] = []
    base = str(pack.base_dir) if getattr(pack, "base_dir", None) else os.getcwd()
    for src in getattr(pack, "skill_sources", []) or []:
        if isinstance(src, dict) and "instructions" in src:
            out.append(Skill(name=src["name"], description=src["description"],
                             mount_as=f"inline/{src['name']}", root="",
                             instructions=src["instructions"], preload=True))
            continue
        path, preload = (src, False) if isinstance(src, str) else \
            (src["path"], bool(src.get("preload", False)))
        if path.startswith("@"):
            log.warning("skill package reference %s needs the PromptPack reconciler's "
                        "manifest; skipped", path)
            continue
        root = path if os.path.isabs(path) else os.path.normpath(os.path.join(base, path))
        dirs = [root] if os.path.isfile(os.path.join(root, "SKILL.md")) else sorted(
            os.path.join(root, d) for d in (os.listdir(root) if os.path.isdir(root) else [])
            if os.path.isfile(os.path.join(root, d, "SKILL.md")))
        if not dirs:
            log.error("pack skill source %s holds no SKILL.md", path)
        for d in dirs:
            rel = os.path.relpath(d, base)
            try:
                s = load_skill(ManifestEntry(mount_as=rel, content_path=d))
            except (OSError, ValueError) as err:
                log.error("pack skill %s skipped: %s", d, err)
                continue
            s.preload = preload
            out.append(s)
    return out


def preloaded_instructions(handler: "SkillsHandler | None") -> str:
    if handler is None:
        return ""
    pre = [s for s in handler.skills.values() if s.preload]
    return "".join(f"\n\n## Skill: {s.name}\n{s.instructions}" for s in pre)


def attach_skills(executor, manifest_path: str | None = None, workflow_prefix: str = "",
                  pack=None):
    """Add the manifest's and the pack's skills to an executor (no-op without
    either)."""
    path = manifest_path if manifest_path is not None else \
        os.environ.get("OMNIA_PROMPTPACK_MANIFEST_PATH", "")
    m = read_manifest(path)
    extra = pack_skills(pack) if pack is not None else []
    if not m.skills and not extra:
        return None
    h = SkillsHandler(m, workflow_prefix, extra=extra)
    executor.add_handler(h)
    return h
