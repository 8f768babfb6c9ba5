"""PromptPack loading, validation and template rendering.

Pack format: ``internal/schema/promptpack.schema.json`` (required: id, name,
version, template_engine, prompts).  A prompt carries ``system_template``,
``user_template``, ``variables`` (name/type/required/default), ``tools``
(names resolved against the pack's ``tools`` map or the ToolRegistry),
``tool_policy`` (tool_choice auto|required|none, max_rounds=5,
max_tool_calls_per_turn=10, blocklist), ``parameters`` (sampling) and
``validators`` (banned_words, max_length, min_length, regex_match, json_schema,
pii_detection).  Templates use ``{{variable}}`` substitution and
``{{fragment_name}}`` / ``{{> fragment_name}}`` fragments (resolved first).

Graph sections (``promptpack.schema.json:200-216``, ``$defs`` WorkflowConfig /
AgentsConfig / SkillSource at ``:1211-1404``):

* ``workflow`` -- a state machine over the prompts: ``entry`` state, ``states``
  {name: {prompt_task, on_event {event: target}, persistence, orchestration,
  skills}}; executed by :mod:`omnia_amd.runtime.workflow`;
* ``agents`` -- multi-agent packs: ``entry`` prompt key plus ``members``
  {prompt key: A2A card metadata}; the entry agent delegates to members;
* ``skills`` -- pack-level skill sources (a path, ``{path, preload}`` or an
  inline ``{name, description, instructions}``).

Cross-references the JSON schema cannot express (entry exists, every
``prompt_task`` / member is a prompt, every ``on_event`` target is a state) are
checked on load.  The entry prompt resolves like ``internal/runtime/
pack_entry.go:54-86``: workflow.entry, then agents.entry, then a sole prompt,
then the configured/"default" name.
The compiled pack lives at ``/etc/omnia/pack/pack.json`` in reconciled pods
(``internal/controller/constants.go:103-127``).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from pathlib import Path

from ..utils import jsonschema

_VAR = re.compile(r"\{\{\s*(>\s*)?([A-Za-z_][\w.\-]*)\s*\}\}")

DEFAULT_MAX_ROUNDS = 5
DEFAULT_MAX_TOOL_CALLS = 10


class PackError(ValueError):
    pass


@dataclass
class ToolPolicy:
    tool_choice: str = "auto"
    max_rounds: int = DEFAULT_MAX_ROUNDS
    max_tool_calls_per_turn: int = DEFAULT_MAX_TOOL_CALLS
    blocklist: list[str] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: dict | None) -> "ToolPolicy":
        d = d or {}
        return cls(tool_choice=d.get("tool_choice", "auto"),
                   max_rounds=int(d.get("max_rounds", DEFAULT_MAX_ROUNDS)),
                   max_tool_calls_per_turn=int(d.get("max_tool_calls_per_turn",
                                                     DEFAULT_MAX_TOOL_CALLS)),
                   blocklist=list(d.get("blocklist", [])))


@dataclass
class Prompt:
    id: str
    name: str
    version: str
    system_template: str
    user_template: str = ""
    variables: list[dict] = field(default_factory=list)
    tools: list[str] = field(default_factory=list)
    tool_policy: ToolPolicy = field(default_factory=ToolPolicy)
    parameters: dict = field(default_factory=dict)
    validators: list[dict] = field(default_factory=list)
    evals: list[dict] = field(default_factory=list)
    raw: dict = field(default_factory=dict)


PACK_SCHEMA = {
    "type": "object",
    "required": ["id", "name", "version", "template_engine", "prompts"],
    "properties": {
        "id": {"type": "string", "minLength": 1},
        "name": {"type": "string", "minLength": 1},
        "version": {"type": "string", "pattern": r"^\d+\.\d+\.\d+"},
        "description": {"type": "string"},
        "template_engine": {"type": "object", "required": ["version", "syntax"],
                            "properties": {"version": {"type": "string"},
                                           "syntax": {"type": "string"},
                                           "features": {"type": "array",
                                                        "items": {"enum": [
                                                            "basic_substitution", "fragments",
                                                            "conditionals", "loops",
                                                            "filters"]}}}},
        "prompts": {"type": "object", "minProperties": 1,
                    "additionalProperties": {"$ref": "#/$defs/Prompt"}},
        "fragments": {"type": "object", "additionalProperties": {"type": "string"}},
        "tools": {"type": "object", "additionalProperties": {"$ref": "#/$defs/Tool"}},
        "workflow": {"$ref": "#/$defs/WorkflowConfig"},
        "agents": {"$ref": "#/$defs/AgentsConfig"},
        "skills": {"type": "array", "items": {"$ref": "#/$defs/SkillSource"}},
        "compositions": {"type": "object",
                         "additionalProperties": {"$ref": "#/$defs/Composition"}},
    },
    "$defs": {
        "WorkflowConfig": {
            "type": "object", "required": ["version", "entry", "states"],
            "additionalProperties": False,
            "properties": {"version": {"type": "integer", "minimum": 1},
                           "entry": {"type": "string"},
                           "states": {"type": "object", "minProperties": 1,
                                      "additionalProperties": {"$ref": "#/$defs/WorkflowState"}},
                           "engine": {"type": "object", "properties": {"budget": {
                               "type": "object", "properties": {
                                   "max_total_visits": {"type": "integer", "minimum": 1},
                                   "max_tool_calls": {"type": "integer", "minimum": 1},
                                   "max_wall_time_sec": {"type": "number",
                                                         "exclusiveMinimum": 0}}}}}}},
        # the published schema file predates PromptKit 1.5; compiled packs in
        # the reference's own samples also carry terminal / max_visits /
        # on_max_visits / artifacts and composition states
        # (config/samples/omnia_v1alpha1_promptpack_deep_research.yaml:383-455,
        # ..._doc_analysis.yaml), so those are part of the accepted shape
        "WorkflowState": {
            "type": "object", "additionalProperties": False,
            "properties": {"prompt_task": {"type": "string"},
                           "description": {"type": "string"},
                           "on_event": {"type": "object",
                                        "additionalProperties": {"type": "string"}},
                           "persistence": {"enum": ["transient", "persistent"]},
                           "orchestration": {"enum": ["internal", "external", "hybrid",
                                                      "composition"]},
                           "composition": {"type": "string"},
                           "skills": {"type": "string"},
                           "terminal": {"type": "boolean"},
                           "max_visits": {"type": "integer", "minimum": 1},
                           "on_max_visits": {"type": "string"},
                           "artifacts": {"type": "object", "additionalProperties": {
                               "type": "object",
                               "properties": {"type": {"type": "string"},
                                              "mode": {"enum": ["append", "replace"]},
                                              "description": {"type": "string"}}}}}},
        "Composition": {
            "type": "object", "required": ["steps"],
            "properties": {"version": {"type": "integer", "minimum": 1},
                           "description": {"type": "string"},
                           "steps": {"type": "array", "minItems": 1,
                                     "items": {"$ref": "#/$defs/Step"}}}},
        "Step": {
            "type": "object", "required": ["id", "kind"],
            "properties": {"id": {"type": "string", "minLength": 1},
                           "kind": {"enum": ["prompt", "parallel", "tool", "branch", "agent"]},
                           "prompt_task": {"type": "string"},
                           "tool": {"type": "string"},
                           "args": {"type": "object"},
                           "depends_on": {"type": "array", "items": {"type": "string"}},
                           "branches": {"type": "array", "minItems": 1,
                                        "items": {"$ref": "#/$defs/Step"}},
                           "reduce": {"type": "object", "properties": {
                               "strategy": {"enum": ["barrier"]},
                               "into": {"type": "string"}}},
                           "predicate": {"type": "object", "required": ["path", "op"],
                                         "properties": {"path": {"type": "string"},
                                                        "op": {"enum": [
                                                            "equals", "not_equals", "contains",
                                                            "exists", "gt", "gte", "lt", "lte",
                                                            "in"]}}},
                           "then": {"type": "string"}, "else": {"type": "string"},
                           "tools": {"type": "array", "items": {"type": "string"}},
                           "termination": {"type": "object", "properties": {
                               "max_steps": {"type": "integer", "minimum": 1}}}}},
        "AgentsConfig": {
            "type": "object", "required": ["entry", "members"], "additionalProperties": False,
            "properties": {"entry": {"type": "string"},
                           "members": {"type": "object", "minProperties": 1,
                                       "additionalProperties": {"$ref": "#/$defs/AgentDef"}}}},
        "AgentDef": {
            "type": "object", "additionalProperties": False,
            "properties": {"description": {"type": "string"},
                           "tags": {"type": "array", "items": {"type": "string"}},
                           "input_modes": {"type": "array", "items": {"type": "string"}},
                           "output_modes": {"type": "array", "items": {"type": "string"}}}},
        "SkillSource": {"oneOf": [{"type": "string"}, {"$ref": "#/$defs/SkillPathSource"},
                                  {"$ref": "#/$defs/InlineSkill"}]},
        "SkillPathSource": {
            "type": "object", "required": ["path"], "additionalProperties": False,
            "properties": {"path": {"type": "string"}, "preload": {"type": "boolean"}}},
        "InlineSkill": {
            "type": "object", "required": ["name", "description", "instructions"],
            "additionalProperties": False,
            "properties": {"name": {"type": "string", "minLength": 1},
                           "description": {"type": "string", "minLength": 1},
                           "instructions": {"type": "string", "minLength": 1}}},
        "Prompt": {
            "type": "object",
            "required": ["id", "name", "version", "system_template"],
            "properties": {
                "system_template": {"type": "string"},
                "variables": {"type": "array", "items": {
                    "type": "object", "required": ["name", "type", "required"]}},
                "tool_policy": {"type": "object", "properties": {
                    "tool_choice": {"enum": ["auto", "required", "none"]},
                    "max_rounds": {"type": "integer", "minimum": 1},
                    "max_tool_calls_per_turn": {"type": "integer", "minimum": 1}}},
                "parameters": {"type": "object", "properties": {
                    "temperature": {"type": "number", "minimum": 0},
                    "max_tokens": {"type": "integer", "minimum": 1},
                    "top_p": {"type": "number", "minimum": 0, "maximum": 1},
                    "top_k": {"type": "integer", "minimum": 0}}},
                "validators": {"type": "array", "items": {
                    "type": "object", "required": ["type", "enabled"],
                    "properties": {"type": {"enum": [
                        "banned_words", "max_length", "min_length", "regex_match",
                        "json_schema", "sentiment", "toxicity", "pii_detection",
                        "custom"]}}}},
            },
        },
        "Tool": {"type": "object", "required": ["name", "description"],
                 "properties": {"name": {"type": "string"}, "description": {"type": "string"},
                                "parameters": {"type": "object"}}},
    },
}


class PromptPack:
    def __init__(self, data: dict, base_dir: str | Path | None = None):
        errs = jsonschema.Validator(PACK_SCHEMA).errors(data)
        if errs:
            raise PackError("invalid pack: " + "; ".join(str(e) for e in errs[:5]))
        self.data = data
        self.base_dir = Path(base_dir) if base_dir is not None else None
        self.id = data["id"]
        self.name = data["name"]
        self.version = data["version"]
        self.fragments: dict[str, str] = dict(data.get("fragments", {}))
        self.tools: dict[str, dict] = dict(data.get("tools", {}))
        self.prompts: dict[str, Prompt] = {}
        for key, p in data["prompts"].items():
            self.prompts[key] = Prompt(
                id=p["id"], name=p["name"], version=p["version"],
                system_template=p["system_template"], user_template=p.get("user_template", ""),
                variables=list(p.get("variables", [])), tools=list(p.get("tools", [])),
                tool_policy=ToolPolicy.from_dict(p.get("tool_policy")),
                parameters=dict(p.get("parameters", {})),
                validators=list(p.get("validators", [])), evals=list(p.get("evals", [])), raw=p)
        self.workflow: dict | None = data.get("workflow")
        self.agents: dict | None = data.get("agents")
        self.skill_sources: list = list(data.get("skills", []))
        self.compositions: dict = dict(data.get("compositions", {}))
        self._check_graph()

    def _check_graph(self):
        """Cross-references of the workflow / agents sections."""
        errs = []
        wf = self.workflow
        if wf:
            states = wf["states"]
            if wf["entry"] not in states:
                errs.append(f"workflow.entry {wf['entry']!r} is not a state")
            for name, st in states.items():
                if st.get("orchestration") == "composition":
                    if st.get("composition") not in self.compositions:
                        errs.append(f"workflow state {name!r}: composition "
                                    f"{st.get('composition')!r} is not defined")
                elif st.get("prompt_task") not in self.prompts:
                    errs.append(f"workflow state {name!r}: prompt_task "
                                f"{st.get('prompt_task')!r} is not a prompt")
                for ev, target in (st.get("on_event") or {}).items():
                    if target not in states:
                        errs.append(f"workflow state {name!r}: event {ev!r} targets "
                                    f"unknown state {target!r}")
                if st.get("on_max_visits") and st["on_max_visits"] not in states:
                    errs.append(f"workflow state {name!r}: on_max_visits targets unknown "
                                f"state {st['on_max_visits']!r}")
        for cname, comp in self.compositions.items():
            errs += self._check_composition(cname, comp)
        ag = self.agents
        if ag:
            if ag["entry"] not in ag["members"]:
                errs.append(f"agents.entry {ag['entry']!r} is not a member")
            for key in ag["members"]:
                if key not in self.prompts:
                    errs.append(f"agents member {key!r} is not a prompt")
        if errs:
            raise PackError("invalid pack: " + "; ".join(errs[:5]))

    def _check_composition(self, cname: str, comp: dict) -> list[str]:
        errs, ids = [], []
        top = [s["id"] for s in comp["steps"]]

        def walk(step):
            ids.append(step["id"])
            k = step["kind"]
            where = f"composition {cname!r} step {step['id']!r}"
            if k in ("prompt", "agent") and step.get("prompt_task") not in self.prompts:
                errs.append(f"{where}: prompt_task {step.get('prompt_task')!r} is not a prompt")
            if k == "tool" and not step.get("tool"):
                errs.append(f"{where}: tool step needs 'tool'")
            if k == "parallel" and not step.get("branches"):
                errs.append(f"{where}: parallel step needs 'branches'")
            if k == "branch":
                if "predicate" not in step or "then" not in step:
                    errs.append(f"{where}: branch step needs 'predicate' and 'then'")
                for tgt in (step.get("then"), step.get("else")):
                    if tgt is not None and tgt not in top:
                        errs.append(f"{where}: branch target {tgt!r} is not a step")
            for d in step.get("depends_on") or []:
                if d not in top:
                    errs.append(f"{where}: depends_on {d!r} is not a step")
            for b in step.get("branches") or []:
                walk(b)

        for st in comp["steps"]:
            walk(st)
        dup = sorted({i for i in ids if ids.count(i) > 1})
        if dup:
            errs.append(f"composition {cname!r}: duplicate step ids {dup}")
        return errs

    def entry(self, fallback: str = "default") -> str:
        """Prompt key the runtime opens the pack at (``pack_entry.go:54-86``).
        A workflow whose entry state runs a composition opens at the first
        prompt (the composition's own steps name theirs)."""
        if self.workflow:
            st = self.workflow["states"][self.workflow["entry"]]
            return st.get("prompt_task") or next(iter(self.prompts))
        if self.agents:
            return self.agents["entry"]
        if len(self.prompts) == 1:
            return next(iter(self.prompts))
        return fallback

    def key_of(self, prompt: "Prompt") -> str:
        for k, p in self.prompts.items():
            if p is prompt:
                return k
        return prompt.id

    @classmethod
    def load(cls, path: str | Path) -> "PromptPack":
        p = Path(path)
        if p.is_dir():
            p = p / "pack.json"
        try:
            return cls(json.loads(p.read_text()), base_dir=p.parent)
        except json.JSONDecodeError as e:
            raise PackError(f"pack.json is not valid JSON: {e}") from e

    @classmethod
    def minimal(cls, system: str = "You are a helpful assistant.") -> "PromptPack":
        return cls({"id": "default", "name": "default", "version": "1.0.0",
                    "template_engine": {"version": "v1", "syntax": "{{variable}}"},
                    "prompts": {"default": {"id": "default", "name": "default",
                                            "version": "1.0.0", "system_template": system}}})

    def prompt(self, name: str | None = None) -> Prompt:
        if name and name in self.prompts:
            return self.prompts[name]
        if name:
            for p in self.prompts.values():
                if p.id == name or p.name == name:
                    return p
            raise PackError(f"prompt {name!r} not in pack {self.id}")
        key = self.entry()
        if key in self.prompts:
            return self.prompts[key]
        return next(iter(self.prompts.values()))

    # ------------------------------------------------------------ rendering
    def _expand_fragments(self, text: str, depth: int = 0) -> str:
        if depth > 8 or not self.fragments:
            return text

        def rep(m):
            name = m.group(2)
            if name in self.fragments:
                return self._expand_fragments(self.fragments[name], depth + 1)
            if name.startswith("fragment.") and name[9:] in self.fragments:
                return self._expand_fragments(self.fragments[name[9:]], depth + 1)
            return m.group(0)

        return _VAR.sub(rep, text)

    def resolve_variables(self, prompt: Prompt, values: dict | None) -> dict:
        values = dict(values or {})
        out = {}
        missing = []
        for v in prompt.variables:
            n = v["name"]
            if n in values:
                out[n] = values[n]
            elif "default" in v:
                out[n] = v["default"]
            elif v.get("required"):
                missing.append(n)
        for k, val in values.items():
            out.setdefault(k, val)
        if missing:
            raise PackError(f"missing required variables: {missing}")
        return out

    def render(self, template: str, variables: dict) -> str:
        text = self._expand_fragments(template)

        def rep(m):
            name = m.group(2)
            if name in variables:
                val = variables[name]
                return val if isinstance(val, str) else json.dumps(val)
            return m.group(0)

        return _VAR.sub(rep, text)

    def render_system(self, prompt: Prompt, variables: dict | None = None,
                      strict: bool = False) -> str:
        try:
            vs = self.resolve_variables(prompt, variables)
        except PackError:
            if strict:
                raise
            vs = dict(variables or {})
        return self.render(prompt.system_template, vs)

    def tool_specs(self, prompt: Prompt, registry_tools: dict | None = None) -> list[dict]:
        """Function specs visible to the model for this prompt (blocklist applied)."""
        if prompt.tool_policy.tool_choice == "none":
            return []
        names = list(prompt.tools)
        if not names and registry_tools:
            names = list(registry_tools)
        specs = []
        for n in names:
            if n in prompt.tool_policy.blocklist:
                continue
            spec = self.tools.get(n) or (registry_tools or {}).get(n)
            if spec is None:
                continue
            specs.append({"name": n, "description": spec.get("description", ""),
                          "parameters": spec.get("parameters",
                                                 spec.get("input_schema",
                                                          {"type": "object"}))})
        return specs


def run_validators(prompt: Prompt, text: str) -> list[str]:
    """Apply enabled guardrail validators; returns violation messages."""
    out = []
    for v in prompt.validators:
        if not v.get("enabled", False):
            continue
        t, p = v["type"], v.get("params", {}) or {}
        if t == "banned_words":
            words = [w.lower() for w in p.get("words", [])]
            low = text.lower()
            hit = [w for w in words if w and w in low]
            if hit:
                out.append(f"banned_words: {hit}")
        elif t == "max_length":
            n = int(p.get("max_characters", p.get("max", p.get("max_length", 10**9))))
            if len(text) > n:
                out.append(f"max_length: {len(text)} > {n}")
        elif t == "min_length":
            n = int(p.get("min_characters", p.get("min", p.get("min_length", 0))))
            if len(text) < n:
                out.append(f"min_length: {len(text)} < {n}")
        elif t == "regex_match":
            pat = p.get("pattern", "")
            if pat and not re.search(pat, text):
                out.append(f"regex_match: {pat!r} not found")
        elif t == "json_schema":
            try:
                jsonschema.validate(json.loads(text), p.get("schema", {}))
            except (json.JSONDecodeError, jsonschema.ValidationError) as e:
                out.append(f"json_schema: {e}")
        elif t == "pii_detection":
            from ..ee.redaction import find_pii

            found = find_pii(text)
            if found:
                out.append(f"pii_detection: {sorted(found)}")
    return out
