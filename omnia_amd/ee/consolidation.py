"""Memory consolidation: policy-driven passes that hand candidate buckets of
memory rows to a consolidation *function* (an AgentRuntime in function mode)
and apply the typed actions it returns, behind a validator.

Parity map (reference, read for behaviour only):

* axes + typed action vocabulary -- ``ee/pkg/memory/consolidation/types.go:26-190``
* scope shapes, buckets -- ``internal/memory/consolidation/types.go``
* pre-filter queries -- ``internal/memory/consolidation/prefilter.go`` (stale
  observations, cross-scope candidates, entity duplicates)
* validator + reasons -- ``ee/pkg/memory/consolidation/validator.go``
* PII gate -- ``ee/pkg/memory/consolidation/pii_gate.go``
* applier + audit outcomes -- ``ee/pkg/memory/consolidation/applier.go``
* function client -- ``ee/pkg/memory/consolidation/client.go``
* worker (lock, per-axis cron due check, anchor-then-run, mark-on-attempt,
  metrics) -- ``ee/pkg/memory/consolidation/worker.go``, ``metrics.go``

Design here: the pre-filters run as plain SQL over the memory store's dialect
layer (SQLite or Postgres), except the entity-duplicate axis, which needs an
all-pairs cosine over entity embeddings: that is one ``E @ E.T`` on the device
the vector index lives on (an MFMA GEMM through hipBLASLt on MI355X) per
(workspace, kind) group instead of the reference's pgvector self-join, so it
works on both dialects and scales with the GPU, not with a quadratic SQL join.
The lock store and the per-axis run tracker are rows in the store's
``memory_meta`` table, so several memory-api replicas sharing one database
coordinate through it (the reference uses Postgres advisory locks + a run
table).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
import uuid
from dataclasses import dataclass, field
from datetime import datetime, timezone

from ..observability import metrics as _m
from ..utils import cron

log = logging.getLogger("omnia.memory.consolidation")

AXIS_STALE = "staleObservations"
AXIS_CROSS_SCOPE = "crossScopeCandidates"
AXIS_ENTITY_DUPES = "entityDuplicateCandidates"
AXES = (AXIS_STALE, AXIS_CROSS_SCOPE, AXIS_ENTITY_DUPES)

SHAPE_INSTITUTIONAL = "institutional"
SHAPE_AGENT = "agent-scoped"
SHAPE_USER = "user-scoped"
SHAPE_USER_FOR_AGENT = "user-for-agent"

MUTABLE = "mutable"
GATE_AGENT = "agentScoped"
GATE_USER = "userScoped"

# validator rejection reasons (validator.go / pii_gate.go)
R_INSTITUTIONAL = "institutional_write_blocked"
R_MUTABILITY = "mutability_blocked"
R_ANONYMITY = "anonymity_below_threshold"
R_OUTSIDE_WS = "scope_outside_workspace"
R_WIDENING = "scope_widening_unsupported"
R_UNKNOWN = "target_unknown"
R_SHAPE = "shape_invalid"
R_PII = "pii_blocked"

APPLIED, REJECTED, APPLY_FAILED = "applied", "rejected_validation", "apply_failed"

PASSES = _m.Counter("omnia_memory_consolidation_passes_total",
                    "Consolidation passes by outcome",
                    ["workspace", "policy", "function", "status"], registry=_m.REGISTRY)
PASS_SECONDS = _m.Histogram("omnia_memory_consolidation_pass_duration_seconds",
                            "Consolidation pass wall time", ["workspace", "policy", "function"],
                            registry=_m.REGISTRY)
ACTIONS = _m.Counter("omnia_memory_consolidation_actions_total",
                     "Consolidation actions by kind and outcome",
                     ["workspace", "policy", "function", "action", "outcome", "tier"],
                     registry=_m.REGISTRY)
FN_SECONDS = _m.Histogram("omnia_memory_consolidation_function_call_duration_seconds",
                          "Consolidation function call latency",
                          ["workspace", "policy", "function"], registry=_m.REGISTRY)


# ------------------------------------------------------------------ model
@dataclass
class Scope:
    workspaceID: str = ""
    agentID: str = ""
    userID: str = ""

    def shape(self) -> str:
        if self.agentID and self.userID:
            return SHAPE_USER_FOR_AGENT
        if self.userID:
            return SHAPE_USER
        if self.agentID:
            return SHAPE_AGENT
        return SHAPE_INSTITUTIONAL

    @classmethod
    def of(cls, d) -> "Scope":
        if isinstance(d, Scope):
            return d
        d = d or {}
        return cls(str(d.get("workspaceID") or ""), str(d.get("agentID") or ""),
                   str(d.get("userID") or ""))

    def to_json(self) -> dict:
        out = {"workspaceID": self.workspaceID}
        if self.agentID:
            out["agentID"] = self.agentID
        if self.userID:
            out["userID"] = self.userID
        return out


@dataclass
class BucketEntry:
    id: str
    content: str
    scope: Scope
    mutability: str = MUTABLE
    sourceType: str = ""
    observedAt: float = 0.0
    metadata: dict = field(default_factory=dict)

    def to_json(self) -> dict:
        out = {"id": self.id, "content": self.content, "scope": self.scope.to_json(),
               "mutability": self.mutability, "sourceType": self.sourceType}
        if self.observedAt:
            out["observedAt"] = datetime.fromtimestamp(
                self.observedAt, timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        if self.metadata:
            out["metadata"] = self.metadata
        return out


@dataclass
class Bucket:
    key: str
    entries: list
    stats: dict = field(default_factory=dict)

    def to_json(self) -> dict:
        out = {"key": self.key, "entries": [e.to_json() for e in self.entries]}
        if self.stats:
            out["stats"] = self.stats
        return out


# the seven typed actions; field names are the wire names of the pack's output
_ACTION_FIELDS = {
    "create_summary": {"fromIDs": list, "scope": Scope.of, "content": str, "metadata": dict},
    "supersede": {"targetIDs": list, "withID": str},
    "rescope": {"targetIDs": list, "newScope": Scope.of, "reason": str},
    "invalidate": {"targetIDs": list, "validUntil": str, "reason": str},
    "merge_entities": {"canonicalID": str, "mergeIDs": list},
    "discard": {"targetIDs": list, "reason": str},
    "rescore": {"targetID": str, "importance": float, "confidence": float},
}


@dataclass
class Action:
    kind: str
    f: dict

    def get(self, k, default=None):
        return self.f.get(k, default)

    def modifying_targets(self) -> list:
        """Rows the action changes (checked for mutability); create_summary writes
        a new row and touches none."""
        k = self.kind
        if k in ("supersede", "rescope", "invalidate", "discard"):
            return list(self.f["targetIDs"])
        if k == "merge_entities":
            return list(self.f["mergeIDs"])
        if k == "rescore":
            return [self.f["targetID"]]
        return []

    def content_fields(self) -> list:
        k = self.kind
        if k == "create_summary":
            return [self.f["content"]]
        if k in ("rescope", "invalidate", "discard"):
            return [self.f["reason"]]
        return []


def _parse_time(v) -> float | None:
    if v in (None, ""):
        return None
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip().replace("Z", "+00:00")
    try:
        dt = datetime.fromisoformat(s)
    except ValueError:
        return None
    if dt.tzinfo is None:
        dt = dt.replace(tzinfo=timezone.utc)
    return dt.timestamp()


def unmarshal_actions(data) -> list[Action]:
    """Decode the function's JSON action array; an unknown action kind or a
    malformed element fails the whole response (no silent drops)."""
    raws = json.loads(data) if isinstance(data, (str, bytes, bytearray)) else data
    if not isinstance(raws, list):
        raise ValueError("decode action array: not a JSON array")
    out = []
    for i, raw in enumerate(raws):
        if not isinstance(raw, dict):
            raise ValueError(f"decode action[{i}] header: not an object")
        kind = raw.get("action")
        spec = _ACTION_FIELDS.get(kind)
        if spec is None:
            raise ValueError(f"decode action[{i}] ({kind}): unknown action kind: {kind!r}")
        f = {}
        for name, conv in spec.items():
            v = raw.get(name)
            if conv is list:
                if v is not None and not isinstance(v, list):
                    raise ValueError(f"decode action[{i}] ({kind}): {name} must be an array")
                f[name] = [str(x) for x in (v or [])]
            elif conv is dict:
                f[name] = {str(a): str(b) for a, b in (v or {}).items()}
            elif conv is float:
                f[name] = float(v or 0.0)
            elif conv is str:
                f[name] = "" if v is None else str(v)
            else:
                f[name] = conv(v)
        if kind == "invalidate":
            f["validUntilTs"] = _parse_time(f["validUntil"])
        out.append(Action(kind, f))
    return out


# ------------------------------------------------------------------ validator
@dataclass
class Result:
    action: Action
    accepted: bool = False
    reason: str = ""


@dataclass
class ValidationContext:
    row_mutability: dict = field(default_factory=dict)
    row_scope: dict = field(default_factory=dict)
    distinct_users: int = 0


class PIIGate:
    """Blocks actions whose free-text fields carry PII when the policy's
    ``safetyGates.requirePIIRedaction`` is on (default on)."""

    def __init__(self, redactor=None):
        self.redactor = redactor

    def check(self, a: Action, gates: dict) -> str:
        if self.redactor is None or not gates_pii_enabled(gates):
            return ""
        for s in a.content_fields():
            if s and self.redactor(s):
                return R_PII
        return ""


def regex_pii_detector(text: str) -> bool:
    from .redaction import find_pii

    return bool(find_pii(text))


def gates_pii_enabled(gates: dict) -> bool:
    v = (gates or {}).get("requirePIIRedaction")
    return True if v is None else bool(v)


class Validator:
    def __init__(self, workspace_id: str, gates: dict | None = None, pii_detector=None):
        self.ws = workspace_id
        self.gates = gates or {}
        self.pii = PIIGate(pii_detector)

    def validate(self, actions: list[Action], ctx: ValidationContext) -> list[Result]:
        return [self._one(a, ctx) for a in actions]

    def _one(self, a: Action, ctx: ValidationContext) -> Result:
        for check in (self._shape, self._mutability, self._institutional, self._anonymity,
                      self._scope):
            r = check(a, ctx)
            if r:
                return Result(a, False, r)
        r = self.pii.check(a, self.gates)
        return Result(a, not r, r)

    @staticmethod
    def _shape(a: Action, ctx) -> str:
        f, k = a.f, a.kind
        ok = {
            "create_summary": lambda: bool(f["fromIDs"]) and bool(f["content"]),
            "supersede": lambda: bool(f["targetIDs"]) and bool(f["withID"]),
            "rescope": lambda: bool(f["targetIDs"]),
            "invalidate": lambda: bool(f["targetIDs"]) and (f.get("validUntilTs") or 0)
            > time.time(),
            "merge_entities": lambda: bool(f["canonicalID"]) and bool(f["mergeIDs"]),
            "discard": lambda: bool(f["targetIDs"]),
            "rescore": lambda: bool(f["targetID"]),
        }[k]()
        return "" if ok else R_SHAPE

    @staticmethod
    def _mutability(a: Action, ctx: ValidationContext) -> str:
        for rid in a.modifying_targets():
            m = ctx.row_mutability.get(rid)
            if m is None:
                return R_UNKNOWN
            if m != MUTABLE:
                return R_MUTABILITY
        return ""

    @staticmethod
    def _institutional(a: Action, ctx) -> str:
        if a.kind == "rescope" and a.f["newScope"].shape() == SHAPE_INSTITUTIONAL:
            return R_INSTITUTIONAL
        return ""

    def _anonymity(self, a: Action, ctx: ValidationContext) -> str:
        if a.kind != "rescope":
            return ""
        key = {SHAPE_AGENT: GATE_AGENT, SHAPE_USER: GATE_USER}.get(a.f["newScope"].shape())
        if key is None:
            return ""
        need = int((self.gates.get("minDistinctUserCount") or {}).get(key) or 0)
        if need and ctx.distinct_users < need:
            return R_ANONYMITY
        return ""

    def _scope(self, a: Action, ctx) -> str:
        if a.kind != "rescope":
            return ""
        w = self.gates.get("maxScopeWidening") or ""
        if w and w != "workspace":
            return R_WIDENING
        if a.f["newScope"].workspaceID != self.ws:
            return R_OUTSIDE_WS
        return ""


# ------------------------------------------------------------------ store side
class ConsolidationStore:
    """The seven writes of the action vocabulary over :class:`MemoryStore`.

    IDs in bucket entries are observation ids (stale / cross-scope axes) or
    entity ids (entity-duplicate axis); every write accepts either: an entity id
    stands for that entity's active observations.  Provenance (pack, time, source
    rows) goes into the entity metadata so a consolidated row can be traced back.
    """

    def __init__(self, store):
        self.s = store

    def _ids(self, db, ids: list[str], workspace: str) -> tuple[list[str], list[str]]:
        """(observation ids, entity ids) of ``ids`` inside ``workspace``."""
        if not ids:
            return [], []
        ph = ",".join("?" * len(ids))
        now = time.time()
        obs = db.execute(
            f"SELECT o.id, o.entity_id FROM memory_observations o JOIN memory_entities e ON "
            f"e.id = o.entity_id WHERE e.workspace_id = ? AND (o.id IN ({ph}) OR "
            f"(o.entity_id IN ({ph}) AND o.superseded_by IS NULL AND (o.valid_until IS NULL "
            f"OR o.valid_until > ?)))", [workspace] + ids + ids + [now]).fetchall()
        return [r[0] for r in obs], sorted({r[1] for r in obs})

    def _provenance(self, db, entity_ids, pack, at, extra=None):
        for eid in entity_ids:
            row = db.execute("SELECT metadata FROM memory_entities WHERE id = ?",
                             (eid,)).fetchone()
            if row is None:
                continue
            meta = json.loads(row[0] or "{}")
            meta.update({"promoted_by_pack": pack, "promoted_at": at})
            meta.update(extra or {})
            db.execute("UPDATE memory_entities SET metadata = ?, updated_at = ? WHERE id = ?",
                       (json.dumps(meta), time.time(), eid))

    def save_summary(self, ws, scope: Scope, content, metadata, from_ids, pack, at) -> str:
        from ..memory.model import SCOPE_AGENT, SCOPE_USER, SCOPE_WORKSPACE, Memory

        sc = {SCOPE_WORKSPACE: ws}
        if scope.userID:
            sc[SCOPE_USER] = scope.userID
        if scope.agentID:
            sc[SCOPE_AGENT] = scope.agentID
        meta = dict(metadata or {})
        meta.update({"promoted_by_pack": pack, "promoted_at": at,
                     "consolidated_from": ",".join(from_ids)})
        res = self.s.save(Memory(type="summary", content=content, scope=sc, metadata=meta),
                          require_user=False)
        return res["observation_id"]

    def supersede(self, ws, target_ids, with_id, pack, at):
        with self.s._tx() as db:
            obs, ents = self._ids(db, target_ids, ws)
            if not obs:
                raise LookupError("no target rows in workspace")
            self.s._log_vectors(db, "delete", obs)
            db.execute(f"UPDATE memory_observations SET superseded_by = ? WHERE id IN "
                       f"({','.join('?' * len(obs))})", [with_id] + obs)
            self._provenance(db, ents, pack, at)

    def rescope(self, ws, target_ids, new_scope: Scope, reason, pack, at):
        with self.s._tx() as db:
            _, ents = self._ids(db, target_ids, ws)
            if not ents:
                raise LookupError("no target rows in workspace")
            for eid in ents:
                db.execute("UPDATE memory_entities SET virtual_user_id = ?, agent_id = ? "
                           "WHERE id = ? AND workspace_id = ?",
                           (new_scope.userID or None, new_scope.agentID or None, eid, ws))
            self._provenance(db, ents, pack, at, {"rescope_reason": reason} if reason else None)
            obs, _ = self._ids(db, ents, ws)
            self.s._log_vectors(db, "upsert", obs)  # scope filters of the index change

    def _end_validity(self, ws, target_ids, until, pack, at, extra):
        with self.s._tx() as db:
            obs, ents = self._ids(db, target_ids, ws)
            if not obs:
                raise LookupError("no target rows in workspace")
            if until <= time.time():
                self.s._log_vectors(db, "delete", obs)
            db.execute(f"UPDATE memory_observations SET valid_until = ? WHERE id IN "
                       f"({','.join('?' * len(obs))})", [until] + obs)
            self._provenance(db, ents, pack, at, extra)

    def invalidate(self, ws, target_ids, until, reason, pack, at):
        self._end_validity(ws, target_ids, until, pack, at,
                           {"invalidate_reason": reason} if reason else None)

    def discard(self, ws, target_ids, reason, pack, at):
        self._end_validity(ws, target_ids, time.time(), pack, at,
                           {"discard_reason": reason} if reason else None)

    def merge_entities(self, ws, canonical_id, merge_ids, pack, at):
        with self.s._tx() as db:
            _, canon = self._ids(db, [canonical_id], ws)
            row = db.execute("SELECT id FROM memory_entities WHERE id = ? AND workspace_id = ? "
                             "AND forgotten = 0", (canonical_id, ws)).fetchone()
            if row is None and not canon:
                raise LookupError(f"canonical entity {canonical_id} not in workspace")
            cid = row[0] if row else canon[0]
            _, ents = self._ids(db, merge_ids, ws)
            ents = [e for e in ents if e != cid]
            if not ents:
                raise LookupError("no mergeable entities in workspace")
            ph = ",".join("?" * len(ents))
            db.execute(f"UPDATE memory_observations SET entity_id = ? WHERE entity_id IN ({ph})",
                       [cid] + ents)
            db.execute(f"UPDATE memory_relations SET source_entity_id = ? WHERE "
                       f"source_entity_id IN ({ph})", [cid] + ents)
            db.execute(f"UPDATE memory_relations SET target_entity_id = ? WHERE "
                       f"target_entity_id IN ({ph})", [cid] + ents)
            for eid in ents:
                meta = json.loads(db.execute("SELECT metadata FROM memory_entities WHERE id = ?",
                                             (eid,)).fetchone()[0] or "{}")
                meta["merged_into"] = cid
                db.execute("UPDATE memory_entities SET forgotten = 1, metadata = ?, updated_at = ?"
                           " WHERE id = ?", (json.dumps(meta), time.time(), eid))
            self._provenance(db, [cid], pack, at, {"merged_from": ",".join(ents)})
            # the canonical entity's active observation set changed: the newest
            # stays active; the index re-reads them all
            obs, _ = self._ids(db, [cid], ws)
            self.s._log_vectors(db, "upsert", obs)

    def rescore(self, ws, target_id, importance, confidence, pack, at):
        with self.s._tx() as db:
            obs, ents = self._ids(db, [target_id], ws)
            if not obs:
                raise LookupError(f"target {target_id} not in workspace")
            if confidence:
                db.execute(f"UPDATE memory_observations SET confidence = ? WHERE id IN "
                           f"({','.join('?' * len(obs))})", [float(confidence)] + obs)
            self._provenance(db, ents, pack, at,
                             {"importance": str(importance)} if importance else None)


class Applier:
    """Applies accepted actions in order, records every outcome to the auditor;
    the first store failure stops the pass (later actions may depend on it)."""

    def __init__(self, store: ConsolidationStore, auditor=None):
        self.store, self.auditor = store, auditor

    def apply(self, ws: str, run_id: str, pack: str, results: list[Result],
              now: float | None = None) -> dict:
        now = now or time.time()
        at = datetime.fromtimestamp(now, timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        counts = {APPLIED: 0, REJECTED: 0, APPLY_FAILED: 0}
        for r in results:
            entry = {"runID": run_id, "workspaceID": ws, "packRef": pack,
                     "actionKind": r.action.kind, "targetIDs": r.action.modifying_targets(),
                     "now": now}
            if not r.accepted:
                counts[REJECTED] += 1
                self._audit(dict(entry, outcome=REJECTED, reason=r.reason))
                continue
            try:
                self._apply_one(ws, pack, at, r.action)
            except Exception as e:  # noqa: BLE001
                counts[APPLY_FAILED] += 1
                self._audit(dict(entry, outcome=APPLY_FAILED, reason=str(e)))
                raise RuntimeError(f"apply {r.action.kind}: {e}") from e
            counts[APPLIED] += 1
            self._audit(dict(entry, outcome=APPLIED, reason=""))
        return counts

    def _audit(self, e: dict):
        if self.auditor is None:
            return
        try:
            self.auditor(e)
        except Exception as ex:  # noqa: BLE001 - audit is best-effort
            log.warning("consolidation audit failed: %s", ex)

    def _apply_one(self, ws, pack, at, a: Action):
        s, f = self.store, a.f
        if a.kind == "create_summary":
            s.save_summary(ws, f["scope"] if f["scope"].workspaceID else Scope(ws),
                           f["content"], f["metadata"], f["fromIDs"], pack, at)
        elif a.kind == "supersede":
            s.supersede(ws, f["targetIDs"], f["withID"], pack, at)
        elif a.kind == "rescope":
            s.rescope(ws, f["targetIDs"], f["newScope"], f["reason"], pack, at)
        elif a.kind == "invalidate":
            s.invalidate(ws, f["targetIDs"], f["validUntilTs"], f["reason"], pack, at)
        elif a.kind == "merge_entities":
            s.merge_entities(ws, f["canonicalID"], f["mergeIDs"], pack, at)
        elif a.kind == "discard":
            s.discard(ws, f["targetIDs"], f["reason"], pack, at)
        elif a.kind == "rescore":
            s.rescore(ws, f["targetID"], f["importance"], f["confidence"], pack, at)
        else:
            raise ValueError(f"unknown action: {a.kind}")


def audit_logger_sink(logger):
    """Auditor writing consolidation outcomes into the EE audit log
    (``ee/audit.py``) as ``memory_consolidated`` events."""
    from .audit import Entry

    def sink(e: dict):
        logger.log_event(Entry(eventType="memory_consolidated", workspace=e["workspaceID"],
                               reason=e.get("reason", ""), resultCount=len(e["targetIDs"]),
                               metadata={k: e[k] for k in ("runID", "packRef", "actionKind",
                                                           "outcome", "targetIDs")}))
    return sink


# ------------------------------------------------------------------ pre-filters
@dataclass
class PreFilterOptions:
    workspace_id: str
    older_than: float = 0.0
    min_group_size: int = 5
    min_distinct_users: int = 0
    similarity_floor: float = 0.85
    max_buckets: int = 100
    max_per_bucket: int = 50


def validate_prefilter_options(axis: str, o: PreFilterOptions):
    if not o.workspace_id:
        raise ValueError(f"preFilter {axis}: WorkspaceID required")
    if axis == AXIS_STALE and (not o.older_than or o.min_group_size <= 0):
        raise ValueError(f"preFilter {axis}: OlderThan + MinGroupSize required")
    if axis == AXIS_CROSS_SCOPE and o.min_distinct_users <= 0:
        raise ValueError(f"preFilter {axis}: MinDistinctUsers required")
    if axis == AXIS_ENTITY_DUPES and o.similarity_floor <= 0:
        raise ValueError(f"preFilter {axis}: SimilarityFloor required")
    if o.max_buckets <= 0:
        raise ValueError(f"preFilter {axis}: MaxBucketsPerPass must be > 0")


_ELIGIBLE = ("SELECT o.id, e.workspace_id, e.virtual_user_id, e.agent_id, e.kind, "
             "coalesce(e.title, e.about_key, ''), o.content, o.observed_at, e.metadata, "
             "coalesce(e.source_type, '') FROM memory_observations o JOIN memory_entities e ON "
             "e.id = o.entity_id WHERE e.workspace_id = ? AND e.forgotten = 0 AND "
             "o.superseded_by IS NULL AND (o.valid_until IS NULL OR o.valid_until > ?) AND "
             "coalesce(e.source_type, '') != 'regulated'")


def _mutability(meta_json) -> str:
    try:
        return str(json.loads(meta_json or "{}").get("mutability") or MUTABLE)
    except ValueError:
        return MUTABLE


class PreFilterRunner:
    """Candidate buckets for each axis from the memory store.  Immutable rows
    (entity metadata ``mutability`` other than ``mutable``), regulated sources,
    superseded / expired observations and forgotten entities never enter a
    bucket."""

    def __init__(self, store, device=None):
        self.s = store
        self.device = device

    def _entry(self, r) -> BucketEntry:
        return BucketEntry(id=r[0], content=r[6] or "",
                           scope=Scope(r[1], r[3] or "", r[2] or ""),
                           mutability=_mutability(r[8]), sourceType=r[9] or "",
                           observedAt=float(r[7] or 0.0))

    def stale_observations(self, o: PreFilterOptions) -> list[Bucket]:
        validate_prefilter_options(AXIS_STALE, o)
        rows = self.s._q(_ELIGIBLE + " AND o.observed_at < ? ORDER BY e.virtual_user_id, "
                         "e.agent_id, e.kind, 6, o.observed_at LIMIT ?",
                         [o.workspace_id, time.time(), o.older_than,
                          o.max_buckets * max(1, o.max_per_bucket)])
        groups: dict = {}
        for r in rows:
            if _mutability(r[8]) != MUTABLE:
                continue
            key = "|".join(str(x or "") for x in (r[2], r[3], r[4], r[5]))
            groups.setdefault(key, []).append(self._entry(r))
        out = []
        for key, ents in groups.items():
            if len(ents) < o.min_group_size:
                continue
            out.append(Bucket(key, ents[:o.max_per_bucket], {"size": len(ents)}))
            if len(out) >= o.max_buckets:
                break
        return out

    def cross_scope_candidates(self, o: PreFilterOptions) -> list[Bucket]:
        validate_prefilter_options(AXIS_CROSS_SCOPE, o)
        rows = self.s._q(_ELIGIBLE + " AND e.virtual_user_id IS NOT NULL ORDER BY e.kind, 6, "
                         "o.observed_at DESC", [o.workspace_id, time.time()])
        groups: dict = {}
        for r in rows:
            if _mutability(r[8]) != MUTABLE:
                continue
            groups.setdefault(f"{r[4]}|{r[5]}", []).append((r[2], self._entry(r)))
        out = []
        for key, items in groups.items():
            users = {u for u, _ in items}
            if len(users) < o.min_distinct_users:
                continue
            out.append(Bucket(key, [e for _, e in items[:o.max_per_bucket]],
                              {"distinctUsers": len(users), "size": len(items)}))
            if len(out) >= o.max_buckets:
                break
        return out

    def entity_duplicate_candidates(self, o: PreFilterOptions) -> list[Bucket]:
        """Pairs of same-kind entities whose active-observation embeddings have
        cosine >= the floor: one normalised ``E @ E.T`` per kind on the index
        device, upper triangle, most similar first."""
        import numpy as np
        import torch

        validate_prefilter_options(AXIS_ENTITY_DUPES, o)
        now = time.time()
        rows = self.s._q(
            "SELECT e.id, e.kind, coalesce(e.title, e.about_key, ''), o.content, "
            f"{self.s.d.vec_select()}, "
            "e.virtual_user_id, e.agent_id, e.metadata, coalesce(e.source_type, ''), "
            "o.observed_at FROM memory_entities e JOIN memory_observations o ON o.entity_id = "
            "e.id WHERE e.workspace_id = ? AND e.forgotten = 0 AND o.superseded_by IS NULL AND "
            "(o.valid_until IS NULL OR o.valid_until > ?) AND o.embedding IS NOT NULL ORDER BY "
            "e.id, o.observed_at DESC", [o.workspace_id, now])
        latest: dict = {}
        for r in rows:
            if r[0] not in latest and _mutability(r[7]) == MUTABLE:
                latest[r[0]] = r
        by_kind: dict = {}
        for r in latest.values():
            by_kind.setdefault(r[1], []).append(r)
        dev = self.device or ("cuda" if torch.cuda.is_available() else "cpu")
        pairs = []
        for kind, ents in by_kind.items():
            if len(ents) < 2:
                continue
            vecs = [np.asarray(self.s._vec(r[4]), dtype=np.float32).ravel() for r in ents]
            dim = max(v.size for v in vecs)
            keep = [i for i, v in enumerate(vecs) if v.size == dim]
            e = torch.from_numpy(np.stack([vecs[i] for i in keep])).to(dev)
            e = torch.nn.functional.normalize(e, dim=1)
            sim = torch.triu(e @ e.T, diagonal=1)
            idx = torch.nonzero(sim >= o.similarity_floor)
            vals = sim[idx[:, 0], idx[:, 1]].cpu().tolist()
            for (i, j), v in zip(idx.cpu().tolist(), vals):
                a, b = ents[keep[i]], ents[keep[j]]
                if a[0] > b[0]:
                    a, b = b, a
                pairs.append((v, kind, a, b))
        pairs.sort(key=lambda p: -p[0])
        out = []
        for v, kind, a, b in pairs[:o.max_buckets]:
            ents = [BucketEntry(id=r[0], content=r[3] or "", scope=Scope(o.workspace_id,
                                r[6] or "", r[5] or ""), mutability=MUTABLE,
                                sourceType=r[8] or "", observedAt=float(r[9] or 0.0),
                                metadata={"name": r[2] or "", "kind": kind}) for r in (a, b)]
            out.append(Bucket(f"{kind}|{a[0]}|{b[0]}", ents,
                              {"similarity": round(float(v), 6), "canonicalID": a[0]}))
        return out

    def run(self, axis: str, o: PreFilterOptions) -> list[Bucket]:
        fn = {AXIS_STALE: self.stale_observations, AXIS_CROSS_SCOPE: self.cross_scope_candidates,
              AXIS_ENTITY_DUPES: self.entity_duplicate_candidates}.get(axis)
        if fn is None:
            raise ValueError(f"unknown axis: {axis}")
        return fn(o)


# ------------------------------------------------------------------ coordination
class MetaLockStore:
    """Per-(workspace, trigger) lease rows in ``memory_meta``: replicas sharing
    the store never run the same workspace's pass concurrently; a crashed
    holder's lease expires after ``ttl_s``."""

    def __init__(self, store, ttl_s: float = 3600.0, owner: str | None = None):
        self.s, self.ttl = store, ttl_s
        self.owner = owner or uuid.uuid4().hex

    def try_lock(self, workspace: str, trigger: str):
        key = f"lock:{trigger}:{workspace}"
        now = time.time()
        with self.s._tx() as db:
            row = db.execute("SELECT value FROM memory_meta WHERE key = ?", (key,)).fetchone()
            if row is not None:
                cur = json.loads(row[0])
                if cur.get("owner") != self.owner and cur.get("until", 0) > now:
                    return False, None
                db.execute("UPDATE memory_meta SET value = ? WHERE key = ?",
                           (json.dumps({"owner": self.owner, "until": now + self.ttl}), key))
            else:
                db.execute("INSERT INTO memory_meta (key, value) VALUES (?, ?)",
                           (key, json.dumps({"owner": self.owner, "until": now + self.ttl})))

        def release():
            with self.s._tx() as db:
                row = db.execute("SELECT value FROM memory_meta WHERE key = ?", (key,)).fetchone()
                if row is not None and json.loads(row[0]).get("owner") == self.owner:
                    db.execute("DELETE FROM memory_meta WHERE key = ?", (key,))
        return True, release


class MetaRunTracker:
    """Last attempt time per (policy, workspace, axis) in ``memory_meta``."""

    def __init__(self, store):
        self.s = store

    @staticmethod
    def _key(policy, ws, axis):
        return f"consolidation_run:{policy}:{ws}:{axis}"

    def last_run(self, policy, ws, axis):
        row = self.s._q("SELECT value FROM memory_meta WHERE key = ?",
                        [self._key(policy, ws, axis)])
        return (float(row[0][0]), True) if row else (0.0, False)

    def mark_run(self, policy, ws, axis, at: float):
        k = self._key(policy, ws, axis)
        with self.s._tx() as db:
            if db.execute("SELECT 1 FROM memory_meta WHERE key = ?", (k,)).fetchone():
                db.execute("UPDATE memory_meta SET value = ? WHERE key = ?", (repr(at), k))
            else:
                db.execute("INSERT INTO memory_meta (key, value) VALUES (?, ?)", (k, repr(at)))


def axis_due(schedule: str, last: float, now: float) -> bool:
    return cron.next_fire(schedule, last) <= now


# ------------------------------------------------------------------ function client
class FunctionClient:
    """POSTs the FunctionInput to the function AgentRuntime's facade
    (``/functions/<name>``) and decodes the action array.  ``base_url``
    overrides the in-cluster address (tests, single-node); ``resolve(name, ns)``
    maps a Service to a local ``host:port`` the way the single-node launcher's
    cluster DNS does."""

    def __init__(self, timeout_s: float = 30.0, base_url: str = "", resolve=None,
                 headers: dict | None = None):
        self.timeout, self.base_url, self.resolve = timeout_s, base_url.rstrip("/"), resolve
        self.headers = headers or {}

    def url_for(self, ref: dict) -> str:
        name, ns = ref.get("name", ""), ref.get("namespace", "")
        if self.base_url:
            return f"{self.base_url}/functions/{name}"
        if not ns:
            raise ValueError("MemoryFunctionRef.namespace required (no global fallback)")
        ep = self.resolve(name, ns) if self.resolve else None
        host = ep or f"{name}.{ns}.svc.cluster.local:8080"
        return f"http://{host}/functions/{name}"

    async def call(self, ref: dict, fn_input: dict, timeout_s: float | None = None):
        import aiohttp

        url = self.url_for(ref)
        t = aiohttp.ClientTimeout(total=timeout_s or self.timeout)
        async with aiohttp.ClientSession(timeout=t) as sess:
            async with sess.post(url, json=fn_input, headers={
                    "Accept": "application/json", **self.headers}) as resp:
                body = await resp.read()
                if resp.status != 200:
                    raise RuntimeError(f"function returned {resp.status}: {body[:512]!r}")
        return unmarshal_actions(body)


# ------------------------------------------------------------------ listers
def workspace_opts_into(ws_obj: dict, policy_name: str) -> bool:
    """A Workspace takes part in a policy's passes when one of its service
    groups' memory block references the policy (``workspace_lister.go``)."""
    for sg in ((ws_obj or {}).get("spec") or {}).get("services") or []:
        ref = ((sg or {}).get("memory") or {}).get("policyRef") or {}
        if ref.get("name") == policy_name:
            return True
    return False


class KubePolicyLister:
    """Cluster-scoped MemoryPolicies with a consolidation block, as
    (name, spec) pairs, from any client with ``list(kind, ns)``
    (``operator/kube.py`` KubeClient, or the in-repo API store)."""

    def __init__(self, client):
        self.client = client

    def __call__(self) -> list:
        return [(o["metadata"]["name"], o.get("spec") or {})
                for o in self.client.list("MemoryPolicy", None)]


class KubeWorkspaceLister:
    """Only this memory-api's own Workspace, and only if it opts into the
    policy; memory rows are keyed by the Workspace UID (its name when the object
    carries no UID, as in single-node mode)."""

    def __init__(self, client, own_workspace: str):
        self.client, self.own = client, own_workspace

    def __call__(self, policy_name: str) -> list:
        if not self.own:
            return []
        getter = getattr(self.client, "try_get", None)
        w = getter("Workspace", self.own, None) if getter else \
            self.client.get("Workspace", self.own, None)
        if not w or not workspace_opts_into(w, policy_name):
            return []
        return [w["metadata"].get("uid") or w["metadata"]["name"]]


# ------------------------------------------------------------------ worker
def resolved_schedule(spec: dict, axis: str) -> str:
    c = (spec or {}).get("consolidation") or {}
    return ((c.get("schedules") or {}).get(axis) or c.get("schedule") or "0 2 * * *")


def resolved_timeouts(spec: dict) -> tuple[float, float]:
    from ..utils.durations import parse_duration

    t = ((spec or {}).get("consolidation") or {}).get("timeouts") or {}
    fn = parse_duration(t["functionCall"]) if t.get("functionCall") else 30.0
    wall = parse_duration(t["passWallClock"]) if t.get("passWallClock") else 600.0
    return fn, wall


def resolved_gates(spec: dict) -> dict:
    g = dict(((spec or {}).get("consolidation") or {}).get("safetyGates") or {})
    g.setdefault("minDistinctUserCount", {})
    g.setdefault("requirePIIRedaction", True)
    return g


class ConsolidationWorker:
    """One pass = for every MemoryPolicy with ``spec.consolidation`` and every
    workspace bound to it: take the workspace lock, and for every axis with a
    functionRef that is due by its cron schedule run pre-filter -> function ->
    validator -> applier.  First sight of an axis only anchors its schedule
    (no catch-up storm on start); the run is marked on attempt, so a failing
    function is retried at the next fire time, not every tick."""

    def __init__(self, store, policies, workspaces=None, client: FunctionClient | None = None,
                 interval_s: float = 60.0, pii_detector=regex_pii_detector, auditor=None,
                 lock_store=None, run_tracker=None, now=time.time, device=None):
        self.store = store
        self.policies = policies  # callable -> [(name, spec)] or a list of them
        self.workspaces = workspaces  # callable(policy_name) -> [workspace ids]
        self.client = client or FunctionClient()
        self.interval = interval_s
        self.pii = pii_detector
        self.applier = Applier(ConsolidationStore(store), auditor)
        self.prefilter = PreFilterRunner(store, device)
        self.locks = lock_store or MetaLockStore(store)
        self.tracker = run_tracker if run_tracker is not None else MetaRunTracker(store)
        self.now = now
        self.call_function = self.client.call
        self.last_results: list = []

    def _policies(self):
        p = self.policies() if callable(self.policies) else self.policies
        return [(n, s) for n, s in p]

    def _workspaces(self, policy_name):
        if self.workspaces is None:
            return [policy_name]
        return list(self.workspaces(policy_name))

    async def run_once(self) -> list[dict]:
        """Returns one record per attempted axis (tests, doctor)."""
        self.last_results = []
        first_err = None
        for name, spec in self._policies():
            if not (spec or {}).get("consolidation"):
                continue
            for ws in self._workspaces(name):
                try:
                    await self._run_workspace(name, spec, ws)
                except Exception as e:  # noqa: BLE001
                    log.error("consolidation workspace %s (policy %s) failed: %s", ws, name, e)
                    first_err = first_err or e
        if first_err is not None:
            raise first_err
        return self.last_results

    async def _run_workspace(self, policy, spec, ws):
        ok, release = self.locks.try_lock(ws, "consolidation")
        if not ok:
            log.debug("consolidation tick skipped: lock_unavailable ws=%s", ws)
            self.last_results.append({"workspace": ws, "status": "lock_unavailable"})
            return
        try:
            _, wall = resolved_timeouts(spec)
            refs = (spec["consolidation"].get("functionRefs") or {})
            gates = resolved_gates(spec)

            async def axes():
                for axis in AXES:
                    if refs.get(axis):
                        await self._maybe_run_axis(axis, refs[axis], policy, spec, ws, gates)
            await asyncio.wait_for(axes(), wall)
        finally:
            release()

    async def _maybe_run_axis(self, axis, ref, policy, spec, ws, gates):
        if self.tracker is None:
            await self._run_axis_logged(axis, ref, policy, spec, ws, gates)
            return
        now = self.now()
        last, seen = self.tracker.last_run(policy, ws, axis)
        if not seen:
            self.tracker.mark_run(policy, ws, axis, now)  # anchor, do not run
            self.last_results.append({"workspace": ws, "axis": axis, "status": "anchored"})
            return
        try:
            due = axis_due(resolved_schedule(spec, axis), last, now)
        except cron.CronError as e:
            log.error("consolidation invalid cron schedule for %s: %s", axis, e)
            return
        if not due:
            self.last_results.append({"workspace": ws, "axis": axis, "status": "not_due"})
            return
        await self._run_axis_logged(axis, ref, policy, spec, ws, gates)
        self.tracker.mark_run(policy, ws, axis, now)  # mark on attempt

    async def _run_axis_logged(self, *a):
        try:
            await self.run_axis(*a)
        except Exception as e:  # noqa: BLE001
            log.error("consolidation axis %s failed: %s", a[0], e)

    def _prefilter_options(self, spec, ws) -> PreFilterOptions:
        c = spec.get("consolidation") or {}
        lim = c.get("candidateLimits") or {}
        gates = resolved_gates(spec)
        return PreFilterOptions(
            workspace_id=ws, older_than=self.now() - 30 * 86400, min_group_size=5,
            min_distinct_users=int((gates.get("minDistinctUserCount") or {}).get(GATE_AGENT)
                                   or 0) or 1,
            similarity_floor=0.85, max_buckets=int(lim.get("maxBucketsPerPass") or 100),
            max_per_bucket=int(lim.get("maxPerBucket") or 50))

    async def run_axis(self, axis, ref, policy, spec, ws, gates) -> dict:
        start = self.now()
        fname = ref.get("name", "")
        rec = {"workspace": ws, "axis": axis, "status": "ok"}
        self.last_results.append(rec)
        try:
            opts = self._prefilter_options(spec, ws)
            try:
                buckets = await asyncio.to_thread(self.prefilter.run, axis, opts)
            except Exception:
                rec["status"] = "prefilter_error"
                raise
            rec["buckets"] = len(buckets)
            if not buckets:
                rec["status"] = "empty"
                return rec
            fn_input = {"axis": axis, "workspaceID": ws,
                        "buckets": [b.to_json() for b in buckets],
                        "gates": {"minDistinctUserCount": gates.get("minDistinctUserCount") or {},
                                  "requirePIIRedaction": gates_pii_enabled(gates)}}
            fn_t, _ = resolved_timeouts(spec)
            t0 = self.now()
            try:
                actions = await asyncio.wait_for(self.call_function(ref, fn_input, fn_t), fn_t)
            except Exception:
                rec["status"] = "function_error"
                raise
            finally:
                FN_SECONDS.labels(ws, policy, fname).observe(max(0.0, self.now() - t0))
            ctx = ValidationContext(distinct_users=max(
                [int(b.stats.get("distinctUsers", 0)) for b in buckets] + [0]))
            for b in buckets:
                for e in b.entries:
                    ctx.row_mutability[e.id] = e.mutability
                    ctx.row_scope[e.id] = e.scope
            results = Validator(ws, gates, self.pii).validate(actions, ctx)
            for r in results:
                tier = r.action.f["newScope"].shape() if r.action.kind == "rescope" else ""
                ACTIONS.labels(ws, policy, fname, r.action.kind,
                               APPLIED if r.accepted else "rejected_" + r.reason, tier).inc()
            rec["results"] = [(r.action.kind, r.accepted, r.reason) for r in results]
            try:
                rec["counts"] = await asyncio.to_thread(
                    self.applier.apply, ws, f"{ws}-{int(self.now())}", fname, results,
                    self.now())
            except Exception:
                rec["status"] = "apply_error"
                raise
            return rec
        finally:
            PASSES.labels(ws, policy, fname, rec["status"]).inc()
            PASS_SECONDS.labels(ws, policy, fname).observe(max(0.0, self.now() - start))

    async def run(self):
        if self.interval <= 0:
            log.info("consolidation worker disabled: interval not set")
            return
        _m.MEMORY_WORKER_RUNNING.labels("consolidation").set(1)
        try:
            while True:
                await asyncio.sleep(self.interval)
                try:
                    await self.run_once()
                except Exception as e:  # noqa: BLE001
                    log.error("consolidation pass failed: %s", e)
        finally:
            _m.MEMORY_WORKER_RUNNING.labels("consolidation").set(0)

