"""MemoryPolicy retention applied to the memory store.

Reference: ``api/v1alpha1/memorypolicy_types.go`` (tiers institutional /
agent / user, modes Manual / TTL / Decay / LRU / Composite, ``perCategory``
leaves, ``softDeleteGraceDays``), ``internal/memory/retention.go`` (the
retention pass), ``ee/pkg/memory`` decay scoring.

A pass over the live (not forgotten) entities of each configured tier:

* **TTL** -- ``ttl.maxAge``: entities created longer ago are forgotten;
  ``ttl.default``: entities without an expiry get ``created + default``
  (the store's own expiry sweep then hard-deletes them);
* **LRU** -- ``lru.staleAfter``: entities whose newest observation was neither
  observed nor accessed within the window are forgotten;
* **Decay** -- score = ``confidenceWeight * confidence + accessFrequencyWeight
  * min(1, accesses / 10) + recencyWeight * 0.5 ** (age_days / halfLifeDays)``
  (weights default 1/3 each, half-life 30 days); below ``minScore`` (default
  0.1) is forgotten;
* **Composite** -- all three; **Manual** -- nothing.

A tier's ``perCategory`` entry overrides it for entities whose consent
category matches.  Forgetting is a soft delete; ``softDeleteGraceDays`` later
the store's purge removes the rows (the retention worker passes the grace).
Tier of an entity: user id set -> user, else agent id set -> agent, else
institutional (``model.derive_tier``; user-for-agent counts as user).
"""
from __future__ import annotations

import time

from ..operator.policies import parse_duration

DEFAULT_HALF_LIFE_DAYS = 30.0
DEFAULT_MIN_SCORE = 0.1


def _tier_of(uid, aid) -> str:
    if uid:
        return "user"
    if aid:
        return "agent"
    return "institutional"


def decay_score(conf: float, accesses: int, age_s: float, dec: dict) -> float:
    f = dec.get("scoreFormula") or {}
    wc = float(f.get("confidenceWeight") or 1 / 3)
    wa = float(f.get("accessFrequencyWeight") or 1 / 3)
    wr = float(f.get("recencyWeight") or 1 / 3)
    half = float(dec.get("halfLifeDays") or DEFAULT_HALF_LIFE_DAYS)
    recency = 0.5 ** (age_s / 86400.0 / half)
    return wc * conf + wa * min(1.0, accesses / 10.0) + wr * recency


def _leaf_for(tier_cfg: dict, category: str | None) -> dict:
    per = tier_cfg.get("perCategory") or {}
    if category and category in per:
        return per[category]
    return tier_cfg


def apply_memory_policy(store, spec: dict, now: float | None = None) -> dict:
    """One retention pass; returns counters per action."""
    now = now or time.time()
    tiers = spec.get("tiers") or {}
    stats = {"ttl_expired": 0, "ttl_defaulted": 0, "lru_forgotten": 0, "decay_forgotten": 0}
    rows = store._q(
        "SELECT e.id, e.virtual_user_id, e.agent_id, e.consent_category, e.created_at, "
        "e.expires_at, max(o.observed_at), max(coalesce(o.accessed_at, 0)), "
        "max(o.confidence), sum(o.access_count) FROM memory_entities e "
        "LEFT JOIN memory_observations o ON o.entity_id = e.id "
        "WHERE e.forgotten = 0 GROUP BY e.id", ())
    forget, set_expiry = [], []
    for (eid, uid, aid, cat, created, expires, observed, accessed, conf, acc) in rows:
        tcfg = tiers.get(_tier_of(uid, aid))
        if not tcfg:
            continue
        leaf = _leaf_for(tcfg, cat)
        mode = leaf.get("mode") or tcfg.get("mode") or "Manual"
        if mode == "Manual":
            continue
        ttl = leaf.get("ttl") or {}
        if mode in ("TTL", "Composite"):
            if ttl.get("maxAge") and created < now - parse_duration(ttl["maxAge"]):
                forget.append(eid)
                stats["ttl_expired"] += 1
                continue
            if ttl.get("default") and expires is None:
                set_expiry.append((created + parse_duration(ttl["default"]), eid))
                stats["ttl_defaulted"] += 1
        lru = leaf.get("lru") or {}
        if mode in ("LRU", "Composite") and lru.get("staleAfter") and \
                lru.get("enabled", True) is not False:
            last = max(observed or 0.0, accessed or 0.0, created)
            if last < now - parse_duration(lru["staleAfter"]):
                forget.append(eid)
                stats["lru_forgotten"] += 1
                continue
        dec = leaf.get("decay") or {}
        if mode in ("Decay", "Composite") and dec and dec.get("enabled", True) is not False:
            s = decay_score(conf if conf is not None else 0.7, int(acc or 0),
                            now - (observed or created), dec)
            if s < float(dec.get("minScore") or DEFAULT_MIN_SCORE):
                forget.append(eid)
                stats["decay_forgotten"] += 1
    with store._tx() as db:
        if set_expiry:
            db.executemany("UPDATE memory_entities SET expires_at = ? WHERE id = ?", set_expiry)
        if forget:
            db.executemany("UPDATE memory_entities SET forgotten = 1, updated_at = ? "
                           "WHERE id = ?", [(now, e) for e in forget])
    return stats


def grace_seconds(spec: dict, default_days: float = 30.0) -> float:
    """The smallest ``softDeleteGraceDays`` of the configured tiers."""
    days = [float(t["softDeleteGraceDays"]) for t in (spec.get("tiers") or {}).values()
            if t and t.get("softDeleteGraceDays") is not None]
    return (min(days) if days else default_days) * 86400.0
