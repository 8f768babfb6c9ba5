"""Ranking math shared by the store and the runtime retriever.

* ``compute_score`` / ``recency_decay``: ``internal/memory/retrieve_multi_tier.go:126-129,
  496-521`` (0.5 confidence + 0.3 log-frequency + 0.2 exp recency with per-tier
  half-life, default 30 days each).
* ``rrf_fuse``: Reciprocal Rank Fusion, k=60 (``internal/runtime/memory_retriever.go:248``).
* ``TierRanker``: MemoryPolicy per-tier bias applied after the base score.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

from .model import Tier

WEIGHT_CONFIDENCE = 0.5
WEIGHT_FREQUENCY = 0.3
WEIGHT_RECENCY = 0.2
FREQ_LOG_CEILING = 100.0
RRF_K = 60.0
HYBRID_FANOUT = 100
ANN_OVERFETCH = 4
CANDIDATE_POOL = 200
DEFAULT_LIMIT = 15
DAY = 86400.0


@dataclass
class HalfLife:
    user: float = 30 * DAY
    agent: float = 30 * DAY
    institutional: float = 30 * DAY

    def for_tier(self, tier: str) -> float:
        if tier in (Tier.USER, Tier.USER_FOR_AGENT):
            return self.user
        if tier == Tier.AGENT:
            return self.agent
        return self.institutional


@dataclass
class TierRanker:
    """score' = score * weight[tier] + boost[tier]  (identity by default)."""

    weights: dict = field(default_factory=dict)
    boosts: dict = field(default_factory=dict)

    def adjust(self, score: float, tier: str) -> float:
        return score * float(self.weights.get(tier, 1.0)) + float(self.boosts.get(tier, 0.0))


def tier_ranker_from_policy(spec: dict | None) -> TierRanker:
    """EE tier precedence (``ee/pkg/memory/tier_ranking.go``): MemoryPolicy
    ``tierPrecedence.multiplicative.{institutional,agent,user}`` weights (decimal
    strings, default 1.0); user-for-agent rows take the user weight.  A weight
    that does not parse makes the whole ranker the identity (fail open to the
    unbiased score, as the reference does)."""
    mult = ((spec or {}).get("tierPrecedence") or {}).get("multiplicative")
    if not mult:
        return TierRanker()
    w = {Tier.INSTITUTIONAL: 1.0, Tier.AGENT: 1.0, Tier.USER: 1.0}
    for tier in (Tier.INSTITUTIONAL, Tier.AGENT, Tier.USER):
        raw = mult.get(tier)
        if raw in (None, ""):
            continue
        try:
            w[tier] = float(raw)
        except (TypeError, ValueError):
            return TierRanker()
    w[Tier.USER_FOR_AGENT] = w[Tier.USER]
    return TierRanker(weights=w)


def half_life_from_policy(spec: dict | None) -> HalfLife:
    """``recall.halfLife.{user,agent,institutional}`` durations ("90d", "720h");
    missing, malformed or non-positive values keep the 30-day default."""
    from ..utils.durations import parse_duration

    hl = HalfLife()
    cfg = (((spec or {}).get("recall") or {}).get("halfLife")) or {}
    for tier in ("user", "agent", "institutional"):
        try:
            v = parse_duration(cfg.get(tier) or "")
        except ValueError:
            continue
        if v > 0:
            setattr(hl, tier, v)
    return hl


def recency_decay(age_s: float, half_life_s: float) -> float:
    if half_life_s <= 0:
        return 1.0
    return math.exp(max(-700.0, -math.log(2) * max(0.0, age_s) / half_life_s))


def compute_score(confidence: float, access_count: int, ref_time: float, now: float,
                  half_life_s: float) -> float:
    freq = math.log1p(max(0, access_count)) / math.log1p(FREQ_LOG_CEILING)
    freq = min(1.0, max(0.0, freq))
    return (WEIGHT_CONFIDENCE * confidence + WEIGHT_FREQUENCY * freq +
            WEIGHT_RECENCY * recency_decay(now - ref_time, half_life_s))


def rrf_fuse(lists, k: float = RRF_K, limit: int | None = None, key=lambda m: m.id):
    """Fuse ranked lists: score += 1/(k + rank + 1); ties keep first-seen order."""
    scores, by_id, order = {}, {}, []
    for lst in lists:
        for rank, m in enumerate(lst or []):
            if m is None:
                continue
            i = key(m)
            if i not in by_id:
                by_id[i] = m
                order.append(i)
            scores[i] = scores.get(i, 0.0) + 1.0 / (k + rank + 1.0)
    order.sort(key=lambda i: -scores[i])  # stable
    out = [by_id[i] for i in order]
    return out[:limit] if limit is not None else out


def rrf_ranks(fts_rank: dict, cos_rank: dict, k: float = RRF_K) -> dict:
    """Per-entity fused score from 1-based rank maps (FULL OUTER JOIN semantics
    of the hybrid SQL, ``retrieve_multi_tier_hybrid.go:157-160``)."""
    out = {}
    for e in set(fts_rank) | set(cos_rank):
        s = 0.0
        if e in fts_rank:
            s += 1.0 / (k + fts_rank[e])
        if e in cos_rank:
            s += 1.0 / (k + cos_rank[e])
        out[e] = s
    return out
