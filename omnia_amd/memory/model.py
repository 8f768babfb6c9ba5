"""Memory record + scope/tier vocabulary (``internal/memory/store.go:35-47``,
``internal/memory/api/handler.go:49-110``)."""
from __future__ import annotations

import time
import uuid
from dataclasses import dataclass, field

SCOPE_WORKSPACE = "workspace_id"
SCOPE_USER = "virtual_user_id"
SCOPE_LEGACY_USER = "user_id"  # pre-#1280 wire name, accepted on input
SCOPE_AGENT = "agent_id"

META_CONSENT_CATEGORY = "consent_category"
META_ABOUT_KIND = "about_kind"
META_ABOUT_KEY = "about_key"
META_TITLE = "title"
META_SOURCE_TYPE = "source_type"
META_PURPOSE = "purpose"

INLINE_BODY_THRESHOLD = 2048  # bytes; larger bodies recall as a preview
PREVIEW_RUNES = 240

AUTO_SUPERSEDE_SIMILARITY = 0.95
SURFACE_DUPLICATE_SIMILARITY = 0.85
DUPLICATE_CANDIDATE_LIMIT = 5

SOURCE_TYPE_WEIGHT = {"user_requested": 1.0, "operator_curated": 1.0, "reflection": 0.85,
                      "conversation_extraction": 0.7, "system_generated": 0.5}
PII_CATEGORIES = ("memory:identity", "memory:location", "memory:health")
PROFILE_CATEGORIES = ("memory:identity", "memory:preferences", "memory:health")


class Tier:
    INSTITUTIONAL = "institutional"
    AGENT = "agent"
    USER = "user"
    USER_FOR_AGENT = "user_for_agent"
    ALL = (INSTITUTIONAL, AGENT, USER, USER_FOR_AGENT)


def derive_tier(scope: dict) -> str:
    u = bool(scope.get(SCOPE_USER))
    a = bool(scope.get(SCOPE_AGENT))
    if u and a:
        return Tier.USER_FOR_AGENT
    if u:
        return Tier.USER
    if a:
        return Tier.AGENT
    return Tier.INSTITUTIONAL


def normalize_scope(scope: dict | None) -> dict:
    s = {k: str(v) for k, v in (scope or {}).items() if v not in (None, "")}
    if SCOPE_LEGACY_USER in s and SCOPE_USER not in s:
        s[SCOPE_USER] = s.pop(SCOPE_LEGACY_USER)
    else:
        s.pop(SCOPE_LEGACY_USER, None)
    return s


def new_id() -> str:
    return str(uuid.uuid4())


@dataclass
class Memory:
    id: str = ""
    type: str = "fact"
    content: str = ""
    confidence: float = 0.7
    scope: dict = field(default_factory=dict)
    metadata: dict = field(default_factory=dict)
    session_id: str = ""
    turn_range: list | None = None
    created_at: float = field(default_factory=time.time)
    accessed_at: float = 0.0
    expires_at: float | None = None
    observation_id: str = ""
    observed_at: float = 0.0
    access_count: int = 0
    title: str = ""
    summary: str = ""
    score: float = 0.0
    tier: str = ""

    def to_json(self, inline_preview: bool = False, related: list | None = None) -> dict:
        d = {"id": self.id, "type": self.type, "content": self.content,
             "confidence": self.confidence, "scope": self.scope, "metadata": self.metadata,
             "created_at": _iso(self.created_at), "tier": self.tier or derive_tier(self.scope)}
        if self.session_id:
            d["session_id"] = self.session_id
        if self.turn_range:
            d["turn_range"] = list(self.turn_range)
        if self.accessed_at:
            d["accessed_at"] = _iso(self.accessed_at)
        if self.access_count:
            d["access_count"] = self.access_count
        if self.expires_at:
            d["expires_at"] = _iso(self.expires_at)
        if self.title:
            d["title"] = self.title
        if self.summary:
            d["summary"] = self.summary
        if self.score:
            d["score"] = self.score
        size = len(self.content.encode())
        if inline_preview and size > INLINE_BODY_THRESHOLD:
            d["content_preview"] = self.content[:PREVIEW_RUNES]
            d["content"] = d["content_preview"]
            d["body_size_bytes"] = size
            d["has_full_body"] = True
        if related:
            d["related"] = related
        return d


def _iso(ts: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(ts)) + f".{int(ts % 1 * 1000):03d}Z"


def parse_time(v) -> float | None:
    if v in (None, ""):
        return None
    if isinstance(v, (int, float)):
        return float(v)
    import datetime as dt

    return dt.datetime.fromisoformat(str(v).replace("Z", "+00:00")).timestamp()
