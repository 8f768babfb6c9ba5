"""Session data model (``internal/session/store.go:40-523``), JSON in the
reference's camelCase field names so dashboards/clients interoperate."""
from __future__ import annotations

import time
import uuid
from dataclasses import asdict, dataclass, field, fields

ROLE_USER, ROLE_ASSISTANT, ROLE_SYSTEM = "user", "assistant", "system"
STATUS_ACTIVE, STATUS_COMPLETED, STATUS_ERROR, STATUS_EXPIRED = (
    "active", "completed", "error", "expired")
TERMINAL = {STATUS_COMPLETED, STATUS_ERROR, STATUS_EXPIRED}


def _camel(s: str) -> str:
    p = s.split("_")
    return p[0] + "".join(x.capitalize() for x in p[1:])


def _snake(s: str) -> str:
    out = []
    for ch in s:
        if ch.isupper():
            out.append("_" + ch.lower())
        else:
            out.append(ch)
    return "".join(out)


class _JSON:
    def to_json(self) -> dict:
        d = {}
        for f in fields(self):
            v = getattr(self, f.name)
            if v in (None, "", [], {}) and f.name not in ("messages",):
                continue
            if isinstance(v, list) and v and hasattr(v[0], "to_json"):
                v = [x.to_json() for x in v]
            d[_camel(f.name)] = v
        return d

    @classmethod
    def from_json(cls, d: dict):
        """Build from a JSON object; a field of the wrong JSON type raises
        ValueError (an API answers 400), ``null`` means "absent"."""
        if d is not None and not isinstance(d, dict):
            raise ValueError(f"{cls.__name__} must be a JSON object")
        ann = {f.name: f.type for f in fields(cls)}
        kw = {}
        for k, v in (d or {}).items():
            sk = _snake(k) if _snake(k) in ann else k
            if sk in ann and v is not None:
                # timestamps travel as epoch seconds or RFC 3339 strings (the
                # reference's wire form): both are accepted as they are
                stamp = sk.endswith("_at") or sk == "timestamp"
                if not (stamp and isinstance(v, str)) and not _json_type_ok(str(ann[sk]), v):
                    raise ValueError(f"{cls.__name__}.{k}: expected {ann[sk]}")
                kw[sk] = v
        return cls(**kw)


_SCALARS = {"str": (str,), "int": (int,), "float": (int, float), "bool": (bool,),
            "dict": (dict,), "list": (list,)}


def _json_type_ok(ann: str, v) -> bool:
    """Does JSON value ``v`` fit the (string) annotation ``ann``?  Unions and
    unknown annotations accept anything they can; bool is not a number."""
    ok = False
    for part in ann.replace(" ", "").split("|"):
        base = part.split("[", 1)[0]
        if base == "None":
            continue
        types = _SCALARS.get(base)
        if types is None:
            return True  # an annotation this check does not model
        if isinstance(v, bool) and bool not in types:
            continue
        if isinstance(v, types) or (base == "int" and isinstance(v, float) and v.is_integer()):
            if base == "list" and "[str]" in part and not all(isinstance(x, str) for x in v):
                continue
            ok = True
    return ok


@dataclass
class Message(_JSON):
    id: str = field(default_factory=lambda: uuid.uuid4().hex)
    role: str = ROLE_USER
    content: str = ""
    timestamp: float = field(default_factory=time.time)
    metadata: dict = field(default_factory=dict)
    input_tokens: int = 0
    output_tokens: int = 0
    cost_usd: float = 0.0
    tool_call_id: str = ""
    sequence_num: int = 0
    has_media: bool = False
    media_types: list = field(default_factory=list)


@dataclass
class Session(_JSON):
    id: str = field(default_factory=lambda: str(uuid.uuid4()))
    agent_name: str = ""
    namespace: str = ""
    created_at: float = field(default_factory=time.time)
    updated_at: float = field(default_factory=time.time)
    expires_at: float = 0.0
    state: dict = field(default_factory=dict)
    workspace_name: str = ""
    status: str = STATUS_ACTIVE
    ended_at: float = 0.0
    message_count: int = 0
    tool_call_count: int = 0
    total_input_tokens: int = 0
    total_output_tokens: int = 0
    estimated_cost_usd: float = 0.0
    tags: list = field(default_factory=list)
    last_message_preview: str = ""
    prompt_pack_name: str = ""
    prompt_pack_version: str = ""
    cohort_id: str = ""
    variant: str = ""
    virtual_user_id: str = ""

    def is_expired(self, now: float | None = None) -> bool:
        return bool(self.expires_at) and (now or time.time()) > self.expires_at


@dataclass
class ToolCall(_JSON):
    id: str = field(default_factory=lambda: uuid.uuid4().hex)
    session_id: str = ""
    call_id: str = ""
    name: str = ""
    arguments: dict = field(default_factory=dict)
    result: object = None
    status: str = "success"  # success | error | pending
    duration_ms: int = 0
    error_message: str = ""
    execution: str = "server"
    created_at: float = field(default_factory=time.time)


@dataclass
class ProviderCall(_JSON):
    id: str = field(default_factory=lambda: uuid.uuid4().hex)
    session_id: str = ""
    provider: str = ""
    model: str = ""
    input_tokens: int = 0
    output_tokens: int = 0
    cached_tokens: int = 0
    cost_usd: float = 0.0
    duration_ms: int = 0
    status: str = "success"
    created_at: float = field(default_factory=time.time)


@dataclass
class RuntimeEvent(_JSON):
    id: str = field(default_factory=lambda: uuid.uuid4().hex)
    session_id: str = ""
    type: str = ""
    data: dict = field(default_factory=dict)
    created_at: float = field(default_factory=time.time)


@dataclass
class EvalResult(_JSON):
    id: str = field(default_factory=lambda: uuid.uuid4().hex)
    session_id: str = ""
    message_id: str = ""
    eval_id: str = ""
    eval_type: str = ""
    passed: bool = True
    score: float = 0.0
    details: dict = field(default_factory=dict)
    source: str = "inline"
    agent_name: str = ""
    namespace: str = ""
    created_at: float = field(default_factory=time.time)
