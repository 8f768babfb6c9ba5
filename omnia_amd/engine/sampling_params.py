"""Sampling parameters -- the PromptPack ``parameters`` block
(``internal/schema/promptpack.schema.json`` ``$defs.Parameters``: temperature,
max_tokens, top_p, top_k, frequency_penalty, presence_penalty) plus the
AgentRuntime ``ProviderDefaults`` (``api/v1alpha1/agentruntime_types.go:431-459``)."""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0  # 0 = disabled
    max_tokens: int = 256
    min_tokens: int = 0
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    repetition_penalty: float = 1.0
    seed: int | None = None
    stop: list[str] = field(default_factory=list)
    stop_token_ids: list[int] = field(default_factory=list)
    ignore_eos: bool = False
    logprobs: bool = False
    # K13 guided decoding: JSON-schema-constrained output / any JSON object
    json_schema: dict | None = None
    json_object: bool = False
    # tool calling on the in-node engine: [{"name", "parameters"}] of the offered
    # tools; "required" constrains the whole answer to one valid Llama-3 tool call,
    # "auto" only once the model opens a JSON object (engine/guided.py)
    tool_grammar: list | None = None
    tool_choice: str = "auto"
    # cross-session KV prefix sharing (engine/kv_manager.py): pages are shared
    # only between requests of one ``cache_salt`` scope, and a prompt publishes
    # at most its first ``share_limit`` tokens (None: all of them; the runtime
    # passes the rendered system prompt + tool schemas length)
    cache_salt: str | None = None
    share_limit: int | None = None

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0

    @property
    def guided(self) -> bool:
        return self.json_schema is not None or self.json_object or bool(self.tool_grammar)

    @property
    def needs_penalties(self) -> bool:
        return (self.frequency_penalty != 0.0 or self.presence_penalty != 0.0
                or self.repetition_penalty != 1.0)

    def validate(self) -> "SamplingParams":
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0.0 < self.top_p <= 1.0:
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k < 0:
            raise ValueError("top_k must be >= 0")
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.repetition_penalty <= 0:
            raise ValueError("repetition_penalty must be > 0")
        for f in ("temperature", "top_p", "frequency_penalty", "presence_penalty",
                  "repetition_penalty"):
            v = getattr(self, f)
            if v != v or v in (float("inf"), float("-inf")):
                raise ValueError(f"{f} must be finite")
        if self.seed is not None and (isinstance(self.seed, bool) or
                                      not isinstance(self.seed, int)):
            raise ValueError("seed must be an integer")
        for f in ("top_k", "max_tokens", "min_tokens"):  # device tensors hold int32
            v = getattr(self, f)
            if isinstance(v, bool) or not isinstance(v, int) or not 0 <= v < 1 << 31:
                raise ValueError(f"{f} must be an integer in [0, 2^31)")
        if self.seed is not None and not -(1 << 63) <= self.seed < 1 << 63:
            # any integer is a valid OpenAI seed: fold it into the sampler's int64 key
            s = self.seed & ((1 << 64) - 1)
            self.seed = s - (1 << 64) if s >= 1 << 63 else s
        if not isinstance(self.stop, (list, tuple)) or not all(isinstance(x, str)
                                                               for x in self.stop):
            raise ValueError("stop must be a string or a list of strings")
        if not isinstance(self.stop_token_ids, (list, tuple, set, frozenset)) or not all(
                isinstance(x, int) for x in self.stop_token_ids):
            raise ValueError("stop_token_ids must be integers")
        if self.json_schema is not None and not isinstance(self.json_schema, dict):
            raise ValueError("json_schema must be an object")
        return self

    @classmethod
    def from_dict(cls, d: dict | None, **defaults) -> "SamplingParams":
        """Build from a PromptPack ``parameters`` / OpenAI-style dict."""
        d = dict(d or {})
        kw = dict(defaults)
        mapping = {
            "temperature": "temperature", "top_p": "top_p", "topP": "top_p", "top_k": "top_k",
            "topK": "top_k", "max_tokens": "max_tokens", "maxTokens": "max_tokens",
            "frequency_penalty": "frequency_penalty", "presence_penalty": "presence_penalty",
            "repetition_penalty": "repetition_penalty", "seed": "seed", "stop": "stop",
            "ignore_eos": "ignore_eos", "min_tokens": "min_tokens", "logprobs": "logprobs",
            "json_schema": "json_schema", "json_object": "json_object",
        }
        for k, v in d.items():
            if k in mapping and v is not None:
                kw[mapping[k]] = v
        rf = d.get("response_format")
        if isinstance(rf, dict):  # OpenAI-style response_format
            if rf.get("type") == "json_object":
                kw["json_object"] = True
            elif rf.get("type") == "json_schema":
                js = rf.get("json_schema") or {}
                kw["json_schema"] = js.get("schema", js) if isinstance(js, dict) else None
        if isinstance(kw.get("stop"), str):
            kw["stop"] = [kw["stop"]]
        for f in ("temperature", "top_p", "frequency_penalty", "presence_penalty",
                  "repetition_penalty"):
            if f in kw:
                kw[f] = float(kw[f])
        for f in ("top_k", "max_tokens", "min_tokens"):
            if f in kw:
                if isinstance(kw[f], float) and not kw[f].is_integer():
                    raise ValueError(f"{f} must be an integer")
                kw[f] = int(kw[f])
        for f in ("ignore_eos", "json_object"):
            if f in kw and not isinstance(kw[f], bool):
                raise ValueError(f"{f} must be a boolean")
        return cls(**kw).validate()
