"""Structured, PII-safe logging (``pkg/logging/logger.go:37-72``, ``sanitize.go:36-68``,
``pkg/logctx/context.go``).

* ``configure()``: ``LOG_LEVEL`` (debug/info/warn/error), ``LOG_FORMAT`` (json|text);
  JSON lines carry ``ts level logger msg`` plus context fields.
* context fields (session_id, trace_id, agent, namespace, request_id) live in
  ``contextvars`` and are stamped onto every record by :class:`ContextFilter`,
  so concurrent turns on one event loop keep their own ids (``logctx``).
* ``sanitize()``: masks bearer tokens / API keys / passwords, redacts PII with
  the EE pattern set, truncates long values; ``safe_fields()`` applies it to
  a dict of log fields.
"""
from __future__ import annotations

import contextvars
import json
import logging
import os
import re
import sys
import time

_CTX: dict[str, contextvars.ContextVar] = {
    k: contextvars.ContextVar(k, default="") for k in
    ("session_id", "trace_id", "agent", "namespace", "request_id", "workspace")}


def bind(**kw):
    """Set context fields for the current task; returns tokens for ``unbind``."""
    return {k: _CTX[k].set(str(v)) for k, v in kw.items() if k in _CTX}


def unbind(tokens: dict):
    for k, t in tokens.items():
        _CTX[k].reset(t)


def context() -> dict:
    return {k: v.get() for k, v in _CTX.items() if v.get()}


class ContextFilter(logging.Filter):
    def filter(self, record):
        for k, v in context().items():
            if not hasattr(record, k):
                setattr(record, k, v)
        return True


_SECRET = re.compile(r"(?i)\b(authorization[=:]\s*(?:bearer\s+|basic\s+)?|bearer\s+|"
                     r"api[_-]?key[=:]\s*|token[=:]\s*|password[=:]\s*|secret[=:]\s*)"
                     r"([^\s,;\"']+)")
MAX_FIELD = 512


def sanitize(value, max_len: int = MAX_FIELD, redact_pii: bool = True) -> str:
    s = value if isinstance(value, str) else repr(value)
    s = _SECRET.sub(lambda m: m.group(1) + "***", s)
    if redact_pii:
        from ..ee.redaction import Redactor

        global _RED
        if _RED is None:
            _RED = Redactor(None, "replace")
        s = _RED(s)
    if len(s) > max_len:
        s = s[:max_len] + f"...(+{len(s) - max_len} chars)"
    return s


_RED = None


def safe_fields(fields: dict) -> dict:
    return {k: sanitize(v) if isinstance(v, str) else v for k, v in fields.items()}


class JSONFormatter(logging.Formatter):
    _STD = set(logging.LogRecord("", 0, "", 0, "", (), None).__dict__) | {"message"}

    def format(self, record):
        d = {"ts": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created)) +
             f".{int(record.msecs):03d}Z", "level": record.levelname.lower(),
             "logger": record.name, "msg": record.getMessage()}
        for k, v in record.__dict__.items():
            if k not in self._STD and not k.startswith("_"):
                d[k] = v if isinstance(v, (int, float, bool)) or v is None else str(v)
        if record.exc_info:
            d["error"] = self.formatException(record.exc_info)
        return json.dumps(d, separators=(",", ":"))


_LEVELS = {"debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING,
           "warning": logging.WARNING, "error": logging.ERROR}


def configure(level: str | None = None, fmt: str | None = None, stream=None):
    level = (level or os.environ.get("LOG_LEVEL", "info")).lower()
    fmt = (fmt or os.environ.get("LOG_FORMAT", "text")).lower()
    h = logging.StreamHandler(stream or sys.stderr)
    h.addFilter(ContextFilter())
    h.setFormatter(JSONFormatter() if fmt == "json" else logging.Formatter(
        "%(asctime)s %(levelname)s %(name)s %(message)s"))
    root = logging.getLogger()
    for old in list(root.handlers):
        root.removeHandler(old)
    root.addHandler(h)
    root.setLevel(_LEVELS.get(level, logging.INFO))
    return root
