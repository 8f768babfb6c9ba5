"""OpenTelemetry-compatible tracing without the otel SDK (not installed).

Reference: ``internal/tracing/tracing.go:36-379`` -- OTLP exporter,
ParentBased(ratio) sampler, batch processor, GenAI span helpers; span names
``omnia.facade.message`` (root), ``omnia.runtime.conversation.turn``,
``genai.chat``, ``omnia.tool.call``; the facade derives the TRACE ID from the
session UUID so every turn of a session shares one trace
(``internal/facade/session.go:160-223``), and a caller's ``traceparent`` becomes
a span LINK.  Engine spans ``omnia.engine.prefill`` / ``omnia.engine.decode_step``
are added.  Spans export as OTLP/HTTP JSON (``/v1/traces``) from a background
batcher, or to an in-memory list for tests.
"""
from __future__ import annotations

import contextvars
import json
import os
import random
import threading
import time
import uuid
from dataclasses import dataclass, field

_current: contextvars.ContextVar = contextvars.ContextVar("omnia_span", default=None)


@dataclass
class Span:
    name: str
    trace_id: str
    span_id: str
    parent_id: str | None
    start_ns: int
    end_ns: int = 0
    attributes: dict = field(default_factory=dict)
    links: list = field(default_factory=list)
    status: str = "UNSET"
    sampled: bool = True
    token: object = None

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-{'01' if self.sampled else '00'}"


class Tracer:
    def __init__(self, service: str = "omnia-runtime", ratio: float = 1.0, exporter=None):
        self.service = service
        self.ratio = ratio
        self.exporter = exporter
        self.enabled = exporter is not None

    def should_sample(self, parent: Span | None) -> bool:
        if parent is not None:
            return parent.sampled  # ParentBased
        return random.random() < self.ratio


_TRACER = Tracer()


def configure(service: str | None = None, endpoint: str | None = None, ratio: float | None = None,
              exporter=None) -> Tracer:
    """OMNIA_TRACING_ENABLED / OMNIA_TRACING_ENDPOINT / OMNIA_TRACING_SAMPLE_RATE."""
    global _TRACER
    env = os.environ
    if exporter is None:
        if endpoint is None and env.get("OMNIA_TRACING_ENABLED", "false").lower() == "true":
            endpoint = env.get("OMNIA_TRACING_ENDPOINT", "http://127.0.0.1:4318")
        if endpoint:
            exporter = OTLPHTTPExporter(endpoint, service or "omnia-runtime")
    _TRACER = Tracer(service or env.get("OMNIA_TRACING_SERVICE", "omnia-runtime"),
                     ratio if ratio is not None else float(env.get("OMNIA_TRACING_SAMPLE_RATE",
                                                                   "1.0")), exporter)
    return _TRACER


def tracer() -> Tracer:
    return _TRACER


def session_trace_id(session_id: str) -> str:
    """Lossless 128-bit trace id from a session UUID (else a hash of it)."""
    try:
        return uuid.UUID(session_id).hex
    except (ValueError, AttributeError, TypeError):
        import hashlib

        return hashlib.sha256(str(session_id).encode()).hexdigest()[:32]


def parse_traceparent(tp: str | None):
    if not tp:
        return None
    p = tp.split("-")
    if len(p) != 4 or len(p[1]) != 32 or len(p[2]) != 16:
        return None
    return {"trace_id": p[1], "span_id": p[2], "sampled": p[3] == "01"}


def start_span(name: str, attributes: dict | None = None, trace_id: str | None = None,
               link: dict | None = None, parent: Span | None = None) -> Span:
    t = _TRACER
    parent = parent if parent is not None else _current.get()
    tid = trace_id or (parent.trace_id if parent else uuid.uuid4().hex)
    sp = Span(name=name, trace_id=tid, span_id=os.urandom(8).hex(),
              parent_id=parent.span_id if parent else None, start_ns=time.time_ns(),
              attributes=dict(attributes or {}), sampled=t.should_sample(parent))
    if link:
        sp.links.append(link)
    sp.token = _current.set(sp)
    return sp


def end_span(sp: Span, attributes: dict | None = None, error: bool = False) -> None:
    if sp is None:
        return
    if attributes:
        sp.attributes.update(attributes)
    sp.end_ns = time.time_ns()
    sp.status = "ERROR" if error else "OK"
    try:
        _current.reset(sp.token)
    except (ValueError, RuntimeError):
        pass
    if _TRACER.enabled and sp.sampled:
        _TRACER.exporter.export(sp)


def record_span(name: str, start_ns: int, end_ns: int, attributes: dict | None = None,
                trace_id: str | None = None) -> Span | None:
    """Export an already-finished root span (engine steps: they overlap when
    pipelined, so they never become the context's current span)."""
    t = _TRACER
    if not t.enabled:
        return None
    sp = Span(name=name, trace_id=trace_id or uuid.uuid4().hex, span_id=os.urandom(8).hex(),
              parent_id=None, start_ns=start_ns, end_ns=end_ns,
              attributes=dict(attributes or {}), status="OK", sampled=t.should_sample(None))
    if sp.sampled:
        t.exporter.export(sp)
    return sp


class MemoryExporter:
    def __init__(self):
        self.spans: list[Span] = []

    def export(self, sp: Span):
        self.spans.append(sp)


class OTLPHTTPExporter:
    """Batching OTLP/HTTP JSON exporter (best effort, drops on failure)."""

    def __init__(self, endpoint: str, service: str, batch: int = 256, interval_s: float = 2.0):
        self.url = endpoint.rstrip("/") + "/v1/traces"
        self.service = service
        self.batch = batch
        self.buf: list[Span] = []
        self.lock = threading.Lock()
        self.dropped = 0
        t = threading.Thread(target=self._loop, args=(interval_s,), daemon=True)
        t.start()

    def export(self, sp):
        with self.lock:
            if len(self.buf) < 8192:
                self.buf.append(sp)
            else:
                self.dropped += 1

    def _loop(self, interval):
        while True:
            time.sleep(interval)
            self.flush()

    def flush(self):
        with self.lock:
            spans, self.buf = self.buf, []
        if not spans:
            return
        import urllib.request

        def attr(k, v):
            if isinstance(v, bool):
                return {"key": k, "value": {"boolValue": v}}
            if isinstance(v, int):
                return {"key": k, "value": {"intValue": str(v)}}
            if isinstance(v, float):
                return {"key": k, "value": {"doubleValue": v}}
            return {"key": k, "value": {"stringValue": str(v)}}

        body = {"resourceSpans": [{
            "resource": {"attributes": [attr("service.name", self.service)]},
            "scopeSpans": [{"scope": {"name": "omnia"}, "spans": [{
                "traceId": s.trace_id, "spanId": s.span_id, "parentSpanId": s.parent_id or "",
                "name": s.name, "kind": 1, "startTimeUnixNano": str(s.start_ns),
                "endTimeUnixNano": str(s.end_ns),
                "attributes": [attr(k, v) for k, v in s.attributes.items()],
                "links": [{"traceId": l["trace_id"], "spanId": l["span_id"]} for l in s.links],
                "status": {"code": 2 if s.status == "ERROR" else 1}} for s in spans]}]}]}
        try:
            req = urllib.request.Request(self.url, data=json.dumps(body).encode(),
                                         headers={"Content-Type": "application/json"})
            urllib.request.urlopen(req, timeout=5).read()
        except Exception:  # noqa: BLE001
            self.dropped += len(spans)
