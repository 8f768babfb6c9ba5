"""OTLP trace protos (``opentelemetry/proto/{common,resource,trace}/v1`` and
``collector/trace/v1/trace_service.proto``), wire-identical, built without protoc
for the session-api's OTLP ingest (reference ``internal/session/otlp/``).

Field numbers and types follow the published OTLP 1.x protos.  The two enums
that upstream nests (``Span.SpanKind``, ``Status.StatusCode``) are file-level
here; enum values travel as varints and keep their names, so the binary and
JSON encodings are unchanged.
"""
from __future__ import annotations

from . import build_file

R = {"repeated": True}
COMMON = "opentelemetry.proto.common.v1"
RESOURCE = "opentelemetry.proto.resource.v1"
TRACE = "opentelemetry.proto.trace.v1"
COLLECTOR = "opentelemetry.proto.collector.trace.v1"
SERVICE = f"{COLLECTOR}.TraceService"
METHOD_EXPORT = f"/{SERVICE}/Export"

_common = build_file("opentelemetry/proto/common/v1/common.proto", COMMON, {
    "AnyValue": [
        ("string_value", 1, "string", {"oneof": "value"}),
        ("bool_value", 2, "bool", {"oneof": "value"}),
        ("int_value", 3, "int64", {"oneof": "value"}),
        ("double_value", 4, "double", {"oneof": "value"}),
        ("array_value", 5, "ArrayValue", {"oneof": "value"}),
        ("kvlist_value", 6, "KeyValueList", {"oneof": "value"}),
        ("bytes_value", 7, "bytes", {"oneof": "value"}),
    ],
    "ArrayValue": [("values", 1, "AnyValue", R)],
    "KeyValueList": [("values", 1, "KeyValue", R)],
    "KeyValue": [("key", 1, "string"), ("value", 2, "AnyValue")],
    "InstrumentationScope": [("name", 1, "string"), ("version", 2, "string"),
                             ("attributes", 3, "KeyValue", R),
                             ("dropped_attributes_count", 4, "uint32")],
}, {}, {})

_resource = build_file("opentelemetry/proto/resource/v1/resource.proto", RESOURCE, {
    "Resource": [("attributes", 1, f".{COMMON}.KeyValue", R),
                 ("dropped_attributes_count", 2, "uint32")],
}, {}, {}, deps=("opentelemetry/proto/common/v1/common.proto",))

_trace = build_file("opentelemetry/proto/trace/v1/trace.proto", TRACE, {
    "TracesData": [("resource_spans", 1, "ResourceSpans", R)],
    "ResourceSpans": [("resource", 1, f".{RESOURCE}.Resource"),
                      ("scope_spans", 2, "ScopeSpans", R), ("schema_url", 3, "string")],
    "ScopeSpans": [("scope", 1, f".{COMMON}.InstrumentationScope"), ("spans", 2, "Span", R),
                   ("schema_url", 3, "string")],
    "Span": [
        ("trace_id", 1, "bytes"), ("span_id", 2, "bytes"), ("trace_state", 3, "string"),
        ("parent_span_id", 4, "bytes"), ("flags", 16, "fixed32"), ("name", 5, "string"),
        ("kind", 6, "enum:SpanKind"), ("start_time_unix_nano", 7, "fixed64"),
        ("end_time_unix_nano", 8, "fixed64"), ("attributes", 9, f".{COMMON}.KeyValue", R),
        ("dropped_attributes_count", 10, "uint32"), ("events", 11, f".{TRACE}.Span.Event", R),
        ("dropped_events_count", 12, "uint32"), ("links", 13, f".{TRACE}.Span.Link", R),
        ("dropped_links_count", 14, "uint32"), ("status", 15, "Status"),
    ],
    "Span.Event": [("time_unix_nano", 1, "fixed64"), ("name", 2, "string"),
                   ("attributes", 3, f".{COMMON}.KeyValue", R),
                   ("dropped_attributes_count", 4, "uint32")],
    "Span.Link": [("trace_id", 1, "bytes"), ("span_id", 2, "bytes"), ("trace_state", 3, "string"),
                  ("attributes", 4, f".{COMMON}.KeyValue", R),
                  ("dropped_attributes_count", 5, "uint32"), ("flags", 6, "fixed32")],
    "Status": [("message", 2, "string"), ("code", 3, "enum:StatusCode")],
}, {
    "SpanKind": [("SPAN_KIND_UNSPECIFIED", 0), ("SPAN_KIND_INTERNAL", 1),
                 ("SPAN_KIND_SERVER", 2), ("SPAN_KIND_CLIENT", 3), ("SPAN_KIND_PRODUCER", 4),
                 ("SPAN_KIND_CONSUMER", 5)],
    "StatusCode": [("STATUS_CODE_UNSET", 0), ("STATUS_CODE_OK", 1), ("STATUS_CODE_ERROR", 2)],
}, {}, deps=("opentelemetry/proto/common/v1/common.proto",
             "opentelemetry/proto/resource/v1/resource.proto"))

_collector = build_file("opentelemetry/proto/collector/trace/v1/trace_service.proto", COLLECTOR, {
    "ExportTraceServiceRequest": [("resource_spans", 1, f".{TRACE}.ResourceSpans", R)],
    "ExportTraceServiceResponse": [("partial_success", 1, "ExportTracePartialSuccess")],
    "ExportTracePartialSuccess": [("rejected_spans", 1, "int64"), ("error_message", 2, "string")],
}, {}, {"TraceService": {"Export": ("ExportTraceServiceRequest", "ExportTraceServiceResponse",
                                    False, False)}},
    deps=("opentelemetry/proto/trace/v1/trace.proto",))

AnyValue = _common["messages"]["AnyValue"]
ArrayValue = _common["messages"]["ArrayValue"]
KeyValueList = _common["messages"]["KeyValueList"]
KeyValue = _common["messages"]["KeyValue"]
InstrumentationScope = _common["messages"]["InstrumentationScope"]
Resource = _resource["messages"]["Resource"]
ResourceSpans = _trace["messages"]["ResourceSpans"]
ScopeSpans = _trace["messages"]["ScopeSpans"]
Span = _trace["messages"]["Span"]
SpanEvent = _trace["messages"]["Span.Event"]
Status = _trace["messages"]["Status"]
ExportTraceServiceRequest = _collector["messages"]["ExportTraceServiceRequest"]
ExportTraceServiceResponse = _collector["messages"]["ExportTraceServiceResponse"]
