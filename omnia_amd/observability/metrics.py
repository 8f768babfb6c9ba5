"""Prometheus metrics with the reference's exact series names (so dashboards and
the KEDA trigger ``sum(omnia_agent_connections_active{...})`` keep working,
``internal/controller/autoscaling.go:319``) plus the new engine series.

Reference sources: facade ``internal/agent/metrics.go:145-350``, facade media /
drain ``internal/facade/metrics.go:23-190``, runtime collector
``pkg/runtime/promptkit/runtime.go:223-255``, compaction ``pkg/metrics/compaction.go``.
All live in one isolated registry (the reference also isolates the runtime's).
"""
from __future__ import annotations

from prometheus_client import (CollectorRegistry, Counter, Gauge, Histogram, Info,
                               generate_latest)

REGISTRY = CollectorRegistry(auto_describe=True)

_REQ_BUCKETS = (0.1, 0.5, 1, 2, 5, 10, 30, 60, 120)  # internal/agent/metrics.go:188-193

# ----------------------------------------------------------------- facade
CONNECTIONS_ACTIVE = Gauge("omnia_agent_connections_active", "Active WebSocket connections",
                           ["agent", "namespace"], registry=REGISTRY)
CONNECTIONS_TOTAL = Counter("omnia_agent_connections_total", "WebSocket connections accepted",
                            ["agent", "namespace"], registry=REGISTRY)
SESSIONS_ACTIVE = Gauge("omnia_agent_sessions_active", "Active sessions", ["agent", "namespace"],
                        registry=REGISTRY)
REQUESTS_INFLIGHT = Gauge("omnia_agent_requests_inflight", "In-flight requests",
                          ["agent", "namespace"], registry=REGISTRY)
REQUESTS_TOTAL = Counter("omnia_agent_requests_total", "Requests handled",
                         ["agent", "namespace", "status"], registry=REGISTRY)
REQUEST_DURATION = Histogram("omnia_agent_request_duration_seconds", "Turn duration",
                             ["agent", "namespace"], buckets=_REQ_BUCKETS, registry=REGISTRY)
MESSAGES_RECEIVED = Counter("omnia_agent_messages_received_total", "Client messages",
                            ["agent", "namespace"], registry=REGISTRY)
MESSAGES_SENT = Counter("omnia_agent_messages_sent_total", "Server messages",
                        ["agent", "namespace"], registry=REGISTRY)
RECORDING_DROPPED = Counter("omnia_facade_recording_dropped_total",
                            "Session recordings dropped (pool full)", registry=REGISTRY)
RATE_LIMITED = Counter("omnia_facade_rate_limited_total", "Messages rejected by rate limit",
                       ["kind"], registry=REGISTRY)
DRAINING = Gauge("omnia_facade_draining", "1 while the facade drains", registry=REGISTRY)
POD_COLD_START = Histogram("omnia_pod_cold_start_seconds",
                           "Agent pod start to ready (process spawn, engine weights + KV, facade)",
                           ["agent", "namespace"],
                           buckets=(1, 2, 5, 10, 20, 30, 60, 120, 300, 600, 900),
                           registry=REGISTRY)
SESSION_API_REQUESTS = Counter("omnia_session_api_requests_total",
                               "session-api HTTP requests by route and status",
                               ["method", "route", "status"], registry=REGISTRY)
SESSION_API_WRITES_DROPPED = Counter("omnia_session_api_writes_dropped_total",
                                     "session-api writes dropped by the privacy middleware",
                                     ["reason"], registry=REGISTRY)
PRIVACY_OUTBOX_STUCK = Gauge("omnia_privacy_outbox_stuck",
                             "consent-revocation outbox rows undelivered past the stuck age",
                             registry=REGISTRY)
MEMORY_CACHE_LOOKUPS = Counter("omnia_memory_cache_lookups_total",
                               "memory-api Redis read-cache lookups", ["op", "result"],
                               registry=REGISTRY)
MEMORY_WORKER_RUNNING = Gauge("omnia_memory_worker_running",
                              "1 while a memory-api background worker loop is alive",
                              ["name"], registry=REGISTRY)
ENGINE_COLD_START = Gauge("omnia_engine_cold_start_seconds",
                          "Engine start-up time by phase (weights, kv_alloc, graph_warmup, total)",
                          ["phase"], registry=REGISTRY)
# realtime blip-resume + drain (internal/agent/metrics.go:298-340)
REALTIME_PARKED = Counter("omnia_facade_realtime_sessions_parked_total",
                          "Realtime sessions parked after a client disconnect", registry=REGISTRY)
REALTIME_REATTACHED = Counter("omnia_facade_realtime_reattach_total",
                              "Clients reattached to a parked realtime session",
                              registry=REGISTRY)
REALTIME_PARK_EXPIRED = Counter("omnia_facade_realtime_park_expired_total",
                                "Parked realtime sessions that expired unclaimed",
                                registry=REGISTRY)
REALTIME_DRAINING = Gauge("omnia_facade_realtime_draining", "1 while realtime calls drain",
                          registry=REGISTRY)
REALTIME_DRAIN_DURATION = Histogram("omnia_facade_realtime_drain_duration_seconds",
                                    "Drain duration", ["reason"], registry=REGISTRY)
REALTIME_DRAINED = Counter("omnia_facade_realtime_calls_drained_total",
                           "Realtime calls that finished during drain", registry=REGISTRY)
REALTIME_FORCE_ENDED = Counter("omnia_facade_realtime_calls_force_ended_total",
                               "Realtime calls still live when drain ended", registry=REGISTRY)
# canary rollouts (internal/controller/rollout_metrics.go:22-28)
ROLLOUT_ACTIVE = Gauge("omnia_rollout_active", "1 while a rollout is in flight",
                       ["namespace", "agent"], registry=REGISTRY)
ROLLOUT_STEPS = Counter("omnia_rollout_step_transitions_total", "Rollout step transitions",
                        ["namespace", "agent", "step_type"], registry=REGISTRY)
ROLLOUT_PROMOTIONS = Counter("omnia_rollout_promotions_total", "Rollout promotions",
                             ["namespace", "agent"], registry=REGISTRY)
ROLLOUT_ROLLBACKS = Counter("omnia_rollout_rollbacks_total", "Rollout rollbacks",
                            ["namespace", "agent", "reason"], registry=REGISTRY)
ROLLOUT_WEIGHT = Gauge("omnia_rollout_traffic_weight", "Traffic weight per track",
                       ["namespace", "agent", "track"], registry=REGISTRY)
ROLLOUT_ANALYSIS = Counter("omnia_rollout_analysis_runs_total", "Rollout analysis runs",
                           ["namespace", "agent", "template", "outcome"], registry=REGISTRY)
A2A_REQUESTS = Counter("omnia_a2a_requests_total", "A2A JSON-RPC requests", ["method", "status"],
                       registry=REGISTRY)
MCP_REQUESTS = Counter("omnia_mcp_requests_total", "MCP requests", ["method", "status"],
                       registry=REGISTRY)
FUNCTION_REQUESTS = Counter("omnia_function_requests_total", "Function-mode invocations",
                            ["function", "status"], registry=REGISTRY)

# ----------------------------------------------------------------- runtime
PROVIDER_INPUT_TOKENS = Counter("omnia_provider_input_tokens_total", "Prompt tokens",
                                ["provider", "model"], registry=REGISTRY)
PROVIDER_OUTPUT_TOKENS = Counter("omnia_provider_output_tokens_total", "Completion tokens",
                                 ["provider", "model"], registry=REGISTRY)
PROVIDER_REQUESTS = Counter("omnia_provider_requests_total", "Provider calls",
                            ["provider", "model", "status"], registry=REGISTRY)
PROVIDER_COST = Counter("omnia_provider_cost_total", "Estimated cost (USD)",
                        ["provider", "model"], registry=REGISTRY)
PROVIDER_DURATION = Histogram("omnia_provider_request_duration_seconds", "Provider call latency",
                              ["provider", "model"], buckets=_REQ_BUCKETS, registry=REGISTRY)
PIPELINES_ACTIVE = Gauge("omnia_runtime_pipelines_active", "Turns in flight", registry=REGISTRY)
PIPELINE_DURATION = Histogram("omnia_runtime_pipeline_duration_seconds", "Turn pipeline latency",
                              buckets=_REQ_BUCKETS, registry=REGISTRY)
TOOL_CALLS = Counter("omnia_runtime_tool_calls_total", "Tool calls", ["tool", "status"],
                     registry=REGISTRY)
TOOL_DURATION = Histogram("omnia_runtime_tool_call_duration_seconds", "Tool call latency",
                          ["tool"], registry=REGISTRY)
VALIDATIONS = Counter("omnia_runtime_validations_total", "Validator runs", ["validator", "result"],
                      registry=REGISTRY)
RUNTIME_INFO = Info("omnia_runtime", "Runtime build/contract info", registry=REGISTRY)

# ----------------------------------------------------------------- policy / data plane
TOOLPOLICY_DECISIONS = Counter("omnia_toolpolicy_decisions_total", "Policy broker decisions",
                               ["decision"], registry=REGISTRY)
TOOLPOLICY_LATENCY = Histogram("omnia_toolpolicy_decision_duration_seconds",
                               "Policy decision latency",
                               buckets=(0.0005, 0.001, 0.005, 0.01, 0.05, 0.1, 0.5),
                               registry=REGISTRY)
COMPACTION_RUNS = Counter("omnia_compaction_runs_total", "Compaction runs", ["result"],
                          registry=REGISTRY)
COMPACTION_SESSIONS = Counter("omnia_compaction_sessions_archived_total",
                              "Sessions archived warm->cold", registry=REGISTRY)
RETENTION_DELETED = Counter("omnia_retention_sessions_deleted_total", "Sessions purged",
                            ["tier"], registry=REGISTRY)

# ----------------------------------------------------------------- engine (new)
TTFT = Histogram("omnia_engine_ttft_seconds", "Time to first token",
                 buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10),
                 registry=REGISTRY)
TURN_SECONDS = Histogram("omnia_engine_turn_seconds", "Engine request latency",
                         buckets=_REQ_BUCKETS, registry=REGISTRY)
STEP_SECONDS = Histogram("omnia_engine_step_seconds", "Engine step latency", ["kind"],
                         buckets=(0.001, 0.0025, 0.005, 0.01, 0.02, 0.04, 0.08, 0.16, 0.32, 1),
                         registry=REGISTRY)
PREFILL_TOKENS = Counter("omnia_engine_prefill_tokens_total", "Prefilled tokens",
                         registry=REGISTRY)
DECODE_TOKENS = Counter("omnia_engine_decode_tokens_total", "Decoded tokens", registry=REGISTRY)
BATCH_SIZE = Histogram("omnia_engine_batch_size", "Decode batch size",
                       buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024), registry=REGISTRY)
ENGINE_FAULTS = Counter("omnia_engine_faults_total", "Engine step faults (recovered or fatal)",
                        ["type"], registry=REGISTRY)
KV_UTIL = Gauge("omnia_engine_kv_utilization", "Fraction of KV pages in use", registry=REGISTRY)
ENGINE_WAITING = Gauge("omnia_engine_requests_waiting", "Queued requests", registry=REGISTRY)
KV_HIT_TOKENS = Counter("omnia_engine_kv_hit_tokens_total",
                        "Prompt tokens served from cached KV (session pages or shared prefix pages)",
                        registry=REGISTRY)
KV_SHARED_HIT_TOKENS = Counter("omnia_engine_kv_shared_hit_tokens_total",
                               "Prompt tokens served from cross-session shared prefix pages",
                               registry=REGISTRY)

# ----------------------------------------------------------------- memory-api
# cmd/memory-api/SERVICE.md "Metrics" (classification + embedding pipeline health)
MEMORY_CLASSIFY_OVERRIDES = Counter("omnia_memory_classify_overrides_total",
                                    "Consent category upgraded by classification",
                                    ["from", "to", "source"], registry=REGISTRY)
MEMORY_CLASSIFY_FILLED = Counter("omnia_memory_classify_filled_total",
                                 "Consent category filled in by classification",
                                 ["category", "source"], registry=REGISTRY)
MEMORY_CLASSIFY_CATEGORY = Counter("omnia_memory_classify_category_total",
                                   "Stored consent categories", ["category", "source"],
                                   registry=REGISTRY)
MEMORY_EMBED_ERRORS = Counter("omnia_memory_classify_errors_total", "Embedding failures",
                              registry=REGISTRY)
MEMORY_EMBED_COVERAGE = Gauge("omnia_memory_embedding_coverage",
                              "Fraction of live entities with an embedded active observation",
                              ["workspace"], registry=REGISTRY)
MEMORY_REEMBED_BACKLOG = Gauge("omnia_memory_reembed_backlog",
                               "Active observations awaiting (re-)embedding", ["workspace"],
                               registry=REGISTRY)
MEMORY_EMBED_SECONDS = Histogram("omnia_memory_embed_seconds", "Embedding batch latency",
                                 registry=REGISTRY)
MEMORY_RETRIEVE_SECONDS = Histogram("omnia_memory_retrieve_seconds", "Retrieval latency",
                                    ["mode"], registry=REGISTRY)
MEMORY_OPS = Counter("omnia_memory_operations_total", "Memory API operations", ["op", "status"],
                     registry=REGISTRY)


def exposition() -> bytes:
    return generate_latest(REGISTRY)


_CHILDREN: dict = {}


def child(metric, *labels):
    """``metric.labels(*labels)`` memoised: the per-turn hot paths (runtime turn
    completion, facade frames) skip prometheus_client's locked label lookup."""
    key = (id(metric), labels)
    c = _CHILDREN.get(key)
    if c is None:
        c = _CHILDREN[key] = metric.labels(*labels)
    return c
