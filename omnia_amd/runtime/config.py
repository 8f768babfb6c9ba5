"""Runtime configuration (``internal/runtime/config.go:31-316``).

Sources, in priority order (as the reference): the AgentRuntime / Provider CRDs
read through the cluster API when available (``config_crd.go:56-260``), then the
``OMNIA_*`` environment injected by the operator, then defaults.  Engine
settings live under ``OMNIA_ENGINE_*``.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

from .context_store import parse_ttl


@dataclass
class RuntimeConfig:
    agent_name: str = "agent"
    namespace: str = "default"
    workspace: str = ""
    workspace_uid: str = ""
    promptpack_path: str = "/etc/omnia/pack"
    promptpack_name: str = ""
    promptpack_version: str = ""
    prompt_name: str = ""
    mode: str = "agent"  # agent | function
    output_format: str = ""  # "" | text | json | json_schema
    output_schema: dict | None = None
    context_type: str = "memory"
    context_url: str = ""
    context_ttl_s: int = 24 * 3600
    provider: dict = field(default_factory=lambda: {"type": "mock"})
    extra_providers: list = field(default_factory=list)  # embedding / stt / tts / judge roles
    duplex: dict = field(default_factory=dict)  # AgentRuntime spec.duplex (audio params)
    context_window: int = 0
    truncation: str = "sliding"
    tools_config_path: str = "/etc/omnia/tools"
    tool_secrets_dir: str = "/etc/omnia/tool-secrets"
    session_api_url: str = ""
    memory_enabled: bool = False
    memory_api_url: str = ""
    memory_strategy: str = "composite"  # keyword | semantic | composite
    memory_deny_cel: str = ""
    memory_limit: int = 10
    policy_broker_url: str = ""
    eval_enabled: bool = False
    eval_inline_groups: list = field(default_factory=list)  # spec.evals.inline.groups
    tracing_enabled: bool = False
    tracing_endpoint: str = ""
    tracing_sample_rate: float = 1.0
    stream_interval_ms: float = 0.0  # Converse text-delta coalescing window (0 = per delta)
    grpc_port: int = 9000
    health_port: int = 9001
    engine: dict = field(default_factory=dict)
    # resolved outbound A2A clients ``[{name, url, exposeAsTools, authTokenEnv}]``
    # (OMNIA_A2A_CLIENTS, ``internal/controller/a2a_client_resolver.go``)
    a2a_clients: list = field(default_factory=list)

    @classmethod
    def from_env(cls, env=None) -> "RuntimeConfig":
        e = env if env is not None else os.environ
        c = cls()
        c.agent_name = e.get("OMNIA_AGENT_NAME", c.agent_name)
        c.namespace = e.get("OMNIA_NAMESPACE", c.namespace)
        c.workspace = e.get("OMNIA_WORKSPACE", "")
        c.workspace_uid = e.get("OMNIA_WORKSPACE_UID", "")
        c.promptpack_path = e.get("OMNIA_PROMPTPACK_PATH", c.promptpack_path)
        c.promptpack_name = e.get("OMNIA_PROMPTPACK_NAME", "")
        c.promptpack_version = e.get("OMNIA_PROMPTPACK_VERSION", "")
        c.prompt_name = e.get("OMNIA_PROMPT_NAME", "")
        c.mode = e.get("OMNIA_MODE", c.mode)
        c.output_format = e.get("OMNIA_OUTPUT_FORMAT", "")
        if e.get("OMNIA_OUTPUT_SCHEMA"):
            c.output_schema = json.loads(e["OMNIA_OUTPUT_SCHEMA"])
        c.context_type = e.get("OMNIA_CONTEXT_TYPE", "redis" if e.get("OMNIA_CONTEXT_URL")
                               else "memory")
        c.context_url = e.get("OMNIA_CONTEXT_URL", "")
        if e.get("OMNIA_CONTEXT_TTL"):
            c.context_ttl_s = parse_ttl(e["OMNIA_CONTEXT_TTL"])
        ptype = e.get("OMNIA_PROVIDER_TYPE") or ("mock" if e.get("OMNIA_MOCK_PROVIDER",
                                                                  "").lower() == "true"
                                                 else "mock")
        c.provider = {"type": ptype, "model": e.get("OMNIA_PROVIDER_MODEL", ""),
                      "baseURL": e.get("OMNIA_PROVIDER_BASE_URL", "")}
        if e.get("OMNIA_PROVIDER_JSON"):
            c.provider.update(json.loads(e["OMNIA_PROVIDER_JSON"]))
        if e.get("OMNIA_EXTRA_PROVIDERS_JSON"):
            c.extra_providers = json.loads(e["OMNIA_EXTRA_PROVIDERS_JSON"])
        if e.get("OMNIA_DUPLEX_JSON"):
            c.duplex = json.loads(e["OMNIA_DUPLEX_JSON"])
        if e.get("OMNIA_MOCK_CONFIG"):
            c.provider.setdefault("mock", {})["path"] = e["OMNIA_MOCK_CONFIG"]
        c.context_window = int(e.get("OMNIA_CONTEXT_WINDOW", "0") or 0)
        c.truncation = e.get("OMNIA_TRUNCATION_STRATEGY", c.truncation)
        c.tools_config_path = e.get("OMNIA_TOOLS_CONFIG_PATH", c.tools_config_path)
        c.tool_secrets_dir = e.get("OMNIA_TOOL_SECRETS_PATH", c.tool_secrets_dir)
        c.session_api_url = e.get("OMNIA_SESSION_API_URL", "")
        c.memory_enabled = e.get("OMNIA_MEMORY_ENABLED", "false").lower() == "true"
        c.memory_api_url = e.get("OMNIA_MEMORY_API_URL", "")
        c.memory_strategy = e.get("OMNIA_MEMORY_STRATEGY", c.memory_strategy)
        c.memory_deny_cel = e.get("OMNIA_MEMORY_DENY_CEL", "")
        c.memory_limit = int(e.get("OMNIA_MEMORY_LIMIT", c.memory_limit))
        c.policy_broker_url = e.get("OMNIA_POLICY_BROKER_URL", "")
        c.eval_enabled = e.get("OMNIA_EVAL_ENABLED", "false").lower() == "true"
        c.eval_inline_groups = [g for g in e.get("OMNIA_EVAL_INLINE_GROUPS", "").split(",") if g]
        c.tracing_enabled = e.get("OMNIA_TRACING_ENABLED", "false").lower() == "true"
        c.tracing_endpoint = e.get("OMNIA_TRACING_ENDPOINT", "")
        c.tracing_sample_rate = float(e.get("OMNIA_TRACING_SAMPLE_RATE", "1.0"))
        c.stream_interval_ms = float(e.get("OMNIA_STREAM_INTERVAL_MS", "0") or 0)
        c.grpc_port = int(e.get("OMNIA_GRPC_PORT", c.grpc_port))
        c.health_port = int(e.get("OMNIA_HEALTH_PORT", c.health_port))
        c.engine = {k[len("OMNIA_ENGINE_"):].lower(): v for k, v in e.items()
                    if k.startswith("OMNIA_ENGINE_")}
        if e.get("OMNIA_A2A_CLIENTS"):
            c.a2a_clients = json.loads(e["OMNIA_A2A_CLIENTS"])
        if e.get("OMNIA_CONFIG_DIR"):
            c = c.with_config_dir(e["OMNIA_CONFIG_DIR"], e)
        return c

    def with_config_dir(self, path: str, env) -> "RuntimeConfig":
        """Cluster-less configuration (``OMNIA_CONFIG_DIR``, the reference's
        fake-client devroot, ``examples/custom-runtime/README.md``): the
        AgentRuntime / Provider / PromptPack / Secret objects are read from every
        ``*.yaml`` / ``*.yml`` in ``path`` and resolved exactly as the operator
        would (CRD values win over env, as ``config_crd.go``); the mounted-file
        paths and ports keep coming from the environment."""
        import base64
        import glob

        import yaml

        docs = []
        for f in sorted(glob.glob(os.path.join(path, "*.yaml")) +
                        glob.glob(os.path.join(path, "*.yml"))):
            with open(f) as fh:
                docs += [d for d in yaml.safe_load_all(fh) if isinstance(d, dict)]

        def find(kind, name=None, ns=None):
            return [d for d in docs if d.get("kind") == kind
                    and (name is None or d["metadata"].get("name") == name)
                    and (ns is None or d["metadata"].get("namespace", "default") == ns)]

        ars = find("AgentRuntime", self.agent_name, self.namespace) or \
            (find("AgentRuntime") if len(find("AgentRuntime")) == 1 else [])
        if not ars:
            raise ValueError(f"OMNIA_CONFIG_DIR {path}: no AgentRuntime "
                             f"{self.namespace}/{self.agent_name}")
        ar = ars[0]
        ar["metadata"].setdefault("namespace", self.namespace)
        ns = ar["metadata"]["namespace"]
        providers = []
        for ref in ar["spec"].get("providers") or []:
            pr = (ref.get("providerRef") or {}).get("name")
            got = find("Provider", pr, ref.get("providerRef", {}).get("namespace", ns))
            if got:
                p = {"metadata": got[0]["metadata"], "spec": dict(got[0]["spec"])}
                if ref.get("name") and ref["name"] != "llm":
                    p["spec"].setdefault("role", ref["name"])
                cred = (p["spec"].get("credential") or {}).get("secretRef") or \
                    p["spec"].get("secretRef")
                if cred:  # the provider key, read like the in-cluster path would
                    sec = find("Secret", cred.get("name"), ns)
                    if sec:
                        data = {k: base64.b64decode(v).decode()
                                for k, v in (sec[0].get("data") or {}).items()}
                        data.update(sec[0].get("stringData") or {})
                        key = cred.get("key") or next(iter(data), None)
                        if key in data:
                            p["spec"]["apiKey"] = data[key]
                providers.append(p)
        pref = (ar["spec"].get("promptPackRef") or {}).get("name", "")
        packs = find("PromptPack", pref, ns)
        pack = packs[0] if packs else {"spec": {"packName": pref,
                                                "version": (ar["spec"].get("promptPackRef")
                                                            or {}).get("version", "")}}
        from ..operator.builders import runtime_config

        c = runtime_config(ar, pack, providers, None)
        for f in ("promptpack_path", "tools_config_path", "grpc_port", "health_port",
                  "session_api_url", "memory_api_url", "workspace", "workspace_uid",
                  "tool_secrets_dir", "a2a_clients", "policy_broker_url", "tracing_enabled",
                  "tracing_endpoint", "stream_interval_ms"):
            setattr(c, f, getattr(self, f))
        if env.get("OMNIA_PROMPTPACK_PATH") is None:
            c.promptpack_path = self.promptpack_path
        if self.engine and not c.engine:
            c.engine = dict(self.engine)
        wss = [w for w in find("Workspace")
               if ((w.get("spec") or {}).get("namespace") or {}).get("name") == ns]
        if wss and not c.workspace:
            c.workspace = wss[0]["metadata"]["name"]
        return c

    def to_env(self) -> dict:
        """Inverse of from_env (used by the operator's pod builder)."""
        env = {
            "OMNIA_AGENT_NAME": self.agent_name, "OMNIA_NAMESPACE": self.namespace,
            "OMNIA_PROMPTPACK_PATH": self.promptpack_path, "OMNIA_PROMPT_NAME": self.prompt_name,
            "OMNIA_MODE": self.mode, "OMNIA_CONTEXT_TYPE": self.context_type,
            "OMNIA_CONTEXT_TTL": f"{self.context_ttl_s}s",
            "OMNIA_GRPC_PORT": str(self.grpc_port), "OMNIA_HEALTH_PORT": str(self.health_port),
            "OMNIA_PROVIDER_JSON": json.dumps(self.provider),
            "OMNIA_TOOLS_CONFIG_PATH": self.tools_config_path,
            "OMNIA_CONTEXT_WINDOW": str(self.context_window),
            "OMNIA_TRUNCATION_STRATEGY": self.truncation,
        }
        if self.context_url:
            env["OMNIA_CONTEXT_URL"] = self.context_url
        if self.stream_interval_ms:
            env["OMNIA_STREAM_INTERVAL_MS"] = str(self.stream_interval_ms)
        if self.extra_providers:
            env["OMNIA_EXTRA_PROVIDERS_JSON"] = json.dumps(self.extra_providers)
        if self.duplex:
            env["OMNIA_DUPLEX_JSON"] = json.dumps(self.duplex)
        if self.output_format:
            env["OMNIA_OUTPUT_FORMAT"] = self.output_format
        if self.output_schema is not None:
            env["OMNIA_OUTPUT_SCHEMA"] = json.dumps(self.output_schema)
        for k, v in (("OMNIA_SESSION_API_URL", self.session_api_url),
                     ("OMNIA_MEMORY_API_URL", self.memory_api_url),
                     ("OMNIA_POLICY_BROKER_URL", self.policy_broker_url),
                     ("OMNIA_WORKSPACE", self.workspace)):
            if v:
                env[k] = v
        if self.memory_enabled:
            env["OMNIA_MEMORY_ENABLED"] = "true"
            env["OMNIA_MEMORY_STRATEGY"] = self.memory_strategy
            env["OMNIA_MEMORY_LIMIT"] = str(self.memory_limit)
            if self.memory_deny_cel:
                env["OMNIA_MEMORY_DENY_CEL"] = self.memory_deny_cel
        if self.eval_enabled:
            env["OMNIA_EVAL_ENABLED"] = "true"
            if self.eval_inline_groups:
                env["OMNIA_EVAL_INLINE_GROUPS"] = ",".join(self.eval_inline_groups)
        if self.a2a_clients:
            env["OMNIA_A2A_CLIENTS"] = json.dumps(self.a2a_clients)
        for k, v in self.engine.items():
            env["OMNIA_ENGINE_" + k.upper()] = str(v)
        return env
