"""Runtime assembly: config -> pack, provider (local engine by default), context
store, tool executor, policy broker, event recording, memory -> RuntimeService.

Mirrors ``pkg/runtime/promptkit/runtime.go:100-330`` (newFromBuilder / Serve /
shutdown) and ``internal/runtime/conversation.go:104-257`` (conversation
options).  ``python -m omnia_amd.runtime`` runs gRPC :9000 + health :9001.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import signal

from ..observability import metrics as M
from ..observability import tracing
from ..tools.executor import OmniaExecutor, PolicyBrokerClient, load_tools_config
from .agent import Agent, AgentConfig
from .config import RuntimeConfig
from .context_store import make_store
from .promptpack import PackError, PromptPack
from .providers import build_provider
from .server import CAPABILITIES, RuntimeService, serve_grpc, serve_health
from ..observability.logging import configure as configure_logging

log = logging.getLogger("omnia.runtime")

_ENGINES: dict = {}


def shared_engine(engine_cfg: dict | None = None):
    """One AsyncLLMEngine per process (the runtime owns the GPU)."""
    from ..engine.engine import AsyncLLMEngine, EngineConfig

    key = json.dumps(engine_cfg or {}, sort_keys=True)
    eng = _ENGINES.get(key)
    if eng is None:
        kw = {}
        ecfg = dict(engine_cfg or {})
        # data-parallel replicas on this node: one engine-core process per GPU,
        # sessions pinned by the rendezvous router (parallel/router.py)
        n_rep = int(ecfg.pop("replicas", 0) or ecfg.pop("dp", 0) or
                    os.environ.get("OMNIA_ENGINE_REPLICAS", "1"))
        for k, v in ecfg.items():
            if k in EngineConfig.__dataclass_fields__:
                t = EngineConfig.__dataclass_fields__[k].type
                kw[k] = (int(v) if "int" in str(t) else float(v) if "float" in str(t)
                         else (str(v).lower() in ("1", "true", "yes", "on")) if "bool" in str(t)
                         else v)
        cfg = EngineConfig.from_env(**kw)
        eng = None
        if n_rep > 1:
            from ..engine.core_proc import EngineCoreClient
            from ..parallel.router import ReplicatedEngine

            if cfg.device == "cuda":
                reps = [EngineCoreClient(cfg, device_index=i * max(1, cfg.tp))
                        for i in range(n_rep)]
            else:
                reps = [AsyncLLMEngine.from_config(cfg) for _ in range(n_rep)]
            eng = ReplicatedEngine(reps)
        elif _use_engine_process(cfg):
            from ..engine.core_proc import EngineCoreClient

            eng = EngineCoreClient(cfg)
        if eng is None:
            eng = AsyncLLMEngine.from_config(cfg)
        _ENGINES[key] = eng
    return eng


def _use_engine_process(cfg) -> bool:
    """Run the engine in its own engine-core process (``engine/core_proc.py``) so the
    serving loop and the engine loop do not share a GIL.  ``OMNIA_ENGINE_PROC``:
    ``1`` / ``0`` / ``auto`` (default: GPU, TP=1, and this process has not
    initialised the GPU yet -- the core must be a fresh child)."""
    import torch

    mode = os.environ.get("OMNIA_ENGINE_PROC", "auto").lower()
    if mode in ("0", "false", "no"):
        return False
    if getattr(cfg, "ep_mode", "tp") == "a2a" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return False  # this process IS rank 0 of the EP group (torchrun env)
    if mode in ("1", "true", "yes"):
        return True
    return (cfg.device == "cuda" and cfg.tp == 1 and torch.cuda.device_count() > 0
            and not torch.cuda.is_initialized())


def response_format_instruction(fmt: str, schema: dict | None) -> str:
    """``internal/runtime/response_format.go``: constrain function-mode output."""
    if fmt in ("json", "json_schema"):
        s = "\n\nRespond ONLY with a single JSON object and no other text."
        if fmt == "json_schema" and schema:
            s += " It must validate against this JSON schema: " + json.dumps(schema)
        return s
    return ""


async def build_runtime(cfg: RuntimeConfig, engine=None, pack: PromptPack | None = None,
                        executor: OmniaExecutor | None = None, provider=None,
                        store=None) -> RuntimeService:
    if pack is None:
        try:
            pack = PromptPack.load(cfg.promptpack_path)
        except (FileNotFoundError, PackError) as e:
            log.warning("prompt pack unavailable (%s); using a minimal default pack", e)
            pack = PromptPack.minimal()
    ptype = (cfg.provider or {}).get("type", "mock")
    if provider is None:
        if ptype in ("local", "omnia", "rocm", "engine") and engine is None:
            engine = shared_engine(cfg.engine)
        provider = build_provider(cfg.provider or {"type": "mock"}, engine=engine)
    extra = {}
    audio = {}
    for p in cfg.extra_providers:
        role = (p.get("role") or "").lower()
        if role in ("stt", "tts"):
            from .duplex import build_audio_provider

            try:
                audio[role] = build_audio_provider(p, role)
            except ValueError as e:
                log.warning("%s provider skipped: %s", role, e)
            continue
        try:
            extra[p.get("role", p.get("name", "extra"))] = build_provider(p, engine=engine)
        except ValueError as e:
            log.warning("extra provider skipped: %s", e)
    store = store or make_store(cfg.context_type, cfg.context_url, cfg.context_ttl_s)
    if executor is None:
        policy = PolicyBrokerClient(cfg.policy_broker_url) if cfg.policy_broker_url else None
        executor = OmniaExecutor(load_tools_config(cfg.tools_config_path),
                                 secrets_dir=cfg.tool_secrets_dir, policy=policy)
    memory = None
    if cfg.memory_enabled and cfg.memory_api_url:
        from ..memory.retriever import HTTPMemoryRetriever
        from ..memory.tools import memory_tools

        ws = cfg.workspace_uid or cfg.workspace
        memory = HTTPMemoryRetriever(cfg.memory_api_url, workspace=ws, agent=cfg.agent_name,
                                     strategy=cfg.memory_strategy, deny_cel=cfg.memory_deny_cel,
                                     limit=cfg.memory_limit)
        executor.add_handler(memory_tools(memory.client, ws, cfg.agent_name))
    for c in cfg.a2a_clients:  # remote agents as tools (client_resolver.go BuildA2AAgentOptions)
        if not c.get("exposeAsTools") or not c.get("url"):
            continue
        from ..facade.a2a import a2a_tool_handler

        headers = {}
        tok = os.environ.get(c.get("authTokenEnv") or "", "")
        if tok:
            headers["Authorization"] = f"Bearer {tok}"
        executor.add_handler(a2a_tool_handler(c["name"], c["url"], c.get("description", ""),
                                              headers=headers, timeout=c.get("timeout")))
        log.info("A2A agent %s (%s) registered as tool ask_%s", c["name"], c["url"],
                 c["name"])
    try:
        from .skills import attach_skills

        # OMNIA_PROMPTPACK_MANIFEST_PATH + the pack's own skills; no-op without either
        attach_skills(executor, pack=pack)
    except (OSError, ValueError) as e:  # unreadable/malformed manifest: serve without skills
        log.error("skill manifest load failed: %s", e)
    try:
        await executor.discover()
    except Exception as e:  # noqa: BLE001
        log.warning("tool discovery failed: %s", e)
    event_sink = None
    if cfg.session_api_url:
        from ..session.httpclient import SessionEventSink

        event_sink = SessionEventSink(cfg.session_api_url)
    evaluator = None
    if cfg.eval_enabled:
        from .evals import InlineEvaluator

        pack_evals = list(pack.data.get("evals") or [])
        for pr in pack.prompts.values():
            pack_evals.extend(pr.evals or [])
        evaluator = InlineEvaluator(event_sink, groups=cfg.eval_inline_groups or None,
                                    pack_evals=pack_evals)
    acfg = AgentConfig(prompt_name=cfg.prompt_name or None, context_window=cfg.context_window,
                       truncation=cfg.truncation, defaults=(cfg.provider or {}).get("defaults",
                                                                                   {}),
                       response_format=cfg.output_format, response_schema=cfg.output_schema)
    tok = getattr(engine, "tokenizer", None) if engine is not None else None
    agent = Agent(pack, provider, store, executor, acfg, extra, memory, event_sink, evaluator,
                  tokenizer=tok)
    invoke_agent = agent
    if cfg.mode == "function" or cfg.output_format:
        prompt = agent.prompt
        instr = response_format_instruction(cfg.output_format or "json", cfg.output_schema)
        fpack = PromptPack(json.loads(json.dumps(pack.data)), base_dir=pack.base_dir)
        for p in fpack.prompts.values():
            if p.id == prompt.id:
                p.system_template = p.system_template + instr
        invoke_agent = Agent(fpack, provider, store, executor, acfg, extra, memory, event_sink,
                             evaluator, tokenizer=tok)
    M.RUNTIME_INFO.info({"agent": cfg.agent_name, "namespace": cfg.namespace,
                         "promptpack": pack.id, "promptpack_version": pack.version,
                         "provider": provider.type, "contract_version": "1.3.0"})
    duplex = None
    if "stt" in audio and "tts" in audio:
        from .duplex import DuplexConfig

        dcfg = cfg.duplex or {}
        aud = dcfg.get("audio") or {}
        duplex = DuplexConfig(audio["stt"], audio["tts"],
                              sample_rate=int(aud.get("sampleRate", 16000)),
                              codec=aud.get("codec", "pcm"), channels=int(aud.get("channels", 1)))
    return RuntimeService(agent, capabilities=list(CAPABILITIES), invoke_agent=invoke_agent,
                          duplex=duplex, stream_interval_s=cfg.stream_interval_ms / 1000.0)


async def run(cfg: RuntimeConfig | None = None):
    cfg = cfg or RuntimeConfig.from_env()
    configure_logging()
    if cfg.tracing_enabled:
        tracing.configure("omnia-runtime", cfg.tracing_endpoint or None, cfg.tracing_sample_rate)
    svc = await build_runtime(cfg)
    server, gport = await serve_grpc(svc, cfg.grpc_port)
    runner, hport = await serve_health(svc, cfg.health_port)
    from ..utils.proc_tune import tune_serving_process

    tune_serving_process()
    log.info("runtime %s/%s serving gRPC :%d health :%d (provider %s)", cfg.namespace,
             cfg.agent_name, gport, hport, svc.agent.provider.type)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:  # pragma: no cover
            pass
    await stop.wait()
    # graceful: stop accepting, drain for 10 s, hard stop (runtime.go:64-67,292-312)
    svc.ready = False
    await runner.cleanup()
    await server.stop(10)
