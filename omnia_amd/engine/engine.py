"""The in-node inference engine: the piece that replaces Omnia's remote
``Provider`` (``internal/runtime/provider.go:95-151``).

``LLMEngine``      synchronous core: add requests, ``step()`` runs one
                   scheduled prefill or decode step, streams tokens through
                   per-sequence callbacks.
``AsyncLLMEngine`` owns a background engine thread and exposes
                   ``async generate()`` yielding incremental text/token events
                   to asyncio consumers (the runtime's agent loop / OpenAI shim).
"""
from __future__ import annotations

import asyncio
import logging
import collections
import os
import sys
import threading
import time
import uuid
from dataclasses import dataclass, field

import torch

from ..models import build_model
from ..models.config import ModelConfig, resolve
from ..models.llama import KVCache
from ..observability import metrics as M
from ..observability import timeline as TL
from ..observability.engine_trace import EngineTrace
from ..utils import failpoints
from .kv_manager import BlockManager
from .model_runner import ModelRunner
from .sampling_params import SamplingParams
from .scheduler import Scheduler, SchedulerConfig
from .model_runner import PLACEHOLDER
from .sequence import FinishReason, Sequence
from .swap import SwapSpace
from .tokenizer import Detokenizer, make_tokenizer

log = logging.getLogger("omnia.engine")


@dataclass
class EngineConfig:
    model: str = "llama-3-8b"
    device: str = "cuda"
    dtype: str = "bfloat16"
    tp: int = 1
    block_size: int = 32
    max_batch: int = 256
    max_model_len: int = 8192
    max_prefill_tokens: int = 16384
    kv_fraction: float = 0.85  # of free HBM after weights
    num_blocks: int | None = None  # override
    use_graphs: bool = True
    seed: int = 0
    swap_gib: float = 0.0  # host-DRAM warm tier for evicted session KV
    tokenizer: str | None = None
    decode_part_size: int = 512
    pipeline: bool = True  # one-deep async decode scheduling
    # >0: mixed steps (running sequences' decode rows + <= this many prefill tokens
    # in one forward) bound inter-token latency under arrivals; 0: separate steps
    mixed_budget: int = 16384
    # >0: mixed steps only while the prefill backlog is <= this many tokens (a
    # burst is then prefilled first); 0: no gate -- a burst's 16K-token chunks
    # carry the running decoders along.  Open loop (profiles/r4/mixed/) mixed
    # steps cut p50 turn latency 1.7x and p95 TTFT 6x.  In the closed loop the
    # ungated default measured +0.6 % tok/s and -0.9 % p50 turn over the 8192
    # gate, 3 of 3 interleaved pairs on one box (p95 TTFT +1.5 %;
    # profiles/r6/bench/mixed_gate/)
    mixed_backlog: int = 0
    # mixed steps under TP (engine/tp.py MIXED; sampled synchronously on rank 0):
    # on since round 5 -- GPU-verified in every TP arrival mode (profiles/r5/tp)
    tp_mixed: bool = True
    checkpoint: str | None = None  # HF safetensors dir (random init when None)
    # MoE expert parallelism: "tp" = experts sharded over the TP group (EP inside
    # TP); "a2a" = data-parallel attention replicas + token all-to-all to the
    # experts' ranks, every rank stepping in lockstep (engine/ep.py)
    ep_mode: str = "tp"
    # >0 (with WORLD_SIZE > 1, tp = 1): prompts of at least this many uncached
    # tokens are prefilled context-parallel by the whole DP group (engine/cp.py)
    cp_threshold: int = 0
    # cross-session prefix sharing (kv_manager.py): sequences map the published
    # KV pages of a prompt prefix another sequence computed (the deployment's
    # shared system prompt) instead of prefilling them
    share_prefix: bool = True

    @classmethod
    def from_env(cls, **kw) -> "EngineConfig":
        env = os.environ
        m = {
            "OMNIA_ENGINE_MODEL": ("model", str), "OMNIA_ENGINE_TP": ("tp", int),
            "OMNIA_ENGINE_MAX_BATCH": ("max_batch", int),
            "OMNIA_ENGINE_KV_FRACTION": ("kv_fraction", float),
            "OMNIA_ENGINE_DTYPE": ("dtype", str),
            "OMNIA_ENGINE_MAX_MODEL_LEN": ("max_model_len", int),
            "OMNIA_ENGINE_BLOCK_SIZE": ("block_size", int),
            "OMNIA_ENGINE_DEVICE": ("device", str),
            "OMNIA_ENGINE_SWAP_GIB": ("swap_gib", float),
            "OMNIA_ENGINE_CHECKPOINT": ("checkpoint", str),
            "OMNIA_ENGINE_USE_GRAPHS": ("use_graphs", lambda v: v.lower() != "false"),
            "OMNIA_ENGINE_MIXED_BUDGET": ("mixed_budget", int),
            "OMNIA_ENGINE_MIXED_BACKLOG": ("mixed_backlog", int),
            "OMNIA_ENGINE_EP_MODE": ("ep_mode", str),
            "OMNIA_ENGINE_CP_THRESHOLD": ("cp_threshold", int),
            "OMNIA_ENGINE_SHARE_PREFIX": ("share_prefix", lambda v: v.lower() not in ("0", "false")),
        }
        for k, (f, t) in m.items():
            if k in env:
                kw.setdefault(f, t(env[k]))
        return cls(**kw)


def engine_model_config(cfg: EngineConfig, model_cfg: ModelConfig | None = None) -> ModelConfig:
    """The model architecture an engine serves: explicit, else the checkpoint's
    ``config.json`` (authoritative when a checkpoint is given -- its name need
    not be a registered preset), else the registered preset ``cfg.model``."""
    if model_cfg is not None:
        return model_cfg
    if cfg.checkpoint:
        from ..models.loader import config_from_hf

        return config_from_hf(cfg.checkpoint, cfg.model)
    return resolve(cfg.model)


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model_cfg: ModelConfig | None = None,
                 weights: dict | None = None):
        self.cfg = cfg
        self.model_cfg = engine_model_config(cfg, model_cfg)
        dev = self._pick_device(cfg)
        self.device = dev
        dtype = getattr(torch, cfg.dtype)
        st = self._ensure_parallel(cfg, dev)
        if st.tp_size > 1 and st.tp_rank != 0:
            raise RuntimeError("TP ranks > 0 run omnia_amd.engine.tp.run_worker, not LLMEngine")
        if dev.type == "cuda":
            from ..ops.gemm_tuning import enable_tuned_gemms

            self.tuned_gemms = enable_tuned_gemms(dev.index or 0)
        t0 = time.perf_counter()
        if weights is None and cfg.checkpoint:
            from ..models.loader import load_hf_checkpoint

            weights = load_hf_checkpoint(cfg.checkpoint, self.model_cfg, st.tp_size, st.tp_rank,
                                         dev, dtype)
        self.model = build_model(self.model_cfg, device=dev, dtype=dtype, seed=cfg.seed,
                                 weights=weights, decode_part_size=cfg.decode_part_size,
                                 ep_mode=cfg.ep_mode)
        self.load_s = time.perf_counter() - t0
        # tile-packed decode weights: allocated before the KV pool is sized from
        # what is left of HBM
        self.packed_bytes = (self.model.prepack_decode(cfg.max_batch)
                             if hasattr(self.model, "prepack_decode") else 0)
        nb = cfg.num_blocks or self.kv_pool_blocks(cfg, self.model_cfg, self.model.tp, dev, dtype)
        runner_cls = ModelRunner
        # DP-attention + EP: every forward is a collective of the EP group
        self.ep_lockstep = cfg.ep_mode == "a2a" and st.world_size > 1
        self._ep_active = 0  # any rank of the lockstep group still busy
        self.cp_lockstep = (cfg.cp_threshold > 0 and st.world_size > 1 and st.tp_size == 1
                            and not self.ep_lockstep)
        self.lockstep = self.ep_lockstep or self.cp_lockstep
        if self.ep_lockstep:
            from .ep import EPModelRunner

            runner_cls = EPModelRunner
        if st.tp_size > 1:
            from .tp import TPModelRunner, agree_num_blocks

            nb = agree_num_blocks(nb, dev)
            runner_cls = TPModelRunner
        t_kv = time.perf_counter()
        self.kv = KVCache.allocate(self.model_cfg, nb, cfg.block_size, dev,
                                   tp_size=self.model.tp, dtype=dtype)
        self.kv_alloc_s = time.perf_counter() - t_kv
        # pod cold-start breakdown (omnia_engine_cold_start_seconds{phase}); decode
        # graphs are captured lazily per bucket and reported as graph_warmup
        M.ENGINE_COLD_START.labels("weights").set(self.load_s)
        M.ENGINE_COLD_START.labels("kv_alloc").set(self.kv_alloc_s)
        self.runner = runner_cls(self.model, self.kv, max_batch=cfg.max_batch,
                                 max_model_len=cfg.max_model_len, use_graphs=cfg.use_graphs,
                                 max_prefill_tokens=cfg.max_prefill_tokens)
        swap = None
        if cfg.swap_gib > 0:  # (on the CPU the "host" tier is a second copy: tests)
            swap = SwapSpace(self.kv, cfg.swap_gib)
            if st.tp_size > 1:
                from .tp import TPSwapProxy

                swap = TPSwapProxy(swap, self.runner.chan)
        self.blocks = BlockManager(nb, cfg.block_size, swap=swap, share_prefix=cfg.share_prefix)
        self._kv_seen: dict = {}  # block-manager hit totals already exported
        self.scheduler = Scheduler(
            SchedulerConfig(max_batch=cfg.max_batch, max_prefill_tokens=cfg.max_prefill_tokens,
                            max_model_len=cfg.max_model_len,
                            # under TP a mixed step is published to the workers (MIXED)
                            # and sampled synchronously on rank 0 (tp_mixed)
                            mixed_budget=cfg.mixed_budget if (self.model.tp == 1 or
                                                              cfg.tp_mixed) else 0,
                            mixed_backlog=cfg.mixed_backlog,
                            cp_threshold=cfg.cp_threshold if self.cp_lockstep else 0),
            self.blocks)
        self.scheduler.on_capped = self._finish_capped
        self.tokenizer = make_tokenizer(self.model_cfg, cfg.tokenizer)
        self.eos = set(self.tokenizer.eos_token_ids)
        self.seqs: dict[int, Sequence] = {}
        self.detok: dict[int, Detokenizer] = {}
        self._guided = None  # K13 grammar registry, built on the first guided request
        self.step_count = 0
        self.inflight = None
        self.counters = {"prefill_tokens": 0, "decode_tokens": 0, "steps_prefill": 0,
                         "steps_decode": 0, "finished": 0}
        # host-side time per phase of pipelined decode (diagnostics; bench reports it)
        self.timing = {"schedule_s": 0.0, "launch_s": 0.0, "collect_wait_s": 0.0,
                       "append_s": 0.0, "pipeline_breaks": 0, "gpu_starved_launches": 0}
        # untraced step timeline (OMNIA_TIMELINE_DIR, observability/timeline.py):
        # host schedule / launch times + timing hipEvents around every step
        self._tl = [] if (TL.ENABLED and dev.type == "cuda") else None
        self._busy = collections.deque()  # (start, end) hipEvents of steps not yet summed
        self._busy_s = 0.0
        self._tap_dir = os.environ.get("OMNIA_LOGIT_TAP_DIR", "")
        # OTel engine spans / roctx ranges / torch.profiler window (all opt-in)
        self.trace = EngineTrace(dev.type)
        M.ENGINE_COLD_START.labels("total").set(time.perf_counter() - t0)
        log.info("engine ready: %s on %s (tp=%d), %d KV blocks x %d tokens, load %.1fs, "
                 "kv alloc %.2fs", self.model_cfg.name, dev, st.tp_size, nb, cfg.block_size,
                 self.load_s, self.kv_alloc_s)

    @staticmethod
    def _pick_device(cfg: EngineConfig) -> torch.device:
        dev = torch.device(cfg.device if (cfg.device != "cuda" or torch.cuda.is_available())
                           else "cpu")
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        return dev

    @staticmethod
    def _ensure_parallel(cfg: EngineConfig, dev):
        from ..parallel import state as pstate

        st = pstate.get_state()
        if cfg.tp > 1 and st.tp_size != cfg.tp:
            st = pstate.init_distributed(tp_size=cfg.tp, device=dev.type)
        elif ((cfg.ep_mode == "a2a" or cfg.cp_threshold > 0) and st.world_size == 1
              and pstate.env_world()[0] > 1):
            st = pstate.init_distributed(tp_size=1, device=dev.type)
        return st

    @staticmethod
    def kv_pool_blocks(cfg: EngineConfig, mc: ModelConfig, tp: int, device, dtype) -> int:
        per_block = (mc.kv_bytes_per_token(torch.tensor([], dtype=dtype).element_size())
                     // tp) * cfg.block_size
        if device.type == "cuda":
            torch.cuda.synchronize()
            free, total = torch.cuda.mem_get_info(device)
            # leave room for activations / graphs
            reserve = 6 * 2**30 + cfg.max_prefill_tokens * mc.hidden_size * 40
            from ..parallel import state as pstate

            share = pstate.ranks_per_device()  # TP ranks rehearsed on one device
            # pods sharing each GPU (the launcher's OMNIA_GPU_SHARE, 288 GB devices):
            # this pod's slice is total / pods, less what it already holds
            pods = max(1, int(os.environ.get("OMNIA_GPU_SHARE", "1") or 1))
            if pods > 1:
                free = max(0, min(free, int(total / pods) - torch.cuda.memory_reserved(device)))
            budget = max(0, int(free * cfg.kv_fraction / share) - reserve)
        else:
            budget = 256 * 2**20
        return int(max(16, budget // per_block))

    def shutdown(self):
        if hasattr(self.runner, "shutdown"):
            self.runner.shutdown()

    # --------------------------------------------------------------- requests
    def add_request(self, prompt: list[int] | str, params: SamplingParams | None = None,
                    session_id: str | None = None, request_id: str | None = None,
                    on_token=None, on_finish=None) -> Sequence:
        params = (params or SamplingParams()).validate()
        if isinstance(prompt, str):
            prompt = self.tokenizer.encode(prompt, add_bos=True)
        s = Sequence(prompt=list(prompt), params=params, session_id=session_id,
                     request_id=request_id or uuid.uuid4().hex, on_token=on_token,
                     on_finish=on_finish)
        if params.guided:
            if self._guided is None:
                from .guided import GuidedRegistry

                self._guided = GuidedRegistry(self.tokenizer)
            s.guide = self._guided.matcher(params)  # raises SchemaError on bad schemas
        self.scheduler.add(s)
        self.seqs[s.seq_id] = s
        self.detok[s.seq_id] = Detokenizer(self.tokenizer)
        M.ENGINE_WAITING.set(len(self.scheduler.waiting))
        return s

    def abort(self, seq_id: int) -> None:
        s = self.scheduler.abort(seq_id)
        if s is not None:
            self._finalize(s)

    def drop_session(self, session_id: str) -> bool:
        return self.blocks.drop_session(session_id)

    # --------------------------------------------------------------- stepping
    def step(self) -> int:
        """Run one engine iteration.  Returns number of tokens produced.

        Decode steps are pipelined one deep ("async scheduling"): step N+1 is
        launched -- its input tokens gathered on the GPU from step N's sampler
        output -- before step N's tokens are pulled to the host and processed,
        so host work (scheduling, detokenisation, streaming, stop checks)
        overlaps the GPU instead of idling it."""
        if failpoints.active():
            failpoints.hit("engine.step")
            failpoints.hit("engine.prefill" if self.scheduler.waiting else "engine.decode_step")
            if failpoints.triggered("engine.hang"):
                time.sleep(float(os.environ.get("OMNIA_FAILPOINT_HANG_S", "5")))
        self.trace.begin(self.step_count)
        try:
            return self._step()
        finally:
            self.trace.end()

    def _step(self) -> int:
        if self.ep_lockstep:
            from .ep import run_ep_step

            return run_ep_step(self)
        if self.cp_lockstep:
            from .cp import run_cp_step

            return run_cp_step(self)
        if self.cfg.pipeline and self.runner.use_graphs:
            return self._step_pipelined()
        return self._step_sync()

    def recover(self, err: Exception) -> int:
        """Engine-fault recovery (SURVEY §5.3 [design]): fail every live sequence
        with ERROR (the runtime answers the turn with an ``ENGINE_FAULT`` error),
        discard the in-flight pipelined step and ALL resident session KV (it may
        hold half-written pages), so the next turn of each session re-prefills
        from its transcript -- the transcript stays authoritative, as in the
        reference's resume path.  Returns the number of sequences failed."""
        self.inflight = None
        self.counters["faults"] = self.counters.get("faults", 0) + 1
        M.ENGINE_FAULTS.labels(type(err).__name__).inc()
        n = 0
        for s in list(self.seqs.values()):
            self.scheduler.abort(s.seq_id)
            s.finish_reason = FinishReason.ERROR
            self._finalize(s)
            n += 1
        for sid in list(self.blocks.sessions.keys()):
            self.blocks.drop_session(sid)
        self.blocks.reset_shared()
        if self.device.type == "cuda":
            try:
                torch.cuda.synchronize(self.device)
            except Exception:  # noqa: BLE001 - a dead context stays dead; health says so
                log.exception("device sync after fault failed")
        log.error("engine fault (%s): failed %d sequences, dropped resident KV", err, n)
        return n

    # ------------------------------------------------------------ timeline
    def _tl_pre(self):
        if self.device.type != "cuda":
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _tl_post(self, e0, kind: str, ts: float, t0: float, rows: int, ntok: int) -> None:
        """Step record: schedule start ``ts``, launch start ``t0``, launch end now;
        device interval = [e0, e1] (e0 completes when the stream reaches the step,
        i.e. when the previous step ends or at launch if the GPU was idle).  Every
        step's interval also feeds the device-busy account (:meth:`busy_seconds`);
        the timeline keeps them only when enabled."""
        if self.trace.active:
            self.trace.on_step(kind, ts, rows, ntok,
                               self.blocks.num_blocks - self.blocks.num_available, self.step_count)
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self._busy.append((e0, e1))
        if len(self._busy) > 512:
            self._busy_harvest(False)
        if self._tl is not None:
            self._tl.append((kind, rows, ntok, ts, t0, time.perf_counter(), e0, e1))

    def _busy_harvest(self, wait: bool) -> None:
        while self._busy and (wait or self._busy[0][1].query()):
            e0, e1 = self._busy.popleft()
            if wait:
                e1.synchronize()
            self._busy_s += e0.elapsed_time(e1) / 1e3

    def busy_seconds(self, reset: bool = False) -> float:
        """Device time covered by engine steps since the last reset: the sum of
        per-step [start, end] hipEvent intervals on the engine stream (steps
        never overlap on it; idle gaps between steps are not counted).  Waits
        for the steps in flight.  None on a CPU engine (no device clock)."""
        if self.device.type != "cuda":
            return None
        self._busy_harvest(True)
        v = self._busy_s
        if reset:
            self._busy_s = 0.0
        return v

    def tl_flush(self) -> None:
        """Resolve the recorded steps' device times onto the host monotonic clock
        and write them (call when idle: it synchronizes the device)."""
        if not self._tl:
            return
        torch.cuda.synchronize(self.device)
        ea, ta = TL.device_anchor()
        for kind, rows, ntok, ts, t0, t1, e0, e1 in self._tl:
            TL.mark_at(ts, "step", kind=kind, rows=rows, ntok=ntok, t_launch=round(t0, 6),
                       t_launched=round(t1, 6), d0=round(ta - e0.elapsed_time(ea) / 1e3, 6),
                       d1=round(ta - e1.elapsed_time(ea) / 1e3, 6))
        self._tl.clear()
        TL.flush()

    def has_work(self) -> bool:
        return self.inflight is not None or self.scheduler.has_work()

    def _flush_inflight(self) -> int:
        h, self.inflight = self.inflight, None
        if h is None:
            return 0
        t0 = time.perf_counter()
        toks = self.runner.collect(h)
        now = time.perf_counter()
        for sq, tok in zip(h.seqs, toks):
            self._append(sq, tok, now)
        tm = self.timing
        tm["collect_wait_s"] += now - t0
        if self._tl is not None:
            TL.mark_at(t0, "collect", kind=h.kind, n=len(toks), t1=now)
        tm["append_s"] += time.perf_counter() - now
        return len(toks)

    def _steady(self) -> bool:
        sch = self.scheduler
        if not self.handoff and (sch.waiting or sch.partial):
            return False
        # every running sequence can take its next token's page without a
        # preemption (never preempt a sequence whose tokens are in flight); pages
        # of idle retained sessions count -- allocation reclaims them (LRU) on the
        # host without touching in-flight work, so a pool full of parked
        # multi-turn sessions does not drop the engine out of pipelined steps
        return self.blocks.num_available >= len(sch.running) + 1

    @property
    def handoff(self) -> bool:
        """Steps of every kind feed in-flight tokens from the device token slots,
        so no step kind waits for the previous one's tokens on the host."""
        return getattr(self.runner, "device_handoff", False)

    def _launched(self, h, prefill, decode=()) -> int:
        """Book-keeping after a step was enqueued: counters advance now, the
        sampled tokens arrive at collect (their PLACEHOLDER is filled then)."""
        for sq in decode:
            sq.num_cached = sq.length  # the fed token's KV is written by this step
            sq.output.append(PLACEHOLDER)
        self.scheduler.on_prefill_done(prefill, {})
        self.export_kv_metrics()
        if self.handoff:
            for sq in h.seqs[len(decode):]:  # completed prompts: token in its slot
                sq.output.append(PLACEHOLDER)
        n = self._flush_inflight()
        self.inflight = h
        ntok = sum(k for _, k in prefill)
        self.counters["prefill_tokens"] += ntok
        M.PREFILL_TOKENS.inc(ntok)
        if decode:
            self.counters["decode_tokens"] += len(decode)
            M.DECODE_TOKENS.inc(len(decode))
        self.step_count += 1
        return n

    def _step_pipelined(self) -> int:
        sch = self.scheduler
        h0 = self.inflight
        if h0 is not None:
            if (h0.kind in ("decode", "mixed") and not self._steady()) or \
                    self.blocks.num_available < len(sch.running) + 1:
                # the next step may preempt: nothing of a sequence it could pick
                # (pages being written, a token not yet collected) may be in flight
                self.timing["pipeline_breaks"] += 1
                return self._flush_inflight()
            if h0.kind == "prefill" and not self.handoff and not (sch.waiting or sch.partial):
                # the next step decodes: it feeds the prefill's sampled tokens
                return self._flush_inflight()
        ts = time.perf_counter()
        plan = sch.schedule()
        if plan.kind == "prefill" and self.runner.can_pipeline_prefill(plan.prefill):
            # prefill N+1 is assembled and enqueued while step N runs on the GPU
            t0 = time.perf_counter()
            self.timing["schedule_s"] += t0 - ts
            e0 = self._tl_pre()
            h = self.runner.launch_prefill(plan.prefill)
            self._tl_post(e0, "prefill", ts, t0, 0, sum(n for _, n in plan.prefill))
            self.timing["launch_s"] += time.perf_counter() - t0
            self.counters["steps_prefill"] += 1
            return self._launched(h, plan.prefill)
        if plan.kind == "mixed" and self.runner.can_pipeline_mixed(plan.decode, plan.prefill):
            # decode rows ride along a prefill chunk; their input tokens (and those
            # of prompts completed by the step before) come from the token slots
            t0 = time.perf_counter()
            self.timing["schedule_s"] += t0 - ts
            e0 = self._tl_pre()
            h = self.runner.launch_mixed(plan.decode, plan.prefill)
            self._tl_post(e0, "mixed", ts, t0, len(plan.decode),
                          sum(n for _, n in plan.prefill))
            self.timing["launch_s"] += time.perf_counter() - t0
            self.counters["steps_mixed"] = self.counters.get("steps_mixed", 0) + 1
            M.BATCH_SIZE.observe(len(plan.decode))
            return self._launched(h, plan.prefill, plan.decode)
        if plan.kind == "mixed":
            # synchronous mixed step (penalties / grammars): drain the in-flight step
            self.counters["steps_mixed_sync"] = self.counters.get("steps_mixed_sync", 0) + 1
            n0 = self._flush_inflight()
            plan.decode = [sq for sq in plan.decode if not sq.is_finished]
            if not plan.decode:
                plan.kind = "prefill"
            return n0 + self._run_plan(plan)
        if h0 is not None and h0.kind == "prefill" and plan.kind != "prefill" and \
                not self.handoff:
            n0 = self._flush_inflight()
            if plan.kind == "decode":
                plan.decode = [sq for sq in plan.decode if not sq.is_finished]
                if not plan.decode:
                    return n0
        else:
            n0 = 0
        if plan.kind == "decode" and self.runner.can_pipeline(plan.decode):
            t0 = time.perf_counter()
            self.timing["schedule_s"] += t0 - ts
            if h0 is not None and h0.event.query():
                self.timing["gpu_starved_launches"] += 1  # GPU drained before this launch
            e0 = self._tl_pre()
            h = self.runner.launch_decode(plan.decode)
            self._tl_post(e0, "decode", ts, t0, len(plan.decode), 0)
            t1 = time.perf_counter()
            self.timing["launch_s"] += t1 - t0
            for sq in plan.decode:
                sq.num_cached = sq.length  # the fed token's KV is written by this step
                sq.output.append(PLACEHOLDER)
            n = self._flush_inflight()
            self.inflight = h
            self.counters["decode_tokens"] += len(plan.decode)
            self.counters["steps_decode"] += 1
            M.DECODE_TOKENS.inc(len(plan.decode))
            M.BATCH_SIZE.observe(len(plan.decode))
            M.STEP_SECONDS.labels("decode").observe(time.perf_counter() - t0)
            self.step_count += 1
            return n0 + n
        n = n0 + self._flush_inflight()
        if plan.kind == "idle":
            return n
        if plan.kind == "decode":
            plan.decode = [sq for sq in plan.decode if not sq.is_finished]
            if not plan.decode:
                return n
        return n + self._run_plan(plan)

    def _step_sync(self) -> int:
        plan = self.scheduler.schedule()
        if plan.kind == "idle":
            return 0
        return self._run_plan(plan)

    def _run_plan(self, plan) -> int:
        t0 = time.perf_counter()
        e0 = self._tl_pre()
        if plan.kind == "mixed":
            toks, sampled = self.runner.run_mixed(plan.decode, plan.prefill)
            done = self.scheduler.on_decode_done(plan.decode, toks)
            done += self.scheduler.on_prefill_done(plan.prefill, sampled)
            ntok = sum(n for _, n in plan.prefill)
            self.counters["prefill_tokens"] += ntok
            self.counters["decode_tokens"] += len(toks)
            self.counters["steps_mixed"] = self.counters.get("steps_mixed", 0) + 1
            M.PREFILL_TOKENS.inc(ntok)
            M.DECODE_TOKENS.inc(len(toks))
        elif plan.kind == "prefill":
            sampled = self.runner.run_prefill(plan.prefill)
            done = self.scheduler.on_prefill_done(plan.prefill, sampled)
            ntok = sum(n for _, n in plan.prefill)
            self.counters["prefill_tokens"] += ntok
            self.counters["steps_prefill"] += 1
            M.PREFILL_TOKENS.inc(ntok)
        else:
            toks = self.runner.run_decode(plan.decode)
            done = self.scheduler.on_decode_done(plan.decode, toks)
            self.counters["decode_tokens"] += len(toks)
            self.counters["steps_decode"] += 1
            M.DECODE_TOKENS.inc(len(toks))
            M.BATCH_SIZE.observe(len(toks))
        self._tl_post(e0, plan.kind + "_sync", t0, t0, len(plan.decode or ()),
                      sum(n for _, n in (plan.prefill or ())))
        dt = time.perf_counter() - t0
        M.STEP_SECONDS.labels(plan.kind).observe(dt)
        now = time.perf_counter()
        for s, tok in done:
            self._append(s, tok, now)
        self.step_count += 1
        self.export_kv_metrics()
        return len(done)

    def export_kv_metrics(self) -> None:
        """KV pool gauges and the prefix-hit counters (from the block manager's
        running totals)."""
        M.KV_UTIL.set(self.blocks.utilization())
        st, seen = self.blocks.stats, self._kv_seen
        for key, metric in (("prefix_hit_tokens", M.KV_HIT_TOKENS),
                            ("shared_hit_tokens", M.KV_SHARED_HIT_TOKENS)):
            d = st.get(key, 0) - seen.get(key, 0)
            if d > 0:
                metric.inc(d)
                seen[key] = st[key]

    def _append(self, s: Sequence, tok: int, now: float) -> None:
        if s.is_finished:
            return
        if s.first_token_time is None:
            s.first_token_time = now
            M.TTFT.observe(now - s.arrival)
        if s.n_real < len(s.output):  # fill the oldest in-flight placeholder
            s.output[s.n_real] = tok
        else:
            s.output.append(tok)
        s.n_real += 1
        nout = s.n_real
        p = s.params
        reason = None
        if s.guide is not None:
            ok = s.guide.accept(tok)
            if not ok:
                log.warning("seq %d: token %d rejected by its grammar", s.seq_id, tok)
            if not ok or s.guide.m.finished:
                reason = FinishReason.STOP  # the document is complete (EOS taken)
        if reason is None:
            if not p.ignore_eos and tok in self.eos and nout > p.min_tokens:
                reason = FinishReason.STOP
            elif tok in p.stop_token_ids:
                reason = FinishReason.STOP
            elif nout >= p.max_tokens:
                reason = FinishReason.LENGTH
            elif len(s.prompt) + nout >= self.cfg.max_model_len:
                reason = FinishReason.LENGTH
        text = ""
        if s.on_token is not None or p.stop:
            if not (reason == FinishReason.STOP and tok in self.eos):
                text = self.detok[s.seq_id].push(tok)
            if p.stop and text:
                s.text_tail = (s.text_tail + text)[-256:]
                for st in p.stop:
                    if st and st in s.text_tail:
                        reason = FinishReason.STOP
                        break
        if s.on_token is not None:
            s.on_token(s, tok, text)
        if reason is not None:
            if s.n_real < len(s.output):  # drop tokens speculatively in flight
                del s.output[s.n_real:]
                s.num_cached = min(s.num_cached, s.length - 1)
            self.scheduler.finish(s, reason)
            self._finalize(s)

    def _finish_capped(self, s: Sequence) -> None:
        """The scheduler finished ``s`` because the KV pool cannot hold its next
        token and nothing else can be preempted."""
        log.warning("sequence %s hit the KV pool capacity (%d tokens): finished as length",
                    s.request_id, s.length)
        if s.n_real < len(s.output):
            del s.output[s.n_real:]
        self._finalize(s)

    def _dump_tap(self, s: Sequence) -> None:
        """``OMNIA_LOGIT_TAP_DIR`` (with the logit tap on): write a finished
        sequence's prompt / output ids and every logits row it was sampled from,
        so a test can check a served pod against ``ops.reference.dense_forward``
        from outside the pod's processes."""
        tap = self.runner.logit_tap
        rows = []
        for ids, r in tap:
            for i, sid in enumerate(ids):
                if sid == s.seq_id:
                    rows.append(r[i])
        # a finished sequence's rows are no longer needed in memory
        self.runner.logit_tap = [(ids, r) for ids, r in tap if any(
            sid in self.seqs and sid != s.seq_id for sid in ids)]
        os.makedirs(self._tap_dir, exist_ok=True)
        torch.save({"prompt": [int(x) for x in s.prompt], "output": [int(x) for x in s.output],
                    "rows": torch.stack(rows) if rows else torch.empty(0)},
                   os.path.join(self._tap_dir,
                                f"seq-{self.model_cfg.name}-{os.getpid()}-{s.seq_id}.pt"))

    def _finalize(self, s: Sequence) -> None:
        self.counters["finished"] += 1
        if self._tap_dir and self.runner.logit_tap is not None:
            self._dump_tap(s)
        rel = getattr(self.runner, "release_slot", None)
        if rel is not None:
            rel(s)
        if s.finish_time is None:
            s.finish_time = time.perf_counter()
        if s.on_token is not None:
            tail = self.detok[s.seq_id].flush()
            if tail:
                s.on_token(s, None, tail)
        self.detok.pop(s.seq_id, None)
        self.seqs.pop(s.seq_id, None)
        M.TURN_SECONDS.observe(s.finish_time - s.arrival)
        if s.on_finish is not None:
            s.on_finish(s)

    def run_until_done(self, max_steps: int = 10**9) -> None:
        n = 0
        if self.lockstep:  # step until the whole EP / CP group is idle
            while n < max_steps:
                self.step()
                n += 1
                if not self._ep_active:
                    return
            return
        while self.has_work() and n < max_steps:
            self.step()
            n += 1

    def generate(self, prompts: list, params: SamplingParams | None = None,
                 session_ids: list | None = None) -> list[Sequence]:
        seqs = [self.add_request(p, params, session_id=(session_ids[i] if session_ids else None))
                for i, p in enumerate(prompts)]
        finished = set()
        while len(finished) < len(seqs):
            self.step()
            for s in seqs:
                if s.is_finished:
                    finished.add(s.seq_id)
        if self.lockstep:
            self.run_until_done()  # keep serving the group's collectives until all idle
        return seqs


# ===================================================================== async
@dataclass
class GenEvent:
    text: str = ""
    token: int | None = None
    n_tokens: int = 1  # tokens coalesced into this event
    finished: bool = False
    finish_reason: str | None = None
    prompt_tokens: int = 0
    output_tokens: int = 0
    cached_tokens: int = 0
    ttft: float | None = None


class _Chan:
    """Per-request delivery buffer (filled on the consumer's loop, drained whole)."""

    __slots__ = ("items", "event")

    def __init__(self):
        self.items: list = []
        self.event = asyncio.Event()


class AsyncLLMEngine:
    """Background engine thread + asyncio streaming API."""

    def __init__(self, engine: LLMEngine):
        # The engine thread and the asyncio serving loop share the GIL.  With the
        # default 5 ms switch interval a busy event loop delays the engine thread's
        # wake-up after every GPU wait by up to 5 ms (a GPU bubble per decode step);
        # hand the GIL over faster.
        sys.setswitchinterval(float(os.environ.get("OMNIA_GIL_SWITCH_INTERVAL", "0.0005")))
        # a cyclic-GC pass holds the GIL for its whole duration (tens of ms on a
        # serving heap full of coroutines and protobuf frames): the engine thread
        # stalls and the GPU drains.  Fewer, larger young-generation passes.
        gct = os.environ.get("OMNIA_GC_THRESHOLD", "")
        if gct:
            import gc

            gc.set_threshold(*[int(x) for x in gct.split(",")])
            if os.environ.get("OMNIA_GC_FREEZE"):
                gc.freeze()
        self.engine = engine
        self._inbox: list = []
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self._outbox: dict = {}  # loop -> [(queue, event)] flushed once per engine step
        self.error: Exception | None = None
        self.healthy = True
        self._fault_times: list = []
        self._step_t0 = None
        self.step_timeout = float(os.environ.get("OMNIA_STEP_TIMEOUT_S", "120"))
        self._thread = threading.Thread(target=self._loop, name="omnia-engine", daemon=True)
        self._thread.start()
        self._watchdog = threading.Thread(target=self._watch, name="omnia-engine-watchdog",
                                          daemon=True)
        self._watchdog.start()

    def _watch(self):
        """Step watchdog: a GPU step that never returns (hung kernel, lost peer in
        a collective) cannot be interrupted from Python, so the watchdog flips
        ``healthy`` off -- readiness fails, the replica router re-homes the
        engine's sessions and the orchestrator restarts the pod."""
        while not self._stop:
            t0 = self._step_t0
            if t0 is not None and self.healthy and time.monotonic() - t0 > self.step_timeout:
                self.healthy = False
                self.error = TimeoutError(f"engine step exceeded {self.step_timeout:.0f}s")
                M.ENGINE_FAULTS.labels("StepTimeout").inc()
                log.error("engine watchdog: step running for >%.0fs, marking unhealthy",
                          self.step_timeout)
            time.sleep(min(1.0, max(0.05, self.step_timeout / 10)))

    def health(self) -> bool:
        return self.healthy and self._thread.is_alive()

    def _emit(self, loop, q, ev):
        self._outbox.setdefault(loop, []).append((q, ev))

    @staticmethod
    def _deliver(batch):
        for ch, ev in batch:
            ch.items.append(ev)
            ch.event.set()

    def _flush(self):
        if self._outbox:
            out, self._outbox = self._outbox, {}
            for loop, batch in out.items():
                try:
                    loop.call_soon_threadsafe(self._deliver, batch)
                except RuntimeError:  # loop closed
                    pass

    @classmethod
    def from_config(cls, cfg: EngineConfig) -> "AsyncLLMEngine":
        return cls(LLMEngine(cfg))

    @property
    def tokenizer(self):
        return self.engine.tokenizer

    def _loop(self):
        eng = self.engine
        if eng.device.type == "cuda":
            torch.cuda.set_device(eng.device)
        while not self._stop:
            with self._lock:
                inbox, self._inbox = self._inbox, []
            for fn in inbox:
                try:
                    fn()
                except Exception as e:  # surface to the submitter
                    log.exception("engine request failed: %s", e)
            if eng.has_work() or eng.lockstep:
                self._step_t0 = time.monotonic()
                try:
                    eng.step()
                except Exception as e:
                    log.exception("engine step failed")
                    self.error = e
                    self._fault_times.append(time.monotonic())
                    try:
                        eng.recover(e)
                    except Exception:  # noqa: BLE001
                        log.exception("engine recovery failed")
                        self._fail_all(e)
                        self.healthy = False
                    recent = [t for t in self._fault_times if time.monotonic() - t < 60.0]
                    self._fault_times = recent
                    if len(recent) >= int(os.environ.get("OMNIA_ENGINE_MAX_FAULTS", "3")):
                        self.healthy = False  # fault storm: stop advertising readiness
                self._step_t0 = None
                self._flush()
                if eng.lockstep and not eng._ep_active:
                    self._wake.wait(0.001)  # group idle: keep the lockstep cadence cheap
                    self._wake.clear()
            else:
                self._flush()
                self._wake.wait(0.05)
                self._wake.clear()

    def _fail_all(self, e: Exception):
        eng = self.engine
        for s in list(eng.seqs.values()):
            eng.scheduler.abort(s.seq_id)
            s.finish_reason = FinishReason.ERROR
            eng._finalize(s)

    def submit(self, fn):
        with self._lock:
            self._inbox.append(fn)
        self._wake.set()

    async def generate(self, prompt, params: SamplingParams | None = None,
                       session_id: str | None = None, request_id: str | None = None):
        from ..utils.arrivals import mark

        mark("runtime_submit")
        loop = asyncio.get_running_loop()
        q = _Chan()
        holder = {}

        def on_token(s, tok, text):
            self._emit(loop, q, GenEvent(text=text or "", token=tok))

        def on_finish(s):
            ev = GenEvent(finished=True, finish_reason=(s.finish_reason.value
                                                        if s.finish_reason else None),
                          prompt_tokens=len(s.prompt), output_tokens=len(s.output),
                          cached_tokens=s.prefix_hit, ttft=s.ttft())
            self._emit(loop, q, ev)

        def add():
            try:
                holder["seq"] = self.engine.add_request(prompt, params, session_id, request_id,
                                                        on_token=on_token, on_finish=on_finish)
            except Exception as e:
                self._emit(loop, q, e)

        self.submit(add)
        try:
            while True:
                await q.event.wait()
                q.event.clear()
                items, q.items = q.items, []
                # adaptive coalescing: tokens that arrived while the consumer was busy
                # are streamed as one chunk (one token per chunk when it keeps up)
                text, last_tok, n = [], None, 0
                for ev in items:
                    if isinstance(ev, Exception):
                        raise ev
                    if ev.finished:
                        if n:
                            yield GenEvent(text="".join(text), token=last_tok, n_tokens=n)
                        yield ev
                        return
                    text.append(ev.text)
                    last_tok = ev.token
                    n += 1
                if n:
                    yield GenEvent(text="".join(text), token=last_tok, n_tokens=n)
        finally:
            s = holder.get("seq")
            if s is not None and not s.is_finished:
                self.submit(lambda: self.engine.abort(s.seq_id))

    def has_session(self, session_id: str) -> bool:
        return self.engine.blocks.has_session(session_id)

    def drop_session(self, session_id: str):
        self.submit(lambda: self.engine.drop_session(session_id))

    def shutdown(self):
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=5)
