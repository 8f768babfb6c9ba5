"""Lockstep execution of DP-attention + EP replicas (``EngineConfig.ep_mode="a2a"``).

Every rank is a full engine (its own scheduler, KV and batch) for attention,
but each Mixtral MoE layer is a collective: tokens go to their experts' rank and
back (:mod:`omnia_amd.parallel.expert`).  So every rank must execute the same
sequence of forwards with the same all-to-all shapes, whatever its own load:

1. each step every rank publishes ``[active, tokens, eager, rows, cols]`` in a
   host shared-memory page and takes the element-wise MAX over the group
   (:class:`omnia_amd.parallel.hostsync.ShmAgreement`: no device collective,
   no device -> host copy);
2. nobody active -> everybody idles;
3. anyone needs an eager forward (a prefill / mixed step, or a decode that
   cannot replay a graph -- penalties, grammars) -> EVERY rank runs eagerly with
   the all-to-all capacity set by the step-global token count: prefill ranks
   prefill, decoding ranks decode eagerly, idle ranks run one padded row;
4. otherwise every rank replays the decode graph of the agreed ``(rows, cols)``
   bucket (idle ranks with all rows padded), so graph captures -- which run the
   collectives too -- happen on all ranks together.

Graph decode steps are pipelined one deep (``run_ep_step``): the agreement
describes the NEXT step from the scheduler's view (in-flight tokens counted as
placeholders), so a rank enqueues step N+1 before collecting step N; a sequence
that finished at step N may ride one speculative step (its token is dropped).
Eager steps drain the in-flight step first.
"""
from __future__ import annotations

import bisect

import torch

from ..parallel import state as pstate
from ..parallel.hostsync import ShmAgreement
from .model_runner import ModelRunner


class EPModelRunner(ModelRunner):
    """ModelRunner whose every forward is agreed across the EP group."""

    fused_launch = False

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        st = pstate.get_state()
        self.group = st.dp_group
        self.ep = st.dp_size
        self.ep_stats = {"steps": 0, "eager_steps": 0, "graph_steps": 0, "idle_fill": 0,
                         "pipelined_steps": 0}
        # per-step agreement over host shared memory: no collective launch, no
        # device -> host copy on the control path (parallel/hostsync.py)
        self.agreement = ShmAgreement.for_group(self.group, 5) if self.ep > 1 else None

    # ------------------------------------------------------------ agreement
    def agree(self, active: int, tokens: int, eager: int, rows: int, cols: int) -> list[int]:
        if self.agreement is None:
            return [active, tokens, eager, rows, cols]
        return self.agreement.max([active, tokens, eager, rows, cols])

    def bucket(self, n: int) -> int:
        return self.buckets[bisect.bisect_left(self.buckets, max(1, n))]

    def describe(self, plan) -> tuple[int, int, int, int, int]:
        if plan.kind == "idle":
            return 0, 0, 0, 0, 0
        if plan.kind in ("prefill", "mixed"):
            n = sum(k for _, k in plan.prefill) + len(plan.decode or [])
            return 1, n, 1, 0, 0
        seqs = plan.decode
        eager = 0 if self.use_graphs and self.can_pipeline(seqs) else 1
        cols = self._ctx_bucket(max(s.length for s in seqs))
        return 1, len(seqs), eager, self.bucket(len(seqs)), cols

    # ------------------------------------------------------------ forwards
    def ep_eager_decode(self, seqs) -> list[int]:
        n = len(seqs)
        ncols = self._ctx_bucket(max(s.length for s in seqs))
        self._decode_inputs(seqs, n, ncols, self.stage[0])
        logits = self._eager_forward(n, ncols)
        self._tap_rows(seqs, logits[:n])
        return self._sample_eager(logits, seqs)

    def ep_idle_forward(self):
        """One padded row through the whole model: this rank still serves the
        MoE all-to-alls of a step in which it has no tokens of its own."""
        ncols = self._ctx_bucket(1)
        self._decode_inputs([], 1, ncols, self.stage[0])
        self._eager_forward(1, ncols)
        self.ep_stats["idle_fill"] += 1

    def ep_graph_decode(self, seqs, nrows: int, ncols: int) -> list[int]:
        n = len(seqs)
        self._decode_inputs(seqs, nrows, ncols, self.stage[0])
        self._replay(nrows, ncols)
        if n == 0:
            self.ep_stats["idle_fill"] += 1
            torch.cuda.current_stream().synchronize()
            return []
        if self._tap is not None:  # correctness tap (the graph copied the rows)
            self._tap_rows(seqs, self._tap[:n])
        return self.out_tok[:n].tolist()


def run_ep_step(engine) -> int:
    """One lockstep engine step (see module docstring).  Returns tokens produced.

    Steady-state decode is pipelined one deep like the single-rank engine: when
    the group agrees on a graph step, a rank with sequences enqueues its replay
    of the agreed bucket (input tokens of the previous, still in-flight step
    gathered on the device from the token slots), THEN collects the previous
    step's tokens -- the host never waits for the GPU between two decode steps.
    Eager steps (someone prefills, penalties, grammars) first drain the
    in-flight step and run synchronously."""
    from . import engine as E
    from .model_runner import PLACEHOLDER

    runner: EPModelRunner = engine.runner
    model = runner.model
    n_pre = 0
    if engine.inflight is not None and not engine._steady():
        # the pool may not give every running sequence its next page without a
        # preemption: never preempt a sequence with a token in flight
        engine.timing["pipeline_breaks"] += 1
        n_pre = engine._flush_inflight()
    plan = engine.scheduler.schedule()
    active, tokens, eager, rows, cols = runner.agree(*runner.describe(plan))
    engine._ep_active = active
    if not active:
        return n_pre + engine._flush_inflight()
    runner.ep_stats["steps"] += 1
    pipelined = engine.cfg.pipeline and runner.use_graphs and runner.device_handoff
    if not eager and pipelined and plan.kind == "decode" and plan.decode:
        runner.ep_stats["graph_steps"] += 1
        runner.ep_stats["pipelined_steps"] = runner.ep_stats.get("pipelined_steps", 0) + 1
        h = runner.launch_decode(plan.decode, rows, cols)
        for sq in plan.decode:
            sq.num_cached = sq.length  # the fed token's KV is written by this step
            sq.output.append(PLACEHOLDER)
        n = engine._flush_inflight()
        engine.inflight = h
        engine.counters["decode_tokens"] += len(plan.decode)
        engine.counters["steps_decode"] += 1
        engine.step_count += 1
        return n_pre + n
    n0 = n_pre + engine._flush_inflight()  # eager / idle-rank steps run on settled state
    if plan.decode:
        plan.decode = [sq for sq in plan.decode if not sq.is_finished]
        if plan.kind == "decode" and not plan.decode:
            plan.kind = "idle"
        elif plan.kind == "mixed" and not plan.decode:
            plan.kind = "prefill"
    done = []
    if eager:
        runner.ep_stats["eager_steps"] += 1
        model.ep_tokens = tokens  # a2a capacity = step-global max tokens x k
        try:
            if plan.kind == "idle":
                runner.ep_idle_forward()
            elif plan.kind == "prefill":
                sampled = runner.run_prefill(plan.prefill)
                done = engine.scheduler.on_prefill_done(plan.prefill, sampled)
                engine.counters["prefill_tokens"] += sum(n for _, n in plan.prefill)
                engine.counters["steps_prefill"] += 1
            elif plan.kind == "mixed":
                toks, sampled = runner.run_mixed(plan.decode, plan.prefill)
                done = engine.scheduler.on_decode_done(plan.decode, toks)
                done += engine.scheduler.on_prefill_done(plan.prefill, sampled)
                engine.counters["prefill_tokens"] += sum(n for _, n in plan.prefill)
                engine.counters["decode_tokens"] += len(toks)
            else:
                toks = runner.ep_eager_decode(plan.decode)
                done = engine.scheduler.on_decode_done(plan.decode, toks)
                engine.counters["decode_tokens"] += len(toks)
                engine.counters["steps_decode"] += 1
        finally:
            model.ep_tokens = 0
    else:
        runner.ep_stats["graph_steps"] += 1
        seqs = plan.decode if plan.kind == "decode" else []
        toks = runner.ep_graph_decode(seqs, rows, cols)
        if seqs:
            done = engine.scheduler.on_decode_done(seqs, toks)
            engine.counters["decode_tokens"] += len(toks)
            engine.counters["steps_decode"] += 1
    import time

    now = time.perf_counter()
    for s, tok in done:
        engine._append(s, tok, now)
    engine.step_count += 1
    engine.export_kv_metrics()
    return n0 + len(done)
