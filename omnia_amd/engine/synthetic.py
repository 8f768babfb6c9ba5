"""Synthetic engine-core: a token source paced like the measured GPU engine.

Capacity rehearsal of the HOST serving path (WebSocket facade -> gRPC runtime
-> engine-core channel -> streamed frames) without a GPU: the engine-core
process (``engine/core_proc.py``) runs this instead of :class:`LLMEngine` when
``OMNIA_ENGINE_SYNTHETIC=1``, so ``bench.py --path ws --engine synthetic
--gpus 8`` drives 8 complete replicas (24 serving processes + the clients) on
one host and shows whether the host path sustains 8x the per-GPU token rate
before an 8-GPU node is available.

Timing model (the engine's own schedule, continuous batching, from the
round-3/4 GPU profiles of Llama-3-8B on one MI355X): waiting prompts are
prefilled in chunks of up to ``max_prefill_tokens`` at ``OMNIA_SYNTH_PREFILL_TOK_S``
tokens/s; otherwise every running sequence gets one token per decode step of
``OMNIA_SYNTH_DECODE_MS`` (+ ``OMNIA_SYNTH_DECODE_MS_PER_ROW`` per row).  The
defaults (165K prefill tok/s, 13 ms + 6 us/row decode) reproduce the measured
~2.7 s wave of 256 x (512 + 128) tokens, i.e. ~12.1K streamed tokens/s per
replica.  Steps sleep instead of computing, so the engine-core process costs
almost no CPU and the rehearsal measures the serving processes alone.

Interface: the subset of :class:`LLMEngine` the engine-core loop uses.
"""
from __future__ import annotations

import collections
import os
import time

from .sequence import FinishReason, Sequence, SeqStatus


class _Blocks:
    num_blocks = 1 << 20

    def __init__(self):
        self.sessions: set = set()

    def has_session(self, sid) -> bool:
        return sid in self.sessions

    def utilization(self) -> float:
        return 0.0


class _Runner:
    use_graphs = False

    def __init__(self):
        self.stats = {"gil_wait_s": 0.0, "captures": 0, "graph_replays": 0}


class _Scheduler:
    def __init__(self, eng):
        self.eng = eng

    def abort(self, seq_id):
        self.eng.abort(seq_id)


class SyntheticEngine:
    TOKEN_TEXT = "a"  # one printable byte token per step: one frame per token

    def __init__(self, cfg):
        from ..models.config import resolve

        self.cfg = cfg
        self.model_cfg = resolve(cfg.model)

        class _Dev:
            type = "cpu"

            def __str__(self):
                return "synthetic"

        self.device = _Dev()
        env = os.environ.get
        self.prefill_tok_s = float(env("OMNIA_SYNTH_PREFILL_TOK_S", "165000"))
        self.decode_s = float(env("OMNIA_SYNTH_DECODE_MS", "13.0")) / 1e3
        self.decode_row_s = float(env("OMNIA_SYNTH_DECODE_MS_PER_ROW", "0.006")) / 1e3
        self.blocks = _Blocks()
        self.runner = _Runner()
        self.scheduler = _Scheduler(self)
        self.timing = {"step_s": 0.0, "sleep_s": 0.0}
        self.counters = collections.Counter()
        self.seqs: dict = {}
        self.waiting: collections.deque = collections.deque()
        self.running: list = []
        self._tok = self._token_id()
        self._next_t = time.perf_counter()

    def _token_id(self) -> int:
        from .tokenizer import make_tokenizer

        try:
            ids = make_tokenizer(self.model_cfg, self.cfg.tokenizer).encode(self.TOKEN_TEXT)
            return int(ids[-1])
        except Exception:  # noqa: BLE001 -- any id: the text is what is streamed
            return 64

    # ------------------------------------------------------------ requests
    def add_request(self, ids, params, session_id=None, request_id=None, on_token=None,
                    on_finish=None):
        s = Sequence(prompt=list(ids), params=params, session_id=session_id,
                     request_id=request_id, on_token=on_token, on_finish=on_finish)
        s._left = len(s.prompt)
        self.seqs[s.seq_id] = s
        self.waiting.append(s)
        if session_id:
            self.blocks.sessions.add(session_id)
        return s

    def abort(self, seq_id):
        s = self.seqs.get(seq_id)
        if s is not None and not s.is_finished:
            self._finish(s, FinishReason.ABORT)

    def drop_session(self, sid):
        self.blocks.sessions.discard(sid)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def _finish(self, s, reason):
        s.finish_reason = reason
        s.status = SeqStatus.FINISHED
        s.finish_time = time.perf_counter()
        self.seqs.pop(s.seq_id, None)
        if s in self.running:
            self.running.remove(s)
        try:
            self.waiting.remove(s)
        except ValueError:
            pass
        if s.on_finish is not None:
            s.on_finish(s)

    def _emit(self, s, now):
        s.output.append(self._tok)
        if s.first_token_time is None:
            s.first_token_time = now
        if s.on_token is not None:
            s.on_token(s, self._tok, self.TOKEN_TEXT)
        if len(s.output) >= s.params.max_tokens:
            self._finish(s, FinishReason.LENGTH)

    # ------------------------------------------------------------ one step
    def step(self):
        t0 = time.perf_counter()
        if self.waiting:  # prefill a chunk of waiting prompts (first token at the end)
            budget = self.cfg.max_prefill_tokens
            done, n = [], 0
            while self.waiting and n < budget:
                s = self.waiting[0]
                take = min(s._left, budget - n)
                s._left -= take
                n += take
                if s._left == 0:
                    done.append(self.waiting.popleft())
            cost = n / self.prefill_tok_s
            self.counters["steps_prefill"] += 1
            self.counters["prefill_tokens"] += n
            self._pace(cost)
            now = time.perf_counter()
            for s in done:
                self.running.append(s)
                self._emit(s, now)
        elif self.running:
            cost = self.decode_s + self.decode_row_s * len(self.running)
            self.counters["steps_decode"] += 1
            self._pace(cost)
            now = time.perf_counter()
            for s in list(self.running):
                self.counters["decode_tokens"] += 1
                self._emit(s, now)
        self.timing["step_s"] += time.perf_counter() - t0

    def _pace(self, cost: float):
        """Sleep until this step's modeled completion (absolute deadlines: host
        overhead of the loop does not stretch the modeled GPU time, as a GPU
        running ahead of its host would not either)."""
        now = time.perf_counter()
        # the GPU runs one step ahead of its host: host time between steps is
        # hidden up to one step's length, beyond that the GPU idled
        base = self._next_t if now - self._next_t <= cost else now
        self._next_t = base + cost
        d = self._next_t - now
        if d > 0:
            self.timing["sleep_s"] += d
            time.sleep(d)

    def recover(self, e):
        for s in list(self.seqs.values()):
            self._finish(s, FinishReason.ERROR)

    def shutdown(self):
        pass
