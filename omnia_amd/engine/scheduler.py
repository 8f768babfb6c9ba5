"""Continuous-batching scheduler with chunked prefill and session-affine KV.

Each engine step is a PREFILL step (new/partially-prefilled sequences, packed
up to ``max_prefill_tokens`` new tokens -- long prompts are chunked), a DECODE
step over every running sequence (the hipGraph-captured hot loop), or -- with
``mixed_budget`` > 0 -- a MIXED step: every running sequence's next token plus
prefill chunks of at most ``mixed_budget`` tokens in ONE forward (the decode
rows ride in the prefill GEMMs, and running sequences never stall behind a
whole prefill chunk: the step time, i.e. their inter-token latency, is bounded
by the budget) -- with ``mixed_backlog`` > 0 taken only while the prefill
backlog is at most that many tokens (arrivals trickling in); a larger backlog
is prefilled first.  Without running sequences prefill uses the full
``max_prefill_tokens`` (throughput); prefill has priority while the running set
is below ``max_batch`` so TTFT stays low.  When the KV pool runs dry, idle session caches are
evicted first (LRU, optionally to host DRAM), then the youngest running
sequence is preempted (its pages are freed and it is re-queued for recompute).
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass

from .kv_manager import BlockManager, OutOfBlocks
from .sequence import FinishReason, Sequence, SeqStatus


@dataclass
class SchedulerConfig:
    max_batch: int = 256
    max_prefill_tokens: int = 16384
    max_model_len: int = 8192
    prefill_chunk: int = 8192  # max new tokens of ONE sequence per prefill step
    mixed_budget: int = 0  # >0: co-schedule decode rows with <= this many prefill tokens
    mixed_backlog: int = 0  # >0: ... only while the prefill backlog is <= this many tokens
    # >0: prompts with at least this many uncached tokens are held for a
    # context-parallel prefill over the DP group (engine/cp.py)
    cp_threshold: int = 0
    # >0: after this many consecutive prefill-first steps with sequences running,
    # the next step serves the running set (decode / mixed) -- a stream of short
    # requests that finish at prefill (so capacity keeps freeing) cannot starve
    # the decoders indefinitely.  A closed-loop wave (<= max_batch prompts) takes
    # far fewer prefill steps and is unaffected.
    max_prefill_streak: int = 16


@dataclass
class StepPlan:
    kind: str  # "prefill" | "decode" | "mixed" | "idle"
    prefill: list  # [(seq, n_new)]
    decode: list  # [seq]


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, blocks: BlockManager):
        self.cfg = cfg
        self.blocks = blocks
        self.waiting: deque[Sequence] = deque()
        self.running: list[Sequence] = []
        self.partial: list[Sequence] = []  # prompts mid-way through chunked prefill
        self.cp_pending: Sequence | None = None  # admitted, waiting for its CP prefill
        self.on_capped = None  # engine hook: a running sequence finished at pool capacity
        self._streak = 0  # consecutive prefill steps taken while sequences were running

    # ------------------------------------------------------------ admission
    def add(self, seq: Sequence) -> None:
        if len(seq.prompt) == 0:
            raise ValueError("empty prompt")
        if len(seq.prompt) >= self.cfg.max_model_len:
            raise ValueError(f"prompt of {len(seq.prompt)} tokens exceeds max_model_len "
                             f"{self.cfg.max_model_len}")
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def abort(self, seq_id: int) -> Sequence | None:
        if self.cp_pending is not None and self.cp_pending.seq_id == seq_id:
            s, self.cp_pending = self.cp_pending, None
            self._free(s, retain=False)
            s.status = SeqStatus.FINISHED
            s.finish_reason = FinishReason.ABORT
            return s
        for q in (self.waiting, self.running, self.partial):
            for s in list(q):
                if s.seq_id == seq_id:
                    q.remove(s)
                    self._free(s, retain=False)
                    s.status = SeqStatus.FINISHED
                    s.finish_reason = FinishReason.ABORT
                    return s
        return None

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self.partial or self.cp_pending)

    @property
    def num_active(self) -> int:
        return len(self.running) + len(self.partial) + (self.cp_pending is not None)

    # ------------------------------------------------------------ context parallel
    def _cp_eligible(self, s: Sequence) -> bool:
        thr = self.cfg.cp_threshold
        return bool(thr) and s.num_cached == 0 and s.length >= thr and not getattr(
            s, "cp_skip", False)

    def cp_candidate(self) -> Sequence | None:
        """The sequence this rank wants prefilled context-parallel (admitted with
        pages for its whole prompt), or None.  Held until :meth:`cp_done`."""
        if self.cp_pending is not None:
            return self.cp_pending
        if not self.cfg.cp_threshold or not self.waiting or self.num_active >= self.cfg.max_batch:
            return None
        s = self.waiting[0]
        if s.num_cached == 0 and not s.blocks:
            self._admit(s)
        if not self._cp_eligible(s):
            return None
        try:
            self._ensure_blocks(s, s.length + 1)
        except OutOfBlocks:
            s.cp_skip = True  # the ordinary chunked path preempts / fails it
            return None
        self.waiting.popleft()
        s.status = SeqStatus.RUNNING
        self.cp_pending = s
        return s

    def cp_done(self, s: Sequence, tok: int) -> list[tuple[Sequence, int]]:
        self.cp_pending = None
        s.num_cached = s.length
        self._publish(s)
        self.running.append(s)
        return [(s, tok)]

    # ------------------------------------------------------------ KV helpers
    def _ensure_blocks(self, s: Sequence, upto_tokens: int) -> None:
        need = self.blocks.blocks_needed(upto_tokens) - len(s.blocks)
        if need > 0:
            s.blocks.extend(self.blocks.allocate(need))

    def _free(self, s: Sequence, retain: bool) -> None:
        if retain and s.session_id:
            self.blocks.retain(s.session_id, s.blocks, s.all_tokens[: s.num_cached])
        else:
            self.blocks.release(s.blocks)
        s.blocks = []

    def _admit(self, s: Sequence) -> None:
        # a prompt held for a context-parallel prefill (engine/cp.py, from token 0)
        # does not map shared pages
        cp = bool(self.cfg.cp_threshold) and s.length >= self.cfg.cp_threshold
        blocks, n = self.blocks.acquire_prefix(s.session_id, s.prompt, share=not cp,
                                               salt=s.params.cache_salt)
        s.blocks = blocks
        s.num_cached = n
        s.prefix_hit = n
        s.pub_pages, s.pub_hash = 0, None

    def _publish(self, s: Sequence) -> None:
        lim = s.params.share_limit
        top = len(s.prompt) if lim is None or lim < 0 else min(lim, len(s.prompt))
        if self.blocks.share_prefix and (s.pub_pages + 1) * self.blocks.block_size <= top:
            s.pub_pages, s.pub_hash = self.blocks.publish(s.prompt, s.blocks, s.num_cached,
                                                          s.pub_pages, s.pub_hash,
                                                          salt=s.params.cache_salt, limit=top)

    def _preempt_one(self, protect: Sequence | None = None) -> bool:
        """Free the youngest page holder: a partially prefilled prompt first (the
        newest admissions; they would otherwise keep their pages while a running
        sequence is cut off at the pool limit), else the youngest running one."""
        for victim in list(reversed(self.partial)) + list(reversed(self.running)):
            if victim is protect:
                continue
            if victim in self.partial:
                self.partial.remove(victim)
            else:
                self.running.remove(victim)
            self.blocks.release(victim.blocks)
            victim.blocks = []
            victim.num_cached = 0
            victim.preemptions += 1
            victim.status = SeqStatus.WAITING
            # re-admission re-prefills prompt + generated-so-far (all_tokens)
            self.waiting.appendleft(victim)
            return True
        return False

    # ------------------------------------------------------------ planning
    def backlog_tokens(self) -> int:
        """Uncached prompt tokens still to prefill (partial + waiting)."""
        return sum(s.num_uncached for s in self.partial) + sum(
            s.length - s.num_cached for s in self.waiting)

    def schedule(self) -> StepPlan:
        plan = self._plan()
        if plan.kind == "prefill" and self.running:
            self._streak += 1
        elif plan.kind != "idle":
            self._streak = 0
        return plan

    def _plan(self) -> StepPlan:
        cfg = self.cfg
        if cfg.max_prefill_streak > 0 and self._streak >= cfg.max_prefill_streak and \
                self.running:
            decode = self._decode_rows()
            if decode:
                if cfg.mixed_budget > 0 and (self.partial or self.waiting):
                    chunks = self._prefill_chunks(
                        max(0, min(cfg.mixed_budget, cfg.max_prefill_tokens) - len(decode)))
                    if chunks:
                        return StepPlan("mixed", chunks, decode)
                return StepPlan("decode", [], decode)
        # mixed steps only for a TRICKLE of prefill work -- a backlog that fits
        # one mixed step (open-loop arrivals while others decode): decoders keep
        # streaming, the new prompt starts at once.  A burst (a closed-loop wave:
        # hundreds of prompts at once) is prefilled by full prefill-first steps
        # on the fused prefill path, which is faster in aggregate.
        if cfg.mixed_budget > 0 and self.running and (self.partial or self.waiting) and (
                cfg.mixed_backlog <= 0 or self.backlog_tokens() <= cfg.mixed_backlog):
            decode = self._decode_rows()
            # the decode rows count against the budget: a full mixed step is exactly
            # mixed_budget tokens, the GEMM shape the prefill GEMMs were tuned for
            chunks = self._prefill_chunks(
                max(0, min(cfg.mixed_budget, cfg.max_prefill_tokens) - len(decode)))
            if chunks and decode:
                return StepPlan("mixed", chunks, decode)
            if chunks:
                return StepPlan("prefill", chunks, [])
            return StepPlan("decode", [], decode) if decode else StepPlan("idle", [], [])
        chunks = self._prefill_chunks(cfg.max_prefill_tokens)
        if chunks:
            return StepPlan("prefill", chunks, [])
        if self.running:
            decode = self._decode_rows()  # may cap the last sequence at pool capacity
            if decode:
                return StepPlan("decode", [], decode)
        return StepPlan("idle", [], [])

    def _prefill_chunks(self, budget: int) -> list:
        cfg = self.cfg
        chunks: list[tuple[Sequence, int]] = []
        # continue chunked prompts first
        for s in list(self.partial):
            n = min(s.num_uncached, cfg.prefill_chunk, budget)
            if n <= 0:
                break
            try:
                self._ensure_blocks(s, s.num_cached + n)
            except OutOfBlocks:
                break
            chunks.append((s, n))
            budget -= n
        while self.waiting and budget > 0 and (self.num_active + len(
                [c for c in chunks if c[0] not in self.partial])) < cfg.max_batch:
            s = self.waiting[0]
            if s.num_cached == 0 and not s.blocks:
                self._admit(s)
            if self._cp_eligible(s):
                break  # the next lockstep step prefills it context-parallel
            n = min(s.num_uncached, cfg.prefill_chunk, budget)
            try:
                self._ensure_blocks(s, s.num_cached + n + (1 if n == s.num_uncached else 0))
            except OutOfBlocks:
                if not chunks and not self.running:
                    # nothing else can free memory: fail the request
                    self.waiting.popleft()
                    self._free(s, retain=False)
                    s.status = SeqStatus.FINISHED
                    s.finish_reason = FinishReason.ERROR
                    if s.on_finish:
                        s.on_finish(s)
                    continue
                break
            self.waiting.popleft()
            s.status = SeqStatus.RUNNING
            chunks.append((s, n))
            budget -= n
            if n < s.num_uncached:
                self.partial.append(s)
        return chunks

    def _decode_rows(self) -> list:
        # every running seq needs a slot for its next token
        for s in list(self.running):
            # a sequence preempted earlier in this pass holds no pages and
            # must not allocate any (that would cascade preemptions)
            if s not in self.running:
                continue
            while True:
                try:
                    self._ensure_blocks(s, s.length)
                    break
                except OutOfBlocks:
                    if not self._preempt_one(protect=s):
                        if self.on_capped is None:
                            raise
                        # nothing left to preempt: the KV pool is this sequence's
                        # context limit -- finish it ("length") instead of faulting
                        self.finish(s, FinishReason.LENGTH)
                        self.on_capped(s)
                        break
        return list(self.running)

    # ------------------------------------------------------------ results
    def on_prefill_done(self, chunks, sampled: dict[int, int]) -> list[tuple[Sequence, int]]:
        """Advance cached counters; returns (seq, token) for completed prompts."""
        out = []
        for s, n in chunks:
            s.num_cached += n
            self._publish(s)
            if s.num_cached >= s.length:
                if s in self.partial:
                    self.partial.remove(s)
                if s not in self.running:
                    self.running.append(s)
                tok = sampled.get(s.seq_id)
                if tok is not None:
                    out.append((s, tok))
        return out

    def on_decode_done(self, seqs: list[Sequence], toks: list[int]) -> list[tuple[Sequence, int]]:
        for s in seqs:
            s.num_cached = s.length  # the fed token's KV is now cached
        return list(zip(seqs, toks))

    def finish(self, s: Sequence, reason: FinishReason) -> None:
        s.status = SeqStatus.FINISHED
        s.finish_reason = reason
        s.finish_time = time.perf_counter()
        if s in self.running:
            self.running.remove(s)
        if s in self.partial:
            self.partial.remove(s)
        self._free(s, retain=reason != FinishReason.ERROR)
