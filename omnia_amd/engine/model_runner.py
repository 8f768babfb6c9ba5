"""Turns scheduled sequences into device batches, runs the model and the fused
sampler, and replays hipGraph-captured decode steps.

Decode graphs are captured lazily per (batch bucket, context bucket); the
context bucket fixes the split-K grid of the paged-attention kernel.  All
per-step host->device metadata goes through ONE pinned staging buffer and one
async copy.  Only sampled token ids come back to the host.
"""
from __future__ import annotations

import bisect
import os
import time

import numpy as np
import torch

from .. import ops
from ..models.llama import ForwardBatch, KVCache
from .sequence import Sequence

BATCH_BUCKETS = [1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384,
                 448, 512, 640, 768, 896, 1024]


class _Staging:
    """Packed pinned host buffer + device twin with typed section views."""

    def __init__(self, spec: dict, device, pin: bool, dev=None):
        self.event = None
        self.nev = None
        self._dsrc = None
        self.off = {}
        o = 0
        for name, (dtype, n) in spec.items():
            o = (o + 63) // 64 * 64
            self.off[name] = (o, dtype, n)
            o += n * torch.tensor([], dtype=dtype).element_size()
        self.nbytes = (o + 63) // 64 * 64
        self.host = torch.zeros(self.nbytes, dtype=torch.uint8, pin_memory=pin)
        self.dev = torch.zeros(self.nbytes, dtype=torch.uint8, device=device) if dev is None \
            else dev
        self.h = {}
        self.d = {}
        for name, (o, dtype, n) in self.off.items():
            es = torch.tensor([], dtype=dtype).element_size()
            self.h[name] = self.host[o:o + n * es].view(dtype)
            self.d[name] = self.dev[o:o + n * es].view(dtype)
        self.np = {k: v.numpy() for k, v in self.h.items()}
        nrows = spec["ids"][1]
        self.row_seq: list = [None] * nrows  # sequence whose data each row holds
        self.row_nb = [0] * nrows  # block-table entries already written for it

    def device_src(self) -> int:
        """Device-visible address of the pinned host buffer (0: not mapped)."""
        if self._dsrc is None:
            self._dsrc = ops.kernels().host_device_ptr(self.host) if self.host.is_pinned() \
                else 0
        return self._dsrc

    def native_event(self):
        if self.nev is None:
            self.nev = _NativeEvent(ops.kernels())
        return self.nev

    def upload(self, nbytes: int | None = None):
        n = self.nbytes if nbytes is None else nbytes
        self.dev[:n].copy_(self.host[:n], non_blocking=True)


class _NativeEvent:
    """Reusable hipEvent (timing disabled) driven through the kernel extension;
    ``synchronize`` only drops the GIL when the event has not completed yet."""

    __slots__ = ("k", "h")

    def __init__(self, k):
        self.k = k
        self.h = k.event_create()

    def synchronize(self) -> int:
        """Wait; returns ns spent re-taking the GIL after the event fired."""
        return self.k.event_sync(self.h)

    def query(self) -> bool:
        return self.k.event_query(self.h)


class ModelRunner:
    # single-call native step launch; TP rank 0 broadcasts the uploaded staging
    # buffer between the H2D copy and the replay, so it keeps the split path
    fused_launch = True
    # decode-step inputs uploaded by a compute-queue kernel reading the mapped
    # pinned staging buffer (ops/csrc/staging.hip) rather than an SDMA copy
    stage_kernel = os.environ.get("OMNIA_STAGE_KERNEL", "1") != "0"
    def __init__(self, model, kv: KVCache, max_batch: int = 256, max_model_len: int = 8192,
                 use_graphs: bool = True, max_prefill_tokens: int = 16384):
        self.model = model
        self.kv = kv
        self.device = model.device
        self.is_gpu = self.device.type == "cuda"
        # OMNIA_SIM_GRAPHS=1 (CPU tests only): the pipelined engine loop on the CPU
        # -- "graphs" replay the decode body eagerly and events are no-ops -- so
        # its scheduling / staging / hand-off logic runs where a bad index raises
        # instead of faulting a GPU
        self.sim = not self.is_gpu and os.environ.get("OMNIA_SIM_GRAPHS") == "1"
        # OMNIA_EAGER_GRAPHS=1 (GPU debugging): "graph replays" run the captured
        # decode body eagerly -- same kernels, same buffers -- so under
        # AMD_SERIALIZE_KERNEL=3 a faulting launch raises at its own Python line
        self.eager_graphs = self.is_gpu and os.environ.get("OMNIA_EAGER_GRAPHS") == "1"
        self.bs = kv.block_size
        self.max_model_len = max_model_len
        self.max_blocks = (max_model_len + self.bs - 1) // self.bs
        self.max_batch = max_batch
        self.max_prefill_tokens = max_prefill_tokens
        self.vocab = model.cfg.vocab_size
        self.use_graphs = use_graphs and (self.is_gpu or self.sim)
        self.buckets = [b for b in BATCH_BUCKETS if b < max_batch] + [max_batch]
        pin = self.is_gpu
        B, MB = max_batch, self.max_blocks
        spec = {
            "ids": (torch.int32, B), "src": (torch.int64, B), "pos": (torch.int32, B),
            "slots": (torch.int64, B), "seq_lens": (torch.int32, B),
            "temp": (torch.float32, B), "top_k": (torch.int32, B),
            "top_p": (torch.float32, B), "seeds": (torch.int64, B), "steps": (torch.int64, B),
            "dst": (torch.int64, B), "bt": (torch.int32, B * MB),
        }
        # double-buffered pinned host staging (step N+1 is prepared while N runs);
        # both halves upload into ONE device twin that the captured graphs read.
        self.dec = _Staging(spec, self.device, pin)
        self.stage = [self.dec, _Staging(spec, self.device, pin, dev=self.dec.dev)]
        self.flip = 0
        self.logits_idx = torch.arange(B, dtype=torch.int64, device=self.device)
        self.out_tok = torch.zeros(B, dtype=torch.int32, device=self.device)
        # device token slots: every sampled token (decode, prefill, mixed step) is
        # also scattered to its sequence's persistent slot, and every step gathers
        # its not-yet-collected input tokens from there -- so a step never waits
        # for the previous one's tokens to reach the host, whatever the step kinds.
        # Slot 0 takes the padded rows' writes.
        self.n_slots = 2 * B + 8
        self.tok_slots = torch.zeros(self.n_slots, dtype=torch.int32, device=self.device)
        self.slot_owner: list = [None] * self.n_slots
        self.free_slots = list(range(self.n_slots - 1, 0, -1))
        self._launch_no = 0
        self.out_hosts = [torch.zeros(B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        # prefill steps are pipelined too: two pinned token buffers + their events
        self.pf_hosts = [torch.zeros(B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.pf_events = [None, None]
        self.pf_flip = 0
        self.graphs: dict = {}
        self.graph_exec: dict = {}  # (rows, cols) -> raw hipGraphExec_t for the fused launch
        self.graph_pool = None
        self.stats = {"graph_replays": 0, "eager_decodes": 0, "prefill_steps": 0,
                      "captures": 0, "capture_s": 0.0,
                      "gil_wait_s": 0.0}
        # correctness tap (tests): fp32 copies of every sampled logits row
        self.logit_tap: list | None = None
        self._tap = None
        self._prefill_host = None  # last packed prefill upload (host), for TP workers
        if os.environ.get("OMNIA_LOGIT_TAP") == "1":  # every TP rank (same collectives)
            self.enable_logit_tap()

    def enable_logit_tap(self):
        """Record ``(seq_ids, fp32 logits rows)`` for every step, for whole-model
        correctness checks against ``ops.reference.dense_forward``.  The decode
        graphs capture one extra copy into a tap buffer, so they are re-captured;
        each pipelined launch snapshots it behind its graph.  Under pipelined
        decode a sequence may run one speculative step past its finish (its token
        is dropped): its trailing extra row is recorded too."""
        self.logit_tap = []
        self._tap = torch.zeros(self.max_batch, self.vocab, dtype=torch.float32,
                                device=self.device)
        self.graphs.clear()
        self.graph_exec.clear()

    def _tap_rows(self, seqs, rows):
        if self.logit_tap is not None:
            self.logit_tap.append(([s.seq_id for s in seqs], rows.float().cpu()))

    # ------------------------------------------------------------------ utils
    def _ctx_bucket(self, max_len: int) -> int:
        """Number of block-table columns (a power-of-two context bucket)."""
        nb = (max_len + self.bs - 1) // self.bs
        c = 1024 // self.bs
        while c < nb:
            c *= 2
        return min(c, self.max_blocks)

    def _penalty_counts(self, seqs: list[Sequence], rows: int):
        if not any(s.params.needs_penalties for s in seqs):
            return None
        counts = torch.zeros(rows, self.vocab, dtype=torch.int32, device=self.device)
        r, t = [], []
        for i, s in enumerate(seqs):
            if s.params.needs_penalties:
                r.extend([i] * len(s.output))
                t.extend(s.output)
        if r:
            counts.index_put_((torch.tensor(r, device=self.device),
                               torch.tensor(t, device=self.device)),
                              torch.ones(len(r), dtype=torch.int32, device=self.device),
                              accumulate=True)
        pen = {
            "freq": torch.tensor([s.params.frequency_penalty for s in seqs], device=self.device),
            "pres": torch.tensor([s.params.presence_penalty for s in seqs], device=self.device),
            "rep": torch.tensor([s.params.repetition_penalty for s in seqs], device=self.device),
        }
        return counts, pen

    # ------------------------------------------------------------------ prefill
    def run_prefill(self, chunks: list[tuple[Sequence, int]]) -> dict[int, int]:
        """chunks: (seq, n_new) -- prefill n_new uncached tokens of each seq.

        Returns {seq_id: sampled token} for sequences whose prompt completed."""
        if self.can_pipeline_prefill(chunks):
            h = self.launch_prefill(chunks)
            return {s.seq_id: t for s, t in zip(h.seqs, self.collect(h))}
        t, meta, sample_seqs = self._prefill_pack(chunks)
        logits = self._prefill_forward(t, meta)
        self.stats["prefill_steps"] += 1
        if not sample_seqs:
            return {}
        self._tap_rows(sample_seqs, logits[: len(sample_seqs)])
        toks = self._sample_eager(logits[: len(sample_seqs)], sample_seqs)
        return {s.seq_id: t for s, t in zip(sample_seqs, toks)}

    @property
    def device_handoff(self) -> bool:
        """Steps feed not-yet-collected tokens from the device token slots (single
        rank; TP workers keep the host hand-off for prefill-sampled tokens)."""
        return (self.is_gpu or self.sim) and self.model.tp == 1

    def _event(self):
        """A recorded stream event (a no-op stand-in in the CPU simulation)."""
        ev = torch.cuda.Event() if self.is_gpu else _SimEvent()
        ev.record()
        return ev

    def can_pipeline_prefill(self, chunks) -> bool:
        return (self.is_gpu or self.sim) and not any(s.params.needs_penalties or s.guide is not None
                                       for s, _ in chunks)

    def launch_prefill(self, chunks: list[tuple[Sequence, int]]) -> "DecodeHandle":
        """Enqueue one prefill step + on-device sampling of the completed prompts and
        the D2H copy of their tokens; returns without waiting.  The sampling
        parameters travel in the same packed upload as the batch metadata, so the
        step issues no synchronous copies and the host can assemble step N+1 while
        the GPU runs step N."""
        t, meta, sample_seqs = self._prefill_pack(chunks, sampling=True)
        tp = self.model.tp > 1
        logits = self._prefill_forward(t, meta, gather=not tp)
        self.stats["prefill_steps"] += 1
        n = len(sample_seqs)
        slot = self.pf_flip
        self.pf_flip ^= 1
        out_host = self.pf_hosts[slot]
        ev = self.pf_events[slot]
        if ev is not None:
            ev.synchronize()  # the pinned token buffer of step N-2 has been read
        if n:
            if tp:
                tok = self._prefill_tp_sample(t, meta, logits, sample_seqs)
            else:
                self._tap_rows(sample_seqs, logits[:n])
                temp, top_k, top_p, seeds, steps = self._prefill_sampling(t, meta)
                tok = ops.sample(logits[:n], temp, top_k, top_p, seeds=seeds, steps=steps)
            if self.device_handoff:  # the next step may feed these tokens on the GPU
                o = meta[5] + 5 * n
                self.tok_slots.index_copy_(0, t[o:o + n], tok.to(torch.int32))
            out_host[:n].copy_(tok, non_blocking=True)
        ev = self._event()
        self.pf_events[slot] = ev
        return DecodeHandle(sample_seqs, out_host, ev, n, "prefill")

    @staticmethod
    def _prefill_sampling(t, meta):
        """(temperature, top_k, top_p, seeds=, steps=) of the sampled rows, sliced
        from the packed prefill upload."""
        n, o = meta[4], meta[5]
        return (t[o:o + n].view(torch.float64).float(), t[o + n:o + 2 * n].int(),
                t[o + 2 * n:o + 3 * n].view(torch.float64).float(),
                t[o + 3 * n:o + 4 * n], t[o + 4 * n:o + 5 * n])

    def _prefill_tp_sample(self, t, meta, local_logits, seqs=None):
        """TP: the distributed sampler (every rank runs it: it is a collective).
        With the logit tap on, every rank first all-gathers the vocab slices
        (rank 0 records the full rows)."""
        from ..parallel import state as pstate
        from ..parallel.tp_sampling import tp_sample

        n = meta[4]
        if self._tap is not None:
            full = pstate.tp_all_gather_lastdim(local_logits[:n].contiguous())
            if seqs is not None:
                self._tap_rows(seqs, full)
        temp, top_k, top_p, seeds, steps = self._prefill_sampling(t, meta)
        return tp_sample(local_logits[:n], self.model.vocab_start, temp, top_k, top_p,
                         seeds=seeds, steps=steps, group=pstate.get_state().tp_group)

    def _prefill_pack(self, chunks, sampling: bool = False):
        """Host-side batch assembly -> (packed int64 device tensor, meta, sampled seqs).
        meta = (T, B, maxb, n_tiles, n_sample[, sampling-params offset])."""
        bs = self.bs
        B = len(chunks)
        lens = np.fromiter((n for _, n in chunks), np.int64, B)
        qsl = np.zeros(B + 1, np.int64)
        np.cumsum(lens, out=qsl[1:])
        T = int(qsl[-1])
        maxb = max(1, max(len(s.blocks) for s, _ in chunks))
        ids = np.empty(T, np.int64)
        pos = np.empty(T, np.int64)
        bt = np.zeros((B, maxb), dtype=np.int64)
        seq_lens = np.empty(B, np.int64)
        sample_rows, sample_seqs = [], []
        for i, (s, n) in enumerate(chunks):
            start = s.num_cached
            q0 = int(qsl[i])
            plen = len(s.prompt)
            if start + n <= plen:
                ids[q0:q0 + n] = s.prompt[start:start + n]
            else:
                ids[q0:q0 + n] = s.all_tokens[start:start + n]
            pos[q0:q0 + n] = np.arange(start, start + n)
            bt[i, :len(s.blocks)] = s.blocks
            seq_lens[i] = start + n
            if start + n == s.length:
                sample_rows.append(q0 + n - 1)
                sample_seqs.append(s)
        # slot of token p of row i = block_table[i][p // bs] * bs + p % bs
        row = np.repeat(np.arange(B), lens)
        slots = bt[row, pos // bs] * bs + pos % bs
        tseq, tq0 = ops.prefill_tiles(lens.tolist())
        parts = [ids, pos, slots, qsl, seq_lens, np.asarray(tseq, np.int64),
                 np.asarray(tq0, np.int64), np.asarray(sample_rows or [0], np.int64),
                 bt.reshape(-1)]
        meta = (T, B, maxb, len(tseq), len(sample_rows))
        if sampling and sample_seqs:
            meta = meta + (sum(len(x) for x in parts),)
            ps = [x.params for x in sample_seqs]
            parts += [np.array([p.temperature for p in ps], np.float64).view(np.int64),
                      np.array([p.top_k for p in ps], np.int64),
                      np.array([p.top_p for p in ps], np.float64).view(np.int64),
                      np.array([p.seed if p.seed is not None else x.seq_id * 7919 + 17
                                for p, x in zip(ps, sample_seqs)], np.int64),
                      np.array([len(x.output) for x in sample_seqs], np.int64)]
            self._launch_no += 1
            parts.append(np.array([self.assign_slot(x) for x in sample_seqs], np.int64))
        t = torch.from_numpy(np.concatenate(parts))
        self._prefill_host = t
        if self.is_gpu:
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t, meta, sample_seqs

    def _prefill_forward(self, t: torch.Tensor, meta, gather: bool = True) -> torch.Tensor:
        T, B, maxb, n_tiles, n_sample = meta[:5]
        o = 0

        def take(n, dtype):
            nonlocal o
            v = t[o:o + n]
            o += n
            return v.to(dtype)

        fb = ForwardBatch(
            input_ids=take(T, torch.int32), positions=take(T, torch.int32),
            slots=take(T, torch.int64), block_tables=None, seq_lens=None, logits_indices=None,
            is_decode=False, num_seqs=B)
        fb.q_start_loc = take(B + 1, torch.int32)
        fb.seq_lens = take(B, torch.int32)
        fb.tile_seq = take(n_tiles, torch.int32)
        fb.tile_q0 = take(n_tiles, torch.int32)
        fb.logits_indices = take(max(1, n_sample), torch.int64)
        fb.block_tables = take(B * maxb, torch.int32).view(B, maxb)
        return self.model.forward(fb, self.kv, gather)

    # ------------------------------------------------------------------ mixed
    def _mixed_forward(self, dseqs: list[Sequence], chunks: list[tuple[Sequence, int]],
                       launch: bool = False):
        """Pack + upload + forward of one mixed step: the running sequences' next
        tokens (decode rows, first) and prefill chunks.  ``launch``: decode rows
        whose input token is still on the device gather it from their token slot,
        and the sampling parameters + destination slots of every sampled row ride
        in the same upload.  Returns (logits, sampled seqs, packed device tensor,
        offset of the sampling tail)."""
        bs = self.bs
        Bd, B = len(dseqs), len(chunks)
        lens = np.fromiter((n for _, n in chunks), np.int64, B)
        qsl = np.zeros(B + 1, np.int64)
        np.cumsum(lens, out=qsl[1:])
        Tp = int(qsl[-1])
        T = Bd + Tp
        ids = np.empty(T, np.int64)
        pos = np.empty(T, np.int64)
        slots = np.empty(T, np.int64)
        src = np.full(Bd, -1, np.int64)
        mbd = self._ctx_bucket(max(s.length for s in dseqs))
        dbt = np.zeros((Bd, mbd), np.int64)
        dlen = np.empty(Bd, np.int64)
        for i, s in enumerate(dseqs):
            p = s.length - 1
            last = s.output[-1] if s.output else s.prompt[-1]
            if last == PLACEHOLDER:
                if not launch:
                    raise RuntimeError("synchronous mixed step with a token in flight")
                src[i] = s.slot
                ids[i] = 0
            else:
                ids[i] = last
            pos[i] = p
            slots[i] = s.blocks[p // bs] * bs + p % bs
            dbt[i, :len(s.blocks)] = s.blocks
            dlen[i] = p + 1
        maxb = max(1, max(len(s.blocks) for s, _ in chunks))
        bt = np.zeros((B, maxb), np.int64)
        seq_lens = np.empty(B, np.int64)
        sample_rows, sample_seqs = list(range(Bd)), list(dseqs)
        for i, (s, n) in enumerate(chunks):
            start, q0 = s.num_cached, Bd + int(qsl[i])
            src_t = s.prompt if start + n <= len(s.prompt) else s.all_tokens
            ids[q0:q0 + n] = src_t[start:start + n]
            pos[q0:q0 + n] = np.arange(start, start + n)
            bt[i, :len(s.blocks)] = s.blocks
            seq_lens[i] = start + n
            blk = bt[i][pos[q0:q0 + n] // bs]
            slots[q0:q0 + n] = blk * bs + pos[q0:q0 + n] % bs
            if start + n == s.length:
                sample_rows.append(q0 + n - 1)
                sample_seqs.append(s)
        tseq, tq0 = ops.prefill_tiles(lens.tolist())
        parts = [ids, pos, slots, qsl, seq_lens, np.asarray(tseq, np.int64),
                 np.asarray(tq0, np.int64), np.asarray(sample_rows, np.int64), bt.reshape(-1),
                 dbt.reshape(-1), dlen]
        tail = None
        if launch:
            parts.append(src)
            tail = sum(len(x) for x in parts)
            ps = [x.params for x in sample_seqs]
            self._launch_no += 1
            parts += [np.array([p.temperature for p in ps], np.float64).view(np.int64),
                      np.array([p.top_k for p in ps], np.int64),
                      np.array([p.top_p for p in ps], np.float64).view(np.int64),
                      np.array([p.seed if p.seed is not None else x.seq_id * 7919 + 17
                                for p, x in zip(ps, sample_seqs)], np.int64),
                      np.array([len(x.output) for x in sample_seqs], np.int64),
                      np.array([self.assign_slot(x) for x in sample_seqs], np.int64)]
        host = torch.from_numpy(np.concatenate(parts))
        # T, B, Bd, maxb, mbd, tiles, n_sample, launch
        meta = (T, B, Bd, maxb, mbd, len(tseq), len(sample_rows), int(launch))
        t = host.pin_memory().to(self.device, non_blocking=True) if self.is_gpu else host
        logits = self._mixed_forward_packed(t, meta, host)
        return logits, sample_seqs, t, tail

    def _mixed_forward_packed(self, t: torch.Tensor, meta, host=None) -> torch.Tensor:
        """Forward of a packed mixed upload (``meta`` = T, B, Bd, maxb, mbd,
        tiles, n_sample, launch) -- the part TP workers replay (``engine/tp.py``
        MIXED).  ``host``: the upload on the host (TP rank 0 publishes it)."""
        T, B, Bd, maxb, mbd, ntiles, nsample, launch = meta
        o = 0

        def take(n, dtype):
            nonlocal o
            v = t[o:o + n]
            o += n
            return v.to(dtype)

        fb = ForwardBatch(input_ids=take(T, torch.int32), positions=take(T, torch.int32),
                          slots=take(T, torch.int64), block_tables=None, seq_lens=None,
                          logits_indices=None, is_decode=False, num_seqs=B)
        fb.q_start_loc = take(B + 1, torch.int32)
        fb.seq_lens = take(B, torch.int32)
        fb.tile_seq = take(ntiles, torch.int32)
        fb.tile_q0 = take(ntiles, torch.int32)
        fb.logits_indices = take(nsample, torch.int64)
        fb.block_tables = take(B * maxb, torch.int32).view(B, maxb)
        fb.dec_block_tables = take(Bd * mbd, torch.int32).view(Bd, mbd)
        fb.dec_seq_lens = take(Bd, torch.int32)
        fb.num_decode = Bd
        if launch and Bd:
            dsrc = t[o:o + Bd]
            ids_d = fb.input_ids[:Bd]
            ids_d.copy_(torch.where(dsrc >= 0, self.tok_slots.index_select(0, dsrc.clamp(min=0)),
                                    ids_d))
        logits = self.model.forward(fb, self.kv)
        self.stats["mixed_steps"] = self.stats.get("mixed_steps", 0) + 1
        return logits

    def run_mixed(self, dseqs: list[Sequence], chunks: list[tuple[Sequence, int]]
                  ) -> tuple[list[int], dict[int, int]]:
        """One synchronous mixed step (eager sampling: penalties, grammars).
        Returns (tokens of ``dseqs``, {seq_id: token} of the prompts this step
        completed)."""
        Bd = len(dseqs)
        logits, sample_seqs, _, _ = self._mixed_forward(dseqs, chunks)
        self._tap_rows(sample_seqs, logits)
        toks = self._sample_eager(logits, sample_seqs)
        return toks[:Bd], {s.seq_id: tk for s, tk in zip(sample_seqs[Bd:], toks[Bd:])}

    def can_pipeline_mixed(self, dseqs, chunks) -> bool:
        return (self.device_handoff and self.can_pipeline(dseqs)
                and self.can_pipeline_prefill(chunks))

    def launch_mixed(self, dseqs: list[Sequence], chunks: list[tuple[Sequence, int]]
                     ) -> "DecodeHandle":
        """Enqueue one mixed step with on-device sampling, the tokens scattered to
        the sampled sequences' slots and copied to a pinned buffer; returns
        without waiting (the handle's seqs = decode rows then completed prompts)."""
        logits, sample_seqs, t, o = self._mixed_forward(dseqs, chunks, launch=True)
        n = len(sample_seqs)
        temp = t[o:o + n].view(torch.float64).float()
        top_k = t[o + n:o + 2 * n].int()
        top_p = t[o + 2 * n:o + 3 * n].view(torch.float64).float()
        tok = ops.sample(logits[:n], temp, top_k, top_p, seeds=t[o + 3 * n:o + 4 * n],
                         steps=t[o + 4 * n:o + 5 * n])
        self.tok_slots.index_copy_(0, t[o + 5 * n:o + 6 * n], tok)
        slot = self.pf_flip
        self.pf_flip ^= 1
        out_host = self.pf_hosts[slot]
        ev = self.pf_events[slot]
        if ev is not None:
            ev.synchronize()  # the pinned token buffer of step N-2 has been read
        if n > out_host.numel():
            self.pf_hosts[slot] = out_host = torch.zeros(
                max(n, 2 * out_host.numel()), dtype=torch.int32, pin_memory=True)
        out_host[:n].copy_(tok, non_blocking=True)
        ev = self._event()
        self.pf_events[slot] = ev
        h = DecodeHandle(sample_seqs, out_host, ev, n, "mixed")
        if self.logit_tap is not None:
            # snapshot now, recorded at collect: the pipelined loop collects the
            # previous step after this launch, and a sequence's rows must stay in order
            h.tap = logits[:n].clone()
        return h

    def _sample_eager(self, logits, seqs: list[Sequence]) -> list[int]:
        n = len(seqs)
        dev = self.device
        temp = torch.tensor([s.params.temperature for s in seqs], dtype=torch.float32, device=dev)
        top_k = torch.tensor([s.params.top_k for s in seqs], dtype=torch.int32, device=dev)
        top_p = torch.tensor([s.params.top_p for s in seqs], dtype=torch.float32, device=dev)
        seeds = torch.tensor([s.params.seed if s.params.seed is not None else s.seq_id * 7919 + 17
                              for s in seqs], dtype=torch.int64, device=dev)
        steps = torch.tensor([len(s.output) for s in seqs], dtype=torch.int64, device=dev)
        pc = self._penalty_counts(seqs, n)
        kw = {}
        if pc is not None:
            kw = dict(counts=pc[0], freq_pen=pc[1]["freq"], pres_pen=pc[1]["pres"],
                      rep_pen=pc[1]["rep"])
        if any(s.guide is not None for s in seqs):
            from .guided import masks_for

            words = (logits.shape[1] + 31) // 32
            m = torch.from_numpy(masks_for([s.guide for s in seqs], words))
            if self.is_gpu:
                m = m.pin_memory().to(dev, non_blocking=True)
            logits = logits[:n]
            if not logits.is_contiguous() and logits.stride(1) != 1:
                logits = logits.contiguous()
            ops.apply_token_mask(logits, m)
        tok = ops.sample(logits, temp, top_k, top_p, seeds=seeds, steps=steps, **kw)
        return tok.cpu().tolist()

    # ------------------------------------------------------------------ slots
    def assign_slot(self, s: Sequence) -> int:
        """The persistent device token slot of ``s`` (allocated on first use)."""
        sl = s.slot
        if sl > 0 and self.slot_owner[sl] is s:
            s.slot_launch = self._launch_no
            return sl
        if not self.free_slots:
            self._reclaim_slots()
        sl = self.free_slots.pop()
        self.slot_owner[sl] = s
        s.slot = sl
        s.slot_launch = self._launch_no
        return sl

    def _reclaim_slots(self):
        """Slot table full (preempted sequences keep theirs): take back slots whose
        owner has no token in flight and is not part of the launch being built."""
        for sl in range(1, self.n_slots):
            o = self.slot_owner[sl]
            if o is None or o.is_finished or (o.n_real == len(o.output) and
                                              getattr(o, "slot_launch", -1) != self._launch_no):
                if o is not None:
                    o.slot = -1
                self.slot_owner[sl] = None
                self.free_slots.append(sl)
        if not self.free_slots:
            raise RuntimeError("device token slots exhausted")

    def release_slot(self, s: Sequence) -> None:
        sl = s.slot
        if sl > 0 and self.slot_owner[sl] is s:
            self.slot_owner[sl] = None
            self.free_slots.append(sl)
        s.slot = -1

    # ------------------------------------------------------------------ decode
    def _decode_inputs(self, seqs: list[Sequence], nrows: int, ncols: int, st: "_Staging",
                       upload: bool = True):
        """Fill a host staging buffer for one decode step.  Each buffer remembers
        which sequence occupied each row and how many block-table entries it
        already holds, so steady-state steps only write what changed (positions,
        slots, steps and newly allocated pages)."""
        n = len(seqs)
        npv = st.np
        ids, pos, slots, lens, src = npv["ids"], npv["pos"], npv["slots"], npv["seq_lens"], \
            npv["src"]
        steps, dst = npv["steps"], npv["dst"]
        bt = npv["bt"].reshape(self.max_batch, self.max_blocks)
        row_seq, row_nb = st.row_seq, st.row_nb
        bs = self.bs
        self._launch_no += 1
        for i, s in enumerate(seqs):
            p = s.length - 1
            last = s.output[-1] if s.output else s.prompt[-1]
            dst[i] = self.assign_slot(s)
            if last == PLACEHOLDER:
                # token still on the device: gather it from the sequence's token slot
                src[i] = s.slot
                ids[i] = 0
            else:
                src[i] = -1
                ids[i] = last
            pos[i] = p
            blocks = s.blocks
            slots[i] = blocks[p // bs] * bs + p % bs
            lens[i] = p + 1
            nb = len(blocks)
            had = row_nb[i]
            # same sequence in the same row with an unchanged block prefix (pages
            # are only ever appended while a sequence runs; preemption / swap
            # re-allocate them, which the endpoint check catches)
            if row_seq[i] is s and 0 < had <= nb and bt[i, 0] == blocks[0] and \
                    bt[i, had - 1] == blocks[had - 1]:
                if nb > had:
                    bt[i, had:nb] = blocks[had:nb]
                    row_nb[i] = nb
            else:
                bt[i, :nb] = blocks
                row_seq[i] = s
                row_nb[i] = nb
                self._fill_row_sampling(npv, i, s)
            steps[i] = len(s.output)
        dst[n:nrows] = 0
        for i in range(n, nrows):  # padded rows -> null page, no KV write
            if row_seq[i] is not _PAD:
                ids[i] = 0
                src[i] = -1
                pos[i] = 0
                slots[i] = -1
                lens[i] = 1
                bt[i, 0] = 0
                npv["temp"][i] = 0.0
                npv["top_k"][i] = 0
                npv["top_p"][i] = 1.0
                row_seq[i] = _PAD
                row_nb[i] = 0
        # upload into the (single) device twin the graphs read from
        if upload:
            self.dec.dev.copy_(st.host, non_blocking=True)

    @staticmethod
    def _fill_row_sampling(npv, i: int, s: Sequence):
        p = s.params
        npv["temp"][i] = p.temperature
        npv["top_k"][i] = p.top_k
        npv["top_p"][i] = p.top_p
        npv["seeds"][i] = p.seed if p.seed is not None else (s.seq_id * 7919 + 17)

    def _decode_fb(self, nrows: int, ncols: int, ids=None) -> ForwardBatch:
        d = self.dec.d
        return ForwardBatch(
            input_ids=d["ids"][:nrows] if ids is None else ids, positions=d["pos"][:nrows],
            slots=d["slots"][:nrows],
            block_tables=d["bt"].view(self.max_batch, self.max_blocks)[:nrows, :ncols],
            seq_lens=d["seq_lens"][:nrows], logits_indices=self.logits_idx[:nrows],
            is_decode=True, num_seqs=nrows)

    def _decode_body(self, nrows: int, ncols: int):
        d = self.dec.d
        fb = self._decode_fb(nrows, ncols)
        # tokens sampled by earlier steps stay on the GPU (async scheduling): the
        # embedding kernel reads them from their slots (no framework op in the graph)
        fb.ids_src, fb.tok_slots = d["src"][:nrows], self.tok_slots
        if self.model.tp > 1:
            # vocab-parallel LM head + distributed sampler: no full-vocab gather
            from ..parallel import state as pstate
            from ..parallel.tp_sampling import tp_sample, tp_sample_device

            local = self.model.forward(fb, self.kv, gather=False)
            if self._tap is not None:  # correctness tap: full rows (a collective)
                self._tap[:nrows].copy_(pstate.tp_all_gather_lastdim(local))
            args = (local, self.model.vocab_start, d["temp"][:nrows], d["top_k"][:nrows],
                    d["top_p"][:nrows])
            kw = dict(seeds=d["seeds"][:nrows], steps=d["steps"][:nrows],
                      out=self.out_tok[:nrows], group=pstate.get_state().tp_group)
            if self.is_gpu and local.dtype == torch.bfloat16:
                # pack kernel -> IPC all-gather -> merge kernel, which also writes each
                # token into its sequence's device slot (no framework op in the graph)
                tp_sample_device(*args, **kw, tok_slots=self.tok_slots, dst=d["dst"][:nrows])
                return
            tp_sample(*args, **kw)
            self.tok_slots.index_copy_(0, d["dst"][:nrows], self.out_tok[:nrows])
            return
        logits = self.model.forward(fb, self.kv)
        if self._tap is not None:
            self._tap[:nrows].copy_(logits)
        # the sampler also writes each token into its sequence's device slot
        ops.sample(logits, d["temp"][:nrows], d["top_k"][:nrows], d["top_p"][:nrows],
                   seeds=d["seeds"][:nrows], steps=d["steps"][:nrows],
                   out=self.out_tok[:nrows], tok_slots=self.tok_slots, dst=d["dst"][:nrows])

    def _capture(self, nrows: int, ncols: int):
        t0 = time.perf_counter()
        if self.sim or self.eager_graphs:  # "replay" = the eager decode body
            g = _SimGraph(lambda: self._decode_body(nrows, ncols))
            self.graphs[(nrows, ncols)] = g
            self.stats["captures"] += 1
            return g
        if self.graph_pool is None:
            self.graph_pool = torch.cuda.graph_pool_handle()
            self._graph_rng_ready = False
        # warm-up/capture must not clobber live sampler outputs of an in-flight step
        saved = self.out_tok.clone()
        saved_slots = self.tok_slots.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._decode_body(nrows, ncols)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # no cyclic-GC pass inside the capture: a collection there can run the
        # deleter of a device tensor from an earlier step (a free on a capturing
        # stream), which aborts the process
        import gc

        gc_was = gc.isenabled()
        gc.disable()
        # framework compute ops / blocks outside the graph pool captured here would
        # replay stale state (engine/capture_guard.py)
        from .capture_guard import CaptureGuard

        guard = CaptureGuard(self.device, f"decode graph rows={nrows} cols={ncols}")
        if not self._graph_rng_ready:
            # PyTorch's CUDA generator allocates its graph seed / offset tensors
            # (2 x 512 B, default pool) when the first live graph registers with
            # it and frees them when the last one goes.  Register an empty graph
            # first, outside the guarded capture, and KEEP it: if it were dropped
            # (or an earlier engine's graphs were collected) the guarded capture
            # would re-allocate them -- a flaky guard violation
            self._rng_anchor = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._rng_anchor, pool=self.graph_pool):
                pass
            self._graph_rng_ready = True
        try:
            with guard.memory_scope():
                # capture on the warm-up stream: per-stream library state (hipBLASLt
                # workspace) already exists there, so nothing is allocated outside
                # the graph pool while capturing
                with torch.cuda.graph(g, pool=self.graph_pool, stream=s):
                    with guard.ops_scope():
                        self._decode_body(nrows, ncols)
        finally:
            if gc_was:
                gc.enable()
        guard.check()
        self.stats["capture_guard_violations"] = \
            self.stats.get("capture_guard_violations", 0) + len(guard.violations())
        self.stats["capture_library_gemms"] = \
            self.stats.get("capture_library_gemms", 0) + sum(guard.library.values())
        torch.cuda.synchronize()
        self.out_tok.copy_(saved)
        self.tok_slots.copy_(saved_slots)
        self.graphs[(nrows, ncols)] = g
        if self.fused_launch:
            self.graph_exec[(nrows, ncols)] = int(g.raw_cuda_graph_exec())
        self.stats["captures"] += 1
        self.stats["capture_s"] += time.perf_counter() - t0
        from ..observability import metrics as M

        M.ENGINE_COLD_START.labels("graph_warmup").set(self.stats["capture_s"])
        return g

    def can_pipeline(self, seqs: list[Sequence]) -> bool:
        # penalties need host token counts, grammars the previous token: synchronous
        return self.use_graphs and not any(s.params.needs_penalties or s.guide is not None
                                           for s in seqs)

    def launch_decode(self, seqs: list[Sequence], nrows: int | None = None,
                      ncols: int | None = None) -> "DecodeHandle":
        """Enqueue one decode step (graph replay) without waiting for it.
        ``nrows`` / ``ncols`` force a larger graph bucket (lockstep EP ranks
        replay the bucket the group agreed on)."""
        n = len(seqs)
        if n > self.max_batch:
            raise ValueError("decode batch exceeds max_batch")
        max_len = max(s.length for s in seqs)
        ncols = max(ncols or 0, self._ctx_bucket(max_len))
        nrows = max(nrows or 0, self.buckets[bisect.bisect_left(self.buckets, n)])
        st = self.stage[self.flip]
        out_host = self.out_hosts[self.flip]
        self.flip ^= 1
        if st.event is not None:
            st.event.synchronize()  # host staging buffer free again
        gx = self.graph_exec.get((nrows, ncols)) if self.fused_launch else None
        if gx is not None:
            # H2D + graph launch + D2H + event record in ONE native call: the GIL is
            # held throughout instead of being dropped/re-taken around each enqueue
            self._decode_inputs(seqs, nrows, ncols, st, upload=False)
            ev = st.native_event()
            src = st.device_src() if self.stage_kernel and ncols % 4 == 0 and \
                self.max_blocks % 4 == 0 else 0
            if src:
                # upload = compute-queue kernel over the mapped pinned buffer, only
                # the block-table window this bucket reads (no SDMA hand-off)
                bt_off = st.off["bt"][0]
                ops.kernels().graph_launch_staged(
                    gx, self.dec.dev.data_ptr(), src, bt_off, bt_off, 4 * self.max_blocks,
                    nrows, 4 * ncols, out_host.data_ptr(), self.out_tok.data_ptr(), 4 * n,
                    ev.h)
            else:
                ops.kernels().graph_launch_step(
                    gx, self.dec.dev.data_ptr(), st.host.data_ptr(), st.nbytes,
                    out_host.data_ptr(), self.out_tok.data_ptr(), 4 * n, ev.h)
            self.stats["graph_replays"] += 1
        else:
            self._decode_inputs(seqs, nrows, ncols, st)
            self._before_replay(nrows, ncols, st)
            self._replay(nrows, ncols)
            out_host[:n].copy_(self.out_tok[:n], non_blocking=True)
            ev = self._event()
        st.event = ev
        h = DecodeHandle(seqs, out_host, ev, n)
        if self._tap is not None:
            # snapshot on the same stream right behind this step's graph: the next
            # (pipelined) step overwrites the tap buffer before this one is collected
            h.tap = self._tap[:n].clone()
        return h

    def _before_replay(self, nrows: int, ncols: int, st: "_Staging | None" = None):
        """Hook: TP runners publish the step inputs (``st.host``) to their workers."""

    def _replay(self, nrows: int, ncols: int):
        g = self.graphs.get((nrows, ncols)) or self._capture(nrows, ncols)
        g.replay()
        self.stats["graph_replays"] += 1

    def collect(self, h: "DecodeHandle") -> list[int]:
        gil_ns = h.event.synchronize()
        if gil_ns:
            self.stats["gil_wait_s"] += gil_ns * 1e-9
        rows = None
        if self._tap is not None and h.kind == "decode":
            rows = h.tap if h.tap is not None else self._tap[: h.n]
        elif h.kind == "mixed" and h.tap is not None:
            rows = h.tap
        if rows is not None:
            # rows of sequences that finished while this step was in flight are
            # speculative (the engine drops their tokens): not part of the record
            keep = [i for i, s in enumerate(h.seqs) if not s.is_finished]
            self._tap_rows([h.seqs[i] for i in keep], rows[keep])
        return h.out_host[: h.n].tolist()

    def run_decode(self, seqs: list[Sequence]) -> list[int]:
        if self.can_pipeline(seqs):
            return self.collect(self.launch_decode(seqs))
        # eager path (CPU engine, penalties): real tokens only
        n = len(seqs)
        ncols = self._ctx_bucket(max(s.length for s in seqs))
        st = self.stage[0]
        self._decode_inputs(seqs, n, ncols, st)
        self._before_eager(n, ncols, st)
        logits = self._eager_forward(n, ncols)
        self._tap_rows(seqs, logits[:n])
        return self._sample_eager(logits, seqs)

    def _before_eager(self, n: int, ncols: int, st: "_Staging | None" = None):
        """Hook: TP runners publish the eager-decode inputs here."""

    def _eager_forward(self, n: int, ncols: int):
        fb = self._decode_fb(n, ncols)
        self.stats["eager_decodes"] += 1
        return self.model.forward(fb, self.kv)


PLACEHOLDER = -1
_PAD = object()  # row_seq marker of a padded (null) row


class _SimEvent:
    """No-op event of the CPU simulation (``ModelRunner.sim``)."""

    def record(self, *a):
        pass

    def synchronize(self):
        return 0

    def query(self):
        return True


class _SimGraph:
    def __init__(self, fn):
        self.fn = fn

    def replay(self):
        self.fn()


class DecodeHandle:
    __slots__ = ("seqs", "out_host", "event", "n", "kind", "tap")

    def __init__(self, seqs, out_host, event, n, kind="decode"):
        self.tap = None
        self.kind = kind
        self.seqs = seqs
        self.out_host = out_host
        self.event = event
        self.n = n
