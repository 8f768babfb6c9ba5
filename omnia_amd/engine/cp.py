"""Context-parallel prefill on the serving path (``EngineConfig.cp_threshold``).

The engine replicas of a DP group are independent (own scheduler, KV pool and
batch), except that a prompt of at least ``cp_threshold`` uncached tokens is
prefilled by the WHOLE group at once: the prompt is cut into 2W zig-zag
chunks, every rank runs the full model over its two chunks, and attention is a
ring over the group (:mod:`omnia_amd.parallel.context_parallel`, the hand
flash-prefill kernel with LSE output per ring step).  The owner writes every
K/V block that goes by into its own paged cache, gets the last position's
hidden state from whichever rank holds it, samples the first token and then
decodes the sequence alone like any other.  TTFT of a long prompt drops by up
to W x while the other ranks lose one step each.

Because a CP prefill is a collective, every rank of the group steps in
lockstep: a host shared-memory all-gather per step (no device collective)
says who (if anyone) has a CP prompt at the head of its queue; with none, each
rank runs its own ordinary step.  When the ranks share a device (the ``ipc``
transport) the ring hops run on the IPC point-to-point kernel instead of RCCL.

The reference bounds context before the remote provider call and has no
sequence parallelism at all (``api/v1alpha1/agentruntime_types.go:417-459``,
SURVEY §5.7 item 3); this is the MI355X-native long-context path.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..models.llama import ForwardBatch
from ..parallel import state as pstate
from ..parallel.context_parallel import CPPrefill
from ..parallel.hostsync import ShmAgreement


def run_cp_prefill(runner, seq, L: int, owner: int, group) -> int | None:
    """Collective prefill of one prompt of L tokens owned by group rank
    ``owner`` (``seq`` on the owner, None elsewhere).  Returns the sampled first
    token on the owner, None on the others."""
    model = runner.model
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    granks = dist.get_process_group_ranks(group)
    dev = runner.device
    is_owner = rank == owner
    cp = CPPrefill(L, world, rank, group, model.hkv, model.cfg.head_dim, runner.bs, dev,
                   model.dtype, owner=is_owner, owner_blocks=seq.blocks if is_owner else None,
                   max_position=model.cfg.max_position)
    ids = torch.zeros(cp.L_pad, dtype=torch.int64, device=dev)
    if is_owner:
        ids[:L] = torch.tensor(seq.all_tokens[:L], dtype=torch.int64)
    if world > 1:
        dist.broadcast(ids, granks[owner], group=group)
    fb = ForwardBatch(input_ids=ids.index_select(0, cp.index).to(torch.int32),
                      positions=cp.positions, slots=cp.slots, block_tables=None,
                      seq_lens=None, logits_indices=None, is_decode=False, cp=cp)
    h = model.hidden_states(fb, runner.kv)
    holder, row = cp.locate(L - 1)
    last = h[row:row + 1].contiguous() if rank == holder else torch.empty(
        1, h.shape[1], dtype=h.dtype, device=dev)
    if world > 1:
        dist.broadcast(last, granks[holder], group=group)
    runner.stats["cp_prefills"] = runner.stats.get("cp_prefills", 0) + 1
    if not is_owner:
        return None
    logits = model.logits(last)
    runner._tap_rows([seq], logits)
    return runner._sample_eager(logits, [seq])[0]


def run_cp_step(engine) -> int:
    """One lockstep step of a CP group (see module docstring)."""
    st = pstate.get_state()
    group, W, r = st.dp_group, st.dp_size, st.dp_rank
    sched = engine.scheduler
    cand = sched.cp_candidate()
    ag = getattr(engine, "_cp_agree", None)
    if ag is None:  # host shared-memory agreement (parallel/hostsync.py), built once
        ag = engine._cp_agree = ShmAgreement.for_group(group, 2)
    got = ag.gather([cand.length if cand is not None else 0, 1 if sched.has_work() else 0])
    lens, busy = [int(x) for x in got[:, 0]], int(got[:, 1].max())
    owners = [i for i, n in enumerate(lens) if n > 0]
    engine._ep_active = 1 if (owners or busy) else 0
    if not owners:
        return engine._step_sync() if sched.has_work() else 0
    owner = owners[0]
    t0 = time.perf_counter()
    tok = run_cp_prefill(engine.runner, cand if owner == r else None, lens[owner], owner, group)
    engine.counters["cp_prefills"] = engine.counters.get("cp_prefills", 0) + 1
    if owner != r:
        return 0
    done = sched.cp_done(cand, tok)
    engine.counters["prefill_tokens"] += lens[owner]
    engine.counters["steps_prefill"] += 1
    engine.timing["cp_prefill_s"] = engine.timing.get("cp_prefill_s", 0.0) + (
        time.perf_counter() - t0)
    now = time.perf_counter()
    for s, t in done:
        engine._append(s, t, now)
    engine.step_count += 1
    return len(done)
