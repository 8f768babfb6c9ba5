"""Scheduler planning under KV pressure (reference has no engine)."""
from omnia_amd.engine.kv_manager import BlockManager
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.engine.scheduler import Scheduler, SchedulerConfig
from omnia_amd.engine.sequence import Sequence, SeqStatus


def _running(sched, n_tokens, out_tok):
    s = Sequence(prompt=list(range(1, n_tokens + 1)), params=SamplingParams(max_tokens=8))
    s.blocks = sched.blocks.allocate(sched.blocks.blocks_needed(n_tokens))
    s.num_cached = n_tokens
    s.output.append(out_tok)
    s.status = SeqStatus.RUNNING
    sched.running.append(s)
    return s


def test_decode_preempts_only_the_youngest():
    """a sequence preempted earlier in the same pass must not then
    allocate pages (which preempted the older sequence too)."""
    bm = BlockManager(9, 4)  # 8 usable pages
    sched = Scheduler(SchedulerConfig(max_batch=8, max_prefill_tokens=64), bm)
    a = _running(sched, 16, 7)  # 4 pages, needs a 5th for its next token
    b = _running(sched, 16, 9)
    assert bm.num_free == 0
    plan = sched.schedule()
    assert [s for s in plan.decode] == [a]
    assert sched.running == [a] and a.preemptions == 0 and len(a.blocks) == 5
    assert b.preemptions == 1 and b.blocks == [] and b.status == SeqStatus.WAITING
    assert list(sched.waiting) == [b]


def test_idle_session_pages_counted_and_reclaimable():
    """``idle_blocks`` always equals the pages parked under idle sessions, and
    ``num_available`` (free + idle) is what an allocation can reach -- the engine
    keeps pipelining when the pool is full of parked multi-turn sessions."""
    import random

    from omnia_amd.engine.kv_manager import BlockManager

    rng = random.Random(0)
    bm = BlockManager(64, 4)
    owned = []
    for step in range(400):
        op = rng.random()
        sid = f"s{rng.randrange(12)}"
        if op < 0.4 and bm.num_available >= 3:
            owned.append((sid, bm.allocate(rng.randrange(1, 4))))
        elif op < 0.7 and owned:
            s, blocks = owned.pop(rng.randrange(len(owned)))
            bm.retain(s, blocks, list(range(rng.randrange(0, 4 * len(blocks) + 1))))
        elif op < 0.85:
            blocks, _ = bm.acquire_prefix(sid, list(range(9)))
            owned.append((sid, blocks))
        else:
            bm.drop_session(sid)
        assert bm.idle_blocks == sum(len(s.blocks) for s in bm.sessions.values())
        assert bm.num_available == bm.num_free + bm.idle_blocks
        held = sum(len(b) for _, b in owned)
        assert bm.num_free + bm.idle_blocks + held == 63
    # a pool full of parked sessions still admits work
    for _, b in owned:
        bm.release(b)
    i = 0
    while bm.num_free:
        bm.retain(f"p{i}", bm.allocate(1), [1, 2, 3])
        i += 1
    assert bm.num_free == 0 and bm.can_allocate(10)
    got = bm.allocate(10)
    assert len(got) == 10 and bm.stats["evictions"] >= 10


def test_prefill_stream_cannot_starve_running_decoders():
    """A stream of one-token requests (each finishes at its prefill, so capacity
    keeps freeing) gets prefill-first steps; after ``max_prefill_streak`` of them
    the running sequence is served anyway, and the streak restarts."""
    from omnia_amd.engine.sequence import FinishReason

    bm = BlockManager(4096, 16)
    sched = Scheduler(SchedulerConfig(max_batch=4, max_prefill_tokens=64,
                                      max_prefill_streak=5), bm)
    r = _running(sched, 16, 3)
    kinds = []
    for i in range(40):
        sched.add(Sequence(prompt=list(range(1, 33)), params=SamplingParams(max_tokens=1)))
        plan = sched.schedule()
        kinds.append(plan.kind)
        for s, _ in plan.prefill:  # the one-token requests finish at their prefill
            if s is not r and s.num_cached + _ >= len(s.prompt):
                s.num_cached = len(s.prompt)
                sched.finish(s, FinishReason.LENGTH)
        if plan.kind == "decode":
            assert plan.decode == [r]
    assert kinds[:6] == ["prefill"] * 5 + ["decode"]
    assert kinds.count("decode") >= 6
    # unbounded (0) keeps the old prefill-first behaviour
    sched2 = Scheduler(SchedulerConfig(max_batch=4, max_prefill_tokens=64,
                                       max_prefill_streak=0), BlockManager(4096, 16))
    _running(sched2, 16, 3)
    sched2.add(Sequence(prompt=list(range(1, 33)), params=SamplingParams(max_tokens=1)))
    assert sched2.schedule().kind == "prefill"
