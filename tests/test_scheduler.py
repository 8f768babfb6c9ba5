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
