"""Property tests of the paged-KV block manager (engine/kv_manager.py): random
interleavings of turns (prefix acquire -> allocate -> retain), aborts, session
drops and LRU evictions never leak, duplicate or lose a page, and the idle-page
count stays exact.  Reference behaviour: the per-session KV residency the
reference's provider layer lacks; the invariants are ours."""
from hypothesis import settings
from hypothesis import strategies as st
from hypothesis.stateful import RuleBasedStateMachine, invariant, precondition, rule

from omnia_amd.engine.kv_manager import BlockManager, OutOfBlocks, common_prefix

NB, BS = 24, 4
SESSIONS = ["a", "b", "c", "d", "e"]


class KVMachine(RuleBasedStateMachine):
    def __init__(self):
        super().__init__()
        self.bm = BlockManager(NB, BS)
        self.live: dict[str, tuple[list[int], list[int]]] = {}  # running turn: blocks, tokens
        self.history: dict[str, list[int]] = {}  # tokens each session last retained

    @rule(sid=st.sampled_from(SESSIONS), extend=st.integers(0, 9), reuse=st.booleans(),
          gen=st.integers(1, 6))
    def turn(self, sid, extend, reuse, gen):
        if sid in self.live:
            return
        base = self.history.get(sid, []) if reuse else []
        prompt = base + [100 + i for i in range(extend + 1)]
        blocks, cached = self.bm.acquire_prefix(sid, prompt)
        assert cached <= len(prompt) - 1
        assert cached <= common_prefix(self.history.get(sid, []), prompt)
        assert len(blocks) == self.bm.blocks_needed(cached)
        tokens = prompt + [7] * gen
        try:
            blocks = blocks + self.bm.allocate(self.bm.blocks_needed(len(tokens)) - len(blocks))
        except OutOfBlocks:
            self.bm.release(blocks)
            return
        self.live[sid] = (blocks, tokens)

    @precondition(lambda self: self.live)
    @rule(data=st.data(), keep=st.booleans())
    def finish(self, data, keep):
        sid = data.draw(st.sampled_from(sorted(self.live)))
        blocks, tokens = self.live.pop(sid)
        if keep:
            self.bm.retain(sid, blocks, tokens)
            self.history[sid] = tokens
        else:  # aborted turn: pages go straight back
            self.bm.release(blocks)

    @rule(sid=st.sampled_from(SESSIONS))
    def drop(self, sid):
        if sid not in self.live:
            self.bm.drop_session(sid)
            self.history.pop(sid, None)

    @invariant()
    def pages_conserved(self):
        held = [b for blocks, _ in self.live.values() for b in blocks]
        parked = [b for s in self.bm.sessions.values() for b in s.blocks]
        every = held + parked + list(self.bm.free)
        assert len(every) == len(set(every)), "a page is owned twice"
        assert set(every) == set(range(1, NB)), "a page leaked (or page 0 escaped)"
        assert self.bm.idle_blocks == len(parked)
        assert self.bm.num_available == len(self.bm.free) + len(parked)

    @invariant()
    def parked_sessions_fit_their_tokens(self):
        for s in self.bm.sessions.values():
            assert len(s.blocks) == self.bm.blocks_needed(len(s.tokens))


TestKVManagerProperties = KVMachine.TestCase
TestKVManagerProperties.settings = settings(max_examples=150, stateful_step_count=40,
                                            deadline=None)


def test_common_prefix_matches_naive():
    from hypothesis import given

    @given(st.lists(st.integers(0, 3), max_size=700), st.lists(st.integers(0, 3), max_size=700))
    @settings(max_examples=200, deadline=None)
    def check(a, b):
        n = 0
        while n < min(len(a), len(b)) and a[n] == b[n]:
            n += 1
        assert common_prefix(a, b) == n

    check()
