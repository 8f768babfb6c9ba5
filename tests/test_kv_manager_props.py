"""Property tests of the paged-KV block manager (engine/kv_manager.py): random
interleavings of turns (prefix acquire -> allocate -> retain), aborts, session
drops and LRU evictions never leak, duplicate or lose a page, and the idle-page
count stays exact.  Reference behaviour: the per-session KV residency the
reference's provider layer lacks; the invariants are ours."""
from hypothesis import given, settings
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


class SharedKVMachine(RuleBasedStateMachine):
    """With cross-session prefix sharing: prompts drawn from a few common
    prefixes, pages published as a turn's prefill completes.  Every page is free,
    table-only, or held; a held shared page is counted once per holder; a
    sequence never owns a shared page in the slot it will write next."""

    PREFIXES = [[1] * 9, [1] * 4 + [2] * 5, [3] * 13]

    def __init__(self):
        super().__init__()
        self.bm = BlockManager(NB, BS, share_prefix=True, max_shared=8)
        self.live: dict[str, tuple[list[int], list[int]]] = {}
        self.history: dict[str, list[int]] = {}

    @rule(sid=st.sampled_from(SESSIONS), pre=st.integers(0, 2), extend=st.integers(0, 6),
          reuse=st.booleans(), gen=st.integers(1, 5))
    def turn(self, sid, pre, extend, reuse, gen):
        if sid in self.live:
            return
        base = self.history.get(sid, []) if reuse else []
        prompt = (base or self.PREFIXES[pre]) + [100 + i for i in range(extend + 1)]
        if not reuse:
            self.bm.drop_session(sid)
            self.history.pop(sid, None)
        blocks, cached = self.bm.acquire_prefix(sid, prompt)
        assert cached <= len(prompt) - 1
        assert len(blocks) == self.bm.blocks_needed(cached)
        if cached % BS:
            assert blocks[-1] not in self.bm.ref, "next write lands in a shared page"
        tokens = prompt + [7] * gen
        try:
            blocks = blocks + self.bm.allocate(self.bm.blocks_needed(len(tokens)) - len(blocks))
        except OutOfBlocks:
            self.bm.release(blocks)
            return
        for b in blocks[cached // BS:]:
            assert b not in self.bm.ref, "a page this turn writes is shared"
        self.bm.publish(prompt, blocks, len(prompt))
        self.live[sid] = (blocks, tokens)

    @precondition(lambda self: self.live)
    @rule(data=st.data(), keep=st.booleans())
    def finish(self, data, keep):
        sid = data.draw(st.sampled_from(sorted(self.live)))
        blocks, tokens = self.live.pop(sid)
        if keep:
            self.bm.retain(sid, blocks, tokens)
            self.history[sid] = tokens
        else:
            self.bm.release(blocks)

    @rule()
    def fault_recovery(self):
        self.bm.reset_shared()

    @invariant()
    def pages_accounted(self):
        bm = self.bm
        held = [b for blocks, _ in self.live.values() for b in blocks]
        parked = [b for s in bm.sessions.values() for b in s.blocks]
        owners = held + parked
        private = [b for b in owners if b not in bm.ref]
        assert len(private) == len(set(private)), "a private page is owned twice"
        for b, r in bm.ref.items():
            tab = int(b in bm.key_of)
            assert r == tab + owners.count(b), f"page {b}: ref {r}, holders {owners.count(b)}"
            assert r >= 1 and (b in bm.evictable) == (r == 1 and tab == 1)
            if tab:
                assert bm.table[bm.key_of[b]] == b
        every = set(private) | set(bm.ref) | set(bm.free)
        assert len(bm.free) == len(set(bm.free))
        assert not (set(bm.free) & (set(private) | set(bm.ref)))
        assert every == set(range(1, NB)), "a page leaked (or page 0 escaped)"
        assert len(bm.table) <= bm.max_shared
        assert bm.idle_blocks == sum(1 for b in parked if b not in bm.ref)


TestSharedKVProperties = SharedKVMachine.TestCase
TestSharedKVProperties.settings = settings(max_examples=150, stateful_step_count=40,
                                           deadline=None)


def test_shared_prefix_maps_published_pages():
    bm = BlockManager(16, 4, share_prefix=True)
    sys_prompt = [5, 6, 7, 8, 9, 10, 11, 12, 13]
    a = sys_prompt + [20, 21]
    blocks_a = bm.allocate(bm.blocks_needed(len(a)))
    assert bm.acquire_prefix("s2", a) == ([], 0)  # nothing published yet
    done, h = bm.publish(a, blocks_a, 6)  # prefill of the first chunk done: page 0
    assert done == 1 and list(bm.table.values()) == [blocks_a[0]]
    bm.publish(a, blocks_a, len(a), done, h)
    assert len(bm.table) == 2  # the third page holds the last token: never full here
    b = sys_prompt + [30]
    got, n = bm.acquire_prefix("s3", b)
    assert got == blocks_a[:2] and n == 8 and bm.stats["shared_hit_tokens"] == 8
    # a prompt that IS the shared prefix leaves its last page to be recomputed
    got2, n2 = bm.acquire_prefix(None, sys_prompt[:8])
    assert got2 == blocks_a[:1] and n2 == 4
    bm.release(got2)
    bm.release(blocks_a)
    assert bm.ref[blocks_a[0]] == 2 and not bm.evictable  # s3 still maps both
    bm.release(got)
    assert set(bm.evictable) == set(blocks_a[:2])
    free0 = bm.num_free
    assert bm.num_available == free0 + 2
    bm.allocate(free0 + 1)  # reclaims one table-only page
    assert len(bm.table) == 1 and bm.stats["shared_evictions"] == 1


def test_unmapped_shared_pages_go_before_parked_sessions():
    bm = BlockManager(12, 4, share_prefix=True)
    one_off = list(range(50, 59))  # a finished sessionless prompt: 2 published pages
    b1 = bm.allocate(3)
    bm.publish(one_off, b1, len(one_off))
    bm.release(b1)
    assert len(bm.evictable) == 2
    conv = list(range(70, 78))  # a parked conversation
    b2 = bm.allocate(2)
    bm.retain("chat", b2, conv)
    bm.allocate(bm.num_free + 2)  # needs both unmapped pages, not the session
    assert bm.has_session("chat") and not bm.table
    assert bm.stats["shared_evictions"] == 2 and bm.stats["evictions"] == 0


def test_forced_digest_collision_maps_nothing():
    """a lookup never maps a page on digest equality alone.  Force a
    collision (a page published under another prompt's digest) and check the
    stored tokens / parent refuse it."""
    bm = BlockManager(16, 4, share_prefix=True)
    victim = [1, 2, 3, 4, 9]
    forged = [66, 66, 66, 66, 9]
    b = bm.allocate(2)
    bm.publish(forged, b, len(forged))
    (page,) = [p for p in bm.table.values()]
    # rewrite the table so the forged page sits under the victim's digest
    vh = bm._chain(bm.seed(None), victim, 0)
    bm.table = {vh: page}
    bm.key_of = {page: vh}
    got, n = bm.acquire_prefix(None, victim)
    assert got == [] and n == 0
    # the honest path still hits
    bm2 = BlockManager(16, 4, share_prefix=True)
    b2 = bm2.allocate(2)
    bm2.publish(victim, b2, len(victim))
    assert bm2.acquire_prefix(None, victim)[1] == 4


def test_chain_digest_is_keyed_per_process():
    a, b = BlockManager(8, 4, share_prefix=True), BlockManager(8, 4, share_prefix=True)
    toks = [3, 1, 4, 1]
    assert a._chain(a.seed(None), toks, 0) != b._chain(b.seed(None), toks, 0)
    assert len(a._chain(a.seed(None), toks, 0)) == 16


@given(st.lists(st.integers(0, 1000), min_size=9, max_size=20), st.text(min_size=1, max_size=8),
       st.text(min_size=1, max_size=8))
@settings(max_examples=60, deadline=None)
def test_salt_scopes_sharing(prompt, s1, s2):
    """Pages published under one cache salt are invisible under another."""
    bm = BlockManager(32, 4, share_prefix=True)
    blocks = bm.allocate(bm.blocks_needed(len(prompt)))
    bm.publish(prompt, blocks, len(prompt), salt=s1)
    assert bm.acquire_prefix(None, prompt, salt=s1)[1] > 0
    if s1 != s2:
        assert bm.acquire_prefix(None, prompt, salt=s2) == ([], 0)
    assert bm.acquire_prefix(None, prompt) == ([], 0)  # no salt: its own scope


def test_share_limit_publishes_only_the_system_prefix():
    bm = BlockManager(16, 4, share_prefix=True)
    sys_part = [7] * 8
    user_a = sys_part + [100, 101, 102, 103, 104, 105, 106, 107, 1]
    b = bm.allocate(bm.blocks_needed(len(user_a)))
    bm.publish(user_a, b, len(user_a), limit=len(sys_part) + 3)
    assert len(bm.table) == 2  # the two system pages, none of the user's
    user_b = sys_part + [100, 101, 102, 103, 999]
    got, n = bm.acquire_prefix(None, user_b)
    assert n == 8  # the other user's conversation page is not visible


def test_shared_prefix_len_covers_system_and_tools_only():
    from omnia_amd.engine.tokenizer import SyntheticTokenizer
    from omnia_amd.runtime.chat import Message, render_llama3, shared_prefix_len

    tok = SyntheticTokenizer(128256, 128000, [128001, 128009])
    enc = lambda t: tok.encode(t, add_bos=False)  # noqa: E731
    tools = [{"name": "lookup", "parameters": {"type": "object"}}]
    msgs = [Message("system", "You are a helpful support agent."), Message("user", "my secret")]
    ids = enc(render_llama3(msgs, tools))
    n = shared_prefix_len(msgs, tools, enc, ids)
    head = enc(render_llama3(msgs[:1], tools, add_generation_prompt=False))
    assert 0 < n <= len(head) < len(ids)
    assert "secret" not in tok.decode(ids[:n])
    assert shared_prefix_len([Message("user", "hi")], None, enc, enc("hi")) == 0
