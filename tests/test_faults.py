"""Failure detection / recovery / fault injection.

* failpoint spec grammar (probability, once, N@K, always, off) and seeding;
* an engine step fault fails only the live sequences with ERROR, drops resident
  KV, and the engine keeps serving (next turn re-prefills);
* the runtime surfaces an engine fault as an ``ENGINE_FAULT`` Error frame;
* a fault storm or a stalled step (watchdog) flips engine health off;
* tool-call and session-write failpoints drive the breaker / error paths."""
import asyncio
import time

import pytest

from omnia_amd.utils import failpoints as fp


@pytest.fixture(autouse=True)
def _clean():
    fp.clear()
    yield
    fp.clear()


def test_spec_grammar():
    pts = fp.parse("a:once,b:2@3,c:always,d:off,e:1.0")
    seq = {k: [pts[k].should_fire(__import__("random").Random(0)) for _ in range(6)]
           for k in pts}
    assert seq["a"] == [True, False, False, False, False, False]
    assert seq["b"] == [False, False, True, True, False, False]
    assert all(seq["c"]) and not any(seq["d"]) and all(seq["e"])
    with pytest.raises(ValueError):
        fp.parse("x:1.5")


def test_hit_raises_and_stats():
    fp.configure("tool.call:once")
    with pytest.raises(fp.FailpointError):
        fp.hit("tool.call")
    fp.hit("tool.call")  # only once
    st = fp.stats()["tool.call"]
    assert st["hits"] == 2 and st["fired"] == 1
    fp.hit("unarmed.point")


def _engine():
    from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig

    cfg = EngineConfig(model="tiny-llama", device="cpu", dtype="float32", num_blocks=64,
                       block_size=16, max_batch=4, max_model_len=512, use_graphs=False)
    return AsyncLLMEngine.from_config(cfg)


def test_engine_fault_recovery_keeps_serving():
    from omnia_amd.engine.sampling_params import SamplingParams

    eng = _engine()
    p = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)

    async def turn(prompt, sid):
        return [ev async for ev in eng.generate(prompt, p, session_id=sid)][-1]

    async def run():
        ok = await turn(list(range(5, 40)), "s1")
        assert ok.finish_reason == "length" and eng.has_session("s1")
        fp.arm("engine.decode_step", "once")
        bad = await turn(list(range(5, 40)) + [1, 2, 3], "s1")
        fp.clear()
        again = await turn(list(range(5, 40)) + [1, 2, 3], "s1")
        return ok, bad, again

    try:
        ok, bad, again = asyncio.run(run())
        assert bad.finish_reason == "error"
        assert again.finish_reason == "length"
        assert again.cached_tokens == 0  # resident KV was discarded by recovery
        assert eng.engine.counters["faults"] == 1 and eng.health()
    finally:
        eng.shutdown()


def test_fault_storm_and_watchdog_mark_unhealthy(monkeypatch):
    from omnia_amd.engine.sampling_params import SamplingParams

    monkeypatch.setenv("OMNIA_ENGINE_MAX_FAULTS", "2")
    eng = _engine()
    p = SamplingParams(temperature=0, max_tokens=3, ignore_eos=True)

    async def turn():
        return [ev async for ev in eng.generate(list(range(3, 20)), p)][-1]

    try:
        fp.arm("engine.step", "always")
        for _ in range(2):
            assert asyncio.run(turn()).finish_reason == "error"
        assert not eng.health()
    finally:
        fp.clear()
        eng.shutdown()

    monkeypatch.setenv("OMNIA_STEP_TIMEOUT_S", "0.3")
    monkeypatch.setenv("OMNIA_FAILPOINT_HANG_S", "1.5")
    eng = _engine()
    try:
        fp.arm("engine.hang", "once")
        t0 = time.time()
        asyncio.run(turn())  # the stalled step still completes
        assert time.time() - t0 >= 1.0
        assert not eng.health() and isinstance(eng.error, TimeoutError)
    finally:
        fp.clear()
        eng.shutdown()


def test_runtime_reports_engine_fault_code():
    from omnia_amd.api.proto import runtime_v1 as pb
    from omnia_amd.runtime.agent import Agent, AgentConfig
    from omnia_amd.runtime.context_store import MemoryContextStore
    from omnia_amd.runtime.promptpack import PromptPack
    from omnia_amd.runtime.providers import LocalEngineProvider
    from omnia_amd.runtime.server import QueueStream, RuntimeService

    eng = _engine()

    async def turn(svc, text):
        st = QueueStream(None)
        task = asyncio.create_task(svc.converse(st))
        await st.inbox.put(pb.ClientMessage(session_id="f1", content=text))
        while True:
            f = await asyncio.wait_for(st.outbox.get(), 10)
            if f.WhichOneof("message") in ("done", "error"):
                break
        st.close()
        await asyncio.wait_for(task, 5)
        return f

    try:
        agent = Agent(PromptPack.minimal("sys"), LocalEngineProvider(eng), MemoryContextStore(),
                      None, AgentConfig(defaults={"maxTokens": 4, "temperature": 0}))
        svc = RuntimeService(agent)
        fp.arm("engine.prefill", "once")
        f = asyncio.run(turn(svc, "hello"))
        assert f.WhichOneof("message") == "error" and f.error.code == "ENGINE_FAULT"
        f = asyncio.run(turn(svc, "hello again"))
        assert f.WhichOneof("message") == "done"
        assert asyncio.run(svc.health()).healthy
    finally:
        eng.shutdown()


def test_tool_call_failpoint_feeds_breaker():
    from omnia_amd.tools.executor import OmniaExecutor
    from omnia_amd.tools.executor import InProcessHandler

    async def echo(args, ctx):
        return {"ok": True}

    ex = OmniaExecutor({"handlers": []})
    ex.add_handler(InProcessHandler("builtin", {"echo": ("echo", {"type": "object"}, echo)}))
    asyncio.run(ex.discover())
    fp.arm("tool.call", "always")
    errs = [asyncio.run(ex.execute("echo", {}))[1] for _ in range(6)]
    assert all(errs)
    fp.clear()
    # 5 consecutive failures opened the breaker: still failing fast while open
    res, is_err = asyncio.run(ex.execute("echo", {}))
    assert is_err and "circuit" in res.lower()


def test_session_write_failpoint():
    from omnia_amd.session.model import Message, Session
    from omnia_amd.session.store import TieredSessionService

    st = TieredSessionService()
    sess = st.create(Session(agent_name="a"))
    fp.arm("session.write", "once")
    with pytest.raises(fp.FailpointError):
        asyncio.run(st.append_message(sess.id, Message(role="user", content="x")))
    m = asyncio.run(st.append_message(sess.id, Message(role="user", content="x")))
    assert m.sequence_num == 0
