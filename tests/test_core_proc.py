"""Engine-core process (``omnia_amd.engine.core_proc``): a child process owns the
engine; the client streams tokens over a socketpair.  CPU (tiny-llama)."""
import asyncio

import pytest

from omnia_amd.engine.core_proc import EngineCoreClient, _Frames, _send
from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams

CFG = dict(model="tiny-llama", device="cpu", num_blocks=256, block_size=32, max_batch=8,
           max_model_len=512)


@pytest.fixture(scope="module")
def client():
    c = EngineCoreClient(EngineConfig(**CFG))
    yield c
    c.shutdown()
    assert c.proc.returncode == 0


def _prompts(n):
    return [list(range(5 + i, 40 + 3 * i)) for i in range(n)]


def test_frames_roundtrip():
    import socket

    a, b = socket.socketpair()
    _send(a, ["out", [["r1", "hé", 7, 2]], []])
    _send(a, ["reply", 3, {"x": [1, 2]}])
    f = _Frames()
    got = []
    data = b.recv(1 << 16)
    # split delivery exercises partial-frame buffering
    got += f.feed(data[:5])
    got += f.feed(data[5:])
    assert got == [["out", [["r1", "hé", 7, 2]], []], ["reply", 3, {"x": [1, 2]}]]
    a.close()
    b.close()


def test_streams_match_in_process_engine(client):
    p = SamplingParams(temperature=0, max_tokens=10, ignore_eos=True)

    async def one(i, ids):
        toks, n = [], 0
        async for ev in client.generate(ids, p, session_id=f"cp{i}"):
            if ev.finished:
                return toks, n, ev
            toks.append(ev.token)
            n += ev.n_tokens

    async def main():
        return await asyncio.gather(*(one(i, ids) for i, ids in enumerate(_prompts(5))))

    res = asyncio.run(main())
    eng = LLMEngine(EngineConfig(**CFG))
    ref = [eng.add_request(ids, p) for ids in _prompts(5)]
    eng.run_until_done()
    for (toks, n, fin), s in zip(res, ref):
        assert n == 10 and fin.output_tokens == 10 and fin.finish_reason == "length"
        assert toks[-1] == s.output[-1]
        assert fin.prompt_tokens == len(s.prompt)
    assert client.has_session("cp1")
    client.drop_session("cp1")
    assert not client.has_session("cp1")
    st = client.stats()
    assert st["counters"]["finished"] >= 5


def test_abort_on_consumer_exit_and_errors(client):
    async def main():
        n = 0
        async for ev in client.generate(_prompts(1)[0], SamplingParams(
                temperature=0, max_tokens=400, ignore_eos=True)):
            n += ev.n_tokens
            if n >= 2:
                break  # consumer leaves: the core must abort the sequence
        with pytest.raises(RuntimeError):
            async for _ in client.generate(list(range(1, 600)), SamplingParams(max_tokens=4)):
                pass  # prompt longer than max_model_len -> error finish

    asyncio.run(main())
    # the aborted request does not keep decoding: the engine drains
    for _ in range(50):
        st = client.stats()
        if st["counters"]["decode_tokens"] < 400 and client.call("has_session", "none") is False:
            break
    assert st["counters"]["decode_tokens"] < 400


@pytest.mark.timeout(240)
def test_request_burst_never_blocks_the_client_during_a_stalled_step():
    """A wave's burst of new prompts arrives while the core sits in a long step
    (here a 3 s simulated hang).  The core's inbox thread keeps draining the
    socket, so the client's sends (made on the serving event loop) return at
    once instead of blocking until the step ends."""
    import time

    c = EngineCoreClient(EngineConfig(**CFG), env={
        "OMNIA_FAILPOINT": "engine.hang:once", "OMNIA_FAILPOINT_HANG_S": "3",
        "OMP_NUM_THREADS": "2"})
    try:
        async def go():
            # first request trips the hang inside the core's next step
            first = asyncio.ensure_future(_drain(c, list(range(5, 60)), 2))
            await asyncio.sleep(0.5)
            big = list(range(256, 512)) * 2  # in-vocab 3-byte msgpack ids: ~1-1.3 KB/frame
            t0 = time.perf_counter()
            tasks = [asyncio.ensure_future(_drain(c, big[: 300 + i % 150], 1))
                     for i in range(400)]
            await asyncio.sleep(0)  # every generate() has sent its add
            sent = time.perf_counter() - t0
            # the claim is about the sends: the stalled turn completes, the burst
            # is aborted (400 CPU prefills take minutes on a loaded box)
            await first
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
            return sent

        sent = asyncio.run(go())
        assert sent < 1.0, f"client sends blocked for {sent:.2f}s behind the stalled step"
    finally:
        c.shutdown()


async def _drain(c, prompt, n):
    out = []
    async for ev in c.generate(prompt, SamplingParams(temperature=0, max_tokens=n,
                                                      ignore_eos=True)):
        out.append(ev)
    return out
