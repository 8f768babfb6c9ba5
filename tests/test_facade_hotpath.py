"""Facade streaming hot path: the pre-serialized chunk frame is byte-identical
to the dict path, and the per-turn inactivity watchdog (which replaced a
``wait_for`` around every streamed frame) still ends a silent turn -- but only
time spent waiting on the runtime counts."""
import asyncio
import json

from omnia_amd.api.proto import runtime_v1 as pb
from omnia_amd.facade import protocol as P
from omnia_amd.facade.handlers import PendingTools, RuntimeHandler, Writer


def test_chunk_text_matches_dict_serialization():
    for sid, content, role in [("abc", 'hé"llo\n ', ""), ("", "x", "assistant"),
                               ("s-1", "", ""), ("s", "\x00\t", "user")]:
        fast = P.chunk_text(json.dumps(sid) if sid else "", content, role)
        ref = P.chunk(sid, content, role)
        ref["timestamp"] = json.loads(fast)["timestamp"]
        assert fast == json.dumps(ref, separators=(",", ":"))
    ts = P.now_rfc3339()
    assert ts.endswith("Z") and "T" in ts and len(ts) in (20, 27)


class _Rec(Writer):
    def __init__(self):
        self.msgs = []

    async def write(self, msg):
        self.msgs.append(msg)


class _Stream:
    def __init__(self, script):
        self.script = list(script)
        self.closed = False

    async def send(self, msg):
        pass

    async def recv(self):
        if not self.script:
            await asyncio.sleep(3600)
        delay, msg = self.script.pop(0)
        await asyncio.sleep(delay)
        return msg

    async def close(self):
        self.closed = True


class _Client:
    def __init__(self, script):
        self.stream = _Stream(script)

    async def open(self, md=None):
        return self.stream


def _chunk(t):
    return pb.ServerMessage(chunk=pb.Chunk(content=t))


def _done():
    return pb.ServerMessage(done=pb.Done(final_content="ab", usage=pb.Usage(output_tokens=2)))


def test_inactivity_watchdog_ends_a_silent_turn():
    async def go():
        c = _Client([(0.01, _chunk("a"))])  # then silence
        w = _Rec()
        h = RuntimeHandler(c, inactivity_s=0.3)
        out = await asyncio.wait_for(h.handle("s", {"content": "hi"}, w, PendingTools(), {}), 5)
        assert out["error"] == "stream inactivity timeout"
        assert w.msgs[0]["type"] == "chunk" and w.msgs[-1]["type"] == "error"
        assert c.stream.closed

    asyncio.run(go())


def test_watchdog_rearms_on_traffic_and_ignores_slow_writes():
    class SlowWriter(_Rec):
        async def write(self, msg):
            await asyncio.sleep(0.25)  # a slow client: not runtime inactivity
            self.msgs.append(msg)

    async def go():
        # frames every 0.2 s for 1 s with a 0.3 s limit: never idle long enough
        c = _Client([(0.2, _chunk("a")) for _ in range(5)] + [(0.05, _done())])
        w = SlowWriter()
        h = RuntimeHandler(c, inactivity_s=0.3)
        out = await h.handle("s", {"content": "hi"}, w, PendingTools(), {})
        assert out["error"] is None and out["usage"]["output_tokens"] == 2
        assert [m["type"] for m in w.msgs] == ["chunk"] * 5 + ["done"]

    asyncio.run(go())


def test_external_cancel_still_propagates():
    async def go():
        c = _Client([])
        h = RuntimeHandler(c, inactivity_s=60)
        t = asyncio.ensure_future(h.handle("s", {"content": "hi"}, _Rec(), PendingTools(), {}))
        await asyncio.sleep(0.05)
        t.cancel()
        try:
            await t
        except asyncio.CancelledError:
            return True
        return False

    assert asyncio.run(go())
