"""Realtime blip-resume (``internal/facade/realtime_registry.go``,
``realtime_registry_test.go``, ``session_resume_test.go``): a duplex call whose
WebSocket drops mid-utterance is parked, a reconnect ``?resume=<sid>`` by the
same owner continues the SAME runtime stream (the utterance spoken across the
two sockets is transcribed as one), the Redis route hint follows the park, and
unclaimed calls expire after the grace window."""
import asyncio
import time

from aiohttp.test_utils import TestClient, TestServer

from omnia_amd.facade import protocol as P
from omnia_amd.facade.auth import AuthChain, SharedTokenValidator
from omnia_amd.facade.realtime import (ROUTE_KEY_PREFIX, MemoryRouteStore, RealtimeRegistry,
                                       RedisRouteStore)
from omnia_amd.facade.runtime_client import InProcessRuntimeClient
from omnia_amd.facade.server import FacadeConfig, FacadeServer
from omnia_amd.observability import metrics as M
from omnia_amd.runtime import duplex as D
from omnia_amd.utils.resp import MiniRedis, RedisClient

from test_duplex import RATE, _service, frames_of, speech


def _frame(i, f, last=False):
    meta = {"codec": "pcm", "sample_rate": RATE, "channels": 1} if i == 0 else None
    return P.encode_frame(P.TYPE_MEDIA_CHUNK, f, meta, i, b"call1", P.FLAG_LAST if last else 0)


async def _collect(ws):
    audio, text, done = b"", "", None
    while done is None:
        m = await ws.receive(timeout=20)
        if m.type.name == "BINARY":
            audio += P.decode_frame(m.data)["payload"]
        elif m.type.name == "TEXT":
            j = m.json()
            if j["type"] == "chunk":
                text += j["content"]
            elif j["type"] in ("done", "error"):
                done = j
        else:
            raise AssertionError(f"socket ended: {m.type}")
    return audio, text, done


def _count(counter):
    return counter._value.get()


def test_dropped_call_parks_and_resumes_on_the_same_stream():
    svc, agent = _service()

    async def run():
        redis = await MiniRedis().start()
        routes = RedisRouteStore(RedisClient(redis.url))
        srv = FacadeServer(FacadeConfig(agent="voice", grace_window_s=30.0,
                                        pod_addr="10.0.0.7:8080"),
                           runtime_client=InProcessRuntimeClient(svc), routes=routes)
        c = TestClient(TestServer(srv.app))
        await c.start_server()
        parked0, re0 = _count(M.REALTIME_PARKED), _count(M.REALTIME_REATTACHED)
        try:
            fs = frames_of(speech("hello there"))
            half = len(fs) // 2
            ws1 = await c.ws_connect("/ws?binary=true")
            sid = (await ws1.receive_json())["session_id"]
            for i in range(half):
                await ws1.send_bytes(_frame(i, fs[i]))
            await asyncio.sleep(0.05)
            await ws1.close()  # a network blip: no hangup
            for _ in range(100):
                if len(srv.parked):
                    break
                await asyncio.sleep(0.02)
            assert sid in srv.parked.parked and srv.audio_sessions == 1
            for _ in range(100):  # the hint is written right after the park
                hint = await RedisClient(redis.url).get(ROUTE_KEY_PREFIX + sid)
                if hint:
                    break
                await asyncio.sleep(0.02)
            assert hint == b"10.0.0.7:8080"
            assert 29000 < redis.exp[(ROUTE_KEY_PREFIX + sid).encode()] * 1000 - \
                time.time() * 1000 <= 30000  # TTL = grace window
            ws2 = await c.ws_connect(f"/ws?binary=true&resume={sid}")
            hello = await ws2.receive_json()
            assert hello["session_id"] == sid and hello["connected"]["resumed"] is True
            assert len(srv.parked) == 0
            assert await RedisClient(redis.url).get(ROUTE_KEY_PREFIX + sid) is None
            for i in range(half, len(fs)):
                await ws2.send_bytes(_frame(i, fs[i], last=i == len(fs) - 1))
            out = await _collect(ws2)
            await ws2.close()
            return (sid, out, _count(M.REALTIME_PARKED) - parked0,
                    _count(M.REALTIME_REATTACHED) - re0)
        finally:
            await c.close()
            await redis.stop()

    sid, (audio, text, done), parked, reattached = asyncio.run(run())
    assert parked == 1 and reattached == 1
    assert done["type"] == "done" and text == "Sure thing. It is sunny today!"
    assert D.FSKCodec(RATE).decode(audio).replace(" ", "") == "Surething.Itissunnytoday!"
    # the runtime heard ONE utterance spanning both sockets
    hist = asyncio.run(agent.store.load(sid))
    assert [m["content"] for m in hist["messages"] if m["role"] == "user"] == ["hello there"]


def test_owner_mismatch_and_expiry():
    svc, _ = _service()
    closed = []

    class Rec:
        async def ensure_session(self, *a, **k):
            pass

        def submit(self, *a, **k):
            pass

        async def close_session(self, sid):
            closed.append(sid)

    async def run():
        routes = MemoryRouteStore()
        auth = AuthChain([SharedTokenValidator("tok")], allow_anonymous=True)
        srv = FacadeServer(FacadeConfig(agent="voice", grace_window_s=0.3, pod_addr="p:1"),
                           runtime_client=InProcessRuntimeClient(svc), routes=routes,
                           auth=auth, recorder=Rec())
        c = TestClient(TestServer(srv.app))
        await c.start_server()
        exp0 = _count(M.REALTIME_PARK_EXPIRED)
        try:
            fs = frames_of(speech("hi"))
            ws1 = await c.ws_connect("/ws?binary=true",
                                     headers={"Authorization": "Bearer tok"})
            sid = (await ws1.receive_json())["session_id"]
            await ws1.send_json({"type": "message", "content": "text first"})  # recorded
            while (await ws1.receive_json())["type"] != "done":
                pass
            await ws1.send_bytes(_frame(0, fs[0]))
            await asyncio.sleep(0.05)
            await ws1.close()
            for _ in range(50):
                if sid in routes.routes:
                    break
                await asyncio.sleep(0.02)
            assert sid in srv.parked.parked
            # an anonymous client may not take an authenticated owner's call
            ws2 = await c.ws_connect(f"/ws?binary=true&resume={sid}")
            await ws2.receive_json()
            assert sid in srv.parked.parked
            await ws2.close()
            await asyncio.sleep(0.6)  # grace window passes unclaimed
            return (sid, len(srv.parked), await routes.get_route(sid), srv.audio_sessions,
                    _count(M.REALTIME_PARK_EXPIRED) - exp0)
        finally:
            await c.close()

    sid, n, route, audio_sessions, expired = asyncio.run(run())
    assert n == 0 and route is None and audio_sessions == 0 and expired == 1
    assert closed == [sid]  # the recorded session reached a terminal status on expiry


def test_hangup_is_not_parked_and_drain_admits_resume():
    svc, _ = _service()

    async def run():
        srv = FacadeServer(FacadeConfig(agent="voice", grace_window_s=30.0, drain_timeout_s=2.0),
                           runtime_client=InProcessRuntimeClient(svc))
        c = TestClient(TestServer(srv.app))
        await c.start_server()
        try:
            fs = frames_of(speech("hi"))
            ws = await c.ws_connect("/ws?binary=true")
            await ws.receive_json()
            await ws.send_bytes(_frame(0, fs[0]))
            await asyncio.sleep(0.05)
            await ws.send_json({"type": "hangup"})
            while (await ws.receive(timeout=5)).type.name not in ("CLOSE", "CLOSED"):
                pass
            for _ in range(100):
                if srv.audio_sessions == 0:
                    break
                await asyncio.sleep(0.02)
            hung = (len(srv.parked), srv.audio_sessions)
            # park one call, then drain: new upgrades are refused, the resume is admitted
            ws = await c.ws_connect("/ws?binary=true")
            sid = (await ws.receive_json())["session_id"]
            await ws.send_bytes(_frame(0, fs[0]))
            await asyncio.sleep(0.05)
            await ws.close()
            for _ in range(50):
                if len(srv.parked):
                    break
                await asyncio.sleep(0.02)
            drain = asyncio.create_task(srv.drain())
            await asyncio.sleep(0.1)
            r = await c.get("/ws")
            refused = r.status
            ws = await c.ws_connect(f"/ws?binary=true&resume={sid}")
            resumed = (await ws.receive_json())["connected"].get("resumed")
            for i in range(1, len(fs)):
                await ws.send_bytes(_frame(i, fs[i], last=i == len(fs) - 1))
            await _collect(ws)
            await ws.close()
            remaining = await asyncio.wait_for(drain, 5)
            return hung, refused, resumed, remaining
        finally:
            await c.close()

    hung, refused, resumed, remaining = asyncio.run(run())
    assert hung == (0, 0)
    assert refused == 503 and resumed is True and remaining == 0


def test_registry_route_store_failures_never_break_parking():
    class Broken:
        async def put_route(self, *a):
            raise ConnectionError("redis down")

        async def delete_route(self, *a):
            raise ConnectionError("redis down")

    class Sess:
        closed = False

        async def close(self):
            Sess.closed = True

    async def run():
        reg = RealtimeRegistry(Broken(), "pod:1", grace_s=0.05)
        await reg.park("s", "u", Sess(), False)
        assert await reg.take("s", "other") is None
        got = await reg.take("s", "u")
        await reg.park("t", "u", Sess(), False)
        await asyncio.sleep(0.2)
        return got, len(reg)

    got, n = asyncio.run(run())
    assert isinstance(got, Sess) and n == 0 and Sess.closed
