"""A fleet session opened ahead of its turn survives the facade's heartbeat
(the TP=2 bench rehearsal's first wave outlived the 30 s ping interval and the
pre-connected sessions were closed under the load generator)."""
import asyncio

from aiohttp import web

from omnia_amd.ee.arena.fleet import FleetSession


def _facade(heartbeat: float):
    async def ws_handler(request):
        ws = web.WebSocketResponse(heartbeat=heartbeat)
        await ws.prepare(request)
        await ws.send_json({"type": "connected", "session_id": "s1"})
        async for msg in ws:
            f = msg.json()
            if f.get("type") == "message":
                await ws.send_json({"type": "chunk", "content": f["content"][::-1]})
                await ws.send_json({"type": "done", "usage": {"output_tokens": 1}})
        return ws

    app = web.Application()
    app.router.add_get("/ws", ws_handler)
    return app


def test_idle_session_answers_heartbeat_pings():
    async def go():
        runner = web.AppRunner(_facade(heartbeat=0.2))
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        try:
            FleetSession.IDLE_AFTER_S = 0.05
            async with FleetSession(f"ws://127.0.0.1:{port}/ws", timeout_s=5) as fs:
                await asyncio.sleep(1.0)  # 5 ping intervals with no turn in flight
                r1 = await fs.turn("abc")
                await asyncio.sleep(1.0)  # and again between two turns
                r2 = await fs.turn("xyz")
            return r1["content"], r2["content"], fs.session_id
        finally:
            FleetSession.IDLE_AFTER_S = 5.0
            await runner.cleanup()

    assert asyncio.run(go()) == ("cba", "zyx", "s1")
