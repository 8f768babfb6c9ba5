"""Fleet mode: drive a deployed agent through its WebSocket facade and time it
(``ee/pkg/arena/fleet/client.go:124-179``, ``fleet/provider.go``).

TTFT = first ``chunk`` (or ``done`` when the agent does not stream) after the
``message`` frame; turn latency = ``done`` arrival.  Client-side tools are
answered with a canned result so tool loops complete.

A session idle between turns for longer than ``IDLE_AFTER_S`` starts one reader
task on its socket: aiohttp answers the facade's heartbeat pings only inside
``receive()``, so a session opened ahead of its turn (load generators
pre-connect the next wave) and left unread for longer than the facade's ping
interval would be closed under it.  Sessions reused within seconds -- a closed-
loop bench wave -- never start one (it cost ~1.5 % of the headline bench's
engine busy time when started on every session)."""
from __future__ import annotations

import asyncio
import contextlib
import json
import os
import time

import aiohttp

from ...utils.arrivals import mark


class FleetSession:
    """One virtual user's WebSocket conversation.  ``http``: a shared
    :class:`aiohttp.ClientSession` (load generators open hundreds of sessions
    through one connector); otherwise the session owns its own."""

    def __init__(self, url: str, agent: str = "", headers: dict | None = None,
                 timeout_s: float = 120.0, http: aiohttp.ClientSession | None = None):
        self.url = url
        self.agent = agent
        self.headers = headers or {}
        self.timeout_s = timeout_s
        self._shared = http
        self._http = None
        self.ws = None
        self.session_id = ""
        self._idle: asyncio.Task | None = None
        self._idle_timer: asyncio.TimerHandle | None = None
        self._idle_msg = None

    async def __aenter__(self):
        if self._shared is None:
            self._http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None))
        http = self._shared or self._http
        url = self.url + (("&" if "?" in self.url else "?") + f"agent={self.agent}"
                          if self.agent else "")
        self.ws = await http.ws_connect(url, headers=self.headers, max_msg_size=0)
        hello = await self.ws.receive_json(timeout=self.timeout_s)
        if hello.get("type") != "connected":
            raise RuntimeError(f"facade handshake failed: {hello}")
        self.session_id = hello.get("session_id", "")
        self._idle_start()
        return self

    IDLE_READ = os.environ.get("OMNIA_FLEET_IDLE_READ", "1") != "0"
    IDLE_AFTER_S = 5.0  # well inside aiohttp's pong deadline (half the ping interval)

    def _idle_start(self):
        """After IDLE_AFTER_S without a turn, read (and so answer pings) until
        the next turn.  The facade sends nothing else between turns; a close or
        error it sends is raised by the next turn."""
        self._idle_msg = None
        if self.IDLE_READ:
            self._idle_timer = asyncio.get_running_loop().call_later(self.IDLE_AFTER_S,
                                                                     self._idle_spawn)

    def _idle_spawn(self):
        self._idle_timer = None
        if self.ws is None or self.ws.closed or self._idle is not None:
            return

        async def idle():
            self._idle_msg = await self.ws.receive()

        self._idle = asyncio.ensure_future(idle())

    async def _idle_stop(self):
        if self._idle_timer is not None:
            self._idle_timer.cancel()
            self._idle_timer = None
        t, self._idle = self._idle, None
        if t is not None and not t.done():
            t.cancel()
            with contextlib.suppress(asyncio.CancelledError):
                await t
        msg, self._idle_msg = self._idle_msg, None
        if msg is not None and msg.type in (aiohttp.WSMsgType.CLOSE, aiohttp.WSMsgType.CLOSED,
                                            aiohttp.WSMsgType.ERROR):
            raise RuntimeError(f"facade closed the idle session ({msg.type})")

    async def __aexit__(self, *exc):
        with contextlib.suppress(RuntimeError):
            await self._idle_stop()
        if self.ws is not None:
            await self.ws.close()
        if self._http is not None:
            await self._http.close()

    async def turn(self, content: str, metadata: dict | None = None,
                   tool_result=lambda name, args: {"ok": True}) -> dict:
        await self._idle_stop()
        t0 = time.perf_counter()
        mark("client_send")
        await self.ws.send_json({"type": "message", "content": content,
                                 "metadata": metadata or {}})
        ttft, text, usage = None, [], {}
        stamps = []  # arrival time of every streamed chunk (inter-token latency)
        while True:
            msg = await self.ws.receive(timeout=self.timeout_s)
            if msg.type != aiohttp.WSMsgType.TEXT:
                raise RuntimeError(f"unexpected websocket frame {msg.type}")
            f = json.loads(msg.data)
            t = f.get("type")
            if t == "chunk":
                now = time.perf_counter()
                if ttft is None:
                    ttft = now - t0
                    mark("client_first")
                stamps.append(now - t0)
                text.append(f.get("content", ""))
            elif t == "tool_call":
                tc = f["tool_call"]
                await self.ws.send_json({"type": "tool_call_ack",
                                         "tool_call_ack": {"call_id": tc["id"]}})
                await self.ws.send_json({"type": "tool_result", "tool_result": {
                    "call_id": tc["id"], "result": tool_result(tc.get("name"),
                                                               tc.get("arguments"))}})
            elif t == "done":
                lat = time.perf_counter() - t0
                mark("client_done")
                if ttft is None:
                    ttft = lat
                final = f.get("content") or "".join(text)
                usage = f.get("usage") or {}
                self._idle_start()
                return {"content": final, "ttft_ms": ttft * 1e3, "latency_ms": lat * 1e3,
                        "usage": usage, "chunk_times_s": stamps}
            elif t == "error":
                err = f.get("error") or {}
                raise RuntimeError(f"{err.get('code')}: {err.get('message')}")
