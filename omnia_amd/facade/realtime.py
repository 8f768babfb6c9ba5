"""Realtime blip-resume: parking a live duplex call across a client reconnect.

Reference: ``internal/facade/realtime_registry.go:27-122`` (park / take /
expire with a grace timer), ``internal/facade/route_store.go`` (best-effort
route hint), ``internal/agent/route_store_redis.go:28-43`` (Redis store, keys
``rt:route:<session>``), wiring ``cmd/agent/websocket.go:211-232``
(``OMNIA_ROUTE_REDIS_URL``, ``OMNIA_GRACE_WINDOW_SECONDS`` default 15,
``POD_IP``:port as the pod address), and ``internal/facade/connection.go:
136-238`` / ``drain.go:40-104`` for the connection side.

When a WebSocket with a live audio call drops without a ``hangup``, the call
(its runtime Converse stream and relay) is parked under its session id and the
owner's identity, and a route hint ``session -> this pod`` is written with the
grace window as TTL so a router can send the reconnect back here.  A reconnect
``?resume=<session>`` by the same owner within the window takes the call back:
the runtime stream never noticed, and runtime output produced while parked is
replayed to the new socket.  Otherwise the grace timer closes the call, drops
the hint and completes the recorded session (only if it had been recorded).
The route store is a hint, never a source of truth: its failures are logged
and never break parking.
"""
from __future__ import annotations

import asyncio
import logging
import math
from dataclasses import dataclass

from ..observability import metrics as M

log = logging.getLogger("omnia.facade.realtime")

ROUTE_KEY_PREFIX = "rt:route:"


class NoopRouteStore:
    async def put_route(self, session_id: str, addr: str, ttl_s: float) -> None:
        return None

    async def delete_route(self, session_id: str) -> None:
        return None

    async def get_route(self, session_id: str) -> str | None:
        return None


class MemoryRouteStore(NoopRouteStore):
    def __init__(self):
        self.routes: dict[str, tuple[str, float]] = {}

    async def put_route(self, session_id, addr, ttl_s):
        self.routes[session_id] = (addr, asyncio.get_running_loop().time() + ttl_s)

    async def delete_route(self, session_id):
        self.routes.pop(session_id, None)

    async def get_route(self, session_id):
        v = self.routes.get(session_id)
        if v is None or v[1] < asyncio.get_running_loop().time():
            return None
        return v[0]


class RedisRouteStore(NoopRouteStore):
    """``SET rt:route:<sid> <addr> PX <ttl>`` over the in-repo RESP client."""

    def __init__(self, client):
        self.r = client

    async def put_route(self, session_id, addr, ttl_s):
        await self.r.execute("SET", ROUTE_KEY_PREFIX + session_id, addr, "PX",
                             max(1, int(math.ceil(ttl_s * 1000))))

    async def delete_route(self, session_id):
        await self.r.delete(ROUTE_KEY_PREFIX + session_id)

    async def get_route(self, session_id):
        v = await self.r.get(ROUTE_KEY_PREFIX + session_id)
        return v.decode() if isinstance(v, bytes) else v


def route_store_from_env(env: dict) -> NoopRouteStore:
    url = env.get("OMNIA_ROUTE_REDIS_URL", "")
    if not url:
        return NoopRouteStore()
    from ..utils.resp import RedisClient

    return RedisRouteStore(RedisClient(url))


@dataclass
class _Parked:
    session: object
    owner: str
    handle: asyncio.TimerHandle
    persisted: bool


class RealtimeRegistry:
    def __init__(self, routes=None, pod_addr: str = "", grace_s: float = 15.0,
                 on_expire=None):
        self.routes = routes or NoopRouteStore()
        self.pod_addr = pod_addr
        self.grace_s = grace_s
        self.on_expire = on_expire  # async (session_id, persisted) -> None
        self.parked: dict[str, _Parked] = {}
        self._tasks: set = set()

    def __len__(self) -> int:
        return len(self.parked)

    async def park(self, session_id: str, owner: str, session, persisted: bool):
        loop = asyncio.get_running_loop()
        old = self.parked.pop(session_id, None)
        if old is not None:  # a second drop of the same call: restart the window
            old.handle.cancel()
        h = loop.call_later(self.grace_s, self._fire, session_id)
        self.parked[session_id] = _Parked(session, owner, h, persisted)
        M.REALTIME_PARKED.inc()
        try:
            await self.routes.put_route(session_id, self.pod_addr, self.grace_s)
        except Exception as e:  # noqa: BLE001 - a hint, never a source of truth
            log.error("realtime route hint write failed for %s: %s", session_id, e)

    async def take(self, session_id: str, owner: str):
        """The parked call if present AND owned by ``owner`` (else None)."""
        p = self.parked.get(session_id)
        if p is None or p.owner != owner:
            return None
        del self.parked[session_id]
        p.handle.cancel()
        try:
            await self.routes.delete_route(session_id)
        except Exception as e:  # noqa: BLE001
            log.error("realtime route hint delete failed for %s: %s", session_id, e)
        M.REALTIME_REATTACHED.inc()
        return p.session

    def _fire(self, session_id: str):
        t = asyncio.get_running_loop().create_task(self.expire(session_id))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    async def expire(self, session_id: str):
        p = self.parked.pop(session_id, None)
        if p is None:
            return
        p.handle.cancel()
        try:
            await p.session.close()
        except Exception as e:  # noqa: BLE001
            log.error("parked session close failed for %s: %s", session_id, e)
        try:
            await self.routes.delete_route(session_id)
        except Exception as e:  # noqa: BLE001
            log.error("realtime route hint delete failed for %s: %s", session_id, e)
        M.REALTIME_PARK_EXPIRED.inc()
        if self.on_expire is not None:
            await self.on_expire(session_id, p.persisted)

    async def close_all(self):
        for sid in list(self.parked):
            await self.expire(sid)
