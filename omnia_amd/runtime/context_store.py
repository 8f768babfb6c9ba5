"""Conversation working-context store (``spec.context``: memory | redis, TTL 24h).

Mirrors the PromptKit statestore the reference configures in
``pkg/runtime/promptkit/serveropts.go:93-146``: the runtime persists each
session's transcript after every turn, ``HasConversation`` answers from the
same store with three states (``runtime.proto:363-394``) and an unreachable
store is reported as UNAVAILABLE, never as an expiry.
"""
from __future__ import annotations

import json
import time

from ..utils.resp import RedisClient

DEFAULT_TTL_S = 24 * 3600  # api/v1alpha1/agentruntime_types.go:258-261


class StoreUnavailable(Exception):
    pass


class MemoryContextStore:
    kind = "memory"

    def __init__(self, ttl_s: int = DEFAULT_TTL_S):
        self.ttl_s = ttl_s
        self._d: dict[str, tuple[float, dict]] = {}
        self.fail = False  # fault injection for tests

    async def load(self, session_id: str) -> dict | None:
        if self.fail:
            raise StoreUnavailable("memory store failure injected")
        v = self._d.get(session_id)
        if v is None:
            return None
        exp, state = v
        if exp < time.time():
            self._d.pop(session_id, None)
            return None
        return json.loads(json.dumps(state))

    async def save(self, session_id: str, state: dict) -> None:
        if self.fail:
            raise StoreUnavailable("memory store failure injected")
        self._d[session_id] = (time.time() + self.ttl_s, json.loads(json.dumps(state)))

    async def delete(self, session_id: str) -> None:
        self._d.pop(session_id, None)

    async def ping(self) -> bool:
        return not self.fail


class RedisContextStore:
    kind = "redis"

    def __init__(self, url: str, ttl_s: int = DEFAULT_TTL_S, prefix: str = "omnia:ctx:"):
        self.client = RedisClient(url)
        self.ttl_s = ttl_s
        self.prefix = prefix

    async def load(self, session_id: str) -> dict | None:
        try:
            v = await self.client.get(self.prefix + session_id)
        except Exception as e:  # noqa: BLE001
            raise StoreUnavailable(str(e)) from e
        return None if v is None else json.loads(v)

    async def save(self, session_id: str, state: dict) -> None:
        try:
            await self.client.set(self.prefix + session_id, json.dumps(state), ex=self.ttl_s)
        except Exception as e:  # noqa: BLE001
            raise StoreUnavailable(str(e)) from e

    async def delete(self, session_id: str) -> None:
        try:
            await self.client.delete(self.prefix + session_id)
        except Exception as e:  # noqa: BLE001
            raise StoreUnavailable(str(e)) from e

    async def ping(self) -> bool:
        try:
            return (await self.client.ping()) == "PONG"
        except Exception:  # noqa: BLE001
            return False


class NoStore:
    """No store configured: every probe is UNAVAILABLE (runtime.proto:388-392)."""

    kind = "none"

    async def load(self, session_id):
        raise StoreUnavailable("no context store configured")

    async def save(self, session_id, state):
        return None

    async def delete(self, session_id):
        return None

    async def ping(self):
        return False


def make_store(kind: str | None, url: str | None = None, ttl_s: int | None = None):
    ttl = ttl_s or DEFAULT_TTL_S
    if kind in (None, "", "memory"):
        return MemoryContextStore(ttl)
    if kind == "redis":
        return RedisContextStore(url or "redis://127.0.0.1:6379/0", ttl)
    if kind == "none":
        return NoStore()
    raise ValueError(f"unknown context store {kind!r}")


def parse_ttl(s: str | None) -> int | None:
    """Go-duration subset: 24h, 30m, 90s, 1h30m."""
    if not s:
        return None
    total, num = 0, ""
    units = {"h": 3600, "m": 60, "s": 1}
    for ch in s.strip():
        if ch.isdigit() or ch == ".":
            num += ch
        elif ch in units and num:
            total += float(num) * units[ch]
            num = ""
        else:
            raise ValueError(f"bad duration {s!r}")
    if num:
        total += float(num)
    return int(total)
