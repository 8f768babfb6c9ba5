"""session-api HTTP client with a fixed-capacity retry ring buffer
(``pkg/session/httpclient/{store,buffer}.go``): failed writes are parked in a
drop-oldest ring and retried in the background, so a session-api outage never
blocks a turn.  Also the runtime's event sink (``internal/runtime/event_store.go``)
and the facade's async recording pool (``internal/facade/recording_pool.go``:
100 workers, 1000-deep queue, drops counted).
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging
import time

from ..observability import metrics as M

log = logging.getLogger("omnia.session.client")


class RingBuffer:
    def __init__(self, capacity: int = 1000):
        self.q: collections.deque = collections.deque(maxlen=capacity)
        self.dropped = 0

    def push(self, item):
        if len(self.q) == self.q.maxlen:
            self.dropped += 1
        self.q.append(item)

    def drain(self, n: int | None = None) -> list:
        out = []
        while self.q and (n is None or len(out) < n):
            out.append(self.q.popleft())
        return out

    def __len__(self):
        return len(self.q)


class SessionHTTPClient:
    def __init__(self, base_url: str, token: str | None = None, buffer: int = 1000,
                 timeout_s: float = 5.0):
        self.base = base_url.rstrip("/")
        self.token = token
        self.ring = RingBuffer(buffer)
        self.timeout_s = timeout_s
        self._session = None

    async def _sess(self):
        import aiohttp

        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout_s))
        return self._session

    def _h(self):
        return {"Authorization": f"Bearer {self.token}"} if self.token else {}

    async def request(self, method: str, path: str, body=None):
        s = await self._sess()
        async with s.request(method, self.base + path, json=body, headers=self._h()) as r:
            if r.status >= 500:
                raise ConnectionError(f"session-api {r.status}")
            if r.status == 204:
                return None
            data = await r.json(content_type=None) if r.content_length != 0 else None
            if r.status >= 400:
                raise KeyError(data)
            return data

    async def write(self, method: str, path: str, body=None) -> bool:
        """Best-effort write; on transport failure park it in the ring buffer."""
        try:
            await self.request(method, path, body)
            return True
        except (ConnectionError, OSError, asyncio.TimeoutError) as e:
            log.debug("session write parked: %s", e)
            self.ring.push((method, path, body, time.time()))
            return False
        except Exception as e:  # noqa: BLE001 - 4xx: not retryable
            log.debug("session write rejected: %s", e)
            return False

    async def flush(self) -> int:
        n = 0
        for method, path, body, _ in self.ring.drain():
            try:
                await self.request(method, path, body)
                n += 1
            except (ConnectionError, OSError, asyncio.TimeoutError):
                self.ring.push((method, path, body, time.time()))
                break
            except Exception:  # noqa: BLE001
                continue
        return n

    # ---- convenience
    async def ensure_session(self, sid, agent, namespace, meta=None):
        return await self.write("POST", "/api/v1/sessions", {
            "id": sid, "agentName": agent, "namespace": namespace,
            "state": {k: str(v) for k, v in (meta or {}).items()},
            "virtualUserId": (meta or {}).get("user", "")})

    async def append(self, sid, role, content, usage=None, meta=None):
        body = {"role": role, "content": content, "metadata": meta or {}}
        if usage:
            body.update(inputTokens=usage.get("input_tokens", 0),
                        outputTokens=usage.get("output_tokens", 0),
                        costUsd=usage.get("cost_usd", 0.0))
        return await self.write("POST", f"/api/v1/sessions/{sid}/messages", body)

    async def close_session(self, sid, status="completed"):
        return await self.write("PATCH", f"/api/v1/sessions/{sid}/status", {"status": status})

    async def get_messages(self, sid):
        return (await self.request("GET", f"/api/v1/sessions/{sid}/messages"))["messages"]

    async def get_privacy_policy(self, namespace: str, agent: str) -> dict | None:
        """``GET /api/v1/privacy-policy`` (``pkg/session/httpclient/store.go:808-848``):
        the effective policy's ``recording`` block for a namespace / agent, or
        None when no policy applies (204).  A config read: it never goes
        through the write ring buffer."""
        from urllib.parse import urlencode

        return await self.request(
            "GET", "/api/v1/privacy-policy?" + urlencode({"namespace": namespace,
                                                           "agent": agent}))

    async def close(self):
        if self._session is not None:
            await self._session.close()


class SessionEventSink:
    """Runtime-side recorder of provider calls / eval results / events."""

    def __init__(self, base_url: str, token: str | None = None):
        self.client = SessionHTTPClient(base_url, token)

    async def record(self, session_id: str, kind: str, payload: dict):
        if kind == "provider_call":
            await self.client.write("POST", f"/api/v1/sessions/{session_id}/provider-calls", {
                "provider": payload.get("provider"), "model": payload.get("model"),
                "inputTokens": payload.get("input_tokens", 0),
                "outputTokens": payload.get("output_tokens", 0),
                "cachedTokens": payload.get("cached_tokens", 0),
                "costUsd": payload.get("cost_usd", 0.0)})
        elif kind == "tool_call":
            body = {"callId": payload.get("call_id", ""), "name": payload.get("name", ""),
                    "status": payload.get("status", "success"),
                    "durationMs": payload.get("duration_ms", 0)}
            if payload.get("arguments") is not None:
                body["arguments"] = payload["arguments"]
            if payload.get("result") is not None:
                body["result"] = payload["result"]
            if payload.get("error"):
                body["errorMessage"] = payload["error"]
            await self.client.write("POST", f"/api/v1/sessions/{session_id}/tool-calls", body)
        elif kind == "eval_result":
            await self.client.write("POST", "/api/v1/eval-results", {
                "sessionId": session_id, "evalId": payload.get("id"),
                "evalType": payload.get("type"), "passed": payload.get("passed", True),
                "score": payload.get("score", 0.0)})
        else:
            await self.client.write("POST", f"/api/v1/sessions/{session_id}/events",
                                    {"type": kind, "data": payload})


def _default_recording() -> dict:
    return {"recording": {"enabled": True, "facadeData": True, "runtimeData": True}}


class RecordingPolicyCache:
    """The facade's view of the effective privacy policy for its one namespace /
    agent (``internal/facade/recording_policy.go``): fetched from session-api,
    cached ``ttl_s``; no policy (204) or a failed fetch records everything
    (fail open, so a transient error never silently drops data)."""

    def __init__(self, fetch, namespace: str, agent: str, ttl_s: float = 60.0,
                 now=time.monotonic):
        self.fetch, self.namespace, self.agent = fetch, namespace, agent
        self.ttl_s, self.now = ttl_s, now
        self.cached: dict | None = None
        self.fetched_at = 0.0
        self.fetches = 0
        self._lock: asyncio.Lock | None = None

    async def get(self) -> dict:
        if self.cached is not None and self.now() - self.fetched_at < self.ttl_s:
            return self.cached
        if self._lock is None:
            self._lock = asyncio.Lock()
        async with self._lock:  # one fetch however many recorders ask at once
            if self.cached is not None and self.now() - self.fetched_at < self.ttl_s:
                return self.cached
            return await self._refresh()

    async def _refresh(self) -> dict:
        self.fetches += 1
        try:
            p = await self.fetch(self.namespace, self.agent)
        except Exception as e:  # noqa: BLE001 - fail open
            log.debug("privacy policy fetch failed, recording enabled: %s", e)
            p = None
        self.cached = p if isinstance(p, dict) and "recording" in p else _default_recording()
        self.fetched_at = self.now()
        return self.cached

    @staticmethod
    def allows(policy: dict | None, role: str) -> bool:
        """User turns are facade data, everything else (assistant turns) runtime
        data; both need ``recording.enabled``."""
        if not policy:
            return True
        rec = policy.get("recording") or {}
        if not rec.get("enabled", True):
            return False
        return bool(rec.get("facadeData" if role == "user" else "runtimeData", True))


class RecordingPool:
    """Facade-side async recorder: N workers over a bounded queue; drops counted.
    ``policy`` (:class:`RecordingPolicyCache`) gates each message by role."""

    def __init__(self, store, workers: int = 100, queue: int = 1000, policy=None):
        self.store = store  # has ensure_session/append/close_session coroutines
        self.policy = policy
        self.gated = 0
        self.q: asyncio.Queue | None = None
        self.workers = workers
        self.queue_size = queue
        self.tasks: list = []
        self.dropped = 0

    def _start(self):
        if self.q is None:
            self.q = asyncio.Queue(self.queue_size)
            for _ in range(self.workers):
                self.tasks.append(asyncio.get_running_loop().create_task(self._work()))

    async def _work(self):
        while True:
            item = await self.q.get()
            try:
                await item()
            except Exception as e:  # noqa: BLE001
                log.debug("recording failed: %s", e)
            finally:
                self.q.task_done()

    async def ensure_session(self, sid, agent, namespace, meta=None):
        await self.store.ensure_session(sid, agent, namespace, meta)

    async def _allowed(self, role) -> bool:
        if self.policy is None:
            return True
        ok = RecordingPolicyCache.allows(await self.policy.get(), role)
        if not ok:
            self.gated += 1
        return ok

    def submit(self, sid, role, content, usage=None):
        self._start()
        try:
            self.q.put_nowait(lambda: self.record(sid, role, content, usage))
        except asyncio.QueueFull:
            self.dropped += 1
            M.RECORDING_DROPPED.inc()

    async def record(self, sid, role, content, usage=None):
        if await self._allowed(role):
            await self.store.append(sid, role, content, usage)

    async def close_session(self, sid):
        await self.store.close_session(sid)

    async def join(self):
        if self.q is not None:
            await self.q.join()

    async def stop(self):
        for t in self.tasks:
            t.cancel()


class LocalSessionStore:
    """In-process adapter over TieredSessionService with the client's API (single-node)."""

    def __init__(self, svc):
        self.svc = svc

    async def ensure_session(self, sid, agent, namespace, meta=None):
        from .model import Session

        self.svc.create(Session(id=sid, agent_name=agent, namespace=namespace,
                                state={k: str(v) for k, v in (meta or {}).items()},
                                virtual_user_id=(meta or {}).get("user", "")))

    async def append(self, sid, role, content, usage=None, meta=None):
        from .model import Message

        u = usage or {}
        await self.svc.append_message(sid, Message(role=role, content=content,
                                                   metadata=meta or {},
                                                   input_tokens=u.get("input_tokens", 0),
                                                   output_tokens=u.get("output_tokens", 0),
                                                   cost_usd=u.get("cost_usd", 0.0)))

    async def close_session(self, sid, status="completed"):
        self.svc.update_status(sid, status)
