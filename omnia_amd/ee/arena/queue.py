"""Arena work queue (``ee/pkg/arena/queue``).

Items are JSON on a Redis Stream ``omnia:arena:queue:<job>`` read through the
consumer group ``arena-workers``; results land in the hash
``omnia:arena:results:<job>`` (item id -> result JSON).  Unacked items idle for
longer than ``visibility_s`` are reclaimed by another worker (``XCLAIM``), up to
``max_attempts``.  :class:`MemoryQueue` has the same interface in-process.
"""
from __future__ import annotations

import asyncio
import json
import time
import uuid
from dataclasses import asdict, dataclass, field

PENDING, PROCESSING, COMPLETED, FAILED = "pending", "processing", "completed", "failed"
GROUP = "arena-workers"


@dataclass
class WorkItem:
    job_id: str
    scenario_id: str
    provider_id: str = ""
    config: dict = field(default_factory=dict)
    id: str = field(default_factory=lambda: uuid.uuid4().hex[:12])
    status: str = PENDING
    attempt: int = 0
    max_attempts: int = 3
    created_at: float = field(default_factory=time.time)
    stream_id: str = ""

    def to_json(self) -> str:
        d = asdict(self)
        d.pop("stream_id")
        return json.dumps(d)

    @classmethod
    def from_json(cls, s, stream_id: str = "") -> "WorkItem":
        d = json.loads(s)
        return cls(**{k: v for k, v in d.items() if k in cls.__dataclass_fields__},
                   stream_id=stream_id)


def _failed(item: WorkItem, error: str) -> dict:
    """The result of an item that exhausted its attempts."""
    return {"passed": False, "error": error or "unknown error", "scenario": item.scenario_id,
            "provider": item.provider_id, "item_id": item.id, "attempt": item.attempt}


class MemoryQueue:
    def __init__(self):
        self.items: dict[str, list[WorkItem]] = {}
        self.results: dict[str, dict[str, dict]] = {}
        self.inflight: dict[str, dict[str, tuple[WorkItem, float]]] = {}
        self._lock = asyncio.Lock()

    async def enqueue(self, items: list[WorkItem]):
        for it in items:
            self.items.setdefault(it.job_id, []).append(it)

    async def claim(self, job_id: str, consumer: str, n: int = 1) -> list[WorkItem]:
        async with self._lock:
            q = self.items.get(job_id, [])
            out, self.items[job_id] = q[:n], q[n:]
            now = time.time()
            for it in out:
                it.attempt += 1
                it.status = PROCESSING
                self.inflight.setdefault(job_id, {})[it.id] = (it, now)
            return out

    async def complete(self, item: WorkItem, result: dict):
        self.inflight.get(item.job_id, {}).pop(item.id, None)
        self.results.setdefault(item.job_id, {})[item.id] = result

    async def fail(self, item: WorkItem, error: str):
        self.inflight.get(item.job_id, {}).pop(item.id, None)
        if item.attempt < item.max_attempts:
            await self.enqueue([item])
        else:
            self.results.setdefault(item.job_id, {})[item.id] = _failed(item, error)

    async def reclaim(self, job_id: str, visibility_s: float) -> int:
        now, n = time.time(), 0
        for iid, (it, t) in list(self.inflight.get(job_id, {}).items()):
            if now - t >= visibility_s:
                del self.inflight[job_id][iid]
                if it.attempt < it.max_attempts:
                    await self.enqueue([it])
                    n += 1
        return n

    async def results_of(self, job_id: str) -> list[dict]:
        return list(self.results.get(job_id, {}).values())

    async def progress(self, job_id: str) -> dict:
        return {"pending": len(self.items.get(job_id, [])),
                "processing": len(self.inflight.get(job_id, {})),
                "done": len(self.results.get(job_id, {}))}


class StreamQueue:
    def __init__(self, redis):
        self.r = redis
        self._groups: set[str] = set()

    @staticmethod
    def _stream(job):
        return f"omnia:arena:queue:{job}"

    async def _group(self, job):
        if job not in self._groups:
            await self.r.xgroup_create(self._stream(job), GROUP, "0")
            self._groups.add(job)

    async def enqueue(self, items: list[WorkItem]):
        for it in items:
            await self._group(it.job_id)
            await self.r.xadd(self._stream(it.job_id), {"item": it.to_json()})
            await self.r.execute("HINCRBY", f"omnia:arena:meta:{it.job_id}", "enqueued", 1)

    async def claim(self, job_id: str, consumer: str, n: int = 1) -> list[WorkItem]:
        await self._group(job_id)
        resp = await self.r.xreadgroup(GROUP, consumer, {self._stream(job_id): ">"}, count=n)
        out = []
        for _stream, entries in resp or []:
            for sid, fields in entries:
                f = dict(zip(fields[::2], fields[1::2]))
                raw = f.get(b"item") or f.get("item")
                it = WorkItem.from_json(raw, sid.decode() if isinstance(sid, bytes) else sid)
                it.attempt += 1
                it.status = PROCESSING
                await self.r.execute("HSET", f"omnia:arena:inflight:{job_id}", it.stream_id,
                                     json.dumps({"t": time.time(), "item": it.to_json()}))
                out.append(it)
        return out

    async def _ack(self, item):
        await self.r.xack(self._stream(item.job_id), GROUP, item.stream_id)
        await self.r.execute("HDEL", f"omnia:arena:inflight:{item.job_id}", item.stream_id)

    async def complete(self, item: WorkItem, result: dict):
        await self.r.execute("HSET", f"omnia:arena:results:{item.job_id}", item.id,
                             json.dumps(result))
        await self._ack(item)

    async def fail(self, item: WorkItem, error: str):
        await self._ack(item)
        if item.attempt < item.max_attempts:
            item.status = PENDING
            await self.r.xadd(self._stream(item.job_id), {"item": item.to_json()})
        else:
            await self.r.execute("HSET", f"omnia:arena:results:{item.job_id}", item.id,
                                 json.dumps(_failed(item, error)))

    async def reclaim(self, job_id: str, visibility_s: float) -> int:
        raw = await self.r.execute("HGETALL", f"omnia:arena:inflight:{job_id}") or []
        now, n = time.time(), 0
        for sid, v in zip(raw[::2], raw[1::2]):
            d = json.loads(v)
            if now - d["t"] < visibility_s:
                continue
            it = WorkItem.from_json(d["item"], sid.decode() if isinstance(sid, bytes) else sid)
            await self._ack(it)
            if it.attempt < it.max_attempts:
                await self.r.xadd(self._stream(job_id), {"item": it.to_json()})
                n += 1
        return n

    async def results_of(self, job_id: str) -> list[dict]:
        raw = await self.r.execute("HGETALL", f"omnia:arena:results:{job_id}") or []
        return [json.loads(v) for v in raw[1::2]]

    async def progress(self, job_id: str) -> dict:
        enq = await self.r.execute("HGET", f"omnia:arena:meta:{job_id}", "enqueued")
        done = len(await self.results_of(job_id))
        infl = await self.r.execute("HGETALL", f"omnia:arena:inflight:{job_id}") or []
        total = int(enq or 0)
        return {"pending": max(0, total - done - len(infl) // 2), "processing": len(infl) // 2,
                "done": done}
