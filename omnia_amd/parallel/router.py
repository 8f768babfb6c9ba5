"""Session-affine data-parallel replica router (SURVEY §2.3 DP row, §7.2 P4).

One engine replica per GPU (Llama-3-8B uses ~16 GB of a 288 GB MI355X, so the
rest is KV for resident sessions).  A session's KV prefix lives on exactly one
replica, so every turn of that session must land there: the router maps
``session_id -> replica`` by rendezvous (highest-random-weight) hashing.

* Stable: adding or losing a replica re-maps only the sessions that hashed to
  it (1/N of them), never reshuffles the rest -- their KV stays resident.
* Failure: a replica marked unhealthy (engine-core died, watchdog fault) drops
  out of the candidate set; its sessions re-hash to survivors and re-prefill
  from the transcript (the transcript is authoritative, as in the reference's
  ``sdk.Resume`` path, ``internal/runtime/conversation.go:260-276``).
* Sessionless requests (function-mode ``Invoke``) go to the least-loaded
  replica.
The reference scales with pod replicas behind a Service (no affinity); the
facade's Redis route table ``rt:route:<sid>`` (``SERVICES.md:178``) is the
cross-pod analogue of this in-node map.
"""
from __future__ import annotations

import hashlib
import threading


def _weight(session_id: str, replica: int) -> int:
    h = hashlib.blake2b(f"{replica}\x00{session_id}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little")


class ReplicaRouter:
    def __init__(self, n: int):
        if n < 1:
            raise ValueError("need at least one replica")
        self.n = n
        self.healthy = [True] * n
        self.inflight = [0] * n
        self.routed = [0] * n
        self._lock = threading.Lock()

    def candidates(self) -> list[int]:
        c = [i for i in range(self.n) if self.healthy[i]]
        if not c:
            raise RuntimeError("no healthy engine replica")
        return c

    def pick(self, session_id: str | None) -> int:
        with self._lock:
            cands = self.candidates()
            if session_id:
                r = max(cands, key=lambda i: _weight(session_id, i))
            else:
                r = min(cands, key=lambda i: (self.inflight[i], i))
            self.routed[r] += 1
            return r

    def acquire(self, r: int) -> None:
        with self._lock:
            self.inflight[r] += 1

    def release(self, r: int) -> None:
        with self._lock:
            self.inflight[r] -= 1

    def mark(self, r: int, healthy: bool) -> None:
        with self._lock:
            self.healthy[r] = healthy

    def snapshot(self) -> dict:
        with self._lock:
            return {"replicas": self.n, "healthy": list(self.healthy),
                    "inflight": list(self.inflight), "routed": list(self.routed)}


class ReplicatedEngine:
    """Drop-in for :class:`~omnia_amd.engine.engine.AsyncLLMEngine` over N replicas.

    ``replicas`` are engine objects with the AsyncLLMEngine surface (in-process
    engines or :class:`~omnia_amd.engine.core_proc.EngineCoreClient`, one per
    GPU).  The router keeps each session on one replica."""

    def __init__(self, replicas: list):
        if not replicas:
            raise ValueError("no replicas")
        self.replicas = replicas
        self.router = ReplicaRouter(len(replicas))
        self.engine = replicas[0].engine  # model_cfg / tokenizer shim

    @property
    def tokenizer(self):
        return self.replicas[0].tokenizer

    def replica_for(self, session_id: str | None) -> int:
        return self.router.pick(session_id)

    async def generate(self, prompt, params=None, session_id: str | None = None, **kw):
        r = self.router.pick(session_id)
        self.router.acquire(r)
        try:
            async for ev in self.replicas[r].generate(prompt, params, session_id=session_id, **kw):
                if getattr(ev, "finish_reason", None) == "error" and \
                        getattr(self.replicas[r], "error", None) is not None:
                    self.router.mark(r, False)  # dead engine-core: re-home its sessions
                yield ev
        finally:
            self.router.release(r)

    def health(self) -> bool:
        """Probe every replica, pull dead ones out of routing; healthy while any
        replica can serve (its sessions re-home to the survivors)."""
        alive = False
        for i, rep in enumerate(self.replicas):
            h = getattr(rep, "health", None)
            ok = bool(h()) if callable(h) else True
            self.router.mark(i, ok)
            alive = alive or ok
        return alive

    def drop_session(self, session_id: str):
        for rep in self.replicas:
            rep.drop_session(session_id)

    def has_session(self, session_id: str) -> bool:
        r = self.router.pick(session_id)
        return self.replicas[r].has_session(session_id)

    def synchronize(self):
        for rep in self.replicas:
            if hasattr(rep, "synchronize"):
                rep.synchronize()

    def stats(self) -> dict:
        per = [rep.stats() if hasattr(rep, "stats") else
               dict(getattr(getattr(rep.engine, "runner", None), "stats", {}) or {})
               for rep in self.replicas]
        out = {"router": self.router.snapshot(), "replicas": per}
        for k in ("generated_tokens", "prefill_tokens", "active"):
            vals = [p.get(k) for p in per if isinstance(p, dict) and isinstance(p.get(k),
                                                                             (int, float))]
            if vals:
                out[k] = sum(vals)
        return out

    def shutdown(self, timeout: float = 30.0):
        for rep in self.replicas:
            try:
                rep.shutdown(timeout)
            except TypeError:
                rep.shutdown()
