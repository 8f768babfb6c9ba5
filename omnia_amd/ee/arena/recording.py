"""Arena run recording into session-api (``ee/cmd/arena-worker/session_recording.go``).

Every conversation an arena worker plays (one scenario x provider x trial run,
or each self-play run) becomes a session in session-api, so the dashboard and
the eval pipeline see arena traffic exactly like live traffic:

* the session id is a name-based UUID (v5) of ``<work item id>:<run id>`` in
  an arena namespace: re-running a reclaimed item writes the SAME session
  instead of a duplicate;
* the agent name is the job, tags mark the origin (``source:arena``,
  ``arena-job:<job>``, ``scenario:<id>``, ``provider:<id>``, ``trial:<n>``) and
  the initial state carries the same facts under ``arena.*`` keys;
* the virtual user id is a pseudonym (keyed hash) of the run id;
* messages are appended turn by turn (user, then assistant with its token
  usage), and the session is closed ``completed`` -- or ``error`` when the run
  failed, so a failed run is visible as such;
* session creation is retried (3 attempts, exponential back-off from 0.5 s); a
  run whose session cannot be created is played but not recorded.
"""
from __future__ import annotations

import asyncio
import hashlib
import hmac
import logging
import uuid

log = logging.getLogger("omnia.arena.recording")

ARENA_SESSION_NS = uuid.UUID("6f6d6e69-612d-4172-656e-612d73657373")  # "omnia-arena-sess"
SOURCE_ARENA = "source:arena"


def session_uuid(work_item_id: str, run_id: str = "") -> str:
    return str(uuid.uuid5(ARENA_SESSION_NS, f"{work_item_id}:{run_id}"))


def pseudonym(run_id: str, key: bytes = b"omnia-arena") -> str:
    return hmac.new(key, run_id.encode(), hashlib.sha256).hexdigest()[:16]


class ArenaSessionRecorder:
    def __init__(self, client, job: str, namespace: str, workspace: str = "",
                 job_type: str = "evaluation", retries: int = 3, base_wait_s: float = 0.5):
        self.client = client  # SessionHTTPClient-like: write(method, path, body) -> bool
        self.job, self.namespace, self.workspace = job, namespace, workspace
        self.job_type = job_type
        self.retries, self.base_wait_s = retries, base_wait_s
        self.recorded: list[str] = []

    def tags(self, item, trial: str = "") -> list[str]:
        t = [SOURCE_ARENA, f"arena-job:{self.job}", f"scenario:{item.scenario_id}",
             f"provider:{item.provider_id}"]
        if trial:
            t.append(f"trial:{trial}")
        return t

    def state(self, item, run_id: str, trial: str = "") -> dict:
        st = {"arena.job": self.job, "arena.job.name": self.job,
              "arena.job.namespace": self.namespace, "arena.scenario": item.scenario_id,
              "arena.scenario.id": item.scenario_id, "arena.provider": item.provider_id,
              "arena.provider.id": item.provider_id, "arena.type": self.job_type}
        if run_id:
            st["arena.run_id"] = run_id
        if trial:
            st["arena.trial.index"] = trial
        return st

    async def _create(self, body: dict) -> bool:
        wait = self.base_wait_s
        for attempt in range(self.retries):
            try:
                if await self.client.write("POST", "/api/v1/sessions", body):
                    return True
            except Exception as e:  # noqa: BLE001 -- retried, then logged
                log.debug("arena session create failed: %s", e)
            if attempt + 1 < self.retries:
                await asyncio.sleep(wait)
                wait *= 2
        return False

    async def record(self, item, result: dict, run_id: str = "") -> str | None:
        """Write one played run; returns the session id (None: not recorded)."""
        trial = str((item.config or {}).get("trial", "")) if hasattr(item, "config") else ""
        run_id = run_id or item.id
        sid = session_uuid(item.id, run_id)
        body = {"id": sid, "agentName": self.job, "namespace": self.namespace,
                "workspaceName": self.workspace, "tags": self.tags(item, trial),
                "state": self.state(item, run_id, trial), "virtualUserId": pseudonym(run_id)}
        if not await self._create(body):
            log.warning("arena run %s of item %s not recorded: session-api unavailable",
                        run_id, item.id)
            return None
        for t in result.get("turns") or []:
            if t.get("user") is not None:
                await self.client.write("POST", f"/api/v1/sessions/{sid}/messages",
                                        {"role": "user", "content": t["user"]})
            u = t.get("usage") or {}
            msg = {"role": "assistant", "content": t.get("content", ""),
                   "metadata": {"ttft_ms": str(round(t.get("ttft_ms") or 0.0, 3)),
                                "latency_ms": str(round(t.get("latency_ms") or 0.0, 3))}}
            if u:
                msg.update(outputTokens=int(u.get("output_tokens") or 0),
                           costUsd=float(u.get("cost") or 0.0))
            await self.client.write("POST", f"/api/v1/sessions/{sid}/messages", msg)
        failed = bool(result.get("error")) or not result.get("passed", True)
        await self.client.write("PATCH", f"/api/v1/sessions/{sid}/status",
                                {"status": "error" if failed else "completed"})
        self.recorded.append(sid)
        return sid
