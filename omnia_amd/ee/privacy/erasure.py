"""DSAR erasure across service groups (``ee/pkg/privacy/fanout_eraser.go``,
``session_group_eraser.go``, ``session_eraser.go``, ``media_deleter.go``).

privacy-api holds no warm-store or object-store credentials: for every service
group of the workspace (:class:`GroupTarget`: session-api + memory-api URLs) the
:class:`FanOutSubjectEraser` asks that group's session-api to erase the subject's
sessions (:class:`SessionGroupEraser` -> ``POST
/api/v1/privacy/sessions/delete-by-user`` with user, workspace and an optional
date range) and that group's memory-api to delete the subject's memories.  A
failing group is recorded and the others still run.

Inside session-api, :class:`SessionTierEraser` does the session half: list the
user's sessions (workspace / date filters), delete each (warm + cold + hot), and
delete each session's media artifacts through a :class:`MediaDeleter` --
:class:`ObjectStoreMediaDeleter` lists and deletes every object under
``<prefix><session_id>/`` through an object-store client
(``list_objects(bucket, prefix)`` / ``delete_objects(bucket, keys)``);
:class:`LocalMediaDeleter` removes ``<root>/sessions/<session_id>/`` of the
local media store.  A per-session failure is recorded and does not abort the
run.
"""
from __future__ import annotations

import logging
import os
import shutil
from dataclasses import dataclass

log = logging.getLogger("omnia.privacy.erasure")


@dataclass
class GroupTarget:
    name: str
    session_url: str = ""
    memory_url: str = ""


@dataclass
class EraseScope:
    virtual_user_id: str
    workspace: str = ""
    date_from: float | None = None  # unix seconds
    date_to: float | None = None

    def to_json(self) -> dict:
        d = {"virtual_user_id": self.virtual_user_id}
        if self.workspace:
            d["workspace"] = self.workspace
        if self.date_from is not None:
            d["date_from"] = self.date_from
        if self.date_to is not None:
            d["date_to"] = self.date_to
        return d


# ------------------------------------------------------------------ media
class MediaDeleter:
    async def delete_session_media(self, session_id: str) -> int:
        return 0


class NoOpMediaDeleter(MediaDeleter):
    pass


class ObjectStoreMediaDeleter(MediaDeleter):
    def __init__(self, client, bucket: str, prefix: str = ""):
        self.client, self.bucket, self.prefix = client, bucket, prefix

    async def delete_session_media(self, session_id: str) -> int:
        keys = await self.client.list_objects(self.bucket, f"{self.prefix}{session_id}/")
        if keys:
            await self.client.delete_objects(self.bucket, keys)
        return len(keys)


class LocalMediaDeleter(MediaDeleter):
    """The local media store's layout (``omnia_amd/media.py``)."""

    def __init__(self, root: str):
        self.root = root

    async def delete_session_media(self, session_id: str) -> int:
        d = os.path.join(self.root, "sessions", session_id)
        if not os.path.isdir(d):
            return 0
        n = sum(1 for f in os.listdir(d) if not f.endswith(".json"))
        shutil.rmtree(d)
        return n


# ------------------------------------------------------------------ session tier
class SessionTierEraser:
    """The session-api half of a DSAR (runs inside session-api)."""

    def __init__(self, svc, media: MediaDeleter | None = None):
        self.svc = svc  # TieredSessionService
        self.media = media or NoOpMediaDeleter()

    async def erase(self, scope: EraseScope) -> dict:
        rows = self.svc.warm.list_sessions(user=scope.virtual_user_id, limit=1_000_000)
        deleted, media, errors = 0, 0, []
        for s in rows:
            if scope.workspace and s.workspace_name not in ("", scope.workspace):
                continue
            created = s.created_at or 0.0
            if scope.date_from is not None and created < scope.date_from:
                continue
            if scope.date_to is not None and created > scope.date_to:
                continue
            try:
                if self.svc.delete(s.id):
                    deleted += 1
                media += await self.media.delete_session_media(s.id)
            except Exception as e:  # noqa: BLE001 - one session never aborts the run
                errors.append(f"session {s.id}: {e}")
        return {"sessions_deleted": deleted, "media_deleted": media, "errors": errors}


# ------------------------------------------------------------------ privacy-api side
class SessionGroupEraser:
    def __init__(self, token: str = "", timeout_s: float = 60.0):
        self.token, self.timeout_s = token, timeout_s

    async def erase(self, session_url: str, scope: EraseScope) -> dict:
        import aiohttp

        headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        async with aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=self.timeout_s)) as s:
            async with s.post(f"{session_url.rstrip('/')}/api/v1/privacy/sessions/"
                              f"delete-by-user", json=scope.to_json(), headers=headers) as r:
                if not 200 <= r.status < 300:
                    raise RuntimeError(f"delete-by-user returned HTTP {r.status}")
                return await r.json()


class MemoryHTTPDeleter:
    def __init__(self, memory_url: str, token: str = ""):
        self.url, self.token = memory_url.rstrip("/"), token

    async def delete_all(self, user: str, workspace: str) -> None:
        import aiohttp

        headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        async with aiohttp.ClientSession() as s:
            async with s.delete(f"{self.url}/api/v1/memories", headers=headers,
                                params={"workspace": workspace, "virtual_user_id": user}) as r:
                if not 200 <= r.status < 300:
                    raise RuntimeError(f"HTTP {r.status}")


class FanOutSubjectEraser:
    def __init__(self, groups: list[GroupTarget], workspaces: list[str] | None = None,
                 session_eraser: SessionGroupEraser | None = None, memory_deleter=None):
        self.groups = groups
        self.workspaces = workspaces or []
        self.session_eraser = session_eraser or SessionGroupEraser()
        self.memory_deleter = memory_deleter or (lambda url: MemoryHTTPDeleter(url))

    async def erase_subject(self, req: dict) -> tuple[int, list[str]]:
        if not self.groups:
            log.info("DSAR fan-out has no service-group targets; nothing erased")
            return 0, []
        scope = EraseScope(req["virtualUserId"], req.get("workspace", ""),
                           req.get("dateFrom"), req.get("dateTo"))
        total, errs = 0, []
        for g in self.groups:
            if g.session_url and req.get("scope", "all") in ("all", "sessions"):
                try:
                    res = await self.session_eraser.erase(g.session_url, scope)
                    total += int(res.get("sessions_deleted", 0))
                    errs += [f"group {g.name}: {e}" for e in res.get("errors") or []]
                except Exception as e:  # noqa: BLE001
                    errs.append(f"group {g.name} sessions: {e}")
            if g.memory_url and req.get("scope", "all") in ("all", "memories"):
                wss = [req["workspace"]] if req.get("workspace") else self.workspaces
                for ws in wss:
                    try:
                        await self.memory_deleter(g.memory_url).delete_all(
                            req["virtualUserId"], ws)
                    except Exception as e:  # noqa: BLE001
                        errs.append(f"group {g.name} memory {ws}: {e}")
        return total, errs
