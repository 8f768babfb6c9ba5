"""Arena scenarios generated from recorded sessions (``ee/pkg/arena/sources``).

Production traffic is the best regression suite: sessions whose evals failed
(or passed) are listed through session-api's cross-session eval-results query,
de-duplicated by session, and each becomes an arena scenario that replays the
conversation's user turns against a provider under test, carrying the evals
that were recorded on it:

* eval results attached to a message (``messageId``) become assertions of the
  turn whose assistant reply that message was;
* session-level results (no ``messageId``) become conversation assertions;
* an assertion's ``params`` are the result's recorded ``details``, its message
  the eval id (``convert.go:evalMessage``) -- and a result whose message id
  is not in the transcript is dropped.

The scenario id is stable (``session-<id prefix>``), so a regenerated suite
overwrites rather than duplicates; ``metadata`` keeps the source session, the
agent it ran on, and which evals it originally failed."""
from __future__ import annotations

ADAPTER = "omnia"


def _assertion(r: dict) -> dict:
    return {"type": r.get("evalType") or r.get("evalId") or "eval",
            "id": r.get("evalId") or "", "params": dict(r.get("details") or {}),
            "recorded": {"passed": bool(r.get("passed")), "score": r.get("score")},
            "message": r.get("evalId") or ""}


def convert_eval_results(results: list[dict], messages: list[dict]):
    """-> (conversation assertions, {message index: [turn assertions]})."""
    idx = {m.get("id"): i for i, m in enumerate(messages) if m.get("id")}
    conv, turns = [], {}
    for r in results:
        mid = r.get("messageId") or ""
        if not mid:
            conv.append(_assertion(r))
        elif mid in idx:
            turns.setdefault(idx[mid], []).append(_assertion(r))
    return conv, turns


def session_to_scenario(session: dict, messages: list[dict], results: list[dict]) -> dict:
    conv, per_msg = convert_eval_results(results, messages)
    turns, system = [], None
    for i, m in enumerate(messages):
        role = m.get("role")
        if role == "system" and system is None:
            system = m.get("content", "")
        elif role == "user":
            turns.append({"user": m.get("content", ""), "assertions": [],
                          "reference": None})
        elif role == "assistant" and turns:
            t = turns[-1]
            if t["reference"] is None:
                t["reference"] = m.get("content", "")
            t["assertions"].extend(per_msg.get(i, []))
    sid = session.get("id", "")
    scen = {"id": f"session-{sid[:12]}", "source": ADAPTER,
            "turns": [t for t in turns if t["user"]],
            "conversation_assertions": conv,
            "metadata": {"sessionId": sid, "agentName": session.get("agentName", ""),
                         "namespace": session.get("namespace", ""),
                         "createdAt": session.get("createdAt"),
                         "failedEvals": sorted({r.get("evalId", "") for r in results
                                                if not r.get("passed")})}}
    if system:
        scen["system"] = system
    return scen


class SessionAPISource:
    """List / fetch recorded sessions as arena scenarios.  ``client`` needs
    ``request(method, path)`` returning parsed JSON (``SessionHTTPClient``)."""

    name = ADAPTER

    def __init__(self, client):
        self.client = client

    async def list(self, passed: bool | None = False, eval_id: str = "",
                   limit: int = 20) -> list[dict]:
        q = []
        if passed is not None:
            q.append(f"passed={'true' if passed else 'false'}")
        if eval_id:
            q.append(f"evalId={eval_id}")
        if limit:
            q.append(f"limit={limit * 5}")  # over-fetch: several results per session
        rows = (await self.client.request("GET", "/api/v1/eval-results" +
                                          ("?" + "&".join(q) if q else "")))["results"]
        seen, out = set(), []
        for r in rows:
            sid = r.get("sessionId")
            if not sid or sid in seen:
                continue
            seen.add(sid)
            s = await self.client.request("GET", f"/api/v1/sessions/{sid}")
            out.append({"id": sid, "source": ADAPTER, "providerId": s.get("agentName", ""),
                        "timestamp": s.get("createdAt"), "messageCount":
                        s.get("messageCount", 0), "evalId": r.get("evalId", "")})
            if limit and len(out) >= limit:
                break
        return out

    async def get(self, session_id: str) -> dict:
        s = await self.client.request("GET", f"/api/v1/sessions/{session_id}")
        msgs = (await self.client.request("GET",
                                          f"/api/v1/sessions/{session_id}/messages"))["messages"]
        res = (await self.client.request(
            "GET", f"/api/v1/sessions/{session_id}/eval-results"))["results"]
        return session_to_scenario(s, msgs, res)

    async def scenarios(self, passed: bool | None = False, eval_id: str = "",
                        limit: int = 20) -> list[dict]:
        return [await self.get(x["id"]) for x in await self.list(passed, eval_id, limit)]
