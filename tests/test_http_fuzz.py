"""HTTP input fuzzing of the session-api REST surface (session/api.py): bad
query parameters and request bodies of the wrong JSON type must come back as
4xx answers, never as a 500 from an unhandled exception.  The reference
validates with typed Go decoders (``internal/session/api``); here the same
contract is asserted over random inputs."""
import asyncio
import json

from aiohttp.test_utils import TestClient, TestServer
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from omnia_amd.session.api import build_app
from omnia_amd.session.model import Message, Session
from omnia_amd.session.store import TieredSessionService

JSON = st.recursive(st.none() | st.booleans() | st.integers(-5, 10**12)
                    | st.floats(allow_nan=False, allow_infinity=False) | st.text(max_size=6),
                    lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=8), c,
                                                                         max_size=3),
                    max_leaves=8)
QVAL = st.one_of(st.text(max_size=5), st.integers(-3, 5).map(str),
                 st.sampled_from(["true", "false", "", "-1", "1e9", "nan", "abc"]))
GETS = ["/api/v1/sessions", "/api/v1/sessions/search", "/api/v1/sessions/s1",
        "/api/v1/sessions/s1/messages", "/api/v1/eval-results", "/api/v1/eval-results/aggregate",
        "/api/v1/sessions/s1/eval-results", "/api/v1/sessions/s1/eval-results/summary",
        "/api/v1/provider-calls/aggregate", "/api/v1/sessions/s1/tool-calls",
        "/api/v1/sessions/nope/messages"]
POSTS = ["/api/v1/sessions", "/api/v1/sessions/s1/messages", "/api/v1/eval-results",
         "/api/v1/sessions/s1/ttl", "/api/v1/sessions/s1/tool-calls",
         "/api/v1/sessions/s1/provider-calls", "/api/v1/provider-usage",
         "/api/v1/sessions/s1/evaluate", "/api/v1/sessions/nope/messages"]
QKEYS = ["limit", "offset", "passed", "evalId", "namespace", "agent", "status", "q", "before",
         "after", "groupBy", "role"]


def _svc():
    svc = TieredSessionService()
    svc.create(Session(id="s1", agent_name="ag", namespace="ns"))
    asyncio.get_event_loop().run_until_complete(
        svc.append_message("s1", Message(role="user", content="hello")))
    return svc


async def _send(reqs):
    svc = TieredSessionService()
    svc.create(Session(id="s1", agent_name="ag", namespace="ns"))
    await svc.append_message("s1", Message(role="user", content="hello"))
    async with TestClient(TestServer(build_app(svc, rate=1e9, burst=1e9))) as c:
        out = []
        for method, path, params, body in reqs:
            if method == "GET":
                r = await c.get(path, params=params)
            else:
                r = await c.post(path, params=params, data=body,
                                 headers={"Content-Type": "application/json"})
            out.append((method, path, params, body, r.status, (await r.text())[:200]))
        return out


BODY_KEYS = ["id", "agentName", "namespace", "role", "content", "ttlSeconds", "status", "evalId",
             "passed", "score", "sessionId", "tags", "state", "messageId", "details", "name",
             "arguments", "result", "model", "inputTokens", "outputTokens", "costUsd", "metadata",
             "workspace", "usage", "endedAt", "expiresAt", "evalType", "durationMs"]
BODY = st.dictionaries(st.sampled_from(BODY_KEYS), JSON, max_size=6).map(json.dumps)

REQ = st.one_of(
    st.tuples(st.just("GET"), st.sampled_from(GETS),
              st.dictionaries(st.sampled_from(QKEYS), QVAL, max_size=3), st.none()),
    st.tuples(st.just("POST"), st.sampled_from(POSTS),
              st.dictionaries(st.sampled_from(QKEYS), QVAL, max_size=2),
              st.one_of(BODY, BODY, JSON.map(json.dumps),
                        st.sampled_from(["", "{", "[]", "null"]))))


@given(st.lists(REQ, min_size=1, max_size=6))
@settings(max_examples=250, deadline=None, suppress_health_check=[HealthCheck.too_slow])
def test_session_api_never_answers_500(reqs):
    for method, path, params, body, status, text in asyncio.run(_send(reqs)):
        assert status < 500, (method, path, params, body, status, text)
