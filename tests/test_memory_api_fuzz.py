"""HTTP input fuzzing of the memory-api REST surface (memory/api.py, EE routes
on): bad query parameters and request bodies of the wrong JSON type answer 4xx,
never a 500 from an unhandled exception (reference: typed Go decoders in
``internal/memory/api``)."""
import asyncio
import json

from aiohttp.test_utils import TestClient, TestServer
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from omnia_amd.memory.api import build_app
from omnia_amd.memory.embedding import HashEmbedder
from omnia_amd.memory.service import MemoryService
from omnia_amd.memory.store import MemoryStore

JSON = st.recursive(st.none() | st.booleans() | st.integers(-3, 10**6)
                    | st.floats(allow_nan=False, allow_infinity=False) | st.text(max_size=6),
                    lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=8), c,
                                                                         max_size=3),
                    max_leaves=8)
QVAL = st.one_of(st.text(max_size=5), st.integers(-3, 5).map(str),
                 st.sampled_from(["true", "", "-1", "1e9", "nan", "abc", "0.5"]))
QKEYS = ["workspace", "user_id", "agent_id", "limit", "offset", "q", "type", "min_confidence",
         "scope", "purpose", "tier", "category", "since", "ids"]
BODY_KEYS = ["content", "type", "workspace", "user_id", "agent_id", "confidence", "metadata",
             "scope", "ids", "query", "limit", "memory_id", "old_id", "new_id", "relation",
             "source_id", "target_id", "purpose", "text", "title", "category", "expires_at",
             "tier", "min_confidence", "types", "event", "granted"]
BODY = st.one_of(st.dictionaries(st.sampled_from(BODY_KEYS), JSON, max_size=6).map(json.dumps),
                 JSON.map(json.dumps), st.sampled_from(["", "{", "[]", "null"]))
GETS = ["/api/v1/memories", "/api/v1/memories/search", "/api/v1/memories/export",
        "/api/v1/memories/aggregate", "/api/v1/memories/conflicts", "/api/v1/memories/stats",
        "/api/v1/memories/m1", "/api/v1/institutional/memories",
        "/api/v1/ingest/summary-candidates", "/api/v1/agent-memories"]
POSTS = ["/api/v1/memories", "/api/v1/memories/supersede", "/api/v1/memories/retrieve",
         "/api/v1/memories/retrieve/semantic", "/api/v1/memories/consent-events",
         "/api/v1/relations", "/api/v1/institutional/memories", "/api/v1/institutional/ingest",
         "/api/v1/ingest/summaries", "/api/v1/agent-memories"]
DELETES = ["/api/v1/memories/batch", "/api/v1/memories/m1", "/api/v1/memories",
           "/api/v1/agent-memories/m1"]
REQ = st.one_of(
    st.tuples(st.just("GET"), st.sampled_from(GETS),
              st.dictionaries(st.sampled_from(QKEYS), QVAL, max_size=3), st.none()),
    st.tuples(st.just("POST"), st.sampled_from(POSTS),
              st.dictionaries(st.sampled_from(QKEYS), QVAL, max_size=2), BODY),
    st.tuples(st.just("DELETE"), st.sampled_from(DELETES),
              st.dictionaries(st.sampled_from(QKEYS), QVAL, max_size=3), BODY))


async def _send(reqs):
    svc = MemoryService(MemoryStore(), HashEmbedder(64), device="cpu", enterprise=True)
    out = []
    async with TestClient(TestServer(build_app(svc, enterprise=True))) as c:
        for method, path, params, body in reqs:
            kw = {"params": params}
            if body is not None:
                kw.update(data=body, headers={"Content-Type": "application/json"})
            r = await asyncio.wait_for(c.request(method, path, **kw), 30)
            out.append((method, path, params, body, r.status, (await r.text())[:200]))
    return out


@given(st.lists(REQ, min_size=1, max_size=5))
@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
def test_memory_api_never_answers_500(reqs):
    for method, path, params, body, status, text in asyncio.run(_send(reqs)):
        assert status < 500, (method, path, params, body, status, text)
