"""JSON-RPC input fuzzing of the A2A endpoint (facade/a2a.py): requests that
are not objects, params / messages / ids of the wrong JSON type, and unknown
methods get a JSON-RPC error (-32600 / -32601 / -32602 / -32001 / -32002) over a
200, never an HTTP 500 from an exception inside the handler."""
import asyncio
import json

from aiohttp.test_utils import TestClient, TestServer
from aiohttp import web
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from omnia_amd.facade.a2a import A2AServer
from omnia_amd.facade.runtime_client import InProcessRuntimeClient

from test_runtime import make_service

JSON = st.recursive(st.none() | st.booleans() | st.integers(-3, 9) | st.text(max_size=5),
                    lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=7), c,
                                                                         max_size=3),
                    max_leaves=8)
MSG = st.fixed_dictionaries({}, optional={
    "role": st.one_of(st.just("user"), JSON), "kind": JSON, "messageId": JSON,
    "taskId": JSON, "contextId": JSON, "metadata": JSON,
    "parts": st.one_of(st.lists(st.fixed_dictionaries({}, optional={
        "kind": st.one_of(st.just("text"), JSON), "text": st.one_of(st.text(max_size=6), JSON),
        "data": JSON}), max_size=2), JSON)})
METHODS = st.sampled_from(["message/send", "tasks/get", "tasks/cancel", "tasks/resubscribe",
                           "message/stream", "nope"])
REQ = st.one_of(
    st.builds(lambda m, p: json.dumps({"jsonrpc": "2.0", "id": 1, "method": m, "params": p}),
              METHODS, st.one_of(st.fixed_dictionaries({}, optional={"message": MSG,
                                                                      "id": JSON}), JSON)),
    JSON.map(json.dumps), st.sampled_from(["", "{", "[1]"]))


async def _run(srv, bodies):
    app = web.Application()
    app.router.add_post("/a2a", srv.rpc)
    out = []
    async with TestClient(TestServer(app)) as c:
        for b in bodies:
            r = await asyncio.wait_for(c.post("/a2a", data=b), 30)
            out.append((b, r.status, (await r.text())[:300]))
    return out


@given(st.lists(REQ, min_size=1, max_size=4))
@settings(max_examples=100, deadline=None, suppress_health_check=[HealthCheck.too_slow])
def test_a2a_rpc_never_answers_500(bodies):
    svc, _, _ = make_service()
    srv = A2AServer(InProcessRuntimeClient(svc), "agent")
    for b, status, text in asyncio.run(_run(srv, bodies)):
        assert status < 500, (b, status, text)
