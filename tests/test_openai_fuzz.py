"""HTTP input fuzzing of the OpenAI-compatible engine server
(engine/openai_server.py) on the CPU tiny-llama engine: requests with fields of
the wrong JSON type, out-of-range token ids, bad sampling parameters or
malformed tools get a 4xx answer; a request that is accepted completes.  No
input reaches the engine thread in a form that would fail a step (which would
fail every request sharing it)."""
import asyncio
import json
import os

import pytest
from aiohttp.test_utils import TestClient, TestServer
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from omnia_amd.engine.engine import AsyncLLMEngine, EngineConfig, LLMEngine
from omnia_amd.engine.openai_server import build_app
from omnia_amd.memory.embedding import HashEmbedder

JSON = st.recursive(st.none() | st.booleans() | st.integers(-5, 300)
                    | st.floats(allow_nan=False, allow_infinity=False, width=32)
                    | st.text(max_size=5),
                    lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=6), c,
                                                                         max_size=3),
                    max_leaves=8)
MSG = st.fixed_dictionaries({"role": st.sampled_from(["user", "system", "assistant", "tool"]),
                             "content": st.one_of(st.text(max_size=12), JSON)})
FIELDS = {"temperature": st.one_of(st.floats(0, 2, width=32), JSON),
          "top_p": st.one_of(st.floats(0.0625, 1, width=32), JSON),
          "top_k": st.one_of(st.integers(0, 50), JSON), "max_tokens": st.one_of(
              st.integers(1, 4), JSON), "seed": JSON, "stop": st.one_of(
              st.text(max_size=3), st.lists(st.text(max_size=3), max_size=2), JSON),
          "n": JSON, "user": JSON, "stream": st.booleans(), "tools": JSON,
          "stream_options": JSON, "response_format": JSON, "ignore_eos": JSON}


@pytest.fixture(scope="module")
def eng():
    e = AsyncLLMEngine(LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=256,
                                              block_size=32, max_batch=8, max_model_len=512)))
    yield e
    e.shutdown()


async def _run(eng, reqs):
    out = []
    async with TestClient(TestServer(build_app(eng, "tiny-llama", HashEmbedder(16)))) as c:
        for path, body in reqs:
            r = await asyncio.wait_for(c.post(path, data=body), 60)
            out.append((path, body, r.status, (await r.text())[:300]))
    return out


CHAT = st.builds(lambda msgs, extra: json.dumps({"model": "tiny-llama", "messages": msgs,
                                                 "max_tokens": 2, **extra}),
                 st.one_of(st.lists(MSG, min_size=1, max_size=3), JSON),
                 st.fixed_dictionaries({}, optional=FIELDS))
COMPL = st.builds(lambda p, extra: json.dumps({"prompt": p, "max_tokens": 2, **extra}),
                  st.one_of(st.text(max_size=10), st.lists(st.integers(-3, 600), max_size=4),
                            JSON),
                  st.fixed_dictionaries({}, optional=FIELDS))
EMB = st.builds(lambda i: json.dumps({"input": i}), JSON)
REQ = st.one_of(st.tuples(st.just("/v1/chat/completions"), CHAT),
                st.tuples(st.just("/v1/completions"), COMPL),
                st.tuples(st.just("/v1/embeddings"), EMB),
                st.tuples(st.sampled_from(["/v1/chat/completions", "/v1/completions"]),
                          st.sampled_from(["", "[]", "null", "{", "7"])))


@given(reqs=st.lists(REQ, min_size=1, max_size=4))
@settings(max_examples=int(os.environ.get("OMNIA_FUZZ_EXAMPLES", "80")), deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
def test_openai_server_rejects_bad_input_with_4xx(eng, reqs):
    for path, body, status, text in asyncio.run(_run(eng, reqs)):
        assert status < 500, (path, body, status, text)
    assert eng.health()
