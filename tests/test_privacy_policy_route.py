"""GET /api/v1/privacy-policy on session-api and the facade recording gate
that reads it (verdict r5 item 6).  Mirrors the reference wiring tests
(``cmd/session-api/wiring_test.go:126-153,315-338``: the route exists in
enterprise AND non-enterprise mode, 204 without a resolver, never 404) and the
facade's ``RecordingPolicyCache`` / ``facadeAllowed`` / ``runtimeAllowed``
(``internal/facade/recording_policy.go``, ``recording_interceptor.go``)."""
import asyncio

import pytest
from aiohttp import web

from omnia_amd.session.api import build_app
from omnia_amd.session.httpclient import RecordingPolicyCache, RecordingPool, SessionHTTPClient
from omnia_amd.session.store import TieredSessionService


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


POLICIES = {("ns1", "quiet"): {"recording": {"enabled": True, "facadeData": False,
                                            "runtimeData": True},
                               "encryption": {"enabled": True, "keyID": "secret-key"}},
            ("ns1", "off"): {"recording": {"enabled": False, "facadeData": True,
                                          "runtimeData": True}}}


def _resolver(ns, agent):
    return POLICIES.get((ns, agent))


def test_route_enterprise_and_non_enterprise():
    async def go():
        out = {}
        for mode, kw in (("ee", {"policy_resolver": _resolver}), ("oss", {})):
            runner, url = await _serve(build_app(TieredSessionService(), **kw))
            c = SessionHTTPClient(url)
            try:
                out[mode] = (await c.get_privacy_policy("ns1", "quiet"),
                             await c.get_privacy_policy("ns1", "nobody"))
                import aiohttp

                async with aiohttp.ClientSession() as s:
                    async with s.get(url + "/api/v1/privacy-policy?namespace=ns1&agent=x") as r:
                        out[mode + "_status"] = r.status
            finally:
                await c.close()
                await runner.cleanup()
        return out

    out = asyncio.run(go())
    pol, none = out["ee"]
    # the facade-visible subset only: the recording block, never encryption config
    assert pol == {"recording": {"enabled": True, "facadeData": False, "runtimeData": True}}
    assert none is None and out["ee_status"] == 204
    # non-enterprise: the route is registered (not 404) and returns 204
    assert out["oss"] == (None, None) and out["oss_status"] == 204


class _Store:
    def __init__(self):
        self.appended = []

    async def append(self, sid, role, content, usage=None):
        self.appended.append((role, content))


@pytest.mark.parametrize("agent,want", [
    ("quiet", [("assistant", "a1")]),             # facadeData off: user turns dropped
    ("off", []),                                  # recording disabled: nothing
    ("nobody", [("user", "u1"), ("assistant", "a1")]),  # no policy (204): fail open
])
def test_facade_recording_gate(agent, want):
    async def go():
        runner, url = await _serve(build_app(TieredSessionService(),
                                             policy_resolver=_resolver))
        client = SessionHTTPClient(url)
        store = _Store()
        pool = RecordingPool(store, workers=2,
                             policy=RecordingPolicyCache(client.get_privacy_policy, "ns1",
                                                         agent))
        try:
            pool.submit("s1", "user", "u1")
            pool.submit("s1", "assistant", "a1")
            await pool.join()
        finally:
            await pool.stop()
            await client.close()
            await runner.cleanup()
        return store.appended, pool

    got, pool = asyncio.run(go())
    assert got == want
    assert pool.policy.fetches == 1  # cached across the session's messages


def test_policy_fetch_failure_records_everything_and_ttl_refreshes():
    t = [0.0]
    calls = []

    async def boom(ns, agent):
        calls.append((ns, agent))
        if len(calls) == 1:
            raise ConnectionError("session-api down")
        return {"recording": {"enabled": False}}

    cache = RecordingPolicyCache(boom, "ns1", "a", ttl_s=30, now=lambda: t[0])

    async def go():
        p1 = await cache.get()
        p2 = await cache.get()
        t[0] = 31.0
        p3 = await cache.get()
        return p1, p2, p3

    p1, p2, p3 = asyncio.run(go())
    assert RecordingPolicyCache.allows(p1, "user") and RecordingPolicyCache.allows(p1, "assistant")
    assert p2 is p1 and len(calls) == 2
    assert not RecordingPolicyCache.allows(p3, "user")


def test_facade_builder_wires_the_gate():
    from omnia_amd.facade.app import build_facade

    f = build_facade({"OMNIA_SESSION_API_URL": "http://127.0.0.1:1", "OMNIA_AGENT_NAME": "ag",
                      "OMNIA_NAMESPACE": "ns9", "OMNIA_HANDLER_MODE": "echo"}, None)
    rec = f.recorder
    assert isinstance(rec.policy, RecordingPolicyCache)
    assert (rec.policy.namespace, rec.policy.agent) == (f.cfg.namespace, f.cfg.agent)
