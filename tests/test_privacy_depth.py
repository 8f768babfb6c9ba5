"""Privacy-API depth (ee/pkg/privacy): embedding consent classifier, consent
outbox + memory-api notifier + replay, media deleters, session-group DSAR
fan-out, SessionPrivacyPolicy watcher, and the privacy middleware of
session-api / memory-api with body redaction -- all against in-repo fakes."""
import asyncio
import json
import os
import time

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.ee.privacy import PrivacyStore
from omnia_amd.ee.privacy.classify import CategoryValidator, EmbeddingClassifier
from omnia_amd.ee.privacy.erasure import (EraseScope, FanOutSubjectEraser, GroupTarget,
                                          LocalMediaDeleter, ObjectStoreMediaDeleter,
                                          SessionTierEraser)
from omnia_amd.ee.privacy.outbox import (MemoryAPINotifier, Outbox, OutboxReplayWorker,
                                         deliver)
from omnia_amd.ee.privacy.policy import (PolicyWatcher, StoreSource, memory_privacy_middleware,
                                         redact_body, session_privacy_middleware)
from omnia_amd.memory.embedding import HashEmbedder


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


class KeywordEmbedder:
    """Deterministic embedder: one axis per topic keyword family."""
    AXES = [("diagnos", "doctor", "therap", "illness", "medic", "allerg", "surgery",
             "blood", "asthma"),
            ("live", "address", "based", "apartment", "office", "house", "moved"),
            ("passport", "social", "legal", "credit", "license", "phone", "id"),
            ("prefer", "like", "favorite", "enjoy"),
            ("project", "meeting", "report", "deadline", "presentation", "migrat", "launch")]

    async def embed(self, texts):
        out = []
        for t in texts:
            low = t.lower()
            v = [float(sum(low.count(k) for k in ax)) for ax in self.AXES]
            out.append(v if any(v) else [0.01] * len(self.AXES))
        return out


# ------------------------------------------------------------------ classifier
def test_embedding_classifier_centroids_threshold_and_validator():
    async def go():
        ec = EmbeddingClassifier(KeywordEmbedder(), threshold=0.7)
        with pytest.raises(RuntimeError):
            await ec.classify("x")
        await ec.prewarm()
        assert set(ec.centroids) == {"memory:health", "memory:location", "memory:identity",
                                     "memory:preferences", "memory:context"}
        h, s = await ec.classify("I see my therapist about my illness")
        loc, _ = await ec.classify("we moved to a house near the office")
        none, s0 = await ec.classify("the weather is nice")
        v = CategoryValidator(ec)
        rule = await v.classify("email me at a@b.io", claimed="memory:preferences")
        emb = await v.classify("I see my therapist weekly", claimed="memory:preferences")
        keep = await v.classify("I enjoy jazz", claimed="memory:health")  # no downgrade
        return h, s, loc, none, s0, rule, emb, keep

    h, s, loc, none, s0, rule, emb, keep = asyncio.run(go())
    assert h == "memory:health" and s > 0.9 and loc == "memory:location"
    assert none == "" and s0 < 0.7
    assert rule == "memory:identity"  # the regex rule is evidence and wins
    assert emb == "memory:health" and keep == "memory:health"


def test_embedding_classifier_on_the_memory_save_path():
    from omnia_amd.memory.model import Memory
    from omnia_amd.memory.service import MemoryService

    async def go():
        svc = MemoryService(enterprise=True)
        svc.embedding_classifier = EmbeddingClassifier(KeywordEmbedder())
        await svc.embedding_classifier.prewarm()
        r = await svc.save(Memory(content="I see my therapist every week",
                                  scope={"workspace_id": "w", "virtual_user_id": "u"}))
        svc.store.revoke_consent("w", "u", "memory:health")
        with pytest.raises(PermissionError):
            await svc.save(Memory(content="my doctor changed the medication",
                                  scope={"workspace_id": "w", "virtual_user_id": "u"}))
        return svc.store.get(r["id"]) if svc.store.get(r["id"]) else r

    got = asyncio.run(go())
    assert isinstance(got, dict) or got.metadata.get("consent_category") == "memory:health"


def test_hash_embedder_centroids_rank_health_first():
    async def go():
        ec = EmbeddingClassifier(HashEmbedder(256), threshold=0.0)
        await ec.prewarm()
        return await ec.classify("my doctor prescribed new medication for my illness")

    cat, _ = asyncio.run(go())
    assert cat == "memory:health"


# ------------------------------------------------------------------ outbox
def test_consent_outbox_notify_replay_prune_and_stuck():
    async def go():
        got, fail = [], {"on": True}
        app = web.Application()

        async def ev(request):
            if fail["on"]:
                return web.json_response({}, status=503)
            got.append((dict(request.query), await request.json()))
            return web.json_response({"deleted_observations": 0})

        app.router.add_post("/api/v1/memories/consent-events", ev)
        r, url = await _serve(app)
        try:
            st = PrivacyStore()
            ob = Outbox(st)
            st.set_consent("alice", ["memory:health"], [])
            oid = ob.revoke_with_outbox("alice", "memory:health")
            assert oid and ob.revoke_with_outbox("alice", "memory:health") is None  # not granted
            assert "memory:health" in st.consent("alice")["denied"]
            n = MemoryAPINotifier([url], workspace="w1")
            assert not await deliver(ob, n, oid, "alice", "memory:health")
            assert [x[0] for x in ob.undelivered(3600)] == [oid]
            w = OutboxReplayWorker(ob, n, stuck_after_s=0.0)
            res1 = await w.run_once()
            fail["on"] = False
            res2 = await w.run_once()
            left = ob.undelivered(3600)
            pruned = ob.prune_delivered(-1)
            return res1, res2, left, pruned, got
        finally:
            await r.cleanup()

    res1, res2, left, pruned, got = asyncio.run(go())
    assert res1["failed"] == 1 and res1["stuck"] == 1
    assert res2["sent"] == 1 and res2["stuck"] == 0 and left == [] and pruned == 1
    assert got == [({"workspace": "w1"}, {"userId": "alice", "category": "memory:health"})]


def test_privacy_api_revocation_reaches_memory_api_through_outbox():
    from omnia_amd.ee.privacy import build_app as privacy_app
    from omnia_amd.memory.api import build_app as memory_app
    from omnia_amd.memory.model import Memory
    from omnia_amd.memory.service import MemoryService

    async def go():
        ms = MemoryService(enterprise=True)
        await ms.save(Memory(content="prefers tea", scope={"workspace_id": "w",
                                                          "virtual_user_id": "bob"},
                             metadata={"consent_category": "memory:preferences"}))
        r1, m_url = await _serve(memory_app(ms, enterprise=True))
        st = PrivacyStore()
        app = privacy_app(st, notifier=MemoryAPINotifier([m_url]))
        r2, p_url = await _serve(app)
        try:
            async with aiohttp.ClientSession() as s:
                r = await s.put(f"{p_url}/api/v1/privacy/preferences/bob/consent",
                                json={"revocations": ["memory:preferences"]})
                body = await r.json()
            return body, ms.store.list({"workspace_id": "w", "virtual_user_id": "bob"}), \
                app["outbox"].undelivered(3600)
        finally:
            await r1.cleanup()
            await r2.cleanup()

    body, left, pending = asyncio.run(go())
    assert "memory:preferences" in body["denied"]
    assert left == [] and pending == []  # erased across workspaces, outbox delivered


# ------------------------------------------------------------------ media / erasure
def test_media_deleters(tmp_path):
    from omnia_amd.media import LocalMediaStorage

    async def go():
        ms = LocalMediaStorage(str(tmp_path))
        for sid in ("s1", "s2"):
            up = await ms.upload_url(sid, {"filename": "a.png", "mime_type": "image/png",
                                           "size_bytes": 3})
            ms.write_upload(up["upload_id"], b"abc")
        n = await LocalMediaDeleter(str(tmp_path)).delete_session_media("s1")

        class FakeObjects:
            def __init__(self):
                self.keys = {"media/s1/a", "media/s1/b", "media/s2/c"}
                self.deleted = []

            async def list_objects(self, bucket, prefix):
                return sorted(k for k in self.keys if k.startswith(prefix))

            async def delete_objects(self, bucket, keys):
                self.deleted += keys
                self.keys -= set(keys)

        fo = FakeObjects()
        m = await ObjectStoreMediaDeleter(fo, "b", "media/").delete_session_media("s1")
        none = await ObjectStoreMediaDeleter(fo, "b", "media/").delete_session_media("zz")
        return n, m, none, fo

    n, m, none, fo = asyncio.run(go())
    assert n == 1 and not os.path.exists(tmp_path / "sessions" / "s1")
    assert os.path.exists(tmp_path / "sessions" / "s2")
    assert m == 2 and none == 0 and fo.keys == {"media/s2/c"}


def _sessions(svc, user, n, created, ws=""):
    from omnia_amd.session.model import Session

    for i in range(n):
        svc.create(Session(id=f"{user}-{ws}-{created}-{i}", namespace="ns",
                           virtual_user_id=user, workspace_name=ws, created_at=created))


def test_session_group_fanout_with_date_range_media_and_failing_group(tmp_path):
    from omnia_amd.memory.api import build_app as memory_app
    from omnia_amd.memory.model import Memory
    from omnia_amd.memory.service import MemoryService
    from omnia_amd.session.api import build_app as session_app
    from omnia_amd.session.store import TieredSessionService

    class CountingMedia(LocalMediaDeleter):
        calls = []

        async def delete_session_media(self, sid):
            self.calls.append(sid)
            return 0

    async def go():
        now = time.time()
        a, b = TieredSessionService(), TieredSessionService()
        _sessions(a, "alice", 2, now - 10 * 86400)
        _sessions(a, "alice", 1, now)
        _sessions(b, "alice", 1, now, ws="w2")
        _sessions(b, "bob", 1, now)
        med = CountingMedia(str(tmp_path))
        ms = MemoryService()
        await ms.save(Memory(content="x", scope={"workspace_id": "w", "virtual_user_id": "alice"}))
        ra, ua = await _serve(session_app(a, media_deleter=med))
        rb, ub = await _serve(session_app(b))
        rm, um = await _serve(memory_app(ms))
        try:
            fan = FanOutSubjectEraser([GroupTarget("g1", ua, um), GroupTarget("g2", ub, ""),
                                       GroupTarget("dead", "http://127.0.0.1:9", "")], ["w"])
            recent = await fan.erase_subject({"virtualUserId": "alice",
                                              "dateFrom": now - 86400})
            rest = await fan.erase_subject({"virtualUserId": "alice"})
            return recent, rest, med.calls, a, b, ms
        finally:
            for r in (ra, rb, rm):
                await r.cleanup()

    recent, rest, calls, a, b, ms = asyncio.run(go())
    assert recent[0] == 2  # one recent in g1 + one in g2; the old ones kept by the range
    assert any("group dead sessions" in e for e in recent[1])  # recorded, others ran
    assert rest[0] == 2 and len(calls) == 3  # media deleted for each erased g1 session
    assert b.warm.list_sessions(user="bob") and not a.warm.list_sessions(user="alice")
    assert ms.store.list({"workspace_id": "w", "virtual_user_id": "alice"}) == []


def test_session_tier_eraser_workspace_filter():
    from omnia_amd.session.store import TieredSessionService

    svc = TieredSessionService()
    _sessions(svc, "u", 2, time.time(), ws="w1")
    _sessions(svc, "u", 1, time.time(), ws="w2")
    res = asyncio.run(SessionTierEraser(svc).erase(EraseScope("u", workspace="w1")))
    assert res["sessions_deleted"] == 2 and len(svc.warm.list_sessions(user="u")) == 1


# ------------------------------------------------------------------ watcher + middleware
def _policy_store():
    from omnia_amd.api import crds
    from omnia_amd.operator.apistore import APIStore

    st = APIStore()

    def pol(name, ns, spec):
        st.apply({"apiVersion": crds.API_VERSION, "kind": "SessionPrivacyPolicy",
                  "metadata": {"name": name, "namespace": ns}, "spec": spec})

    pol("default", "omnia-system", {"recording": {"enabled": True, "runtimeData": True}})
    pol("strict", "team", {"recording": {"enabled": False}})
    pol("group", "team", {"recording": {"enabled": True, "runtimeData": False,
                                        "pii": {"redact": True, "strategy": "replace"}},
                          "userOptOut": {"enabled": True}})
    st.apply({"apiVersion": crds.API_VERSION, "kind": "Workspace", "metadata": {"name": "ws"},
              "spec": {"displayName": "W", "namespace": {"name": "team"},
                       "services": [{"name": "default", "mode": "external",
                                     "external": {"sessionURL": "http://s:8080",
                                                  "memoryURL": "http://m:8080"},
                                     "privacyPolicyRef": {"name": "group"}}]}})
    for name, ref in (("a-strict", "strict"), ("a-plain", None)):
        spec = {"promptPackRef": {"name": "p"}, "facades": [{"type": "websocket"}]}
        if ref:
            spec["privacyPolicyRef"] = {"name": ref}
        st.apply({"apiVersion": crds.API_VERSION, "kind": "AgentRuntime",
                  "metadata": {"name": name, "namespace": "team"}, "spec": spec})
    return st


def test_policy_watcher_precedence_and_change_events():
    st = _policy_store()
    w = PolicyWatcher(StoreSource(st), own_workspace="ws", own_namespace="team")
    changes = []
    w.on_change = lambda old, new: changes.append((old is None, new is None))
    asyncio.run(w.load_all())
    assert w.effective("team", "a-strict")["recording"]["enabled"] is False  # agent ref
    assert w.effective("team", "a-plain")["recording"]["runtimeData"] is False  # group ref
    assert w.effective("other", "x")["recording"]["runtimeData"] is True  # global default
    assert len(changes) == 3 and all(c == (True, False) for c in changes)
    st.delete("SessionPrivacyPolicy", "strict", "team")
    asyncio.run(w.load_all())
    assert changes[-1] == (False, True)  # evicted
    assert w.effective("team", "a-strict")["recording"]["runtimeData"] is False  # -> group


def test_session_api_privacy_middleware_drop_optout_and_redaction():
    from omnia_amd.session.api import build_app as session_app, session_resolver
    from omnia_amd.session.model import Session
    from omnia_amd.session.store import TieredSessionService

    st = _policy_store()
    w = PolicyWatcher(StoreSource(st), own_workspace="ws", own_namespace="team")
    asyncio.run(w.load_all())
    prefs = PrivacyStore()
    prefs.opt_out("carol")

    async def go():
        svc = TieredSessionService()
        svc.create(Session(id="s-strict", namespace="team", agent_name="a-strict"))
        svc.create(Session(id="s-plain", namespace="team", agent_name="a-plain"))
        app = session_app(svc, privacy_middleware=session_privacy_middleware(
            w, session_resolver(svc), prefs))
        r, url = await _serve(app)
        out = {}
        try:
            async with aiohttp.ClientSession() as s:
                async def post(sid, path, body, **h):
                    resp = await s.post(f"{url}/api/v1/sessions/{sid}/{path}", json=body,
                                        headers=h)
                    return resp.status
                out["strict"] = await post("s-strict", "messages",
                                           {"role": "user", "content": "hi"})
                out["rt_assistant"] = await post("s-plain", "messages",
                                                 {"role": "assistant", "content": "a"},
                                                 **{"X-Omnia-Source": "runtime"})
                out["facade_assistant"] = await post(
                    "s-plain", "messages", {"role": "assistant", "content": "from facade"},
                    **{"X-Omnia-Source": "facade"})
                out["user_pii"] = await post("s-plain", "messages",
                                             {"role": "user", "content": "mail me at z@x.io"})
                out["opted_out"] = await post("s-plain", "messages",
                                              {"role": "user", "content": "secret"},
                                              **{"X-Omnia-User-ID": "carol"})
                out["tool"] = await post("s-plain", "tool-calls",
                                         {"name": "t", "arguments": {"to": "z@x.io"},
                                          "callId": "c1"})
                msgs = await (await s.get(f"{url}/api/v1/sessions/s-plain/messages")).json()
                tools = await (await s.get(f"{url}/api/v1/sessions/s-plain/tool-calls")).json()
                strict = await (await s.get(f"{url}/api/v1/sessions/s-strict/messages")).json()
            return out, msgs, tools, strict
        finally:
            await r.cleanup()

    out, msgs, tools, strict = asyncio.run(go())
    assert out["strict"] == 204 and strict.get("messages") == []
    assert out["rt_assistant"] == 204 and out["opted_out"] == 204
    assert out["facade_assistant"] < 300 and out["user_pii"] < 300 and out["tool"] < 300
    contents = [m["content"] for m in msgs["messages"]]
    assert contents == ["from facade", "mail me at [REDACTED_EMAIL]"]
    assert json.dumps(tools["tool-calls"][0]["arguments"]) == '{"to": "[REDACTED_EMAIL]"}'


def test_memory_api_privacy_middleware_redacts_saves():
    from omnia_amd.memory.api import build_app as memory_app
    from omnia_amd.memory.service import MemoryService

    st = _policy_store()
    w = PolicyWatcher(StoreSource(st), own_workspace="ws", own_namespace="team")
    asyncio.run(w.load_all())

    async def go():
        svc = MemoryService()
        app = memory_app(svc)
        app.middlewares.append(memory_privacy_middleware(w, "team"))
        r, url = await _serve(app)
        try:
            async with aiohttp.ClientSession() as s:
                resp = await s.post(f"{url}/api/v1/memories", headers={
                    "x-omnia-agent-name": "a-plain"}, json={
                    "content": "my email is q@w.io", "scope": {"workspace_id": "w",
                                                                "virtual_user_id": "u"}})
                return resp.status, await resp.json()
        finally:
            await r.cleanup()

    st_, body = asyncio.run(go())
    assert st_ == 201 and body["memory"]["content"] == "my email is [REDACTED_EMAIL]"


def test_redact_body_rules():
    from omnia_amd.ee.redaction import Redactor

    red = Redactor(None, "replace")
    out = json.loads(redact_body(b'{"content": "x@y.io", "role": "user"}',
                                 "/api/v1/sessions/s/messages", red))
    assert out == {"content": "[REDACTED_EMAIL]", "role": "user"}
    same = redact_body(b'{"content": "x@y.io"}', "/api/v1/sessions/s/ttl", red)
    assert json.loads(same)["content"] == "x@y.io"  # endpoint without free text
    with pytest.raises(ValueError):
        redact_body(b"not json", "/api/v1/sessions/s/messages", red)
