"""Single-node KEDA (BASELINE config 4's "KEDA scale-to-zero on the
active-connection metric"): the PromQL subset, the ScaledObject replica math
(``internal/controller/autoscaling.go:167-325`` semantics: threshold per pod,
immediate scale-up, scale-down to minReplicaCount after cooldownPeriod), the
activator that parks connections while a replica cold-starts, and the whole
loop under ``omnia serve``'s process launcher: connect -> scale from zero -> the
turn streams from a TP=2 engine -> idle -> scale to zero."""
import asyncio
import os
import time

import aiohttp
import pytest
from aiohttp import web

from omnia_amd.api import crds
from omnia_amd.operator.apistore import APIStore, get_condition
from omnia_amd.operator.keda import Activator, KedaScaler, eval_query, parse_prom_text

PROM = """# HELP omnia_agent_connections_active Active WebSocket connections
# TYPE omnia_agent_connections_active gauge
omnia_agent_connections_active{agent="a",namespace="default"} 150.0
omnia_agent_connections_active{agent="a",namespace="other"} 7.0
omnia_agent_connections_active{agent="b",namespace="default"} 3.0
omnia_agent_requests_total{agent="a",namespace="default",status="ok"} 12.0
"""


def test_prom_text_and_query_subset():
    s = parse_prom_text(PROM)
    assert len(s) == 4 and s[0] == ("omnia_agent_connections_active",
                                    {"agent": "a", "namespace": "default"}, 150.0)
    q = 'sum(omnia_agent_connections_active{agent="a",namespace="default"})'
    assert eval_query(q, s) == 150.0
    assert eval_query('sum(omnia_agent_connections_active{namespace="default"})', s) == 153.0
    assert eval_query('max(omnia_agent_connections_active{agent=~"a|b"})', s) == 150.0
    assert eval_query('count(omnia_agent_connections_active{namespace!="default"})', s) == 1.0
    assert eval_query('sum(omnia_agent_connections_active{agent="zz"})', s) is None
    assert eval_query('sum(omnia_agent_connections_active{agent="zz"}) or vector(0)', s) == 0.0
    assert eval_query('omnia_agent_requests_total{status="ok"}', s) == 12.0
    with pytest.raises(ValueError):
        eval_query("rate(x[5m])", s)


def _store_with(min_r=0, max_r=4, poll=1, cool=3, threshold="200", replicas=1):
    st = APIStore()
    st.apply({"apiVersion": "apps/v1", "kind": "Deployment",
              "metadata": {"name": "a", "namespace": "default"},
              "spec": {"replicas": replicas, "template": {"metadata": {}, "spec": {}}}})
    st.apply({"apiVersion": "keda.sh/v1alpha1", "kind": "ScaledObject",
              "metadata": {"name": "a", "namespace": "default"},
              "spec": {"scaleTargetRef": {"name": "a"}, "minReplicaCount": min_r,
                       "maxReplicaCount": max_r, "pollingInterval": poll, "cooldownPeriod": cool,
                       "triggers": [{"type": "prometheus", "metadata": {
                           "query": 'sum(omnia_agent_connections_active{agent="a",'
                                    'namespace="default"})', "threshold": threshold}}]}})
    return st


def test_scaler_replica_math_and_cooldown():
    st = _store_with()
    now = [1000.0]
    conns = [0.0]

    async def samples(ns, name):
        return [("omnia_agent_connections_active", {"agent": "a", "namespace": "default"},
                 conns[0])]

    sc = KedaScaler(st, samples, clock=lambda: now[0])
    reps = lambda: st.get("Deployment", "a", "default")["spec"]["replicas"]  # noqa: E731

    async def run():
        out = []
        for t, c in [(0, 0), (1, 0), (2, 0), (3, 0), (4, 450), (4.5, 450), (5, 450), (6, 10),
                     (7, 10), (8, 10), (9, 10), (10, 0), (11, 0), (12, 0), (13, 0)]:
            now[0] = 1000.0 + t
            conns[0] = c
            await sc.tick()
            out.append(reps())
        return out

    got = asyncio.run(run())
    # idle from the start: cooldown (3 s) then min (0); 450 conns / 200 -> 3 pods at once
    # (polling interval 1 s skips t=4.5); 10 conns hold 3 pods until the cooldown after
    # the scale-up (t=7), then ceil(10/200)=1; idle from t=10 -> 0 once the last
    # activity (t=9) is 3 s old
    assert got == [1, 1, 1, 0, 3, 3, 3, 3, 1, 1, 1, 1, 1, 0, 0], got
    so = st.get("ScaledObject", "a", "default")
    assert get_condition(so, "Ready")["status"] == "True"
    assert get_condition(so, "Active")["status"] == "False"
    assert so["status"]["currentReplicas"] == 0 and "lastActiveTime" in so["status"]


def test_scaler_respects_min_and_max():
    st = _store_with(min_r=2, max_r=3, cool=0, replicas=2)

    async def samples(ns, name):
        return [("omnia_agent_connections_active", {"agent": "a", "namespace": "default"},
                 5000.0)]

    sc = KedaScaler(st, samples, clock=lambda: 0.0)
    asyncio.run(sc.tick())
    assert st.get("Deployment", "a", "default")["spec"]["replicas"] == 3

    async def idle(ns, name):
        return []

    sc2 = KedaScaler(st, idle, clock=lambda: 100.0)
    asyncio.run(sc2.tick())
    assert st.get("Deployment", "a", "default")["spec"]["replicas"] == 2  # never below min


def test_activator_parks_until_a_backend_is_ready_then_relays():
    async def run():
        up = web.Application()

        async def ws(request):
            w = web.WebSocketResponse()
            await w.prepare(request)
            async for m in w:
                await w.send_str("echo:" + m.data)
            return w

        up.router.add_get("/ws", ws)
        up.router.add_get("/hello", lambda r: web.json_response({"q": r.query.get("x")}))
        runner = web.AppRunner(up)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        be = f"127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
        act = Activator("a", "default", timeout_s=10)
        ep = await act.start()
        try:
            async with aiohttp.ClientSession() as s:
                task = asyncio.ensure_future(s.ws_connect(f"ws://{ep}/ws"))
                for _ in range(100):
                    if act.parked:
                        break
                    await asyncio.sleep(0.02)
                parked = act.parked
                assert act.samples()[0][2] == 1.0  # counted as an active connection
                act.set_backends([be])
                w = await asyncio.wait_for(task, 5)
                await w.send_str("hi")
                msg = await w.receive_str(timeout=5)
                await w.close()
                r = await s.get(f"http://{ep}/hello?x=1")
                body = await r.json()
                act.set_backends([])
                act.timeout_s = 0.2
                r2 = await s.get(f"http://{ep}/hello")
                return parked, msg, body, r2.status
        finally:
            await act.stop()
            await runner.cleanup()

    parked, msg, body, late = asyncio.run(run())
    assert parked == 1 and msg == "echo:hi" and body == {"q": "1"} and late == 503


EXAMPLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "examples",
                       "llama3-70b-tp8", "manifests.yaml")
AGENT = "assistant-70b"


def _example_docs(engine: dict, max_tokens: int = 6, poll: int = 1, cool: int = 3):
    """The shipped config-4 manifests with the engine swapped for a test-sized
    one and the KEDA periods shortened."""
    import json

    import yaml

    with open(EXAMPLE) as f:
        docs = [d for d in yaml.safe_load_all(f) if d]
    for d in docs:
        d.setdefault("apiVersion", crds.API_VERSION)
        if d["kind"] == "Provider":
            d["spec"]["engine"] = dict(engine)
            d["spec"]["model"] = engine["model"]
        elif d["kind"] == "ConfigMap":
            pack = json.loads(d["data"]["pack.json"])
            pack["prompts"]["default"]["parameters"] = {"temperature": 0,
                                                        "max_tokens": max_tokens,
                                                        "ignore_eos": True}
            d["data"]["pack.json"] = json.dumps(pack)
        elif d["kind"] == "AgentRuntime":
            d["spec"]["runtime"]["autoscaling"]["keda"].update(pollingInterval=poll,
                                                               cooldownPeriod=cool)
    return docs


def _scale_cycle(engine: dict, gpu_count: int = 0):
    from omnia_amd.ee.arena.fleet import FleetSession
    from omnia_amd.operator.launcher import LocalLauncher
    from omnia_amd.operator.manager import Manager, new_store

    docs = _example_docs(engine)

    async def go():
        store = new_store()
        mgr = Manager(store)
        await mgr.start()
        launcher = LocalLauncher(store, mode="process", gpu_count=gpu_count)
        launcher.start()
        try:
            for d in docs:
                store.apply(d)
            ep = None
            for _ in range(300):
                svc = store.try_get("Service", AGENT)
                ep = ((svc or {}).get("status") or {}).get("endpoint")
                if ep and store.try_get("ScaledObject", AGENT) is not None:
                    break
                await asyncio.sleep(0.1)
            assert ep, "activator endpoint never published"
            assert not launcher.replicas.get(("default", AGENT))  # at zero: no pod
            t0 = time.monotonic()
            async with FleetSession(f"ws://{ep}/ws", timeout_s=600) as fs:
                r = await fs.turn("hello there")
            first_turn_s = time.monotonic() - t0
            dep = store.get("Deployment", AGENT)
            cold = dep["status"].get("coldStartSeconds")
            up = dep["spec"]["replicas"]
            # idle: cooldown 3 s, poll 1 s -> back to zero, pod stopped
            for _ in range(300):
                if store.get("Deployment", AGENT)["spec"]["replicas"] == 0 and \
                        not launcher.replicas.get(("default", AGENT)):
                    break
                await asyncio.sleep(0.1)
            down = store.get("Deployment", AGENT)["spec"]["replicas"]
            so = store.get("ScaledObject", AGENT)
            return r, up, down, cold, first_turn_s, so, launcher.replicas.get(("default", AGENT))
        finally:
            await launcher.stop()
            await mgr.stop()

    r, up, down, cold, first_s, so, reps = asyncio.run(go())
    assert (r["usage"] or {}).get("output_tokens") == 6 and not r.get("error"), r
    assert up == 1 and down == 0 and not reps
    assert cold and 0 < cold < first_s
    assert get_condition(so, "Ready")["status"] == "True"
    print(f"scale-from-zero: pod cold start {cold:.1f}s, first turn {first_s:.1f}s")
    return cold, first_s


def test_serve_scales_from_zero_and_back_to_zero_tp2_cpu():
    _scale_cycle({"model": "tiny-llama", "tp": 2, "maxBatch": 4, "maxModelLen": 512,
                  "numBlocks": 64, "blockSize": 16, "dtype": "float32", "useGraphs": False,
                  "device": "cpu"})


@pytest.mark.gpu
def test_serve_scales_from_zero_llama3_8b_gpu():
    """GPU variant: Llama-3-8B TP=1 on the box's one MI355X (graphs on); the pod's
    cold start covers weights, KV pool and decode-graph capture."""
    from conftest import release_gpu_memory

    release_gpu_memory()
    cold, first = _scale_cycle({"model": "llama-3-8b", "tp": 1, "maxBatch": 64,
                                "maxModelLen": 4096, "kvFraction": 0.5}, gpu_count=1)
    assert cold < 300


@pytest.mark.gpu
def test_serve_tp2_70b_shape_pod_scale_cycle_matches_oracle_gpu(tmp_path, monkeypatch):
    """BASELINE config 4 through the whole serving stack on the one MI355X: the
    operator reconciles the shipped TP manifests, the activator parks the first
    connection, the launcher starts a TP=2 pod whose two ranks share the GPU
    (``OMNIA_RANKS_PER_GPU=2`` -> ``ipc`` transport), the rank-0 runtime loads a
    Llama-3-70B-shaped 2-layer checkpoint (``Provider.spec.engine.checkpoint``,
    safetensors, sharded per rank on load), the turn streams through facade ->
    gRPC -> TP engine (graph decode, hand TP sampler), and the pod scales back to
    zero.  Every logits row of the turn (dumped by the engine's logit tap) equals
    the fp32 dense oracle of the checkpoint; a swapped kv head fails the gate."""
    from conftest import release_gpu_memory
    from served_oracle import check_tap, full_llama_weights, swapped_kv_head, to_f32

    from omnia_amd.models.config import resolve
    from omnia_amd.models.loader import save_hf_checkpoint

    release_gpu_memory()
    mc = resolve("llama-3-70b").replace(name="llama-3-70b-2l", num_layers=2)
    w = full_llama_weights(mc)
    ckpt = tmp_path / "ckpt"
    save_hf_checkpoint(w, mc, ckpt)
    w32 = to_f32(w)
    del w
    tap = tmp_path / "tap"
    monkeypatch.setenv("OMNIA_RANKS_PER_GPU", "2")
    monkeypatch.setenv("OMNIA_LOGIT_TAP", "1")
    monkeypatch.setenv("OMNIA_LOGIT_TAP_DIR", str(tap))
    cold, first = _scale_cycle({"model": "llama-3-70b-2l", "tp": 2, "checkpoint": str(ckpt),
                                "maxBatch": 8, "maxModelLen": 1024, "numBlocks": 256,
                                "blockSize": 16}, gpu_count=1)
    frac, worst, n = check_tap(str(tap), mc, w32)
    print(f"TP=2 pod: {n} rows, worst rel err {worst:.4f}, cold start {cold:.1f}s")
    assert n >= 6 and frac == 1.0, (frac, worst)
    bfrac, bworst, _ = check_tap(str(tap), mc, swapped_kv_head(w32, mc))
    assert bfrac < 1.0 and bworst > 0.05


def test_serve_tp2_checkpoint_pod_matches_oracle_cpu(tmp_path, monkeypatch):
    """CPU twin of the config-4 GPU oracle test: a TP=2 pod (gloo) loads an HF
    checkpoint named only by ``Provider.spec.engine.checkpoint`` (an unregistered
    model name -- the checkpoint's config.json is the architecture), serves the
    turn after scale-from-zero, and every logits row the engine dumped equals
    the fp32 dense oracle of that checkpoint."""
    import torch
    from served_oracle import check_tap, swapped_kv_head, to_f32

    from omnia_amd.models.config import resolve
    from omnia_amd.models.loader import save_hf_checkpoint

    mc = resolve("tiny-llama").replace(name="ckpt-llama")
    g = torch.Generator().manual_seed(5)
    d, D = mc.hidden_size, mc.head_dim

    def init(shape, std):
        return (torch.randn(shape, generator=g) * std).float()

    w = {"embed": init((mc.vocab_size, d), 0.5), "lm_head": init((mc.vocab_size, d), 0.5),
         "final_norm": torch.ones(d), "layers": []}
    for _ in range(mc.num_layers):
        w["layers"].append({"in_norm": torch.ones(d), "post_norm": torch.ones(d),
                            "qkv": init(((mc.num_heads + 2 * mc.num_kv_heads) * D, d), 0.08),
                            "o": init((d, mc.num_heads * D), 0.05),
                            "gate_up": init((2 * mc.intermediate_size, d), 0.08),
                            "down": init((d, mc.intermediate_size), 0.05)})
    ckpt = tmp_path / "ckpt"
    save_hf_checkpoint(w, mc, ckpt)
    tap = tmp_path / "tap"
    monkeypatch.setenv("OMNIA_LOGIT_TAP", "1")
    monkeypatch.setenv("OMNIA_LOGIT_TAP_DIR", str(tap))
    _scale_cycle({"model": "ckpt-llama", "tp": 2, "checkpoint": str(ckpt), "maxBatch": 4,
                  "maxModelLen": 512, "numBlocks": 64, "blockSize": 16, "dtype": "float32",
                  "useGraphs": False, "device": "cpu"})
    frac, worst, n = check_tap(str(tap), mc, to_f32(w), rel_tol=1e-3)
    assert n >= 6 and frac == 1.0, (frac, worst)
    bfrac, _, _ = check_tap(str(tap), mc, swapped_kv_head(to_f32(w), mc), rel_tol=1e-3)
    assert bfrac < 1.0
