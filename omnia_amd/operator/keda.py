"""Single-node KEDA: ScaledObject evaluation + a scale-from-zero activator.

In a cluster the reference delegates to KEDA (``internal/controller/
autoscaling.go:167-325``): the AgentRuntime reconciler writes a ScaledObject
whose default trigger is ``sum(omnia_agent_connections_active{agent, namespace})``
against a per-pod threshold (``constants.go:47-49``: 200), with ``minReplicas: 0``
enabling scale-to-zero (``api/v1alpha1/agentruntime_types.go:318-375``).  On a
single 8x MI355X node (``omnia serve``) nothing runs KEDA, so the launcher runs
this module instead:

* :class:`KedaScaler` evaluates every ScaledObject each ``pollingInterval``
  seconds.  Prometheus triggers are evaluated locally (:func:`eval_query`, the
  PromQL subset the operator itself emits: ``sum|max|min|avg|count(selector)``
  with an optional ``or vector(c)``) over samples scraped from the target's
  ready facades plus the activator's parked connections; ``cron`` triggers are
  honoured too.  Replica math follows KEDA/HPA: active -> ``ceil(value /
  threshold)`` clamped to ``[max(1, min), max]``, scale-up immediately,
  scale-down after ``cooldownPeriod`` without activity (to ``minReplicaCount``,
  possibly 0).  The Deployment's ``spec.replicas`` is patched (the AgentRuntime
  reconciler keeps an autoscaled Deployment's replica count) and the
  ScaledObject gets KEDA-shaped status (``Ready`` / ``Active`` conditions,
  ``lastActiveTime``, ``currentReplicas``).
* :class:`Activator` is the scale-from-zero front (the KEDA HTTP add-on
  interceptor's role): when a ScaledObject allows zero replicas the Service's
  stable endpoint is the activator, which relays WebSocket and HTTP traffic to a
  ready replica, and when there is none PARKS the connection (counted as an
  active connection of the agent, so the trigger fires), waits for the first
  replica to become ready, then relays.  A parked request that outlives
  ``OMNIA_ACTIVATOR_TIMEOUT_S`` (default 900 s: a TP=8 70B cold start) gets 503.
"""
from __future__ import annotations

import asyncio
import logging
import math
import random
import re
import time

log = logging.getLogger("omnia.keda")

ANN_COLD_START = "omnia.altairalabs.ai/cold-start-seconds"


# ------------------------------------------------------------------ PromQL subset
_SAMPLE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{(.*)\})?\s+(\S+)')
_LABEL = re.compile(r'([a-zA-Z_][a-zA-Z0-9_]*)\s*(=~|!=|=)\s*"((?:[^"\\]|\\.)*)"')


def parse_prom_text(text: str) -> list[tuple[str, dict, float]]:
    """Prometheus text exposition -> ``[(name, labels, value)]``."""
    out = []
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        m = _SAMPLE.match(line)
        if not m:
            continue
        labels = {k: v for k, _, v in _LABEL.findall(m.group(3) or "")}
        try:
            out.append((m.group(1), labels, float(m.group(4))))
        except ValueError:
            continue
    return out


def _selector(sel: str):
    m = re.fullmatch(r'\s*([a-zA-Z_:][a-zA-Z0-9_:]*)\s*(\{(.*)\})?\s*', sel)
    if not m:
        raise ValueError(f"unsupported selector: {sel!r}")
    matchers = _LABEL.findall(m.group(3) or "")

    def match(name, labels):
        if name != m.group(1):
            return False
        for k, op, v in matchers:
            have = labels.get(k, "")
            if op == "=" and have != v:
                return False
            if op == "!=" and have == v:
                return False
            if op == "=~" and not re.fullmatch(v, have):
                return False
        return True

    return match


def eval_query(query: str, samples: list[tuple[str, dict, float]]) -> float | None:
    """Evaluate ``agg(selector) [or vector(c)]`` or a bare selector; ``None`` when
    no series matched and there is no ``or vector`` fallback."""
    q = query.strip()
    fallback = None
    m = re.fullmatch(r"(.*?)\s+or\s+vector\(\s*([-0-9.eE+]+)\s*\)", q)
    if m:
        q, fallback = m.group(1).strip(), float(m.group(2))
    m = re.fullmatch(r"(sum|max|min|avg|count)\s*(?:by\s*\([^)]*\)\s*)?\((.*)\)", q, re.S)
    agg, sel = (m.group(1), m.group(2)) if m else (None, q)
    match = _selector(sel)
    vals = [v for n, lab, v in samples if match(n, lab)]
    if not vals:
        return fallback
    if agg in (None, "sum"):
        return float(sum(vals))
    if agg == "max":
        return float(max(vals))
    if agg == "min":
        return float(min(vals))
    if agg == "avg":
        return float(sum(vals) / len(vals))
    return float(len(vals))


def _cron_active(md: dict, now: float) -> bool:
    """KEDA cron trigger: active between ``start`` and ``end`` (5-field crons):
    inside a window exactly when the next ``end`` comes before the next ``start``."""
    from ..utils.cron import next_fire

    try:
        return next_fire(md["end"], now) < next_fire(md["start"], now)
    except Exception:  # noqa: BLE001 - malformed: never active
        return False


# ------------------------------------------------------------------ scaler
class KedaScaler:
    """Evaluates ScaledObjects of ``store`` and patches their Deployments.

    ``samples_fn(ns, name) -> list[(metric, labels, value)]`` returns the
    target's current metric samples (the launcher scrapes its facades and adds
    the activator's parked connections)."""

    def __init__(self, store, samples_fn, clock=time.monotonic):
        self.store = store
        self.samples_fn = samples_fn
        self.clock = clock
        self.state: dict[tuple, dict] = {}

    def scale_to_zero_targets(self) -> set[tuple]:
        return {(so["metadata"]["namespace"], so["spec"]["scaleTargetRef"]["name"])
                for so in self.store.list("ScaledObject")
                if int(so["spec"].get("minReplicaCount", 0) or 0) == 0}

    async def tick(self):
        now = self.clock()
        live = set()
        for so in self.store.list("ScaledObject"):
            ns, name = so["metadata"]["namespace"], so["metadata"]["name"]
            key = (ns, name)
            live.add(key)
            spec = so["spec"]
            st = self.state.setdefault(key, {"last_poll": -1e18, "last_active": now,
                                             "last_up": -1e18, "last_ready": -1e18,
                                             "ready": 0})
            if now - st["last_poll"] < float(spec.get("pollingInterval", 30)):
                continue
            st["last_poll"] = now
            target = spec["scaleTargetRef"]["name"]
            dep = self.store.try_get("Deployment", target, ns)
            if dep is None:
                continue
            try:
                samples = await self.samples_fn(ns, target)
            except Exception as e:  # noqa: BLE001 - a scrape failure keeps the count
                log.warning("scaledobject %s/%s: metrics unavailable: %s", ns, name, e)
                continue
            ready = int((dep.get("status") or {}).get("readyReplicas", 0) or 0)
            if ready > st["ready"]:
                st["last_ready"] = now  # cooldown counts from a replica becoming ready
            st["ready"] = ready
            lo = int(spec.get("minReplicaCount", 0) or 0)
            hi = int(spec.get("maxReplicaCount", 100) or 100)
            cur = int(dep["spec"].get("replicas", 0) or 0)
            active, want, metric = False, 0, None
            for trig in spec.get("triggers") or []:
                md = trig.get("metadata") or {}
                if trig.get("type") == "prometheus":
                    v = eval_query(md.get("query", ""), samples)
                    v = 0.0 if v is None else v
                    metric = v if metric is None else max(metric, v)
                    if v > float(md.get("activationThreshold", 0) or 0):
                        active = True
                        thr = max(1e-9, float(md.get("threshold", 1) or 1))
                        want = max(want, math.ceil(v / thr))
                elif trig.get("type") == "cron":
                    if _cron_active(md, time.time()):
                        active = True
                        want = max(want, int(md.get("desiredReplicas", 1) or 1))
            cool = float(spec.get("cooldownPeriod", 300))
            if active:
                st["last_active"] = now
                desired = min(hi, max(want, lo, 1))
                if desired < cur and now - st["last_up"] < cool:
                    desired = cur  # hold a recent scale-up (HPA stabilisation)
            elif now - max(st["last_active"], st["last_ready"]) >= cool:
                desired = lo
            else:
                desired = max(cur, lo)
            if desired != cur:
                if desired > cur:
                    st["last_up"] = now
                dep["spec"]["replicas"] = desired
                dep["metadata"].pop("resourceVersion", None)
                self.store.apply(dep)
                log.info("scaledobject %s/%s: %s -> %d replicas (metric %s)", ns, name, cur,
                         desired, metric)
            self._status(so, active, desired, metric, st)
        for key in [k for k in self.state if k not in live]:
            self.state.pop(key)

    def _status(self, so, active, replicas, metric, st):
        from .apistore import set_condition

        gen = so["metadata"].get("generation", 1)
        s = dict(so.get("status") or {})
        before = dict(s)
        set_condition(s, "Ready", True, "ScaledObjectReady", "single-node scaler", gen)
        set_condition(s, "Active", active, "ScalerActive" if active else "ScalerNotActive",
                      "", gen)
        s["currentReplicas"] = replicas
        if metric is not None:
            s["metricValue"] = metric
        if active:
            s["lastActiveTime"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        if s != before:
            so["status"] = s
            so["metadata"].pop("resourceVersion", None)
            self.store.update_status(so)


# ------------------------------------------------------------------ activator
class Activator:
    """Stable front of a scale-to-zero agent (WebSocket + HTTP relay).

    ``backends`` is a list of ``host:port`` of ready facades (kept current by the
    launcher); :attr:`parked` counts connections waiting for the first one."""

    def __init__(self, agent: str, namespace: str, timeout_s: float | None = None):
        import os

        self.agent, self.namespace = agent, namespace
        self.backends: list[str] = []
        self.parked = 0
        self.connecting = 0  # released from parking, upstream handshake not done yet
        self.relayed = 0
        self.timeout_s = timeout_s if timeout_s is not None else float(
            os.environ.get("OMNIA_ACTIVATOR_TIMEOUT_S", "900"))
        self._ready = asyncio.Event()
        self.runner = None
        self.endpoint = None
        self._session = None

    def set_backends(self, eps: list[str]):
        self.backends = list(eps)
        if self.backends:
            self._ready.set()
        else:
            self._ready.clear()

    def samples(self) -> list[tuple[str, dict, float]]:
        """Connections the facades cannot see yet: parked ones, and released ones
        whose upstream handshake is still in flight (once it completes the
        facade's own ``omnia_agent_connections_active`` counts them)."""
        return [("omnia_agent_connections_active",
                 {"agent": self.agent, "namespace": self.namespace},
                 float(self.parked + self.connecting))]

    async def _backend(self) -> str | None:
        if self.backends:
            return random.choice(self.backends)
        self.connecting -= 1  # counted as parked while it waits
        self.parked += 1
        try:
            await asyncio.wait_for(self._ready.wait(), self.timeout_s)
        except asyncio.TimeoutError:
            return None
        finally:
            self.parked -= 1
            self.connecting += 1
        return random.choice(self.backends) if self.backends else None

    async def start(self, host: str = "127.0.0.1", port: int = 0) -> str:
        import aiohttp
        from aiohttp import web

        self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None))
        app = web.Application(client_max_size=32 * 2**20)
        app.router.add_get("/activator/healthz", self._health)
        app.router.add_route("*", "/{tail:.*}", self._handle)
        self.runner = web.AppRunner(app)
        await self.runner.setup()
        site = web.TCPSite(self.runner, host, port)
        await site.start()
        self.endpoint = f"{host}:{site._server.sockets[0].getsockname()[1]}"
        return self.endpoint

    async def stop(self):
        if self.runner is not None:
            await self.runner.cleanup()
        if self._session is not None:
            await self._session.close()

    async def _health(self, _request):
        from aiohttp import web

        return web.json_response({"backends": len(self.backends), "parked": self.parked})

    async def _handle(self, request):
        tok = {"counted": True}
        self.connecting += 1
        try:
            return await self._route(request, tok)
        finally:
            self._release(tok)

    def _release(self, tok):
        """The request is now visible to a facade (or done): stop counting it."""
        if tok["counted"]:
            tok["counted"] = False
            self.connecting -= 1

    async def _route(self, request, tok):
        from aiohttp import web

        be = await self._backend()
        if be is None:
            return web.json_response({"error": "no replica became ready"}, status=503,
                                     headers={"Retry-After": "5"})
        self.relayed += 1
        url = f"http://{be}{request.rel_url}"
        hop = {"host", "connection", "upgrade", "sec-websocket-key", "sec-websocket-version",
               "sec-websocket-extensions", "sec-websocket-protocol", "content-length",
               "transfer-encoding"}
        headers = {k: v for k, v in request.headers.items() if k.lower() not in hop}
        if request.headers.get("Upgrade", "").lower() == "websocket":
            return await self._relay_ws(request, url.replace("http://", "ws://", 1), headers,
                                        tok)
        body = await request.read()
        async with self._session.request(request.method, url, data=body or None,
                                         headers=headers) as r:
            resp = web.StreamResponse(status=r.status, headers={
                k: v for k, v in r.headers.items()
                if k.lower() not in ("content-length", "transfer-encoding", "connection")})
            await resp.prepare(request)
            async for chunk in r.content.iter_chunked(1 << 16):
                await resp.write(chunk)
            await resp.write_eof()
            return resp

    async def _relay_ws(self, request, url, headers, tok):
        import aiohttp
        from aiohttp import web

        protos = [p.strip() for p in request.headers.get("Sec-WebSocket-Protocol", "").split(",")
                  if p.strip()]
        try:
            up = await self._session.ws_connect(url, headers=headers, protocols=protos,
                                                max_msg_size=16 * 2**20)
        except aiohttp.WSServerHandshakeError as e:
            return web.json_response({"error": "upstream refused"}, status=e.status or 502)
        self._release(tok)  # the facade counts this connection now
        down = web.WebSocketResponse(protocols=(up.protocol,) if up.protocol else (),
                                     max_msg_size=16 * 2**20)
        await down.prepare(request)

        async def pump(src, dst):
            async for m in src:
                if m.type == aiohttp.WSMsgType.TEXT:
                    await dst.send_str(m.data)
                elif m.type == aiohttp.WSMsgType.BINARY:
                    await dst.send_bytes(m.data)
                elif m.type in (aiohttp.WSMsgType.CLOSE, aiohttp.WSMsgType.CLOSING,
                                aiohttp.WSMsgType.CLOSED, aiohttp.WSMsgType.ERROR):
                    break
            await dst.close()

        t1 = asyncio.ensure_future(pump(up, down))
        t2 = asyncio.ensure_future(pump(down, up))
        await asyncio.wait([t1, t2], return_when=asyncio.FIRST_COMPLETED)
        for t in (t1, t2):
            t.cancel()
        await asyncio.gather(t1, t2, return_exceptions=True)
        await up.close()
        await down.close()
        return down
