"""Drive bench waves through the full runtime turn path in-process.

Each synthetic turn is a real ``omnia.runtime.v1`` Converse exchange against a
:class:`RuntimeService` (hello -> chunks -> Done{usage}) whose agent renders the
PromptPack + Llama-3 chat template and streams from the in-node engine.  TTFT =
first Chunk frame, turn latency = Done, tokens = Done.usage.output_tokens -- the
arena fleet client's definitions (``ee/pkg/arena/fleet/client.go:124-157``).
"""
from __future__ import annotations

import asyncio
import os
import threading
import time

from ..api.proto import runtime_v1 as pb
from .agent import Agent, AgentConfig
from .context_store import MemoryContextStore
from .promptpack import PromptPack
from .providers import LocalEngineProvider
from .server import QueueStream, RuntimeService


class _TokenIdProvider(LocalEngineProvider):
    """Local provider fed pre-tokenised synthetic prompts (exact prompt length)."""

    def __init__(self, engine, params, prompts: dict):
        super().__init__(engine)
        self.params = params
        self.prompts = prompts
        self.trace = None

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        from .providers import ProviderEvent, Usage

        ids = self.prompts.pop(session_id)
        usage = Usage(input_tokens=len(ids))
        tr = self.trace.setdefault(session_id, {}) if self.trace is not None else None
        if tr is not None:
            tr["submit"] = time.perf_counter()
        async for ev in self.engine.generate(ids, self.params, session_id=session_id):
            if tr is not None and "first" not in tr:
                tr["first"] = time.perf_counter()
            if ev.text or ev.token is not None:
                yield ProviderEvent("text", text=ev.text or " ")
            if ev.finished:
                if tr is not None:
                    tr["finished"] = time.perf_counter()
                usage.output_tokens = ev.output_tokens
                usage.cached_tokens = ev.cached_tokens
                yield ProviderEvent("done", usage=usage, finish_reason=ev.finish_reason or "")
                return


class RuntimeBenchDriver:
    def __init__(self, aeng, params):
        """``aeng``: an :class:`AsyncLLMEngine` or an engine-core client."""
        self.aeng = aeng
        self.params = params
        self.prompts: dict = {}
        self.provider = _TokenIdProvider(self.aeng, params, self.prompts)
        if os.environ.get("OMNIA_BENCH_TRACE"):
            self.provider.trace = {}
        agent = Agent(PromptPack.minimal("You are a benchmark agent."), self.provider,
                      MemoryContextStore(), None, AgentConfig())
        self.svc = RuntimeService(agent)
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self.loop.run_forever, daemon=True)
        self.thread.start()

    async def _one(self, sid: str):
        st = QueueStream({"x-omnia-session-id": sid})
        task = asyncio.ensure_future(self.svc.converse(st))
        t0 = time.perf_counter()
        await st.inbox.put(pb.ClientMessage(session_id=sid, content="bench"))
        ttft = None
        out_tokens = 0
        while True:
            f = await st.outbox.get()
            k = f.WhichOneof("message")
            if k == "chunk" and ttft is None:
                ttft = time.perf_counter() - t0
            elif k == "done":
                out_tokens = f.done.usage.output_tokens
                break
            elif k == "error":
                break
        lat = time.perf_counter() - t0
        st.close()
        await task
        return ttft, lat, out_tokens

    async def _wave(self, prompts, step):
        sids = []
        for i, p in enumerate(prompts):
            sid = f"bench-{step}-{i}"
            self.prompts[sid] = p
            sids.append(sid)
        t_w = time.perf_counter()
        res = await asyncio.gather(*(self._one(s) for s in sids))
        t_end = time.perf_counter()
        for s in sids:
            self.aeng.drop_session(s)
        if self.provider.trace is not None:
            self._report(t_w, t_end, sids)
        return res

    def _report(self, t_w, t_end, sids):
        import sys

        tr = [self.provider.trace.pop(s, {}) for s in sids]

        def q(key):
            v = sorted(t[key] - t_w for t in tr if key in t)
            return (f"{key}: min {v[0]*1e3:.0f} p50 {v[len(v)//2]*1e3:.0f} "
                    f"max {v[-1]*1e3:.0f} ms") if v else f"{key}: -"

        print(f"[wave] {q('submit')} | {q('first')} | {q('finished')} | "
              f"end {(t_end - t_w)*1e3:.0f} ms", file=sys.stderr)

    def run_wave(self, prompts, step):
        fut = asyncio.run_coroutine_threadsafe(self._wave(prompts, step), self.loop)
        return fut.result()

    def close(self):
        self.aeng.shutdown()
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(timeout=5)
