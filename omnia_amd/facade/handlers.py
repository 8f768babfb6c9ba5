"""Facade message handlers (``internal/agent/{runtime,echo,demo}_handler.go``).

``RuntimeHandler`` opens one Converse stream per user message (as the
reference, ``runtime_handler.go:135``), relays chunk/done/error frames, forwards
CLIENT tool calls to the WebSocket client, waits for the client's ack (5 s)
and result (60 s), sends ``ClientToolResult`` back on the stream, and aborts
the turn after 120 s without runtime traffic (``:38-46``).  Server-side tool
calls and RuntimeHello are consumed, never forwarded.
"""
from __future__ import annotations

import asyncio
import json
import time

from ..utils.arrivals import mark
from ..api.proto import runtime_v1 as pb
from . import protocol as P

STREAM_INACTIVITY_S = 120.0
TOOL_ACK_TIMEOUT_S = 5.0
TOOL_RESULT_TIMEOUT_S = 60.0


class Writer:
    """Sink for server messages of one connection/turn."""

    async def write(self, msg: dict) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    async def write_chunk(self, session_id: str, session_json: str, content: str,
                          role: str = "") -> None:
        """A streamed ``chunk`` frame; writers that can send text override this
        with the pre-serialized fast path (``protocol.chunk_text``)."""
        await self.write(P.chunk(session_id, content, role))


class PendingTools:
    """Client-tool waits of the active turn, fed by the connection read loop."""

    def __init__(self):
        self.acks: dict[str, asyncio.Future] = {}
        self.results: dict[str, asyncio.Future] = {}

    def expect(self, call_id: str):
        loop = asyncio.get_running_loop()
        self.acks[call_id] = loop.create_future()
        self.results[call_id] = loop.create_future()

    def ack(self, call_id: str, ok: bool = True, reason: str = "") -> bool:
        f = self.acks.get(call_id)
        if f is None or f.done():
            return False
        f.set_result((ok, reason))
        if not ok:
            r = self.results.get(call_id)
            if r is not None and not r.done():
                r.set_result({"rejected": True, "reason": reason})
        return True

    def result(self, call_id: str, res: dict) -> bool:
        f = self.results.get(call_id)
        if f is None or f.done():
            return False
        a = self.acks.get(call_id)
        if a is not None and not a.done():
            a.set_result((True, ""))
        f.set_result(res)
        return True

    def clear(self, call_id: str):
        self.acks.pop(call_id, None)
        self.results.pop(call_id, None)


class RuntimeHandler:
    name = "runtime"

    def __init__(self, client, inactivity_s: float = STREAM_INACTIVITY_S,
                 ack_timeout_s: float = TOOL_ACK_TIMEOUT_S,
                 result_timeout_s: float = TOOL_RESULT_TIMEOUT_S):
        self.client = client
        self.inactivity_s = inactivity_s
        self.ack_timeout_s = ack_timeout_s
        self.result_timeout_s = result_timeout_s

    async def handle(self, session_id: str, msg: dict, writer: Writer, pending: PendingTools,
                     metadata: dict) -> dict:
        """Run one turn.  Returns {"content", "usage", "error"} for recording."""
        cm = pb.ClientMessage(session_id=session_id, content=msg.get("content", ""),
                              metadata={str(k): str(v) for k, v in
                                        (msg.get("metadata") or {}).items()},
                              consent_grants=list(msg.get("consent_grants") or []))
        for p in msg.get("parts") or []:
            part = cm.parts.add()
            part.type = p.get("type", "text")
            part.text = p.get("text", "")
            media = p.get("media") or {}
            part.media.data = media.get("data", "")
            part.media.url = media.get("url", "")
            part.media.mime_type = media.get("mime_type", "")
            part.media.storage_ref = media.get("storage_ref", "")
        stream = await self.client.open(metadata)
        out = {"content": "", "usage": None, "error": None, "ttft": None}
        t0 = time.perf_counter()
        sj = json.dumps(session_id) if session_id else ""
        # stream inactivity: one re-arming timer per turn instead of a wait_for
        # (a task + a timer) around every streamed frame
        loop = asyncio.get_running_loop()
        task = asyncio.current_task()
        wd = {"last": loop.time(), "fired": False, "h": None, "recv": False}

        def watchdog():
            if not wd["recv"]:  # only a wait on the runtime counts as inactivity
                wd["last"] = loop.time()
            idle = loop.time() - wd["last"]
            if idle >= self.inactivity_s:
                wd["fired"] = True
                task.cancel()
            else:
                wd["h"] = loop.call_later(self.inactivity_s - idle, watchdog)

        wd["h"] = loop.call_later(self.inactivity_s, watchdog)
        try:
            await stream.send(cm)
            while True:
                wd["recv"] = True
                wd["last"] = loop.time()  # idle = time in THIS wait on the runtime
                try:
                    resp = await stream.recv()
                except asyncio.CancelledError:
                    if not wd["fired"]:
                        raise
                    out["error"] = "stream inactivity timeout"
                    await writer.write(P.error(session_id, P.E_INTERNAL,
                                               "agent did not respond in time"))
                    return out
                wd["recv"] = False
                if resp is None:
                    out["error"] = "runtime stream closed"
                    await writer.write(P.error(session_id, P.E_AGENT_UNAVAILABLE,
                                               "agent stream closed unexpectedly"))
                    return out
                kind = resp.WhichOneof("message")
                if kind == "chunk":
                    if out["ttft"] is None:
                        out["ttft"] = time.perf_counter() - t0
                    c = resp.chunk
                    await writer.write_chunk(session_id, sj, c.content, c.role)
                elif kind == "done":
                    d = resp.done
                    usage = {"input_tokens": d.usage.input_tokens,
                             "output_tokens": d.usage.output_tokens,
                             "cost_usd": round(d.usage.cost_usd, 8)}
                    if d.usage.cached_tokens:  # prompt tokens served from cached KV
                        usage["cached_tokens"] = d.usage.cached_tokens
                    parts = [{"type": p.type, "text": p.text} for p in d.parts] or None
                    out.update(content=d.final_content, usage=usage)
                    mark("facade_done")
                    await writer.write(P.done(session_id, d.final_content, parts, usage))
                    return out
                elif kind == "error":
                    out["error"] = resp.error.code
                    await writer.write(P.error(session_id, resp.error.code or P.E_INTERNAL,
                                               resp.error.message))
                    return out
                elif kind == "tool_call":
                    tc = resp.tool_call
                    if tc.execution != pb.TOOL_EXECUTION_CLIENT:
                        continue  # server-side tools never reach the client
                    await self._client_tool(session_id, tc, writer, pending, stream)
                elif kind == "media_chunk":
                    import base64

                    mc = resp.media_chunk
                    await writer.write(P.server_msg(P.MEDIA_CHUNK, session_id, media_chunk={
                        "media_id": mc.media_id, "sequence": mc.sequence, "is_last": mc.is_last,
                        "mime_type": mc.mime_type,
                        "data": base64.b64encode(mc.data).decode()}))
                elif kind == "interruption":
                    await writer.write(P.server_msg(P.INTERRUPT, session_id))
                # runtime_hello: consumed
        finally:
            if wd["h"] is not None:
                wd["h"].cancel()
            await stream.close()

    async def _client_tool(self, session_id, tc, writer, pending: PendingTools, stream):
        try:
            args = json.loads(tc.arguments_json or "{}")
        except json.JSONDecodeError:
            args = {}
        pending.expect(tc.id)
        await writer.write(P.tool_call(session_id, tc.id, tc.name, args, tc.consent_message,
                                       list(tc.categories)))
        result = pb.ClientToolResult(call_id=tc.id)
        try:
            ok, reason = await asyncio.wait_for(pending.acks[tc.id], self.ack_timeout_s)
            if not ok:
                result.is_rejected = True
                result.rejection_reason = reason or "client rejected the tool call"
            else:
                res = await asyncio.wait_for(pending.results[tc.id], self.result_timeout_s)
                if res.get("rejected"):
                    result.is_rejected = True
                    result.rejection_reason = res.get("reason", "")
                elif res.get("error"):
                    result.result_json = json.dumps({"error": res["error"]})
                else:
                    result.result_json = json.dumps(res.get("result"))
        except asyncio.TimeoutError:
            result.is_rejected = True
            result.rejection_reason = "client tool timed out"
        finally:
            pending.clear(tc.id)
        await stream.send(pb.ClientMessage(session_id=session_id, client_tool_result=result))


class EchoHandler:
    name = "echo"

    async def handle(self, session_id, msg, writer, pending, metadata):
        content = msg.get("content", "")
        await writer.write(P.chunk(session_id, content))
        await writer.write(P.done(session_id, content))
        return {"content": content, "usage": None, "error": None}


class DemoHandler:
    """Canned streaming + simulated tool call, no runtime needed (demo_handler.go)."""

    name = "demo"

    async def handle(self, session_id, msg, writer, pending, metadata):
        text = msg.get("content", "")
        if "weather" in text.lower():
            await writer.write(P.server_msg(P.TOOL_CALL, session_id, tool_call={
                "id": "demo-1", "name": "get_weather", "arguments": {"city": "Paris"}}))
            reply = "It is 21°C and sunny in Paris."
        else:
            reply = f"You said: {text}. This is the Omnia demo agent."
        for w in reply.split(" "):
            await writer.write(P.chunk(session_id, w + " "))
            await asyncio.sleep(0)
        await writer.write(P.done(session_id, reply))
        return {"content": reply, "usage": None, "error": None}
