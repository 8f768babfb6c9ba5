"""Facade -> runtime client (``internal/facade/runtime_client.go:41-247``).

``GrpcRuntimeClient`` dials the runtime container over gRPC (gzip on Converse,
x-omnia-* identity metadata, never the raw Authorization header).
``InProcessRuntimeClient`` drives a :class:`RuntimeService` directly -- the
single-process "standalone" layout (``deployment_builder.go:174-176``) and the
tests.  Both expose the same small API.
"""
from __future__ import annotations

import asyncio

from ..utils import failpoints
from ..api.proto import runtime_v1 as pb


class RuntimeStream:
    async def send(self, msg: pb.ClientMessage):  # pragma: no cover - interface
        raise NotImplementedError

    async def recv(self) -> pb.ServerMessage | None:  # pragma: no cover
        raise NotImplementedError

    async def close(self):  # pragma: no cover
        pass


class _GrpcStream(RuntimeStream):
    def __init__(self, call, grpc_mod):
        self.call = call
        self.grpc = grpc_mod

    async def send(self, msg):
        await self.call.write(msg)

    async def recv(self):
        m = await self.call.read()
        return None if m is self.grpc.aio.EOF else m

    async def close(self):
        try:
            await self.call.done_writing()
        except Exception:  # noqa: BLE001
            pass
        self.call.cancel()


class GrpcRuntimeClient:
    def __init__(self, target: str = "127.0.0.1:9000", compression: bool = True):
        import grpc

        self.grpc = grpc
        self.target = target
        self.ch = grpc.aio.insecure_channel(target, options=[
            ("grpc.max_receive_message_length", 32 * 2**20)])
        comp = grpc.Compression.Gzip if compression else grpc.Compression.NoCompression
        self._converse = self.ch.stream_stream(
            pb.METHOD_CONVERSE, request_serializer=pb.ClientMessage.SerializeToString,
            response_deserializer=pb.ServerMessage.FromString)
        self._comp = comp
        self._invoke = self.ch.unary_unary(pb.METHOD_INVOKE,
                                           request_serializer=pb.InvocationRequest.SerializeToString,
                                           response_deserializer=pb.InvocationResponse.FromString)
        self._health = self.ch.unary_unary(pb.METHOD_HEALTH,
                                           request_serializer=pb.HealthRequest.SerializeToString,
                                           response_deserializer=pb.HealthResponse.FromString)
        self._has = self.ch.unary_unary(
            pb.METHOD_HAS_CONVERSATION,
            request_serializer=pb.HasConversationRequest.SerializeToString,
            response_deserializer=pb.HasConversationResponse.FromString)

    async def open(self, metadata: dict | None = None) -> RuntimeStream:
        md = tuple((k.lower(), str(v)) for k, v in (metadata or {}).items())
        call = self._converse(metadata=md, compression=self._comp)
        return _GrpcStream(call, self.grpc)

    async def invoke(self, req, metadata=None, timeout=None):
        md = tuple((k.lower(), str(v)) for k, v in (metadata or {}).items())
        return await self._invoke(req, metadata=md, timeout=timeout)

    async def health(self, timeout=5.0):
        return await self._health(pb.HealthRequest(), timeout=timeout)

    async def has_conversation(self, session_id, timeout=5.0):
        return await self._has(pb.HasConversationRequest(session_id=session_id), timeout=timeout)

    async def wait_ready(self, attempts: int = 60, delay: float = 0.5) -> bool:
        """Dial with retry (cmd/agent/runtime_dial.go:47-112)."""
        for _ in range(attempts):
            try:
                failpoints.hit("runtime.dial")
                h = await self.health(timeout=2.0)
                if h.healthy:
                    return True
            except Exception:  # noqa: BLE001
                pass
            await asyncio.sleep(delay)
        return False

    async def close(self):
        await self.ch.close()


class _QStream(RuntimeStream):
    def __init__(self, svc, md):
        from ..runtime.server import QueueStream

        self.q = QueueStream(md)
        self.task = asyncio.get_running_loop().create_task(svc.converse(self.q))
        self._closed = False

    async def send(self, msg):
        await self.q.inbox.put(msg)

    async def recv(self):
        get = asyncio.ensure_future(self.q.outbox.get())
        done, _ = await asyncio.wait({get, self.task}, return_when=asyncio.FIRST_COMPLETED)
        if get in done:
            return get.result()
        get.cancel()
        if not self.q.outbox.empty():
            return self.q.outbox.get_nowait()
        return None

    async def close(self):
        if not self._closed:
            self._closed = True
            self.q.close()
            try:
                await asyncio.wait_for(self.task, 5)
            except Exception:  # noqa: BLE001
                self.task.cancel()


class InProcessRuntimeClient:
    def __init__(self, svc):
        self.svc = svc

    async def open(self, metadata=None) -> RuntimeStream:
        return _QStream(self.svc, dict(metadata or {}))

    async def invoke(self, req, metadata=None, timeout=None):
        return await asyncio.wait_for(self.svc.invoke(req, metadata), timeout)

    async def health(self, timeout=5.0):
        return await self.svc.health()

    async def has_conversation(self, session_id, timeout=5.0):
        return await self.svc.has_conversation(pb.HasConversationRequest(session_id=session_id))

    async def wait_ready(self, attempts=1, delay=0.0):
        return True

    async def close(self):
        pass
