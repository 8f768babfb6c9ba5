"""Protocol conformance suite for ``omnia.runtime.v1`` runtimes.

Re-implementation of ``pkg/runtime/conformance/conformance.go:45-100`` /
``checks.go:44-230`` (CLI ``cmd/runtime-conformance/main.go:39-89``): protocol
only, no model-quality assertions.  Checks:

  health/contract          Health healthy, semver contract_version, capabilities
  hello-first              first ServerMessage is RuntimeHello, caps == Health's
  text-turn-shape          a turn ends with Done; no Done before the hello
  graceful-malformed-input empty ClientMessage{session_id} -> no Internal/Unknown/DataLoss
  invoke-honesty           advertised invoke => not Unimplemented; else Unimplemented
  duplex-honesty           advertised duplex_audio => DuplexStart yields an on-protocol frame

Usage: ``python -m omnia_amd.runtime.conformance --target 127.0.0.1:9000``
"""
from __future__ import annotations

import argparse
import asyncio
import re
import sys
import uuid
from dataclasses import dataclass

from ..api.proto import runtime_v1 as pb

SEMVER = re.compile(r"^\d+\.\d+\.\d+(-[0-9A-Za-z.-]+)?$")


@dataclass
class CheckResult:
    name: str
    passed: bool
    detail: str = ""


class Client:
    def __init__(self, target: str, timeout: float = 30.0):
        import grpc

        self.grpc = grpc
        self.ch = grpc.aio.insecure_channel(target)
        self.timeout = timeout
        self.health = self.ch.unary_unary(pb.METHOD_HEALTH,
                                          request_serializer=pb.HealthRequest.SerializeToString,
                                          response_deserializer=pb.HealthResponse.FromString)
        self.invoke = self.ch.unary_unary(
            pb.METHOD_INVOKE, request_serializer=pb.InvocationRequest.SerializeToString,
            response_deserializer=pb.InvocationResponse.FromString)
        self.has_conv = self.ch.unary_unary(
            pb.METHOD_HAS_CONVERSATION,
            request_serializer=pb.HasConversationRequest.SerializeToString,
            response_deserializer=pb.HasConversationResponse.FromString)
        self.converse = self.ch.stream_stream(
            pb.METHOD_CONVERSE, request_serializer=pb.ClientMessage.SerializeToString,
            response_deserializer=pb.ServerMessage.FromString)

    async def turn(self, msgs: list, max_frames: int = 10000, stop_on_done=True):
        """Send msgs, collect frames until Done/Error (or stream end)."""
        call = self.converse(timeout=self.timeout)
        for m in msgs:
            await call.write(m)
        frames = []
        try:
            while len(frames) < max_frames:
                f = await call.read()
                if f is self.grpc.aio.EOF:
                    break
                frames.append(f)
                kind = f.WhichOneof("message")
                if stop_on_done and kind in ("done", "error"):
                    break
        finally:
            await call.done_writing()
            call.cancel()
        return frames

    async def close(self):
        await self.ch.close()


async def run(target: str, timeout: float = 30.0) -> list[CheckResult]:
    c = Client(target, timeout)
    out: list[CheckResult] = []
    try:
        # health/contract
        h = await c.health(pb.HealthRequest(), timeout=timeout)
        caps = list(h.capabilities)
        ok = h.healthy and bool(SEMVER.match(h.contract_version)) and len(caps) > 0
        out.append(CheckResult("health/contract", ok,
                               f"healthy={h.healthy} version={h.contract_version} caps={caps}"))
        sid = str(uuid.uuid4())
        frames = await c.turn([pb.ClientMessage(session_id=sid, content="conformance ping")])
        kinds = [f.WhichOneof("message") for f in frames]
        hello_ok = bool(frames) and kinds[0] == "runtime_hello" and \
            sorted(frames[0].runtime_hello.capabilities) == sorted(caps)
        out.append(CheckResult("hello-first", hello_ok, f"frames={kinds[:4]}"))
        shape_ok = "done" in kinds and kinds.index("done") > 0 and kinds[-1] == "done"
        out.append(CheckResult("text-turn-shape", shape_ok, f"frames={kinds[-3:]}"))
        # malformed input
        try:
            frames = await c.turn([pb.ClientMessage(session_id=str(uuid.uuid4()))])
            out.append(CheckResult("graceful-malformed-input", True,
                                   f"frames={[f.WhichOneof('message') for f in frames]}"))
        except c.grpc.aio.AioRpcError as e:
            bad = e.code() in (c.grpc.StatusCode.INTERNAL, c.grpc.StatusCode.UNKNOWN,
                               c.grpc.StatusCode.DATA_LOSS)
            out.append(CheckResult("graceful-malformed-input", not bad, str(e.code())))
        # invoke honesty
        adv = pb.CAP_INVOKE in caps
        try:
            await c.invoke(pb.InvocationRequest(input_json='{"ping":true}',
                                                invocation_id=str(uuid.uuid4())),
                           timeout=timeout)
            out.append(CheckResult("invoke-honesty", adv, "invoke answered"))
        except c.grpc.aio.AioRpcError as e:
            unimpl = e.code() == c.grpc.StatusCode.UNIMPLEMENTED
            out.append(CheckResult("invoke-honesty", (not adv) == unimpl or (adv and not unimpl),
                                   str(e.code())))
        # duplex honesty
        adv = pb.CAP_DUPLEX_AUDIO in caps
        if adv:
            try:
                frames = await c.turn([pb.ClientMessage(
                    session_id=str(uuid.uuid4()),
                    duplex_start=pb.DuplexStart(codec="pcm", sample_rate=16000, channels=1))],
                    max_frames=1, stop_on_done=False)
                out.append(CheckResult("duplex-honesty", bool(frames),
                                       f"frames={[f.WhichOneof('message') for f in frames]}"))
            except c.grpc.aio.AioRpcError as e:
                out.append(CheckResult("duplex-honesty", False, str(e.code())))
        else:
            out.append(CheckResult("duplex-honesty", True, "duplex_audio not advertised"))
    finally:
        await c.close()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="omnia.runtime.v1 conformance suite")
    ap.add_argument("--target", default="127.0.0.1:9000")
    ap.add_argument("--timeout", type=float, default=30.0)
    a = ap.parse_args(argv)
    res = asyncio.run(run(a.target, a.timeout))
    for r in res:
        print(f"[{'PASS' if r.passed else 'FAIL'}] {r.name}: {r.detail}")
    sys.exit(0 if all(r.passed for r in res) else 1)


if __name__ == "__main__":
    main()
