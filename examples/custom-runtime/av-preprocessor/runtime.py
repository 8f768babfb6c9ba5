"""A third-party ``omnia.runtime.v1`` runtime: an audio/video preprocessor that
any AgentRuntime can use in place of the stock runtime (the facade only speaks
the gRPC contract).  Behaviour mirrors the reference example
(``examples/custom-runtime/av-preprocessor/main.go``): Health advertises the
contract version and ``invoke``; Converse sends ``RuntimeHello`` first, then a
chunk + done per client message; Invoke answers JSON; HasConversation says the
runtime keeps no conversations.

The preprocessing stage is MI355X-native where the reference wires a PromptKit
video-to-frames stage: PCM16 audio parts (``audio/pcm`` or ``audio/L16``, base64)
become 80-bin log-mel frames through ``torch.stft`` on the GPU when one is
visible (the CPU otherwise); the reply reports the frame count.

It depends only on the contract module (``omnia_amd.api.proto.runtime_v1``), not
on the stock runtime.  Run it with ``python runtime.py`` (``OMNIA_GRPC_PORT``,
default 9000) and check it with ``omnia conformance --target 127.0.0.1:9000``;
``conformance_test.py`` next to this file does both.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
from omnia_amd.api.proto import runtime_v1 as pb  # noqa: E402

GREETING = "hello from av-preprocessor"
CAPABILITIES = [pb.CAP_INVOKE]
log = logging.getLogger("av-preprocessor")


class LogMelStage:
    """PCM16 mono -> [frames, n_mels] log-mel features (25 ms window, 10 ms hop)."""

    def __init__(self, sample_rate: int = 16000, n_mels: int = 80):
        import torch

        self.torch = torch
        self.sr, self.n_mels = sample_rate, n_mels
        self.n_fft, self.hop = int(0.025 * sample_rate), int(0.010 * sample_rate)
        self.device = "cuda" if torch.cuda.is_available() else "cpu"
        self.window = torch.hann_window(self.n_fft, device=self.device)
        self.fbank = self._mel_fbank().to(self.device)

    def _mel_fbank(self):
        t = self.torch
        n_freq = self.n_fft // 2 + 1
        mel = lambda f: 2595.0 * t.log10(1.0 + f / 700.0)  # noqa: E731
        inv = lambda m: 700.0 * (10 ** (m / 2595.0) - 1.0)  # noqa: E731
        pts = inv(t.linspace(mel(t.tensor(0.0)), mel(t.tensor(self.sr / 2.0)),
                             self.n_mels + 2))
        freqs = t.linspace(0, self.sr / 2.0, n_freq)
        lo, ce, hi = pts[:-2, None], pts[1:-1, None], pts[2:, None]
        up = (freqs[None] - lo) / (ce - lo)
        down = (hi - freqs[None]) / (hi - ce)
        return t.clamp(t.minimum(up, down), min=0.0)  # [n_mels, n_freq]

    def __call__(self, pcm16: bytes):
        t = self.torch
        x = t.frombuffer(bytearray(pcm16), dtype=t.int16).to(self.device, t.float32) / 32768.0
        if x.numel() < self.n_fft:
            return t.zeros(0, self.n_mels)
        spec = t.stft(x, self.n_fft, self.hop, window=self.window, return_complex=True,
                      center=False).abs().pow(2)  # [n_freq, frames]
        return t.log(self.fbank @ spec + 1e-6).t().cpu()


_stage = None


def stage() -> LogMelStage:
    global _stage
    if _stage is None:
        _stage = LogMelStage()
    return _stage


def describe(parts) -> str:
    frames = 0
    for p in parts:
        m = p.media if p.HasField("media") else None
        if m is not None and m.mime_type.split(";")[0] in ("audio/pcm", "audio/L16") and m.data:
            frames += int(stage()(base64.b64decode(m.data)).shape[0])
    return f" ({frames} log-mel frames)" if frames else ""


async def health(req, context):
    return pb.HealthResponse(healthy=True, status="ok", contract_version=pb.CONTRACT_VERSION,
                             capabilities=CAPABILITIES)


async def converse(request_iterator, context):
    yield pb.ServerMessage(runtime_hello=pb.RuntimeHello(capabilities=CAPABILITIES))
    async for msg in request_iterator:
        text = GREETING + describe(msg.parts)
        yield pb.ServerMessage(chunk=pb.Chunk(content=text))
        yield pb.ServerMessage(done=pb.Done(final_content=text))


async def invoke(req, context):
    return pb.InvocationResponse(output_json=json.dumps({"message": GREETING}),
                                 invocation_id=req.invocation_id)


async def has_conversation(req, context):
    return pb.HasConversationResponse(state=pb.RESUME_STATE_NOT_FOUND)


def handler():
    import grpc

    return grpc.method_handlers_generic_handler(pb.SERVICE, {
        "Converse": grpc.stream_stream_rpc_method_handler(
            converse, request_deserializer=pb.ClientMessage.FromString,
            response_serializer=pb.ServerMessage.SerializeToString),
        "Invoke": grpc.unary_unary_rpc_method_handler(
            invoke, request_deserializer=pb.InvocationRequest.FromString,
            response_serializer=pb.InvocationResponse.SerializeToString),
        "Health": grpc.unary_unary_rpc_method_handler(
            health, request_deserializer=pb.HealthRequest.FromString,
            response_serializer=pb.HealthResponse.SerializeToString),
        "HasConversation": grpc.unary_unary_rpc_method_handler(
            has_conversation, request_deserializer=pb.HasConversationRequest.FromString,
            response_serializer=pb.HasConversationResponse.SerializeToString)})


async def serve(port: int, host: str = "0.0.0.0"):
    import grpc

    server = grpc.aio.server()
    server.add_generic_rpc_handlers((handler(),))
    bound = server.add_insecure_port(f"{host}:{port}")
    await server.start()
    return server, bound


async def _main():
    logging.basicConfig(level=logging.INFO)
    server, port = await serve(int(os.environ.get("OMNIA_GRPC_PORT", "9000")))
    log.info("av-preprocessor: serving omnia.runtime.v1 on :%d (log-mel stage on %s)", port,
             "cuda" if __import__("torch").cuda.is_available() else "cpu")
    await server.wait_for_termination()


if __name__ == "__main__":
    asyncio.run(_main())
