"""Duplex (realtime audio) sessions, SURVEY §3.4.

Real PCM16 signals end to end: the mock STT/TTS speak an FSK "voice" (text <->
tones), so VAD segmentation, transcription, the agent turn, sentence-wise TTS,
MediaChunk framing, barge-in and the facade's binary audio path are all
exercised without a speech model."""
import asyncio

import pytest

from omnia_amd.api.proto import runtime_v1 as pb
from omnia_amd.runtime import duplex as D
from omnia_amd.runtime.agent import Agent, AgentConfig
from omnia_amd.runtime.context_store import MemoryContextStore
from omnia_amd.runtime.promptpack import PromptPack
from omnia_amd.runtime.providers import MockProvider, Provider, ProviderEvent, Usage
from omnia_amd.runtime.server import QueueStream, RuntimeService

RATE = 16000
FRAME = RATE // 50 * 2  # 20 ms of pcm16


def speech(text: str, lead_ms=100, tail_ms=400) -> bytes:
    return D.pcm16_silence(lead_ms) + D.FSKCodec(RATE).encode(text) + D.pcm16_silence(tail_ms)


def frames_of(pcm: bytes):
    return [pcm[i:i + FRAME] for i in range(0, len(pcm), FRAME)]


def test_fsk_roundtrip_and_vad_segmentation():
    codec = D.FSKCodec(RATE)
    assert codec.decode(codec.encode("Hello, MI355X!")) == "Hello, MI355X!"
    # misaligned start (7 ms of silence) still decodes
    assert codec.decode(D.pcm16_silence(7) + codec.encode("abc")) == "abc"
    vad = D.EnergyVAD(RATE)
    events = []
    for f in frames_of(speech("first") + speech("second one")):
        events += vad.feed(f)
    kinds = [e[0] for e in events]
    assert kinds == ["start", "end", "start", "end"]
    assert [codec.decode(e[1]) for e in events if e[0] == "end"] == ["first", "second one"]


def _service(provider=None):
    prov = provider or MockProvider(scenarios={"default_response":
                                               "Sure thing. It is sunny today!"})
    agent = Agent(PromptPack.minimal("voice agent"), prov, MemoryContextStore(), None,
                  AgentConfig())
    cfg = D.DuplexConfig(D.MockSTT(RATE), D.MockTTS(RATE), sample_rate=RATE)
    return RuntimeService(agent, duplex=cfg), agent


async def _call(svc, utterances, gap_ms=0, pace=0.0):
    st = QueueStream(None)
    task = asyncio.create_task(svc.converse(st))
    await st.inbox.put(pb.ClientMessage(session_id="v1", duplex_start=pb.DuplexStart(
        codec="pcm", sample_rate=48000, channels=1)))
    pcm = b"".join(speech(u) + D.pcm16_silence(gap_ms) for u in utterances)
    fs = frames_of(pcm)
    for i, f in enumerate(fs):
        await st.inbox.put(pb.ClientMessage(audio_input=pb.AudioInputChunk(
            data=f, sequence=i, is_last=i == len(fs) - 1)))
        if pace:
            await asyncio.sleep(pace)
    out = []
    while True:
        f = await asyncio.wait_for(st.outbox.get(), 20)
        if f is None:
            break
        out.append(f)
        if task.done() and st.outbox.empty():
            break
    await asyncio.wait_for(task, 20)
    while not st.outbox.empty():
        f = st.outbox.get_nowait()
        if f is not None:
            out.append(f)
    return out


def test_runtime_duplex_turn():
    svc, agent = _service()
    assert pb.CAP_DUPLEX_AUDIO in svc.capabilities
    out = asyncio.run(_call(svc, ["what is the weather"]))
    kinds = [f.WhichOneof("message") for f in out]
    assert kinds[0] == "runtime_hello"
    hello = out[0].runtime_hello
    assert hello.media.sample_rate == RATE and pb.CAP_DUPLEX_AUDIO in hello.capabilities
    text = "".join(f.chunk.content for f in out if f.WhichOneof("message") == "chunk")
    assert text == "Sure thing. It is sunny today!"
    media = [f.media_chunk for f in out if f.WhichOneof("message") == "media_chunk"]
    assert media[-1].is_last and [m.sequence for m in media] == list(range(len(media)))
    spoken = D.FSKCodec(RATE).decode(b"".join(m.data for m in media))
    assert spoken.replace(" ", "") == "Surething.Itissunnytoday!"
    assert kinds[-1] == "done"
    hist = asyncio.run(agent.store.load("v1"))
    assert any(m["role"] == "user" and m["content"] == "what is the weather"
               for m in hist["messages"])


class SlowProvider(Provider):
    type = "slow"

    async def stream(self, messages, tools, params, session_id=None, metadata=None):
        for w in ("one. ", "two. ", "three. ", "four. ", "five. ", "six. "):
            await asyncio.sleep(0.08)
            yield ProviderEvent("text", text=w)
        yield ProviderEvent("done", usage=Usage(input_tokens=3, output_tokens=6))


def test_barge_in_interrupts_response():
    svc, _ = _service(SlowProvider())
    out = asyncio.run(_call(svc, ["hi", "stop"], pace=0.002))
    kinds = [f.WhichOneof("message") for f in out]
    assert "interruption" in kinds
    assert kinds.count("done") == 1  # the interrupted response never completes


def test_no_duplex_is_honest():
    agent = Agent(PromptPack.minimal("x"), MockProvider(), MemoryContextStore(), None,
                  AgentConfig())
    svc = RuntimeService(agent)
    assert pb.CAP_DUPLEX_AUDIO not in svc.capabilities

    async def go():
        st = QueueStream(None)
        t = asyncio.create_task(svc.converse(st))
        await st.inbox.put(pb.ClientMessage(session_id="x", duplex_start=pb.DuplexStart()))
        f = await asyncio.wait_for(st.outbox.get(), 5)
        await asyncio.wait_for(t, 5)
        return f

    assert asyncio.run(go()).error.code == "DUPLEX_UNSUPPORTED"


def test_facade_binary_audio_call():
    from aiohttp.test_utils import TestClient, TestServer

    from omnia_amd.facade import protocol as P
    from omnia_amd.facade.runtime_client import InProcessRuntimeClient
    from omnia_amd.facade.server import FacadeConfig, FacadeServer

    svc, _ = _service()

    async def run():
        srv = FacadeServer(FacadeConfig(agent="voice"), runtime_client=InProcessRuntimeClient(svc))
        c = TestClient(TestServer(srv.app))
        await c.start_server()
        try:
            ws = await c.ws_connect("/ws?binary=true")
            await ws.receive_json()  # connected
            fs = frames_of(speech("hello there"))
            for i, f in enumerate(fs):
                meta = {"codec": "pcm", "sample_rate": RATE, "channels": 1} if i == 0 else None
                await ws.send_bytes(P.encode_frame(P.TYPE_MEDIA_CHUNK, f, meta, i, b"call1",
                                                   P.FLAG_LAST if i == len(fs) - 1 else 0))
            got_cfg, audio, text, done = None, b"", "", None
            while done is None:
                m = await ws.receive(timeout=20)
                if m.type.name == "BINARY":
                    fr = P.decode_frame(m.data)
                    assert fr["type"] == P.TYPE_MEDIA_CHUNK
                    audio += fr["payload"]
                else:
                    j = m.json()
                    if j["type"] == "session_config":
                        got_cfg = j
                    elif j["type"] == "chunk":
                        text += j["content"]
                    elif j["type"] in ("done", "error"):
                        done = j
            await ws.close()
            return got_cfg, audio, text, done
        finally:
            await c.close()

    cfg, audio, text, done = asyncio.run(run())
    assert cfg["media"]["sample_rate"] == RATE
    assert done["type"] == "done" and text == "Sure thing. It is sunny today!"
    assert D.FSKCodec(RATE).decode(audio).replace(" ", "") == "Surething.Itissunnytoday!"
