"""Duplex (realtime audio) sessions (reference
``internal/runtime/duplex.go`` + ``internal/facade/audio_session.go``).

The reference hands the audio stream to a realtime vendor model through the
PromptKit SDK (``sdk.OpenDuplex``).  Here the pipeline is assembled in the
runtime around the same agent loop that serves text turns, so a local
(MI355X-engine) provider can serve voice:

    AudioInputChunk (pcm16) -> VAD (utterance segmentation, barge-in)
      -> STT provider -> agent turn (PromptPack, tools, provider stream)
      -> Chunk frames (text) + TTS provider per sentence -> MediaChunk (pcm16)

Protocol semantics kept from the reference:
* the facade's ``DuplexStart`` is a PROPOSAL; the runtime answers with a
  ``RuntimeHello`` carrying the media counter-offer (``MediaNegotiation``:
  codec / sample rate / channels it requires); ``duplex_audio`` is advertised
  only when an STT and a TTS provider are configured (capability honesty --
  the conformance suite's duplex check);
* ``AudioInputChunk.is_last`` ends the call: the pending utterance is flushed,
  the response finishes, the stream ends;
* barge-in: user speech while the agent is still speaking cancels the response
  and emits an ``Interruption`` frame (``interruption`` capability).
Audio providers: ``mock`` STT/TTS implement an FSK "voice" (text <-> tones) so
the whole path is exercised on real PCM signals in tests; ``openai``-compatible
STT (``/v1/audio/transcriptions``) and TTS (``/v1/audio/speech``) for real
speech models behind an OpenAI-style endpoint.
"""
from __future__ import annotations

import asyncio
import io
import re
import uuid
import wave

import numpy as np

from ..api.proto import runtime_v1 as pb


# ------------------------------------------------------------------ VAD
class EnergyVAD:
    """Frame-energy voice activity detector with onset/hangover hysteresis."""

    def __init__(self, sample_rate: int = 16000, frame_ms: int = 20,
                 threshold_dbfs: float = -40.0, start_frames: int = 2, end_frames: int = 15):
        self.frame_bytes = sample_rate * frame_ms // 1000 * 2
        self.threshold = threshold_dbfs
        self.start_frames, self.end_frames = start_frames, end_frames
        self.buf = b""
        self.in_speech = False
        self.voiced = 0
        self.silent = 0
        self.pre: list[bytes] = []
        self.utt: list[bytes] = []

    @staticmethod
    def dbfs(frame: bytes) -> float:
        x = np.frombuffer(frame, dtype="<i2").astype(np.float64)
        rms = np.sqrt(np.mean(x * x)) if x.size else 0.0
        return 20 * np.log10(rms / 32768.0) if rms > 0 else -120.0

    def feed(self, pcm: bytes) -> list[tuple]:
        """Returns events: ("start",) and ("end", utterance_pcm)."""
        self.buf += pcm
        ev = []
        while len(self.buf) >= self.frame_bytes:
            fr, self.buf = self.buf[:self.frame_bytes], self.buf[self.frame_bytes:]
            speech = self.dbfs(fr) > self.threshold
            if not self.in_speech:
                self.pre = (self.pre + [fr])[-self.start_frames:]
                self.voiced = self.voiced + 1 if speech else 0
                if self.voiced >= self.start_frames:
                    self.in_speech, self.silent = True, 0
                    self.utt = list(self.pre)
                    ev.append(("start",))
            else:
                self.utt.append(fr)
                self.silent = 0 if speech else self.silent + 1
                if self.silent >= self.end_frames:
                    ev.append(("end", b"".join(self.utt[:-self.silent])))
                    self.in_speech, self.voiced, self.utt, self.pre = False, 0, [], []
        return ev

    def flush(self) -> bytes | None:
        if self.in_speech and self.utt:
            out = b"".join(self.utt[:len(self.utt) - self.silent] if self.silent else self.utt)
            self.in_speech, self.utt = False, []
            return out
        return None


# ------------------------------------------------------------------ FSK "voice"
class FSKCodec:
    """Text <-> PCM16 tones: each byte is two 4-bit symbols, each symbol a
    ``sym_ms`` tone at ``base + value * step`` Hz.  Deterministic and robust
    enough to round-trip through the VAD and framing with no speech model."""

    def __init__(self, sample_rate: int = 16000, sym_ms: int = 20, base: float = 1000.0,
                 step: float = 200.0, amp: float = 0.3):
        self.rate, self.n = sample_rate, sample_rate * sym_ms // 1000
        self.base, self.step, self.amp = base, step, amp
        t = np.arange(self.n) / self.rate
        self.tones = [(amp * 32767 * np.sin(2 * np.pi * (base + v * step) * t)).astype("<i2")
                      for v in range(16)]

    def encode(self, text: str) -> bytes:
        out = []
        for b in text.encode("utf-8"):
            out.append(self.tones[b >> 4])
            out.append(self.tones[b & 15])
        return np.concatenate(out).tobytes() if out else b""

    def _symbols(self, x: np.ndarray) -> list[tuple[int, float, float]]:
        """(symbol, tone purity, window energy) per ``sym_ms`` window."""
        n = self.n
        freqs = np.fft.rfftfreq(n, 1 / self.rate)
        bins = [int(np.argmin(np.abs(freqs - (self.base + v * self.step)))) for v in range(16)]
        out = []
        for i in range(0, len(x) - n + 1, n):
            spec = np.abs(np.fft.rfft(x[i:i + n]))[bins]
            out.append((int(np.argmax(spec)), float(spec.max() / (spec.sum() + 1e-9)),
                        float(spec.max())))
        return out

    def decode(self, pcm: bytes) -> str:
        x = np.frombuffer(pcm, dtype="<i2").astype(np.float64)
        if len(x) < self.n:
            return ""
        x = np.concatenate([x, np.zeros(self.n)])  # a clipped last symbol still decodes
        # symbol alignment: pick the offset whose windows are most tone-pure
        best, best_q = 0, -1.0
        for off in range(0, self.n, max(1, self.n // 16)):
            syms = self._symbols(x[off:])
            loud = [s[1] for s in syms if s[2] > 0]
            q = float(np.mean(loud)) if loud else 0.0
            if q > best_q:
                best, best_q = off, q
        syms = self._symbols(x[best:])
        peak = max((s[2] for s in syms), default=0.0)
        vals = [s[0] for s in syms if s[2] > 0.25 * peak]  # drop silent windows
        data = bytes((vals[i] << 4) | vals[i + 1] for i in range(0, len(vals) - 1, 2))
        return data.decode("utf-8", errors="ignore")


class MockSTT:
    type = "mock"

    def __init__(self, sample_rate: int = 16000):
        self.codec = FSKCodec(sample_rate)

    async def transcribe(self, pcm: bytes, sample_rate: int) -> str:
        return self.codec.decode(pcm)


class MockTTS:
    type = "mock"

    def __init__(self, sample_rate: int = 16000):
        self.codec = FSKCodec(sample_rate)

    async def synthesize(self, text: str, sample_rate: int) -> bytes:
        return self.codec.encode(text)


def pcm_to_wav(pcm: bytes, rate: int, channels: int = 1) -> bytes:
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(pcm)
    return buf.getvalue()


class OpenAIAudio:
    """OpenAI-compatible speech endpoints (whisper-style STT, tts-style TTS)."""

    type = "openai"

    def __init__(self, base_url: str, model: str = "", api_key: str | None = None,
                 voice: str = "alloy"):
        self.base = base_url.rstrip("/")
        self.model, self.key, self.voice = model, api_key, voice

    def _h(self):
        return {"Authorization": f"Bearer {self.key}"} if self.key else {}

    async def transcribe(self, pcm: bytes, sample_rate: int) -> str:
        import aiohttp

        form = aiohttp.FormData()
        form.add_field("model", self.model or "whisper-1")
        form.add_field("file", pcm_to_wav(pcm, sample_rate), filename="audio.wav",
                       content_type="audio/wav")
        async with aiohttp.ClientSession() as s:
            async with s.post(f"{self.base}/audio/transcriptions", data=form, headers=self._h(),
                              timeout=aiohttp.ClientTimeout(total=60)) as r:
                r.raise_for_status()
                return (await r.json(content_type=None)).get("text", "")

    async def synthesize(self, text: str, sample_rate: int) -> bytes:
        import aiohttp

        body = {"model": self.model or "tts-1", "input": text, "voice": self.voice,
                "response_format": "pcm", "sample_rate": sample_rate}
        async with aiohttp.ClientSession() as s:
            async with s.post(f"{self.base}/audio/speech", json=body, headers=self._h(),
                              timeout=aiohttp.ClientTimeout(total=60)) as r:
                r.raise_for_status()
                return await r.read()


def build_audio_provider(spec: dict, role: str, sample_rate: int = 16000):
    t = (spec.get("type") or "mock").lower()
    if t == "mock":
        return MockSTT(sample_rate) if role == "stt" else MockTTS(sample_rate)
    if t in ("openai", "vllm", "local-audio"):
        return OpenAIAudio(spec.get("baseURL") or "https://api.openai.com/v1",
                           spec.get("model", ""), spec.get("apiKey"),
                           (spec.get("audio") or {}).get("voice", "alloy"))
    if role == "tts":
        from .vendors import build_tts_provider

        tts = build_tts_provider(spec, spec.get("apiKey"))
        if tts is not None:
            return tts
    raise ValueError(f"unsupported {role} provider type {t!r}")


# ------------------------------------------------------------------ session
class DuplexConfig:
    def __init__(self, stt, tts, sample_rate: int = 16000, codec: str = "pcm",
                 channels: int = 1, vad: dict | None = None, media_chunk_ms: int = 200):
        self.stt, self.tts = stt, tts
        self.sample_rate, self.codec, self.channels = sample_rate, codec, channels
        self.vad = vad or {}
        self.media_chunk_ms = media_chunk_ms

    @property
    def mime(self) -> str:
        return f"audio/pcm;rate={self.sample_rate};channels={self.channels}"


_SENTENCE = re.compile(r"(.+?[.!?\n])(\s|$)", re.S)


class _DuplexIO:
    """TurnIO for a spoken response: text chunks go out as Chunk frames and are
    cut into sentences that are synthesized and streamed as MediaChunks."""

    def __init__(self, sess: "DuplexSession"):
        self.s = sess
        self.pending = ""
        self.media_id = uuid.uuid4().hex[:12]
        self.seq = 0

    async def chunk(self, text: str) -> None:
        await self.s.send(pb.ServerMessage(chunk=pb.Chunk(content=text, role="assistant")))
        self.pending += text
        while True:
            m = _SENTENCE.match(self.pending)
            if not m:
                break
            self.pending = self.pending[m.end():]
            await self.speak(m.group(1))

    async def speak(self, text: str, last: bool = False) -> None:
        cfg = self.s.cfg
        audio = await cfg.tts.synthesize(text.strip(), cfg.sample_rate) if text.strip() else b""
        step = cfg.sample_rate * cfg.media_chunk_ms // 1000 * 2
        parts = [audio[i:i + step] for i in range(0, len(audio), step)] or ([b""] if last else [])
        for i, p in enumerate(parts):
            await self.s.send(pb.ServerMessage(media_chunk=pb.MediaChunk(
                media_id=self.media_id, sequence=self.seq, mime_type=cfg.mime, data=p,
                is_last=last and i == len(parts) - 1)))
            self.seq += 1

    async def finish(self) -> None:
        await self.speak(self.pending, last=True)
        self.pending = ""

    async def client_tool_calls(self, calls, meta):
        raise RuntimeError("client tools are not available in a voice session")


class DuplexSession:
    def __init__(self, agent, cfg: DuplexConfig, stream, session_id: str, ctx=None,
                 metadata: dict | None = None):
        self.agent, self.cfg, self.stream = agent, cfg, stream
        self.sid = session_id
        self.ctx = ctx
        self.metadata = metadata or {}
        self.vad = EnergyVAD(cfg.sample_rate, **cfg.vad)
        self.task: asyncio.Task | None = None
        self.turns = 0
        self.interruptions = 0
        self._send_lock = asyncio.Lock()

    async def send(self, msg) -> None:
        async with self._send_lock:
            await self.stream.send(msg)

    def hello(self, start) -> pb.ServerMessage:
        return pb.ServerMessage(runtime_hello=pb.RuntimeHello(
            capabilities=[pb.CAP_DUPLEX_AUDIO, pb.CAP_INTERRUPTION],
            media=pb.MediaNegotiation(codec=self.cfg.codec, sample_rate=self.cfg.sample_rate,
                                      channels=self.cfg.channels)))

    async def _respond(self, pcm: bytes) -> None:
        text = (await self.cfg.stt.transcribe(pcm, self.cfg.sample_rate)).strip()
        if not text:
            return
        io_ = _DuplexIO(self)
        res = await self.agent.run_turn(self.sid, text, io_, metadata={
            **self.metadata, "modality": "voice"}, ctx=self.ctx)
        await io_.finish()
        self.turns += 1
        await self.send(pb.ServerMessage(done=pb.Done(
            final_content=res.content, usage=pb.Usage(
                input_tokens=res.usage.input_tokens, output_tokens=res.usage.output_tokens,
                cost_usd=res.cost))))

    async def _barge_in(self) -> None:
        if self.task is not None and not self.task.done():
            self.task.cancel()
            try:
                await self.task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self.interruptions += 1
            await self.send(pb.ServerMessage(interruption=pb.Interruption()))

    async def _utterance(self, pcm: bytes) -> None:
        if self.task is not None and not self.task.done():
            await self.task  # one response at a time (in-flight cap 1)
        self.task = asyncio.get_running_loop().create_task(self._respond(pcm))

    async def run(self, start_msg) -> None:
        await self.send(self.hello(start_msg))
        while True:
            msg = await self.stream.recv()
            if msg is None:
                break
            if not msg.HasField("audio_input"):
                continue
            ai = msg.audio_input
            for ev in self.vad.feed(bytes(ai.data)):
                if ev[0] == "start":
                    await self._barge_in()
                else:
                    await self._utterance(ev[1])
            if ai.is_last:
                tail = self.vad.flush()
                if tail:
                    await self._utterance(tail)
                break
        if self.task is not None:
            try:
                await self.task
            except asyncio.CancelledError:
                pass


def pcm16_silence(ms: int, sample_rate: int = 16000) -> bytes:
    return b"\0\0" * (sample_rate * ms // 1000)
