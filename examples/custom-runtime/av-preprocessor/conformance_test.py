"""The example runtime must pass the omnia.runtime.v1 conformance suite (as the
reference's ``conformance_test.go``), and its log-mel stage must match a plain
fp32 reference.  Collected by the repo test suite (tests/test_custom_runtime.py)."""
import asyncio
import base64
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import runtime as avp  # noqa: E402

from omnia_amd.api.proto import runtime_v1 as pb  # noqa: E402
from omnia_amd.runtime import conformance  # noqa: E402


def test_example_runtime_is_conformant():
    async def go():
        server, port = await avp.serve(0, "127.0.0.1")
        try:
            return await conformance.run(f"127.0.0.1:{port}", timeout=20)
        finally:
            await server.stop(0)

    res = asyncio.run(go())
    for r in res:
        print(f"{r.name:26s} {'PASS' if r.passed else 'FAIL'} {r.detail}")
    assert res and all(r.passed for r in res), res


def test_log_mel_stage_against_numpy_reference():
    sr = 16000
    t = np.arange(sr // 2) / sr
    pcm = (0.4 * np.sin(2 * np.pi * 440 * t) * 32767).astype(np.int16)
    st = avp.LogMelStage(sr)
    got = st(pcm.tobytes()).numpy()
    x = pcm.astype(np.float64) / 32768.0
    n_fft, hop = st.n_fft, st.hop
    win = np.hanning(n_fft + 1)[:-1]  # periodic Hann, as torch.hann_window
    frames = 1 + (len(x) - n_fft) // hop
    spec = np.stack([np.abs(np.fft.rfft(x[i * hop:i * hop + n_fft] * win)) ** 2
                     for i in range(frames)], 1)
    want = np.log(st.fbank.cpu().double().numpy() @ spec + 1e-6).T
    assert got.shape == want.shape == (frames, 80)
    assert np.abs(got - want).max() < 1e-3 * max(1.0, np.abs(want).max())
    # the 440 Hz tone lands in one mel band
    band = int(np.argmax(want.mean(0)))
    centers = st.fbank.argmax(1).cpu().numpy() * (sr / 2) / (n_fft // 2)
    assert abs(centers[band] - 440) < 120


def test_converse_reports_frames_for_audio_parts():
    async def go():
        server, port = await avp.serve(0, "127.0.0.1")
        try:
            c = conformance.Client(f"127.0.0.1:{port}", 20)
            pcm = (np.random.default_rng(0).standard_normal(16000) * 3000).astype(np.int16)
            part = pb.ContentPart(type="audio", media=pb.MediaContent(
                mime_type="audio/pcm", data=base64.b64encode(pcm.tobytes()).decode()))
            frames = await c.turn([pb.ClientMessage(session_id="s", content="hi", parts=[part])])
            await c.close()
            return frames
        finally:
            await server.stop(0)

    frames = asyncio.run(go())
    done = [f for f in frames if f.WhichOneof("message") == "done"][0]
    assert done.done.final_content == "hello from av-preprocessor (98 log-mel frames)"
