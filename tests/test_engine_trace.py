"""Engine-step observability (SURVEY §5.1 [design]): OTel engine spans with
step attributes, the roctx marker hooks and the torch.profiler window -- on the
CPU engine (roctx is exercised through a stub: the CPU engine never emits it)."""
import json

import pytest

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.observability import engine_trace, tracing


def _engine():
    return LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_blocks=64,
                                  max_batch=4, max_model_len=256, use_graphs=False))


def test_engine_steps_export_spans_with_step_attributes():
    mem = tracing.MemoryExporter()
    tracing.configure(exporter=mem, ratio=1.0)
    try:
        eng = _engine()
        eng.generate([list(range(3, 40)), list(range(5, 20))],
                     SamplingParams(temperature=0, max_tokens=4, ignore_eos=True))
    finally:
        tracing.configure(exporter=None, endpoint="")
    names = [s.name for s in mem.spans]
    assert "omnia.engine.prefill" in names and "omnia.engine.decode_step" in names
    for sp in mem.spans:
        a = sp.attributes
        assert {"omnia.engine.batch_size", "omnia.engine.tokens", "omnia.engine.kv_pages_used",
                "omnia.engine.step"} <= set(a)
        assert sp.end_ns >= sp.start_ns and sp.parent_id is None and sp.status == "OK"
    pre = [s for s in mem.spans if s.name == "omnia.engine.prefill"]
    assert sum(s.attributes["omnia.engine.tokens"] for s in pre) == 37 + 15
    dec = [s for s in mem.spans if s.name == "omnia.engine.decode_step"]
    assert all(s.attributes["omnia.engine.batch_size"] in (1, 2) for s in dec)
    assert all(s.attributes["omnia.engine.kv_pages_used"] > 0 for s in dec)


def test_tracing_off_costs_nothing():
    tracing.configure(exporter=None, endpoint="")
    eng = _engine()
    assert not eng.trace.active
    eng.generate([list(range(3, 20))], SamplingParams(temperature=0, max_tokens=3,
                                                      ignore_eos=True))
    assert eng.trace.spans == 0


def test_roctx_ranges_bracket_every_step(monkeypatch):
    calls = []

    class Nvtx:
        def range_push(self, m):
            calls.append(("push", m))

        def range_pop(self):
            calls.append(("pop",))

        def mark(self, m):
            calls.append(("mark", m))

    monkeypatch.setattr(engine_trace, "_nvtx", lambda: Nvtx())
    tr = engine_trace.EngineTrace("cuda", env={"OMNIA_ROCTX": "1"})
    assert tr.active
    for step in range(3):
        tr.begin(step)
        tr.on_step("decode", 0.0, 8, 0, 10, step)
        tr.end()
    assert [c[0] for c in calls] == ["push", "mark", "pop"] * 3
    assert calls[1][1].startswith("omnia.engine.decode_step rows=8")
    # no roctx on a CPU engine
    assert not engine_trace.EngineTrace("cpu", env={"OMNIA_ROCTX": "1"}).roctx


def test_torch_profiler_window_writes_a_chrome_trace(tmp_path):
    tr = engine_trace.EngineTrace("cpu", env={"OMNIA_TORCH_PROFILE_DIR": str(tmp_path),
                                              "OMNIA_TORCH_PROFILE_STEPS": "2:4"})
    import torch

    for step in range(6):
        tr.begin(step)
        torch.ones(8).sum()
        tr.end()
    files = list(tmp_path.glob("engine_steps_*.json"))
    assert len(files) == 1
    assert "traceEvents" in json.loads(files[0].read_text())
    assert tr.prof_window is None  # one window per process


@pytest.mark.parametrize("spec,window", [("5:9", (5, 9)), ("7", (7, 17))])
def test_profile_window_parsing(spec, window):
    tr = engine_trace.EngineTrace("cpu", env={"OMNIA_TORCH_PROFILE_DIR": "/nonexistent",
                                              "OMNIA_TORCH_PROFILE_STEPS": spec})
    assert tr.prof_window == window
