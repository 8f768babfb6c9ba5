"""Decode hipGraphs captured under the STRICT capture guard (verdict r5 item
5): the decode step is hand kernels and copies only -- no framework compute op
(the old where / clamp / index_select / index_copy token plumbing now lives in
the embedding and sampler kernels) and no block allocated outside the graph
pool -- and the graphs still replay to the eager result."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams


@pytest.mark.parametrize("model,batch", [("tiny-llama", 8), ("llama-3-8b", 256)])
def test_decode_graphs_pass_strict_guard(monkeypatch, model, batch):
    """tiny-llama: every bucket; Llama-3-8B at the serving bucket (256 rows, the
    bench's decode shape), where every projection is on a hand kernel."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OMNIA_CAPTURE_GUARD", "strict")
    monkeypatch.setenv("OMNIA_CAPTURE_GUARD_TRACE", "1")
    big = model == "llama-3-8b"

    def run(graphs):
        e = LLMEngine(EngineConfig(model=model, device="cuda", num_blocks=2048 if big else 512,
                                   block_size=32, max_batch=batch, max_model_len=2048,
                                   use_graphs=graphs, mixed_budget=0))
        p = SamplingParams(temperature=0, max_tokens=6 if big else 12, ignore_eos=True)
        prompts = [list(range(100 + i, 140 + i)) for i in range(batch)]
        out = [s.output for s in e.generate(prompts, p)]
        st = dict(e.runner.stats)
        del e
        torch.cuda.empty_cache()
        return out, st

    g, st = run(True)
    assert st["captures"] > 0 and st["graph_replays"] > 0
    assert st.get("capture_guard_violations", 0) == 0
    if big:  # the serving decode step: hand kernels and copies only, no library GEMM
        assert st.get("capture_library_gemms", 0) == 0
    if not big:
        assert g == run(False)[0]


def test_strict_guard_after_an_earlier_engine_is_collected(monkeypatch):
    """PyTorch's CUDA generator allocates its graph seed / offset tensors when
    the first live graph registers and frees them with the last one: once an
    earlier engine's graphs are collected, the next engine's first capture would
    allocate them (2 x 512 B outside the graph pool) -- unless the runner keeps
    its warm-up registration graph alive (model_runner._capture)."""
    import gc

    monkeypatch.setenv("OMNIA_CAPTURE_GUARD", "strict")

    def engine():
        return LLMEngine(EngineConfig(model="tiny-llama", device="cuda", num_blocks=256,
                                      block_size=32, max_batch=4, max_model_len=512,
                                      use_graphs=True, mixed_budget=0))

    p = SamplingParams(temperature=0, max_tokens=4, ignore_eos=True)
    e = engine()
    e.generate([list(range(5, 40))], p)
    del e
    gc.collect()  # every graph of the first engine is gone
    torch.cuda.empty_cache()
    e2 = engine()
    e2.generate([list(range(5, 40)), list(range(9, 30))], p)
    assert e2.runner.stats.get("capture_guard_violations", 0) == 0
    assert e2.runner.stats["captures"] > 0
