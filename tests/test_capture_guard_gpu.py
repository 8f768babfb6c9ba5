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
