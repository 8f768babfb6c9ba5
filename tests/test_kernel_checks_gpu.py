"""OMNIA_KERNEL_CHECKS on the GPU: a corrupt block table is refused before the
decode-attention launch (nothing reaches the device), and a whole engine run
with the checks on -- eager and graph-captured -- raises nothing and generates
the same tokens as with them off."""
import pytest
import torch

from omnia_amd import ops
from omnia_amd.ops import checks

pytestmark = pytest.mark.gpu


def test_corrupt_table_refused_before_launch(monkeypatch):
    monkeypatch.setattr(checks, "ENABLED", True)
    nb, hkv, bs = 8, 8, 32
    kc = torch.zeros(nb, hkv, bs, 128, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    bt = torch.zeros(2, 4, dtype=torch.int32, device="cuda")
    bt[1, 1] = 1 << 20  # would read far outside the cache
    sl = torch.tensor([40, 40], dtype=torch.int32, device="cuda")
    q = torch.randn(2, 32, 128, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(checks.KernelCheckError, match="row 1 page 1"):
        ops.decode_attention(q, kc, vc, bt, sl, 0.1)
    bt[1, 1] = 2
    ops.decode_attention(q, kc, vc, bt, sl, 0.1)  # fixed table: launches
    torch.cuda.synchronize()


@pytest.mark.parametrize("graphs", [False, True])
def test_engine_run_is_clean_under_checks(monkeypatch, graphs):
    from omnia_amd.engine.engine import EngineConfig, LLMEngine
    from omnia_amd.engine.sampling_params import SamplingParams

    def run(on):
        monkeypatch.setattr(checks, "ENABLED", on)
        e = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", num_blocks=128,
                                   max_batch=8, max_model_len=1024, use_graphs=graphs))
        p = SamplingParams(temperature=0, max_tokens=8, ignore_eos=True)
        return [s.output for s in e.generate([list(range(3, 90)), list(range(40, 300))], p)]

    assert run(True) == run(False)
