"""Mid-size step dispatch (ops.midm_config, ops/tuned/midm_mi355x.json): bucket
mapping, the decode / prefill-tile boundaries, mode-1 (gate_up) unsplit
entries, and the OMNIA_MIDM kill switch -- pure table logic, CPU."""
import json
import os

from omnia_amd import ops


def test_table_file_is_well_formed():
    p = os.path.join(os.path.dirname(ops.__file__), "tuned", "midm_mi355x.json")
    t = json.load(open(p))
    for k, S in t.items():
        mode, b, N, K = (int(x) for x in k.split(":"))
        assert mode in (0, 1) and b in ops.MIDM_BUCKETS
        assert S >= 1 and K % S == 0 and (K // S) % 128 == 0  # pgemm split-K constraints
        assert mode == 1 or N % 256 == 0


def test_bucket_mapping_and_boundaries():
    cfg = ops.midm_config(600, 4096, 14336, 0)  # down at 600 rows -> the 768 bucket
    assert cfg == (256, ops.PGEMM_SPLIT, 4)
    assert ops.midm_config(512, 4096, 14336, 0)[2] == 8
    assert ops.midm_config(256, 4096, 14336, 0) is None  # decode sizes: the tile table
    assert ops.midm_config(5000, 4096, 14336, 0) is None  # past the last bucket
    assert ops.midm_config(1500, 6144, 4096, 0) is None  # qkv: the library wins there
    assert ops.midm_config(1024, 14336, 4096, 1)[2] == 1  # gate_up: unsplit fused tile
    assert ops.midm_config(700, 1234, 4096, 0) is None  # unknown shape


def test_kill_switch(monkeypatch):
    monkeypatch.setattr(ops, "_midm_on", False)
    assert ops.midm_config(600, 4096, 14336, 0) is None
