"""OMNIA_KERNEL_CHECKS bounds checks (SURVEY §5.2 [design]): a corrupt block
table, an over-long sequence or an out-of-cache KV slot is refused before the
launch with the op and row named; valid inputs (incl. padded -1 slots and
unused table tails full of garbage) pass.  The checks are plain torch ops, so
they run here on CPU tensors; the GPU test drives them through the ops."""
import pytest
import torch

from omnia_amd.ops import checks

NB, HKV, BS, D = 16, 2, 32, 128


def _cache():
    return torch.zeros(NB, HKV, BS, D, dtype=torch.bfloat16)


def test_valid_tables_and_slots_pass():
    bt = torch.full((3, 4), 999, dtype=torch.int32)  # unused tail: garbage is fine
    bt[0, :1] = torch.tensor([3])
    bt[1, :3] = torch.tensor([0, 5, 15])
    sl = torch.tensor([17, 65, 0], dtype=torch.int32)
    checks.paged("decode_attention", bt, sl, _cache())
    checks.slots("rope_kv", torch.tensor([-1, 0, NB * BS - 1]), _cache())


@pytest.mark.parametrize("row,page,val", [(1, 2, NB), (0, 0, -3)])
def test_page_outside_the_cache_is_named(row, page, val):
    bt = torch.zeros(2, 4, dtype=torch.int32)
    bt[row, page] = val
    sl = torch.tensor([BS * 4, BS * 4], dtype=torch.int32)
    with pytest.raises(checks.KernelCheckError, match=f"row {row} page {page}"):
        checks.paged("decode_attention", bt, sl, _cache())


def test_sequence_longer_than_its_table_row():
    bt = torch.zeros(2, 2, dtype=torch.int32)
    with pytest.raises(checks.KernelCheckError, match="seq_len 65 of row 1"):
        checks.paged("prefill_attention", bt, torch.tensor([3, 65], dtype=torch.int32),
                     _cache())


def test_rows_limit_ignores_trailing_rows():
    bt = torch.zeros(2, 2, dtype=torch.int32)
    bt[1, 0] = 10 ** 6
    checks.paged("decode_attention", bt, torch.tensor([5, 5], dtype=torch.int32), _cache(),
                 rows=1)


@pytest.mark.parametrize("bad", [-2, NB * BS])
def test_slot_outside_the_cache(bad):
    with pytest.raises(checks.KernelCheckError, match=f"KV slot {bad} of row 1"):
        checks.slots("splitk_rope_kv", torch.tensor([0, bad]), _cache())


def test_off_by_default_and_inactive_when_disabled(monkeypatch):
    monkeypatch.setattr(checks, "ENABLED", False)
    assert not checks.active(torch.zeros(1))
    monkeypatch.setattr(checks, "ENABLED", True)
    assert checks.active(torch.zeros(1))
