"""Capture guard (engine/capture_guard.py): framework compute ops and blocks
allocated outside the graph pool during a hipGraph capture are violations
(verdict r5 item 5).  The op recorder runs on CPU here; the GPU test captures
real decode graphs under the strict guard (tests/test_capture_guard_gpu.py)."""
import pytest
import torch

from omnia_amd.engine.capture_guard import ALLOWED, CaptureGuard, CaptureGuardError


def test_views_allocation_and_copies_are_allowed():
    x = torch.arange(12.0)
    with CaptureGuard("cpu", "t", mode="strict") as g:
        y = x.view(3, 4)[1:, :2].t()
        z = torch.empty(4)
        z.copy_(x[:4])
        _ = y.unsqueeze(0).expand(2, -1, -1)
    assert g.violations() == []


def test_framework_compute_ops_fail_strict():
    src = torch.tensor([1, -1, 0])
    slots = torch.tensor([7, 8, 9])
    ids = torch.tensor([3, 4, 5])
    with pytest.raises(CaptureGuardError, match="aten::where|aten::clamp|aten::index_select"):
        with CaptureGuard("cpu", "decode", mode="strict"):
            torch.where(src >= 0, slots.index_select(0, src.clamp(min=0)), ids)


def test_warn_mode_records_without_raising(caplog):
    with CaptureGuard("cpu", "decode", mode="warn") as g:
        torch.zeros(3).index_copy_(0, torch.tensor([0]), torch.ones(1))
    assert any("index_copy" in v for v in g.violations())
    assert "capture-guard violation" in caplog.text


def test_off_mode_checks_nothing():
    with CaptureGuard("cpu", "decode", mode="off") as g:
        torch.ones(2) + 1
    assert g.violations() == []


def test_allowed_set_has_no_compute_ops():
    for bad in ("aten::where", "aten::index_copy_", "aten::clamp", "aten::eq", "aten::add"):
        assert bad not in ALLOWED


def test_split_scopes_like_the_model_runner():
    """The runner records ops INSIDE the capture and memory OUTSIDE it, then
    calls check() -- the same protocol on CPU."""
    g = CaptureGuard("cpu", "split", mode="strict")
    with g.memory_scope():
        torch.ones(2).fill_(3.0)  # outside the op scope: not counted (capture_begin's work)
        with g.ops_scope():
            torch.empty(4).view(2, 2)
    g.check()
    assert g.violations() == []
    g2 = CaptureGuard("cpu", "split", mode="strict")
    with g2.memory_scope():
        with g2.ops_scope():
            torch.zeros(3).add_(1)
    with pytest.raises(CaptureGuardError, match="aten::add"):
        g2.check()
