"""Decode-step staging upload kernel (ops/csrc/staging.hip) vs a host slice copy:
the scalar head and the [rows x row_bytes] block-table window land byte-exact in
the device twin; everything outside the window is left untouched."""
import pytest
import torch

from omnia_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(1, 64), (77, 128), (256, 512)])
def test_stage_copy_window(rows, cols):
    k = ops.kernels()
    MB, B = 512, 256
    head = 14 * 1024
    nbytes = head + B * MB * 4
    g = torch.Generator().manual_seed(rows)
    host = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, generator=g).pin_memory()
    dev = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    src = k.host_device_ptr(host)
    assert src != 0, "pinned buffer is not device-mapped"
    k.stage_copy(dev.data_ptr(), src, head, head, 4 * MB, rows, 4 * cols)
    torch.cuda.synchronize()
    got = dev.cpu()
    want = torch.zeros_like(host)
    want[:head] = host[:head]
    bt_h = host[head:].view(B, MB * 4)
    bt_w = want[head:].view(B, MB * 4)
    bt_w[:rows, :4 * cols] = bt_h[:rows, :4 * cols]
    assert torch.equal(got, want)


def test_stage_copy_rejects_misaligned():
    k = ops.kernels()
    host = torch.zeros(4096, dtype=torch.uint8).pin_memory()
    dev = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError, match="stage_copy"):
        k.stage_copy(dev.data_ptr(), k.host_device_ptr(host), 100, 128, 64, 2, 64)
    with pytest.raises(RuntimeError, match="stage_copy"):
        k.stage_copy(dev.data_ptr(), k.host_device_ptr(host), 128, 128, 64, 2, 128)
