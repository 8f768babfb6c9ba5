"""The multi-GPU preflight's device steps on the one-GPU box (verdict r5 item
4: "on the one-GPU box it reports rccl_world: 1 correctly"): a fresh child
initialises RCCL, all-reduces, runs the IPC one-shot / two-shot kernels
(comm.hip) and checks them bit-for-bit against RCCL, and reads the
peer-access matrix."""
import socket

import pytest
import torch

from omnia_amd.parallel import preflight as pf

pytestmark = pytest.mark.gpu


def test_single_gpu_preflight_reports_world_one():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rep = pf.spawn(0, 1, 0, port, "nccl", timeout_s=90.0)
    assert rep["errors"] == [], rep
    assert rep["rccl_world"] == 1 and rep["rccl_ok"] and rep["ipc_ok"]
    n = rep["device_count"]
    assert len(rep["p2p"]) == n and all(rep["p2p"][i][i] for i in range(n))
    summ = pf.summarize([rep])
    assert summ["rccl_world"] == 1 and summ["p2p_ok"] and summ["failures"] == []
    assert set(summ["ipc_allreduce_us_max"]) == {"16KiB", "32MiB"}
