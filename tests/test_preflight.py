"""Multi-GPU first-contact preflight plumbing (verdict r5 item 4), on CPU over
gloo: fresh child per rank, rendezvous, all-reduce check, per-rank failure
report, job summary, and the bench integration at N = 1.  The device steps
(peer-access matrix, RCCL, IPC vs RCCL) run only on the GPU box
(``tests/test_preflight_gpu.py``)."""
import concurrent.futures as cf
import os
import socket
import sys

import pytest

from omnia_amd.parallel import preflight as pf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(n, env=None, timeout=60.0):
    port = _port()
    with cf.ThreadPoolExecutor(n) as ex:
        return list(ex.map(lambda r: pf.spawn(r, n, r, port, "gloo", timeout, env), range(n)))


@pytest.mark.parametrize("n", [2, 4])
def test_gloo_job_reports_world_and_checks(n):
    reps = _job(n)
    s = pf.summarize(reps)
    assert s["ranks"] == n and s["rccl_world"] == n
    assert s["rccl_ok"] is True and s["failures"] == []
    assert s["ipc_ok"] is None and s["p2p_ok"] is None  # device steps: GPU only
    assert set(s["rccl_allreduce_us_max"]) == {"16KiB", "32MiB"}


def test_a_bad_rank_is_named_not_hung():
    env = dict(os.environ, OMNIA_PREFLIGHT_INJECT="1:rccl")
    s = pf.summarize(_job(3, env))
    assert s["rccl_ok"] is False
    assert [f["rank"] for f in s["failures"]] == [1]
    assert "mismatch" in s["failures"][0]["errors"][0]


def test_rank_that_never_joins_times_out_with_errors_everywhere():
    env = dict(os.environ, OMNIA_PREFLIGHT_INJECT="1:init")
    reps = _job(2, env, timeout=8.0)
    s = pf.summarize(reps)
    assert {f["rank"] for f in s["failures"]} == {0, 1}
    assert any("injected init failure" in e for e in reps[1]["errors"])


def test_dead_child_is_reported(tmp_path):
    orig = sys.executable
    try:
        sys.executable = str(tmp_path / "no-python")  # the child cannot start
        rep = pf.spawn(0, 1, 0, _port(), "gloo", 5.0)
    finally:
        sys.executable = orig
    assert rep["rccl_world"] is None
    assert "preflight child exited" in rep["errors"][0] and "spawn failed" in rep["errors"][0]


def test_bench_job_preflight_single_rank():
    sys.path.insert(0, ROOT)
    import bench

    a = bench.parse(["--device", "cpu"])
    s = bench.job_preflight(a, 1, 0, 0, "gloo")
    assert s["rccl_world"] == 1 and s["rccl_ok"] and s["failures"] == []
