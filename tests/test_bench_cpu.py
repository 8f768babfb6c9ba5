"""bench.py contract on CPU: the WebSocket pod path (facade + runtime processes),
``--gpus N`` spawning N rank processes itself, and the aggregated JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--model", "tiny-llama", "--prompt-len", "96", "--gen-len", "6",
                        "--warmup", "1", *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_ws_path_two_ranks_spawned_by_bench():
    rec = _bench("--gpus", "2", "--concurrency", "3", "--steps", "2")
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2
    assert len(rec["per_rank_tokens_per_s"]) == 2 and all(v > 0 for v in
                                                          rec["per_rank_tokens_per_s"])
    assert rec["config"]["path"] == "ws" and rec["config"]["parallelism"] == "dp2"
    assert rec["turns"] == 2 * 2 * 3
    # every turn streamed gen_len tokens: value = tokens / elapsed of the slowest rank
    tokens = 2 * 2 * 3 * 6
    assert abs(rec["value"] - tokens / (rec["ms_per_step"] * rec["steps"] / 1000)) < 1.0


def test_open_loop_poisson_reports_latency_percentiles():
    rec = _bench("--concurrency", "4", "--steps", "1", "--arrival", "poisson", "--rate", "40",
                 "--stream-interval-ms", "0")
    assert rec["config"]["arrival"].startswith("poisson")
    assert rec["turns"] == 4 and rec["p95_tpot_ms"] is not None and rec["p95_ttft_ms"]


def test_tp2_pod_serves_over_ws():
    """--tp K: one TP pod per K ranks (torchrun'd runtime ranks, TP-rank 0 serves
    gRPC), the other bench ranks only join the aggregation (CPU, gloo)."""
    rec = _bench("--gpus", "2", "--tp", "2", "--concurrency", "2", "--steps", "1")
    assert rec["config"]["parallelism"] == "dp1-tp2" and rec["n_gpus"] == 2
    assert rec["turns"] == 2 and rec["per_rank_tokens_per_s"][1] == 0.0
    assert rec["value"] > 0


def test_driver_torchrun_invocation_two_ranks():
    """The driver's exact N>1 launch: torch.distributed.run starts one rank per
    GPU with RANK/WORLD_SIZE set; bench.py must not spawn ranks again, and rank 0
    prints one aggregated line."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu",
                        "--model", "tiny-llama", "--prompt-len", "96", "--gen-len", "6",
                        "--concurrency", "3"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["steps"] == 2
    assert len(rec["per_rank_tokens_per_s"]) == 2 and rec["config"]["parallelism"] == "dp2"


def test_streamed_frames_cross_check_usage():
    """The headline's token count (done.usage.output_tokens) must agree with the
    frames the client timed; a drifting server count aborts the bench."""
    sys.path.insert(0, ROOT)
    import pytest

    from bench import check_streamed

    ok = [(0.1, 1.0, 8, 96, [0.1 * i for i in range(8)])]
    assert check_streamed(ok, 8, True) == 8
    merged = [(0.1, 1.0, 128, 96, [0.0] * 126)]  # two tokens held back into neighbours
    assert check_streamed(merged, 128, True) == 126
    with pytest.raises(SystemExit, match="output tokens"):
        check_streamed([(0.1, 1.0, 7, 96, [0.0] * 7)], 8, True)  # short turn
    with pytest.raises(SystemExit, match="frames"):
        check_streamed([(0.1, 1.0, 128, 96, [0.0] * 60)], 128, True)  # inflated usage
    with pytest.raises(SystemExit, match="frames"):
        check_streamed([(0.1, 1.0, 8, 96, [0.0] * 12)], 8, True)
    assert check_streamed([(0.1, 1.0, 8, 96, [])], 8, False) == 0
    assert check_streamed([(0.1, 1.0, 8, 96, [0.0])], 8, True, strict=False) == 1


def test_ws_path_reports_streamed_frames():
    rec = _bench("--concurrency", "2", "--steps", "1", "--stream-interval-ms", "0")
    # tiny-llama's vocab is mostly raw bytes: frames are counted, not matched
    assert 1 <= rec["streamed_frames_rank0"] <= rec["turns"] * 7
