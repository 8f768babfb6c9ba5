"""Pod listen ports (operator/pods.py ``free_port``): with ``OMNIA_PORT_BASE``
(bench.py sets one window per local rank) ports come sequentially from the
rank's own window, skipping taken ones -- replicas starting together cannot
draw the same port the way concurrent bind(0) calls can."""
import socket

from omnia_amd.operator import pods


def test_port_window_is_sequential_and_skips_taken(monkeypatch):
    monkeypatch.setenv("OMNIA_PORT_BASE", "23100")
    monkeypatch.setenv("OMNIA_PORT_SPAN", "6")
    monkeypatch.setattr(pods, "_next_port", {})
    hold = socket.socket()
    hold.bind(("127.0.0.1", 23101))
    hold.listen()
    try:
        got = [pods.free_port() for _ in range(5)]
    finally:
        hold.close()
    assert got == [23100, 23102, 23103, 23104, 23105]


def test_rank_windows_are_disjoint(monkeypatch):
    seen = {}
    for rank in range(8):
        monkeypatch.setenv("OMNIA_PORT_BASE", str(21000 + 200 * rank))
        monkeypatch.setattr(pods, "_next_port", {})
        seen[rank] = {pods.free_port() for _ in range(12)}
        assert all(21000 + 200 * rank <= p < 21200 + 200 * rank for p in seen[rank])
    allp = [p for s in seen.values() for p in s]
    assert len(allp) == len(set(allp))


def test_without_a_window_falls_back_to_the_kernel(monkeypatch):
    monkeypatch.delenv("OMNIA_PORT_BASE", raising=False)
    p = pods.free_port()
    assert 1024 < p < 65536
