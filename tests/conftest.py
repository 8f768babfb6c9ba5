import os
import sys

# Under pytest-xdist every worker (and every engine / pod process its tests
# start) would otherwise run torch's CPU ops on as many OpenMP threads as the
# machine has cores: with 4 workers on 8 cores the spinning thread pools
# oversubscribe the CPUs and tiny-model tests slow down 20-100x (a 6 s property
# test past a 600 s timeout).  Give each worker its share; children inherit it.
_workers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "0") or 0)
if _workers > 1 and "OMP_NUM_THREADS" not in os.environ:
    os.environ["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // _workers))

# concurrent multi-rank bench jobs on different workers get disjoint pod port
# windows (bench.py: OMNIA_BENCH_PORT_BASE + 200 * local rank)
_wid = os.environ.get("PYTEST_XDIST_WORKER", "gw0")[2:]
if _wid.isdigit():
    os.environ.setdefault("OMNIA_BENCH_PORT_BASE", str(21000 + 1800 * int(_wid)))

import pytest  # noqa: E402

try:  # property tests draw fresh examples every run: no on-disk example database,
    # and hypothesis's own caches go to a temp dir, not the repository
    import tempfile

    os.environ.setdefault("HYPOTHESIS_STORAGE_DIRECTORY",
                          os.path.join(tempfile.gettempdir(), "omnia-hypothesis"))
    from hypothesis import settings as _hyp_settings

    _hyp_settings.register_profile("omnia", database=None)
    _hyp_settings.load_profile("omnia")
except ImportError:  # pragma: no cover
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def release_gpu_memory():
    """Free what earlier GPU tests left in this pytest process: the runtime's
    process-wide cached engines (each holds a KV pool sized from free HBM) and
    the caching allocator's blocks -- before a test that shares the card with
    child processes."""
    import gc

    try:
        import torch
    except Exception:  # pragma: no cover
        return
    try:
        from omnia_amd.runtime import app

        for eng in list(app._ENGINES.values()):
            try:
                eng.shutdown()
            except Exception:  # noqa: BLE001
                pass
        app._ENGINES.clear()
    except Exception:  # noqa: BLE001
        pass
    gc.collect()
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """GPU tests that legitimately run quiet for minutes (pod cold starts, TP
    groups) print a heartbeat to the real stderr every 30 s, past pytest's
    capture, so a remote runner does not take them for hung."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import threading
    import time

    stop = threading.Event()
    t0 = time.monotonic()

    def beat():
        while not stop.wait(30):
            sys.__stderr__.write(f"[heartbeat] {request.node.name} "
                                 f"{time.monotonic() - t0:.0f}s\n")
            sys.__stderr__.flush()

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
