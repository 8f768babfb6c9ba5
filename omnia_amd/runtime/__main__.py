"""``python -m omnia_amd.runtime`` -- the runtime container entrypoint (cmd/runtime/main.go).

Under tensor parallelism the runtime is launched one process per GPU
(``torchrun --nproc-per-node N -m omnia_amd.runtime`` with ``OMNIA_ENGINE_TP=N``):
TP-rank 0 serves gRPC and drives the engine, the other ranks run the engine's
TP worker loop until rank 0 shuts down.

Expert parallelism with DP attention (``OMNIA_ENGINE_EP_MODE=a2a``, world =
``OMNIA_ENGINE_EP`` ranks, BASELINE config 5): rank 0 serves gRPC; every other
rank is an attention replica with its own (here: empty) queue that steps in
lockstep with rank 0 and serves its experts to the group's all-to-alls.
"""
import asyncio
import os


def _ep_member():
    """A non-serving rank of an EP (a2a) group: run the lockstep engine loop."""
    import threading

    from .app import shared_engine
    from .config import RuntimeConfig

    shared_engine(RuntimeConfig.from_env().engine)  # same engine config as rank 0
    threading.Event().wait()  # the pod's process group is stopped as a whole


def main():
    tp = int(os.environ.get("OMNIA_ENGINE_TP", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("OMNIA_ENGINE_EP_MODE", "tp") == "a2a" and \
            int(os.environ.get("WORLD_SIZE", "1")) > 1 and rank != 0:
        _ep_member()
        return
    if tp > 1 and rank % tp != 0:
        from ..engine import tp as tpmod
        from ..engine.engine import EngineConfig

        tpmod.start(EngineConfig.from_env())
        return
    from .app import run
    from ..utils.pyprof import maybe_start

    maybe_start("runtime")
    asyncio.run(run())


if __name__ == "__main__":
    main()
