"""``python -m omnia_amd.runtime`` -- the runtime container entrypoint (cmd/runtime/main.go).

Under tensor parallelism the runtime is launched one process per GPU
(``torchrun --nproc-per-node N -m omnia_amd.runtime`` with ``OMNIA_ENGINE_TP=N``):
TP-rank 0 serves gRPC and drives the engine, the other ranks run the engine's
TP worker loop until rank 0 shuts down.
"""
import asyncio
import os


def main():
    tp = int(os.environ.get("OMNIA_ENGINE_TP", "1"))
    if tp > 1 and int(os.environ.get("RANK", "0")) % tp != 0:
        from ..engine import tp as tpmod
        from ..engine.engine import EngineConfig

        tpmod.start(EngineConfig.from_env())
        return
    from .app import run

    asyncio.run(run())


if __name__ == "__main__":
    main()
