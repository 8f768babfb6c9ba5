"""``python -m omnia_amd.facade`` -- the facade container entrypoint.

Dials the runtime sidecar over gRPC (retrying until ready), serves WebSocket /
REST functions (+ A2A / MCP when enabled), and the management-plane twin
(18080 / 19999 / 19998) behind its mgmt-only chain when the operator allocated it and drains gracefully on SIGTERM
(in-flight turns finish, new connections refused, ``omnia_facade_draining`` = 1)."""
import asyncio
import logging
import os
import signal

from .app import build_facade, dial_runtime, start_facade, stop_facade
from ..observability.logging import configure as configure_logging


async def main():
    from ..utils.pyprof import maybe_start

    maybe_start("facade")
    configure_logging()
    env = dict(os.environ)
    client = await dial_runtime(env.get("OMNIA_RUNTIME_ADDRESS", "127.0.0.1:9000"))
    fac = build_facade(env, client)
    await start_facade(fac, env)
    from ..utils.proc_tune import tune_serving_process

    tune_serving_process()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    await stop.wait()
    await stop_facade(fac)


if __name__ == "__main__":
    asyncio.run(main())
