"""``python -m omnia_amd.runtime`` -- the runtime container entrypoint (cmd/runtime/main.go)."""
import asyncio

from .app import run

if __name__ == "__main__":
    asyncio.run(run())
