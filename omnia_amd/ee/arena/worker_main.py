"""Arena worker pod entry point (``ee/cmd/arena-worker/main.go``).

``python -m omnia_amd.ee.arena.worker_main`` is what the ArenaJob controller's
worker Job runs (``ArenaJobController(worker_mode="pods")``).  Everything comes
from the environment the controller sets on the pod:

* ``ARENA_JOB_NAME`` / ``ARENA_JOB_NAMESPACE`` / ``ARENA_JOB_TYPE``;
* ``REDIS_URL`` -- the Redis-Streams work queue shared with the controller
  (``omnia:arena:queue:<job>``, consumer group, reclaim of stale claims);
* ``ARENA_CONFIG_FILE`` -- the resolved job config (scenarios, providers; direct
  providers carry their Provider ``spec``), mounted from the job's ConfigMap;
* ``ARENA_VUS_PER_WORKER``, ``ARENA_RAMP_UP`` / ``ARENA_RAMP_DOWN`` (seconds),
  ``ARENA_BUDGET`` (this worker's share of ``budgetLimit``);
* ``ARENA_PROVIDER_SECRET_<ID>`` -- a direct provider's API key (from its
  Secret via ``secretKeyRef``; never written into the ConfigMap).

The worker drains the queue with its virtual-user pool and exits 0 when the
queue is empty (non-zero on a configuration error), so the Job's completions
count finished workers.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import re
import sys

from .profile import LoadProfile
from .queue import StreamQueue
from .worker import ArenaWorker

log = logging.getLogger("omnia.arena.worker_main")


def secret_env_name(provider_id: str) -> str:
    return "ARENA_PROVIDER_SECRET_" + re.sub(r"[^A-Za-z0-9]", "_", provider_id).upper()


def build_providers(cfg_providers: list[dict], env=os.environ) -> dict:
    from ...runtime.providers import build_provider

    out = {}
    for p in cfg_providers:
        p = dict(p)
        if p.get("mode") == "direct":
            key = env.get(secret_env_name(p["id"]))
            spec = dict(p.get("spec") or {"type": "mock"})
            secrets = {(spec.get("credential") or {}).get("secretRef", {}).get(
                "key", "api-key"): key} if key else None
            p["object"] = build_provider(spec, secrets=secrets)
        out[p["id"]] = p
    for p in out.values():
        if p.get("persona"):
            p["persona_object"] = out[p["persona"]]["object"]
    return out


async def amain(env=os.environ) -> int:
    from ...utils.resp import RedisClient

    job = env["ARENA_JOB_NAME"]
    with open(env["ARENA_CONFIG_FILE"]) as f:
        cfg = json.load(f)
    scenarios = {s["id"]: s for s in cfg.get("scenarios", [])}
    providers = build_providers(cfg.get("providers", []), env)
    q = StreamQueue(RedisClient(env["REDIS_URL"]))
    budget = float(env["ARENA_BUDGET"]) if env.get("ARENA_BUDGET") else None
    recorder = sess = None
    if env.get("SESSION_API_URL"):  # played runs recorded as sessions (source:arena)
        from ...session.httpclient import SessionHTTPClient
        from .recording import ArenaSessionRecorder

        sess = SessionHTTPClient(env["SESSION_API_URL"])
        recorder = ArenaSessionRecorder(sess, job, env.get("ARENA_JOB_NAMESPACE", "default"),
                                        env.get("OMNIA_WORKSPACE_NAME", ""),
                                        env.get("ARENA_JOB_TYPE") or "evaluation")
    w = ArenaWorker(q, job, scenarios, providers,
                    LoadProfile(max(1, int(env.get("ARENA_VUS_PER_WORKER") or 1)),
                                float(env.get("ARENA_RAMP_UP") or 0),
                                float(env.get("ARENA_RAMP_DOWN") or 0)),
                    budget=budget, job_type=env.get("ARENA_JOB_TYPE") or "evaluation",
                    consumer=env.get("HOSTNAME") or None, recorder=recorder)
    try:
        await w.run()
    finally:
        if sess is not None:
            await sess.close()
    log.info("worker for %s done: %d item(s)", job, w.done)
    return 0


def main() -> int:
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO").upper())
    try:
        return asyncio.run(amain())
    except (KeyError, FileNotFoundError, json.JSONDecodeError, ValueError) as e:
        log.error("worker misconfigured: %s", e)
        return 2


if __name__ == "__main__":
    sys.exit(main())
