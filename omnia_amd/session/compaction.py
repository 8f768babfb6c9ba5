"""Storage compaction CronJob: warm -> cold archival, warm-only purge, cold
expiry, hot invalidation (``cmd/compaction``, ``internal/compaction/engine.go:53-351``).

NB: Omnia's "compaction" is storage tiering, not LLM context
compaction.  The KV analogue (HBM -> DRAM -> transcript) lives in
``omnia_amd.engine.kv_manager``.

``python -m omnia_amd.session.compaction --db sessions.db --cold-dir /archive``
"""
from __future__ import annotations

import argparse
import logging
import time
from dataclasses import dataclass

from ..observability import metrics as M
from .store import ColdArchive, HotCache, LocalBlobStore, TierError, WarmStore

log = logging.getLogger("omnia.compaction")


@dataclass
class CompactionConfig:
    warm_retention_s: float = 7 * 86400  # older than this moves to cold (or is purged)
    cold_retention_s: float = 365 * 86400
    batch_size: int = 200
    max_retries: int = 3
    retry_backoff_s: float = 0.5
    dry_run: bool = False


@dataclass
class CompactionResult:
    archived: int = 0
    purged: int = 0
    cold_expired: int = 0
    skipped: int = 0
    errors: int = 0


class CompactionEngine:
    def __init__(self, warm: WarmStore, cold: ColdArchive | None, hot: HotCache | None = None,
                 cfg: CompactionConfig | None = None, sleep=time.sleep):
        self.warm, self.cold, self.hot = warm, cold, hot
        self.cfg = cfg or CompactionConfig()
        self.sleep = sleep

    def _retry(self, fn):
        last = None
        for i in range(self.cfg.max_retries):
            try:
                return fn()
            except TierError as e:
                last = e
                self.sleep(self.cfg.retry_backoff_s * (2 ** i))
        raise last

    def run(self, now: float | None = None) -> CompactionResult:
        now = now or time.time()
        res = CompactionResult()
        cutoff = now - self.cfg.warm_retention_s
        try:
            while True:
                ids = self._retry(lambda: self.warm.sessions_older_than(cutoff,
                                                                        self.cfg.batch_size))
                if not ids:
                    break
                batch = []
                for sid in ids:
                    try:
                        s = self.warm.get_session(sid)
                        msgs = self.warm.messages(sid, limit=10**9)
                    except TierError:
                        res.skipped += 1  # never delete what we could not read
                        continue
                    if s is not None:
                        batch.append((s, msgs))
                if self.cfg.dry_run:
                    res.archived += len(batch)
                    break
                if self.cold is not None and batch:
                    self._retry(lambda: self.cold.archive(batch))
                    res.archived += len(batch)
                    M.COMPACTION_SESSIONS.inc(len(batch))
                elif batch:
                    res.purged += len(batch)
                    M.RETENTION_DELETED.labels("warm").inc(len(batch))
                for s, _ in batch:
                    self._retry(lambda sid=s.id: self.warm.delete_session(sid))
                    if self.hot is not None:
                        self.hot.invalidate(s.id)
                if res.skipped and len(batch) == 0:
                    break
            if self.cold is not None and not self.cfg.dry_run:
                res.cold_expired = self.cold.expire(now - self.cfg.cold_retention_s)
                M.RETENTION_DELETED.labels("cold").inc(res.cold_expired)
            M.COMPACTION_RUNS.labels("success").inc()
        except Exception:  # noqa: BLE001
            res.errors += 1
            M.COMPACTION_RUNS.labels("error").inc()
            log.exception("compaction run failed")
        return res


def run_remote(url: str, warm_s: float | None, cold_s: float | None, dry_run: bool,
               token: str = "", timeout_s: float = 600.0) -> dict:
    """Drive one compaction run on a session-api replica
    (``POST /api/v1/admin/compaction``): the CronJob form for deployments whose
    warm store lives inside the session-api pod."""
    import json
    import urllib.request

    body = {"dryRun": dry_run}
    if warm_s is not None:
        body["warmRetentionSeconds"] = warm_s
    if cold_s is not None:
        body["coldRetentionSeconds"] = cold_s
    req = urllib.request.Request(url.rstrip("/") + "/api/v1/admin/compaction",
                                 data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    if token:
        req.add_header("Authorization", f"Bearer {token}")
    with urllib.request.urlopen(req, timeout=timeout_s) as r:
        return json.loads(r.read() or b"{}")


def main(argv=None):
    ap = argparse.ArgumentParser("compaction")
    ap.add_argument("--db", default="", help="warm store (SQLite path / postgres DSN)")
    ap.add_argument("--session-api", default="",
                    help="run the compaction inside this session-api replica instead")
    ap.add_argument("--token", default="")
    ap.add_argument("--cold-dir", default="")
    ap.add_argument("--warm-retention", type=float, default=None,
                    help="seconds (default: the policy's, else 7 days)")
    ap.add_argument("--cold-retention", type=float, default=None,
                    help="seconds (default: the policy's, else 365 days)")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--retention-config", default="",
                    help="retention.yaml of a SessionRetentionPolicy (operator ConfigMap "
                         "retention-policy-<name>); overrides the two retention flags")
    a = ap.parse_args(argv)
    if a.session_api:
        res = run_remote(a.session_api, a.warm_retention, a.cold_retention, a.dry_run,
                         a.token)
        print(res)
        return 1 if res.get("errors") else 0
    if not a.db:
        ap.error("--db or --session-api is required")
    warm_s = a.warm_retention if a.warm_retention is not None else 7 * 86400
    cold_s = a.cold_retention if a.cold_retention is not None else 365 * 86400
    if a.retention_config:
        import yaml

        from ..operator.policies import retention_from_config

        with open(a.retention_config) as f:
            r = retention_from_config(yaml.safe_load(f) or {})
        warm_s, cold_s = r.get("warm_retention_s", warm_s), r.get("cold_retention_s", cold_s)
    cold = ColdArchive(LocalBlobStore(a.cold_dir)) if a.cold_dir else None
    eng = CompactionEngine(WarmStore(a.db), cold, None, CompactionConfig(
        warm_s, cold_s, dry_run=a.dry_run))
    print(eng.run())


if __name__ == "__main__":
    import sys

    sys.exit(main(sys.argv[1:]))
