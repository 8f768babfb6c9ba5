"""Arena job result aggregation (``ee/pkg/arena/aggregator/aggregator.go:114-475``).

Folds the per-item results a job's workers wrote (one per scenario x provider x
trial) into:

* totals -- items, passed / failed, pass rate (percent), summed and mean item
  duration, output tokens, cost;
* ``byScenario`` / ``byProvider`` -- the same figures per group, so a job over
  several providers reads as a comparison table;
* ``errors`` -- failure messages grouped by text with the ids of the items that
  hit them (an empty message counts as "unknown error");
* ``assertions`` -- every turn assertion rolled up by name in first-seen order:
  total / passed / failed, pass rate, and the distinct failure messages.

:func:`to_job_result` renders the CRD ``status.result`` shape: a flat
``summary`` of strings (``passRate``, ``totalItems``, ... for kubectl columns)
plus a ``details`` entry holding the JSON breakdown.  Per-turn latency / TTFT
percentiles stay in :mod:`.stats` (threshold evaluation)."""
from __future__ import annotations

import json


def _status(r: dict) -> str:
    if "status" in r:
        return "pass" if r["status"] == "pass" else "fail"
    return "pass" if r.get("passed") and not r.get("error") else "fail"


def _duration_ms(r: dict) -> float:
    if r.get("duration_ms") is not None:
        return float(r["duration_ms"])
    turns = r.get("turns") or []
    if turns:
        return float(sum(t.get("latency_ms") or 0.0 for t in turns))
    return float(r.get("latency_ms") or 0.0)


def _new_group() -> dict:
    return {"total": 0, "passed": 0, "failed": 0, "passRate": 0.0, "totalDurationMs": 0.0,
            "avgDurationMs": 0.0, "totalTokens": 0, "totalCost": 0.0}


def _add(g: dict, ok: bool, dur: float, tokens: int, cost: float) -> None:
    g["total"] += 1
    g["passed" if ok else "failed"] += 1
    g["totalDurationMs"] += dur
    g["totalTokens"] += tokens
    g["totalCost"] += cost


def _finish(g: dict) -> dict:
    if g["total"]:
        g["passRate"] = round(100.0 * g["passed"] / g["total"], 4)
        g["avgDurationMs"] = round(g["totalDurationMs"] / g["total"], 3)
    g["totalDurationMs"] = round(g["totalDurationMs"], 3)
    g["totalCost"] = round(g["totalCost"], 8)
    return g


def _assertions(r: dict) -> list[dict]:
    out = list(r.get("assertions_flat") or [])
    if not out:
        for t in r.get("turns") or []:
            out.extend(t.get("assertions") or [])
        if not r.get("turns"):
            out.extend(a for a in (r.get("assertions") or []) if isinstance(a, dict))
    return [a for a in out if isinstance(a, dict) and not a.get("skipped")]


def aggregate(results: list[dict]) -> dict:
    """Aggregate item results (dicts as written by :class:`ArenaWorker`)."""
    tot = _new_group()
    tot.pop("passRate")
    by_s: dict[str, dict] = {}
    by_p: dict[str, dict] = {}
    errors: dict[str, dict] = {}
    asum: dict[str, dict] = {}
    for r in results:
        ok = _status(r) == "pass"
        dur = _duration_ms(r)
        tokens = int(r.get("output_tokens") or (r.get("metrics") or {}).get("tokens") or 0)
        cost = float(r.get("cost") or (r.get("metrics") or {}).get("cost") or 0.0)
        _add(tot, ok, dur, tokens, cost)
        if r.get("scenario"):
            _add(by_s.setdefault(r["scenario"], _new_group()), ok, dur, tokens, cost)
        if r.get("provider"):
            _add(by_p.setdefault(r["provider"], _new_group()), ok, dur, tokens, cost)
        if not ok and (r.get("error") is not None):
            msg = r.get("error") or "unknown error"
            e = errors.setdefault(msg, {"message": msg, "count": 0, "workItemIds": []})
            e["count"] += 1
            if r.get("item_id"):
                e["workItemIds"].append(r["item_id"])
        for a in _assertions(r):
            name = a.get("id") or a.get("name") or a.get("type") or "assertion"
            s = asum.setdefault(name, {"name": name, "total": 0, "passed": 0, "failed": 0,
                                       "passRate": 0.0, "failures": []})
            s["total"] += 1
            if a.get("passed"):
                s["passed"] += 1
            else:
                s["failed"] += 1
                m = a.get("message") or ""
                if m and m not in s["failures"]:
                    s["failures"].append(m)
    out = {
        "totalItems": tot["total"], "passedItems": tot["passed"], "failedItems": tot["failed"],
        "passRate": round(100.0 * tot["passed"] / tot["total"], 4) if tot["total"] else 0.0,
        "totalDurationMs": round(tot["totalDurationMs"], 3),
        "avgDurationMs": round(tot["totalDurationMs"] / tot["total"], 3) if tot["total"] else 0.0,
        "totalTokens": tot["totalTokens"], "totalCost": round(tot["totalCost"], 8),
    }
    if by_s:
        out["byScenario"] = {k: _finish(v) for k, v in sorted(by_s.items())}
    if by_p:
        out["byProvider"] = {k: _finish(v) for k, v in sorted(by_p.items())}
    if errors:
        out["errors"] = sorted(errors.values(), key=lambda e: (-e["count"], e["message"]))
    if asum:
        for s in asum.values():
            s["passRate"] = round(100.0 * s["passed"] / s["total"], 4)
            if not s["failures"]:
                s.pop("failures")
        out["assertions"] = list(asum.values())
    return out


def to_job_result(agg: dict) -> dict:
    """``status.result`` of an ArenaJob: flat string summary + JSON details."""
    summary = {
        "passRate": f"{agg['passRate']:.1f}",
        "totalItems": str(agg["totalItems"]),
        "passedItems": str(agg["passedItems"]),
        "failedItems": str(agg["failedItems"]),
        "avgDurationMs": str(int(round(agg["avgDurationMs"]))),
    }
    if agg.get("totalTokens"):
        summary["totalTokens"] = str(agg["totalTokens"])
    if agg.get("totalCost"):
        summary["totalCost"] = f"{agg['totalCost']:.6f}"
    details = {
        "scenarios": [{"name": k, **{f: v[f] for f in ("total", "passed", "failed", "passRate",
                                                         "avgDurationMs", "totalTokens",
                                                         "totalCost")}}
                      for k, v in (agg.get("byScenario") or {}).items()],
        "providers": [{"name": k, **{f: v[f] for f in ("total", "passed", "failed", "passRate",
                                                         "avgDurationMs", "totalTokens",
                                                         "totalCost")}}
                      for k, v in (agg.get("byProvider") or {}).items()],
        "assertions": agg.get("assertions") or [],
        "errors": agg.get("errors") or [],
    }
    summary["details"] = json.dumps(details, separators=(",", ":"), sort_keys=True)
    return {"summary": summary}
