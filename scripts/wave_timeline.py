"""Per-wave wall-time attribution from an untraced timeline run.

Run the bench with ``OMNIA_TIMELINE_DIR=<dir>`` (every process of the serving
tree buffers its stage marks and the engine-core its per-step host times +
hipEvent device intervals, observability/timeline.py), then:

    python scripts/wave_timeline.py <dir> --concurrency 256 [--json out.json]

A closed-loop wave = ``concurrency`` consecutive ``client_send`` marks up to
the last ``client_done`` of the group.  The wave's wall time splits EXACTLY into

    head   first client send -> first GPU step of the wave starts
    busy   device time inside engine steps (prefill / mixed / decode)
    gaps   device idle between consecutive steps (the host launched late)
    tail   last step ends -> last client receives its done frame

and the head / gaps are further attributed to the host stages that sit there.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics


def load(d: str) -> list[dict]:
    evs = []
    for p in glob.glob(os.path.join(d, "*.jsonl")):
        with open(p) as f:
            for line in f:
                line = line.strip()
                if line:
                    e = json.loads(line)
                    e["src"] = os.path.basename(p)
                    evs.append(e)
    evs.sort(key=lambda e: e["t"])
    return evs


def spread(ts: list[float], t0: float) -> dict:
    if not ts:
        return {}
    ts = sorted(ts)
    return {"first_ms": round(1e3 * (ts[0] - t0), 2),
            "p50_ms": round(1e3 * (ts[len(ts) // 2] - t0), 2),
            "last_ms": round(1e3 * (ts[-1] - t0), 2), "n": len(ts)}


def analyse(evs: list[dict], C: int) -> list[dict]:
    by = {}
    for e in evs:
        by.setdefault(e["ev"], []).append(e)
    sends = [e["t"] for e in by.get("client_send", [])]
    dones = [e["t"] for e in by.get("client_done", [])]
    steps = sorted(by.get("step", []), key=lambda e: e["d0"])
    waves = []
    for w in range(len(sends) // C):
        t_start = sends[w * C]
        t_next = sends[(w + 1) * C] if (w + 1) * C < len(sends) else float("inf")
        t_end = max(t for t in dones if t_start <= t < t_next) if any(
            t_start <= t < t_next for t in dones) else None
        if t_end is None:
            continue
        ws = [s for s in steps if t_start <= s["d1"] and s["d0"] <= t_end]
        if not ws:
            continue
        busy = {"prefill": 0.0, "decode": 0.0, "mixed": 0.0, "other": 0.0}
        gaps = {}
        gap_list = []
        prev = None
        for s in ws:
            d0, d1 = max(s["d0"], t_start), min(s["d1"], t_end)
            k = s["kind"].replace("_sync", "")
            if prev is not None and d0 > prev["d1"]:
                g = d0 - prev["d1"]
                key = f"{prev['kind'].replace('_sync', '')}->{k}"
                gaps[key] = gaps.get(key, 0.0) + g
                # the host launched late: how far the launch started after the GPU
                # drained, and how long schedule + launch took
                gap_list.append({"after": prev["kind"], "before": s["kind"], "gap_ms": 1e3 * g,
                                 "sched_ms": 1e3 * (s["t_launch"] - s["t"]),
                                 "launch_ms": 1e3 * (s["t_launched"] - s["t_launch"]),
                                 "host_start_after_drain_ms": 1e3 * (s["t"] - prev["d1"])})
            lo = d0 if prev is None else max(d0, prev["d1"])
            if d1 > lo:
                busy[k if k in busy else "other"] += d1 - lo
            prev = s if prev is None or s["d1"] > prev["d1"] else prev
        first_d0, last_d1 = max(ws[0]["d0"], t_start), min(max(s["d1"] for s in ws), t_end)
        head, tail = first_d0 - t_start, t_end - last_d1
        wall = t_end - t_start
        tot_busy, tot_gap = sum(busy.values()), sum(gaps.values())
        marks = {k: spread([e["t"] for e in by.get(k, []) if t_start <= e["t"] <= t_end],
                           t_start)
                 for k in ("client_send", "facade_msg", "runtime_turn", "runtime_submit",
                           "engine_add", "client_first", "engine_finish", "runtime_done",
                           "facade_done", "client_done")}
        big = sorted(gap_list, key=lambda g: -g["gap_ms"])[:8]
        n_dec = sum(1 for s in ws if s["kind"].startswith("decode"))
        waves.append({
            "wave": w, "wall_ms": round(1e3 * wall, 2),
            "head_ms": round(1e3 * head, 2), "busy_ms": round(1e3 * tot_busy, 2),
            "gap_ms": round(1e3 * tot_gap, 2), "tail_ms": round(1e3 * tail, 2),
            "sum_check_ms": round(1e3 * (head + tot_busy + tot_gap + tail), 2),
            "gpu_busy_frac": round(tot_busy / wall, 4),
            "busy_by_kind_ms": {k: round(1e3 * v, 2) for k, v in busy.items() if v},
            "gaps_by_transition_ms": {k: round(1e3 * v, 2) for k, v in
                                      sorted(gaps.items(), key=lambda x: -x[1])},
            "steps": len(ws), "decode_steps": n_dec,
            "decode_step_device_ms_p50": round(1e3 * statistics.median(
                [s["d1"] - s["d0"] for s in ws if s["kind"] == "decode"]), 3) if n_dec else None,
            "largest_gaps": [{k: (round(v, 3) if isinstance(v, float) else v)
                              for k, v in g.items()} for g in big],
            "stage_marks_rel_ms": marks,
        })
    return waves


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    waves = analyse(load(a.dir), a.concurrency)
    for w in waves:
        print(f"wave {w['wave']}: wall {w['wall_ms']:.1f} ms = head {w['head_ms']:.1f} + "
              f"busy {w['busy_ms']:.1f} + gaps {w['gap_ms']:.1f} + tail {w['tail_ms']:.1f} "
              f"(sum {w['sum_check_ms']:.1f}); GPU busy {100 * w['gpu_busy_frac']:.1f} %")
        print("   busy by kind:", w["busy_by_kind_ms"])
        print("   gaps by transition:", w["gaps_by_transition_ms"])
        for k, v in w["stage_marks_rel_ms"].items():
            if v:
                print(f"   {k:15s} {v}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(waves, f, indent=1)


if __name__ == "__main__":
    main()
