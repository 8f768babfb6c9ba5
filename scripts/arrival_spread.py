"""Per-wave arrival spreads of a turn's start across the serving stages, from the
OMNIA_TRACE_ARRIVALS files (client_send -> facade_msg -> runtime_turn ->
runtime_submit -> engine_add).  Usage: python scripts/arrival_spread.py DIR"""
import collections
import glob
import os
import sys


def main(d):
    ev = []
    for f in glob.glob(os.path.join(d, "*.txt")):
        for line in open(f):
            t, tag = line.split()
            ev.append((float(t), tag))
    ev.sort()
    sends = [t for t, g in ev if g == "client_send"]
    if not sends:
        print("no client_send marks")
        return
    # waves: client sends separated by > 0.5 s
    waves, cur = [], [sends[0]]
    for t in sends[1:]:
        if t - cur[-1] > 0.5:
            waves.append(cur)
            cur = []
        cur.append(t)
    waves.append(cur)
    order = ["client_send", "facade_msg", "runtime_turn", "runtime_submit", "engine_add"]
    dorder = ["engine_finish", "runtime_done", "facade_done", "client_done"]
    for w in waves:
        t0, t1 = w[0], w[-1] + 0.5
        by = collections.defaultdict(list)
        for t, g in ev:
            if t0 <= t < t1 + 2.0:
                by[g].append(t)
        print(f"wave at {t0:.3f}: {len(w)} turns")
        for g in order:
            ts = sorted(by.get(g, []))[:len(w)]
            if ts:
                print(f"  {g:15s} first +{(ts[0] - t0) * 1e3:7.1f} ms  last +{(ts[-1] - t0) * 1e3:7.1f}"
                      f" ms  spread {(ts[-1] - ts[0]) * 1e3:7.1f} ms  n={len(ts)}")
    # turn ends: the previous wave's finishes before each wave's first send
    print("wave ends (relative to the first engine finish of the wave):")
    bounds = [w[0] for w in waves] + [float("inf")]
    for a, b in zip(bounds, bounds[1:]):
        by = collections.defaultdict(list)
        for t, g in ev:
            if a <= t < b and g in dorder:
                by[g].append(t)
        fin = sorted(by.get("engine_finish", []))
        if not fin:
            continue
        e0 = fin[0]
        for g in dorder:
            ts = sorted(by.get(g, []))
            if ts:
                print(f"  {g:15s} first +{(ts[0] - e0) * 1e3:7.1f} ms  last "
                      f"+{(ts[-1] - e0) * 1e3:7.1f} ms  n={len(ts)}")
        if b != float("inf"):
            print(f"  next wave's first send +{(b - e0) * 1e3:7.1f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
