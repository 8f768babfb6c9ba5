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


if __name__ == "__main__":
    main(sys.argv[1])
