"""Device idle time between kernels from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d <dir> -- python3 bench.py ...
    python scripts/kernel_gaps.py <dir> [--out summary.md]

For the process / queue that ran the most kernel time (the engine-core), the
kernels are ordered by start time; every gap between one kernel's end and the
next one's start is device idle time on that queue.  The gaps are summed per
"phase" (a prefill-GEMM neighbourhood vs graph decode) and the largest gaps are
listed with the kernels on both sides -- which tells a launch-bound host from a
synchronisation point from a copy on another engine.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    i = n.find("(")
    n = n[:i] if i > 0 else n
    return n[:70]


def load(d: str):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append(r)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last-ms", type=float, default=0.0,
                    help="analyse only the final window of this many ms (the timed waves)")
    ap.add_argument("--dump", default="", help="write the window's kernels as a gzip CSV")
    a = ap.parse_args(argv)
    rows = load(a.dir)
    if not rows:
        raise SystemExit(f"no kernel_trace.csv under {a.dir}")
    key = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    busy = collections.Counter()
    for r in rows:
        busy[(r.get("Process_Id", ""), r.get(key, ""))] += int(r["End_Timestamp"]) - int(
            r["Start_Timestamp"])
    (pid, q), _ = busy.most_common(1)[0]
    ks = sorted((r for r in rows if r.get("Process_Id", "") == pid and r.get(key, "") == q),
                key=lambda r: int(r["Start_Timestamp"]))
    if a.last_ms > 0:
        end = max(int(r["End_Timestamp"]) for r in ks)
        lo = end - int(a.last_ms * 1e6)
        ks = [r for r in ks if int(r["Start_Timestamp"]) >= lo]
    if a.dump:
        import gzip

        with gzip.open(a.dump, "wt") as f:
            f.write("start_ns,end_ns,kernel\n")
            for r in ks:
                f.write(f"{r['Start_Timestamp']},{r['End_Timestamp']},{short(r['Kernel_Name'])}\n")
    out = []
    t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    kern = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks)
    out.append(f"process {pid} queue {q}: {len(ks)} kernels, span {(t1 - t0) / 1e6:.1f} ms, "
               f"kernel time {kern / 1e6:.1f} ms ({100 * kern / (t1 - t0):.1f} %)")
    gaps = []
    by_prev = collections.Counter()
    by_phase = collections.Counter()
    nbig = collections.Counter()
    for a_, b in zip(ks, ks[1:]):
        g = int(b["Start_Timestamp"]) - int(a_["End_Timestamp"])
        if g <= 0:
            continue
        pa, pb = short(a_["Kernel_Name"]), short(b["Kernel_Name"])
        phase = "prefill" if ("pgemm" in pa or "pgemm" in pb or "prefill_attn" in pa
                              or "prefill_attn" in pb) else "other"
        by_phase[phase] += g
        by_prev[(pa, pb)] += g
        if g > 50_000:
            nbig[phase] += 1
        gaps.append((g, pa, pb, int(a_["End_Timestamp"]) - t0))
    tot = sum(g for g, *_ in gaps)
    out.append(f"idle between kernels: {tot / 1e6:.1f} ms ({100 * tot / (t1 - t0):.1f} % of "
               f"the span); by phase: " + ", ".join(f"{k} {v / 1e6:.1f} ms" for k, v in
                                                    by_phase.most_common()))
    out.append(f"gaps > 50 us: {dict(nbig)}")
    out.append("\n| idle ms | after -> before |")
    out.append("|---:|---|")
    for (pa, pb), g in by_prev.most_common(a.top):
        out.append(f"| {g / 1e6:.2f} | {pa} -> {pb} |")
    out.append("\nlargest single gaps:")
    for g, pa, pb, at in sorted(gaps, reverse=True)[:a.top]:
        out.append(f"  {g / 1e3:9.1f} us at +{at / 1e6:9.1f} ms: {pa} -> {pb}")
    # kernel time by name
    kt = collections.Counter()
    kn = collections.Counter()
    for r in ks:
        n = short(r["Kernel_Name"])
        kt[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        kn[n] += 1
    out.append("\n| kernel ms | calls | kernel |")
    out.append("|---:|---:|---|")
    for n, v in kt.most_common(a.top):
        out.append(f"| {v / 1e6:.1f} | {kn[n]} | {n} |")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
