"""Summarise GPU idle gaps from a rocprofv3 kernel-trace CSV (one process or
many): busy time (union of kernel intervals), gaps by size, the largest gaps.
Usage: python scripts/gap_analysis.py <kernel_trace.csv> [out.md]"""
import csv
import sys


def main(path, out=None):
    iv = []
    with open(path) as f:
        r = csv.DictReader(f)
        for row in r:
            try:
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]),
                           row.get("Kernel_Name", "")[:60]))
            except (KeyError, ValueError):
                continue
    iv.sort()
    busy, gaps = 0, []
    cs, ce, last_name = iv[0][0], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, ce, last_name, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        last_name = n
    busy += ce - cs
    span = iv[-1][1] - iv[0][0]
    lines = [f"kernels: {len(iv)}", f"span: {span / 1e9:.3f} s", f"busy: {busy / 1e9:.3f} s "
             f"({100 * busy / span:.1f} %)", f"idle: {(span - busy) / 1e9:.3f} s"]
    for lo, hi in ((0, 1e4), (1e4, 1e5), (1e5, 1e6), (1e6, 1e7), (1e7, 1e12)):
        g = [x[0] for x in gaps if lo <= x[0] < hi]
        lines.append(f"gaps {lo / 1e3:>8.0f}-{hi / 1e3:<10.0f}us: n={len(g):7d} "
                     f"total={sum(g) / 1e6:9.1f} ms")
    # where the mid-size gaps (0.1-10 ms: host-side stalls inside a wave, not the
    # wave-boundary waits) sit: by the kernel pair around them
    from collections import Counter

    pairs = Counter()
    tot = Counter()
    for g, t, a, b in gaps:
        if 1e5 <= g < 1e7:
            k = f"{a[:45]} -> {b[:45]}"
            pairs[k] += 1
            tot[k] += g
    lines.append("0.1-10 ms gaps by kernel pair (count, total ms):")
    for k, n in pairs.most_common(12):
        lines.append(f"  {n:5d} {tot[k] / 1e6:9.1f} ms  {k}")
    # timeline of the mid-size gaps: count per 100 ms bucket of the run
    buckets = Counter(int((t - iv[0][0]) / 1e8) for g, t, a, b in gaps if 1e5 <= g < 1e7)
    if buckets:
        lines.append("0.1-10 ms gaps per 100 ms of the run (bucket: count): " + ", ".join(
            f"{k / 10:.1f}s:{v}" for k, v in sorted(buckets.items())))
    lines.append("largest gaps (ms, at s from start, after -> before):")
    for g, t, a, b in sorted(gaps, reverse=True)[:25]:
        lines.append(f"  {g / 1e6:8.2f} ms at {(t - iv[0][0]) / 1e9:8.3f} s  {a} -> {b}")
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
