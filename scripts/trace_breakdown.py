"""Per-phase breakdown of a rocprofv3 kernel trace of the WS bench.

Splits the timeline into prefill segments (any prefill-only kernel: pgemm epi
1-3, prefill attention, hipBLASLt prefill tiles, silu_mul / rope_kv) and decode
steps (segments between consecutive ``sample_kernel`` launches with no prefill
kernel inside), then reports per-kernel time per decode step, prefill time per
131K-token wave, and GPU idle inside / between phases.

    python scripts/trace_breakdown.py gpurun_out/r4_3/prof/run_kernel_trace.csv
"""
import collections
import csv
import re
import sys

# prefill-only kernels of the fused path (the library path's prefill GEMMs share
# their hipBLASLt names with the decode LM head and are not separable by name)
PREFILL = re.compile(r"pgemm_kernel<[123]|prefill_attn|silu_mul|(?<!splitk_)rope_kv_kernel|"
                     r"row_sumsq|(?<!splitk_add_)rmsnorm_kernel<\d+, true")


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0]
    return n[:70]


def main(path: str, tokens_per_wave: int = 256 * 512):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # decode steps: from one sample_kernel end to the next, no prefill kernel inside
    samples = [i for i, r in enumerate(rows) if "sample_kernel" in r[2]]
    dec = collections.Counter()
    dec_steps = 0
    dec_busy = dec_span = 0
    for a, b in zip(samples, samples[1:]):
        seg = rows[a + 1:b + 1]
        if any(PREFILL.search(r[2]) for r in seg):
            continue
        dec_steps += 1
        for s, e, n in seg:
            dec[short(n)] += e - s
            dec_busy += e - s
        dec_span += rows[b][1] - rows[a][1]
    pre = collections.Counter()
    pre_tokens_waves = 0.0
    for s, e, n in rows:
        if PREFILL.search(n):
            pre[short(n)] += e - s
    t0, t1 = rows[0][0], rows[-1][1]
    busy = sum(e - s for s, e, _ in rows)
    print(f"trace span {(t1 - t0) / 1e6:.1f} ms, kernels busy {busy / 1e6:.1f} ms "
          f"({100 * busy / (t1 - t0):.1f} %)")
    if dec_steps:
        print(f"\n{dec_steps} pure decode steps: busy {dec_busy / dec_steps / 1e3:.1f} us/step, "
              f"span {dec_span / dec_steps / 1e3:.1f} us/step")
        print("| us / step | kernel |\n|---:|---|")
        for n, t in dec.most_common(14):
            print(f"| {t / dec_steps / 1e3:8.1f} | {n} |")
    tot_pre = sum(pre.values())
    calls = sum(1 for r in rows if "pgemm_kernel<1" in r[2] or "silu_mul" in r[2])
    print(f"\nprefill kernels: {tot_pre / 1e6:.1f} ms total")
    print("| ms total | kernel |\n|---:|---|")
    for n, t in pre.most_common(12):
        print(f"| {t / 1e6:8.1f} | {n} |")
    return dec, pre


if __name__ == "__main__":
    main(sys.argv[1])
