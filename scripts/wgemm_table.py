"""Turn a wgemm sweep (scripts/wgemm_sweep.py JSON) into the dispatch table
``omnia_amd/ops/tuned/wgemm_mi355x.json``: ``mode:Mbucket:N:K -> [nw, nwaves, S]``
for the shapes where the weight-streaming kernel plus the cost of its split-K
consumer reading the fp32 slabs (charged at 4 TB/s) beats tuned hipBLASLt by
>= 5 %.  Every other shape stays on the library path."""
import json
import sys


def main(src, dst):
    res = json.load(open(src))
    table = {}
    for key, r in sorted(res.items()):
        best = None
        for t, nw, nwaves, S in r["top"]:
            mode_out = 2 if (S > 1 or r["mode"] == 0) else 1
            slab = r["slab_bytes_per_split"] * S if mode_out == 2 else 0
            cost = t + slab / 4e6  # us at 4 TB/s
            if best is None or cost < best[0]:
                best = (cost, nw, nwaves, S)
        if best and best[0] < 0.95 * r["lib_us"]:
            table[f"{r['mode']}:{r['M']}:{r['N']}:{r['K']}"] = list(best[1:])
            print(f"{key:18s} lib {r['lib_us']:7.1f}  wgemm+slab {best[0]:7.1f}  -> {best[1:]}")
        else:
            print(f"{key:18s} lib {r['lib_us']:7.1f}  wgemm+slab {best[0] if best else 0:7.1f}"
                  "  -> lib")
    json.dump(table, open(dst, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "omnia_amd/ops/tuned/wgemm_mi355x.json")
