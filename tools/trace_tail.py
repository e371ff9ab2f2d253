"""Per-kernel averages over the LAST fraction of a rocprofv3 kernel trace
(steady state of a sampler run whose first part is burn-in).

    python tools/trace_tail.py <kernel_trace.csv> [--frac 0.3]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frac", type=float, default=0.3)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    t1 = int(rows[-1]["End_Timestamp"])
    cut = t1 - (t1 - t0) * a.frac
    agg = collections.defaultdict(list)
    busy = 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= cut:
            agg[r["Kernel_Name"][:64]].append((e - s) / 1e3)
            busy += e - s
    span = (t1 - cut) / 1e3
    print(f"window {span / 1e3:.1f} ms, kernels busy {busy / 1e6:.1f} ms")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{k:64s} n={len(v):6d} avg={sum(v) / len(v):8.1f} med={v[len(v) // 2]:8.1f} "
              f"p90={v[int(len(v) * .9)]:8.1f} total={sum(v) / 1e3:8.1f} ms")


if __name__ == "__main__":
    main()
