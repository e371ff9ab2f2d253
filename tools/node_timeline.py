"""Per-call kernel timeline of the batched node call from a rocprofv3 kernel
trace of tools/node_call_probe.py: medians of each kernel's duration and of
the gaps, per call kind (full / simple DDM, the probe's two parameter sets in
order).

    python tools/node_timeline.py <trace dir>
"""
import csv
import glob
import statistics as st
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if name.startswith("void wfpt::node_") or name.startswith("wfpt::segment_publish"):
            cur.append(r)
            if name.startswith("wfpt::segment_publish"):
                calls.append(cur)
                cur = []
        else:
            cur = []
    kinds = {}
    for c in calls:
        key = tuple(r["Kernel_Name"].split("(")[0].replace("void wfpt::", "") for r in c)
        kinds.setdefault(key, []).append(c)
    for key, cs in kinds.items():
        # the probe runs truth then start per family: split each kind in halves
        for half, sel in (("first", cs[:len(cs) // 2]), ("second", cs[len(cs) // 2:])):
            if not sel:
                continue
            parts = []
            for k in range(len(key)):
                d = st.median(int(c[k]["End_Timestamp"]) - int(c[k]["Start_Timestamp"]) for c in sel)
                parts.append(f"{key[k][:22]} {d / 1e3:.1f}")
                if k + 1 < len(key):
                    g = st.median(int(c[k + 1]["Start_Timestamp"]) - int(c[k]["End_Timestamp"])
                                  for c in sel)
                    parts.append(f"gap {g / 1e3:.1f}")
            tot = st.median(int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"]) for c in sel)
            print(f"  {half:6s} x{len(sel):3d}: " + " | ".join(parts) + f" | total {tot / 1e3:.1f} us")


if __name__ == "__main__":
    main()
