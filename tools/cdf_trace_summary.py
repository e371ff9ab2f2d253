"""Per-kernel durations of the CDF probe's calls from a rocprofv3 kernel trace
(tools/gpu_cdf_prof.sh): the table, lane-pass and wave kernels of each call,
split into the probe's full-DDM and simple halves.

    python tools/cdf_trace_summary.py gpurun_out/cdf_prof/<variant>/run_kernel_trace.csv
"""
import csv
import sys

import numpy as np


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "cdf_table_kernel" in n:
            cur = {"table": d, "t0": int(r["Start_Timestamp"])}
            calls.append(cur)
        elif cur is not None and "dmat_cdf_kernel" in n:
            cur["lane"] = d
        elif cur is not None and "cdf_wave_kernel" in n:
            cur["wave"] = d
            cur["span"] = (int(r["End_Timestamp"]) - cur["t0"]) / 1e3
    half = len(calls) // 2
    for name, cs in (("full", calls[:half]), ("simple", calls[half:])):
        out = {k: np.array([c[k] for c in cs]) for k in ("table", "lane", "wave", "span")}
        print(name, " ".join(f"{k} {np.median(v):6.1f} (max {v.max():6.1f})" for k, v in out.items()), "us")


if __name__ == "__main__":
    main(sys.argv[1])
