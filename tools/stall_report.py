"""Per-launch stall attribution of one kernel from tools/gpu_stall_pmc.sh output.

    python tools/stall_report.py gpurun_out/stall/<variant> [kernel-prefix]
"""
import csv
import os
import sys


def per_launch(path, kernel):
    vals, n = {}, set()
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith(kernel):
            continue
        n.add(r["Dispatch_Id"])
        vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return {k: v / max(len(n), 1) for k, v in vals.items()}


def main():
    d = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "void wfpt::lean_kernel<3, false, 0>"
    c = {}
    for p in ("p1", "p2"):
        f = os.path.join(d, p, f"{p}_counter_collection.csv")
        if os.path.exists(f):
            c.update(per_launch(f, kern))
    st = list(csv.DictReader(open(os.path.join(d, "trace", "trace_kernel_stats.csv"))))
    ns = next(float(r["AverageNs"]) for r in st if r["Name"].startswith(kern))
    wc = c.get("SQ_WAVE_CYCLES", 0)
    out = {"kernel_us": ns / 1e3}
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        out[k + "/WAVE_CYCLES"] = c.get(k, 0) / wc if wc else None
    w = c.get("SQ_WAVES", 1)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_IFETCH",
              "SQ_INSTS_VSKIPPED"):
        out[k + "_per_wave"] = c.get(k, 0) / w
    if c.get("SQ_ACTIVE_INST_VALU"):
        out["lane_activity"] = c.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * c["SQ_ACTIVE_INST_VALU"])
    out["wave_cycles_per_wave(quad)"] = wc / w
    out["smem_cycles_per_wave"] = c.get("SQ_INST_CYCLES_SMEM", 0) / w
    for k, v in out.items():
        print(f"{k:32s} {v:.4g}" if isinstance(v, float) else f"{k:32s} {v}")


if __name__ == "__main__":
    main()
