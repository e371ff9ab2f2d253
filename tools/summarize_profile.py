"""Summarise a tools/gpu_profile.sh run (gpurun_out/prof) into profiles/<tag>/.

Writes <tag>/pmc_summary.json with per-launch averages of the main likelihood
kernel, and profiles/traffic.json (read by bench.py) with HBM bytes per launch,
corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) reads half
the bytes of a wide coalesced stream on gfx950, so it is doubled; WRITE_SIZE
(KiB) is taken as is.

    python tools/summarize_profile.py r02 [--kernel 'void wfpt::fast_kernel<3, false, 0>']

traffic.json carries the source digest of hddm_amd/lib/libwfpt_amd.so (flags +
sources of the build that was shipped to the GPU box and profiled,
hddm_amd.build.source_digest): bench.py uses the executed-work figures only
while the library it loads was built from those sources.
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")


def per_launch(path, kernel):
    agg = collections.defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith(kernel):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count",
                                      "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size",
                                      "LDS_Block_Size")}
    return {k: sum(v) / len(v) for k, v in agg.items()}, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="void wfpt::lean_kernel<3, false, 0>")
    ap.add_argument("--trials", type=int, default=1_000_000)
    ap.add_argument("--bytes-per-trial", type=float, default=8.0,
                    help="algorithmic HBM bytes per trial: 8 for the summing kernels (rt in, "
                         "a sum out), 16 for per-trial outputs (x in, value out)")
    ap.add_argument("--prof-dir", default=PROF, help="tools/gpu_profile*.sh output directory")
    ap.add_argument("--name", default="pmc_summary", help="summary file name under profiles/<tag>/")
    ap.add_argument("--no-traffic", action="store_true",
                    help="do not write profiles/traffic.json (secondary kernels)")
    ap.add_argument("--traffic-out", default="traffic.json",
                    help="file under profiles/ for the digest-matched figures bench.py reads "
                         "(traffic.json: the headline kernel; traffic_stress.json: the engine "
                         "on the stress sets)")
    a = ap.parse_args()
    prof = a.prof_dir
    out_dir = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out_dir, exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(prof, "trace", "trace_kernel_stats.csv"))))
    k_ns = next(float(r["AverageNs"]) for r in stats if r["Name"].startswith(a.kernel))
    res, meta = {}, {}
    for grp in ("fetch", "write", "sq", "f64"):
        p = os.path.join(prof, grp, f"{grp}_counter_collection.csv")
        if os.path.exists(p):
            r, m = per_launch(p, a.kernel)
            res.update(r)
            meta = meta or m
    t = k_ns * 1e-9
    fetch_b = res.get("FETCH_SIZE", 0.0) * 1024 * 2  # gfx950: FETCH_SIZE reads half
    write_b = res.get("WRITE_SIZE", 0.0) * 1024
    f64 = sum(v for k, v in res.items() if k.startswith("SQ_INSTS_VALU_") and k.endswith("F64")
              and "MFMA" not in k)
    valu = res.get("SQ_INSTS_VALU", 0.0)
    clk = res.get("GRBM_GUI_ACTIVE", 0.0) / 8 / t if t else 0.0
    # issue-time model: a wave64 fp64 VALU op occupies a SIMD-32 for 4 cycles, others 2
    simd_cycles = (4 * f64 + 2 * (valu - f64)) / 1024.0
    summary = {
        "kernel": a.kernel, "trials": a.trials, "kernel_avg_ns": k_ns, **meta,
        "counters_per_launch": res,
        "hbm_read_bytes": fetch_b, "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "algorithmic_bytes_per_launch": a.bytes_per_trial * a.trials,
        "valu_lane_ops_per_trial": valu * 64 / a.trials,
        "fp64_lane_ops_per_trial": f64 * 64 / a.trials,
        "fp64_lane_ops_per_s": f64 * 64 / t,
        "effective_clock_hz": clk,
        "valu_issue_utilisation": simd_cycles / (t * clk) if clk else None,
        "valu_busy_wave": res.get("SQ_ACTIVE_INST_VALU", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1),
    }
    shutil.copy(os.path.join(prof, "trace", "trace_kernel_stats.csv"),
                os.path.join(out_dir, "kernel_stats.csv" if a.name == "pmc_summary"
                             else a.name + "_kernel_stats.csv"))
    # the digest of the library the GPU run profiled (tools/gpu_profile.sh
    # records it next to the counters), not whatever is built here now
    with open(os.path.join(prof, "src_sha1.txt")) as fh:
        sha = fh.read().strip()
    summary["src_sha1"] = sha
    with open(os.path.join(out_dir, a.name + ".json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    if a.no_traffic:
        print(json.dumps(summary, indent=1))
        return
    with open(os.path.join(ROOT, "profiles", a.traffic_out), "w") as fh:
        json.dump({"src_sha1": sha, "source": f"profiles/{a.tag}/{a.name}.json", "kernel": a.kernel,
                   "n_trials": a.trials, "hbm_bytes_per_launch": fetch_b + write_b,
                   "hbm_bytes_per_trial": (fetch_b + write_b) / a.trials,
                   "valu_issue_utilisation": summary["valu_issue_utilisation"],
                   "fp64_lane_ops_per_trial": summary["fp64_lane_ops_per_trial"],
                   "valu_lane_ops_per_trial": summary["valu_lane_ops_per_trial"]}, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
