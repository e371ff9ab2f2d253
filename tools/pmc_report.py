"""Per-launch counter report for tools/gpu_pmc_variants.sh output."""
import collections, csv, glob, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_*"))):
    v = os.path.basename(d)[4:]
    stats = list(csv.DictReader(open(os.path.join(d, "trace", "trace_kernel_stats.csv"))))
    main = max(stats, key=lambda r: float(r["TotalDurationNs"]))
    kname = main["Name"]
    res = collections.defaultdict(list)
    meta = {}
    for grp in ("sq", "f64"):
        for r in csv.DictReader(open(os.path.join(d, grp, f"{grp}_counter_collection.csv"))):
            if r["Kernel_Name"] == kname:
                res[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("VGPR_Count", "Scratch_Size", "Grid_Size", "Workgroup_Size")}
    c = {k: sum(x) / len(x) for k, x in res.items()}
    t = float(main["AverageNs"]) * 1e-9
    f64 = sum(c.get(k, 0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_FMA_F64",
                                    "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
    valu = c.get("SQ_INSTS_VALU", 0)
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / t
    util = (4 * f64 + 2 * (valu - f64)) / 1024 / (t * clk) if clk else 0
    wc = c.get("SQ_WAVE_CYCLES", 1)
    print(f"{v:10s} {kname[:48]:48s} {t*1e6:8.1f}us valu/wave={valu/max(c.get('SQ_WAVES',1),1):7.0f} "
          f"f64={f64/max(valu,1):.2f} util={util:.2f} clk={clk/1e9:.2f} "
          f"active={c.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f} wait_inst={c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
          f"wait_any={c.get('SQ_WAIT_ANY',0)/wc:.2f} {meta}")
