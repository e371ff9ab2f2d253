"""Per-node latency of the drop-in likelihood: the call HDDM
makes once per observed node per logp (hddm/likelihoods.py:52-55 via
base.py:754-757), on one 250-trial node, simple and full DDM.

Rows (median over --reps calls after warm-up, microseconds):
  capi_resident   bare ctypes call of wfpt_wiener_like on a resident dataset
  dataset         hddm_amd.wfpt.Dataset.wiener_like (Python wrapper)
  wfpt_like_res   hddm_amd.likelihoods wfpt_like on a DataFrame slice (the
                  resident cache; what install() binds for HDDM's Wfpt class)
  ref_wfpt_like   the reference's own wfpt_like body with install()ed wfpt:
                  x['rt'].abs().max() < 998, then wfpt.wiener_like(x['rt'].values)
                  (host array uploaded per call)
  module_host     hddm_amd.wfpt.wiener_like on a host array
  cpu_oracle      the C restatement of the reference (1 thread), for scale

    python tools/bench_node_latency.py [--reps 2000] [--json out.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KN = dict(err=1e-4, n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3, w_outlier=0.1)
SETS = {"simple": (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0),
        "full": (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)}


def timeit(fn, reps, warm=50):
    for _ in range(warm):
        fn()
    ts = np.empty(reps)
    for i in range(reps):
        t0 = time.perf_counter_ns()
        fn()
        ts[i] = time.perf_counter_ns() - t0
    return {"median_us": float(np.median(ts)) / 1e3, "p10_us": float(np.percentile(ts, 10)) / 1e3,
            "p90_us": float(np.percentile(ts, 90)) / 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--trials", type=int, default=250)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import pandas as pd
    import oracle
    from hddm_amd import _lib, likelihoods, wfpt
    out = {"trials": a.trials, "reps": a.reps, "rows": {}}
    for name, p in SETS.items():
        np.random.seed(20261017)
        x = wfpt.gen_rts_from_cdf(*p, samples=a.trials, dt=1e-4)
        df = pd.DataFrame({"rt": x, "response": (x > 0).astype(float), "subj_idx": 0})
        node = df[df.subj_idx == 0]
        rows = {}
        ds = wfpt.Dataset(x)
        ctx = ds.ctx
        P = _lib.make_params(*p, 0.05)
        K = _lib.make_knobs(KN["err"], KN["n_st"], KN["n_sz"], KN["use_adaptive"],
                            KN["simps_err"], KN["w_outlier"])
        res = ctypes.c_double()
        f = _lib.wfpt_wiener_like
        h, dh = ctx.handle, ds.handle
        pp, kp, rp = ctypes.byref(P), ctypes.byref(K), ctypes.byref(res)
        rows["capi_resident"] = timeit(lambda: f(h, dh, pp, kp, rp), a.reps)
        rows["dataset"] = timeit(lambda: ds.wiener_like(*p, p_outlier=0.05, **KN), a.reps)
        like = likelihoods.make_wfpt_like(KN)
        rows["wfpt_like_res"] = timeit(lambda: like(node, *p, p_outlier=0.05), a.reps)

        def ref_body():  # hddm/likelihoods.py:52-55 with wfpt = hddm_amd.wfpt
            if node["rt"].abs().max() < 998:
                return wfpt.wiener_like(node["rt"].values, *p, p_outlier=0.05, **KN)
        rows["ref_wfpt_like"] = timeit(ref_body, a.reps)
        xh = np.ascontiguousarray(x)
        rows["module_host"] = timeit(lambda: wfpt.wiener_like(xh, *p, p_outlier=0.05, **KN),
                                     a.reps)
        kn = (KN["err"], KN["n_st"], KN["n_sz"], KN["use_adaptive"], KN["simps_err"], 0.05,
              KN["w_outlier"])
        rows["cpu_oracle"] = timeit(lambda: oracle.wiener_like(xh, *p, *kn),
                                    max(50, a.reps // 10), warm=5)
        vals = {"resident": ds.wiener_like(*p, p_outlier=0.05, **KN),
                "host": wfpt.wiener_like(xh, *p, p_outlier=0.05, **KN),
                "oracle": oracle.wiener_like(xh, *p, *kn)}
        rows["values"] = vals
        out["rows"][name] = rows
        print(name, json.dumps(rows), flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
