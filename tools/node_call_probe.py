"""Batched per-node call of config 4 (wiener_like_nodes over 400 nodes x 250
trials: the call the hierarchical sampler makes per slice evaluation), per
call wall time (median) and node-kernel time (HIP events), at the generating
parameters and at HDDM's starting values, full and simple DDM.

    python tools/node_call_probe.py [--reps 300]
Set WFPT_NODE_SPLIT=0 for the one-lane-per-trial level 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    from hddm_amd import _lib
    from hddm_amd.hierarchical import HDDM, gen_data
    ctx = _lib.context(0)
    for full in (True, False):
        inter = dict(sv=0.1, sz=0.1, st=0.1) if full else {}
        data, truth = gen_data(n_subj=200, n_trials=500, **inter)
        m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05)
        start = m.node_table()
        P = start.copy()
        for j, (s, c) in enumerate(m.node_keys):
            P[j, 0] = truth["v"][c][s]
            P[j, 2] = truth["a"][s]
            P[j, 5] = truth["t"][s]
            for k, col in (("sv", 1), ("sz", 4), ("st", 6)):
                P[j, col] = inter.get(k, 0.0)
        for name, T in (("truth", P), ("start", start)):
            ds = m.dataset
            for _ in range(20):
                ds.wiener_like_nodes(T, **m.wp)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = ds.wiener_like_nodes(T, **m.wp)
                ts.append(time.perf_counter() - t0)
            ctx.profile(1)
            ctx.profile_read(reset=True)
            for _ in range(50):
                ds.wiener_like_nodes(T, **m.wp)
            ms, nl, _ = ctx.profile_read(reset=True)
            ctx.profile(ctx.PROF_EVALS)  # one counting call: the deferred-trial tallies
            ctx.profile_lists(reset=True)
            ds.wiener_like_nodes(T, **m.wp)
            lists = ctx.profile_lists(reset=True)
            ctx.profile(0)
            print(json.dumps({"full": full, "params": name,
                              "split": os.environ.get("WFPT_NODE_SPLIT", "1"),
                              "path": ctx.last_path(),
                              "call_us_median": float(np.median(ts)) * 1e6,
                              "call_us_p10": float(np.percentile(ts, 10)) * 1e6,
                              "node_kernels_us": ms / nl * 1e3, "sum": float(np.sum(r)),
                              "deferred": lists.get("node_deferred"),
                              "exact": lists.get("exact"), "walk": lists.get("walk")}),
                  flush=True)


if __name__ == "__main__":
    main()
