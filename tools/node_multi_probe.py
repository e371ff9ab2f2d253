"""Multi-table node calls on config 4's data (wfpt_wiener_like_nodes_multi):
per-call wall time and node-kernel time (HIP events) for T = 1, 2, 4, 8, 16
parameter tables (T chains' tables around the generating parameters), full
and simple DDM; per chain-call = call / T.

    python tools/node_multi_probe.py [--reps 100]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--tables", default="1,2,4,8,16")
    ap.add_argument("--full-only", action="store_true")
    a = ap.parse_args()
    from hddm_amd import _lib
    from test_nodes_multi import _c4, _chain_tables
    ctx = _lib.context(0)
    for full in ((True,) if a.full_only else (True, False)):
        m, _, start, P = _c4(full)
        ds = m.dataset
        for T in [int(v) for v in a.tables.split(",")]:
            tabs = _chain_tables(np.random.default_rng(T), P, T, full)
            for _ in range(5):
                ds.wiener_like_nodes_multi(tabs, **m.wp)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                ds.wiener_like_nodes_multi(tabs, **m.wp)
                ts.append(time.perf_counter() - t0)
            ctx.profile(ctx.PROF_EVENTS)
            ctx.profile_read(reset=True)
            for _ in range(a.reps):
                ds.wiener_like_nodes_multi(tabs, **m.wp)
            k_ms, nl, _ = ctx.profile_read(reset=True)
            ctx.profile(0)
            ctx.profile(ctx.PROF_EVALS)
            ctx.profile_lists(reset=True)
            ds.wiener_like_nodes_multi(tabs, **m.wp)
            _, _, ne = ctx.profile_read(reset=True)
            lists = ctx.profile_lists(reset=True)
            ctx.profile(0)
            med = float(np.median(ts)) * 1e6
            print(json.dumps({"full": full, "tables": T, "call_us_median": med,
                              "per_table_us": med / T, "node_kernels_us": k_ms / max(nl, 1) * 1e3,
                              "trials_per_call": T * m.n_trials,
                              "evals_per_trial": ne / (T * m.n_trials),
                              "records": lists.get("node_deferred"),
                              "segments": lists.get("segments")}), flush=True)
        m.dataset.close()


if __name__ == "__main__":
    main()
