"""Replay a batched per-node likelihood call saved by
`tools/bench_hier.py --slow-dump` (data + parameter table of the slowest
call of a run) and report where its time goes: call time, kernel lists
(deferred records, exact-path trials, per-lane walks) and evaluations per
trial, plus the same call at the run's typical parameters for scale.

    python tools/slow_node_probe.py gpurun_out/hier/slow.npz [--reps 5]
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
    ap.add_argument("dump")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import pandas as pd
    from hddm_amd import _lib
    from hddm_amd.hierarchical import HDDM
    d = np.load(a.dump)
    P = d["params"]
    data = pd.DataFrame({"rt": d["rt"], "response": d["response"], "subj_idx": d["subj_idx"],
                         "cond": np.where(d["cond"], "c1", "c0")})
    m = HDDM(data, depends_on={"v": "cond"}, include=("sv", "sz", "st"),
             p_outlier=float(P[0, 7]), seed=1)
    ctx = m.dataset.ctx
    out = {"saved_call_ms": float(d["seconds"]) * 1e3,
           "params_range": {n: [float(P[:, i].min()), float(P[:, i].max())]
                            for i, n in enumerate(("v", "sv", "a", "z", "sz", "t", "st", "p_out"))}}
    for tag, tab in (("saved", P), ("typical", None)):
        if tab is None:
            tab = P.copy()
            tab[:, 0] = np.where(np.arange(len(P)) % 2, 1.0, 0.5)
            tab[:, 1], tab[:, 2], tab[:, 4], tab[:, 5], tab[:, 6] = 0.1, 2.0, 0.1, 0.3, 0.1
        m.dataset.wiener_like_nodes(tab)
        ctx.synchronize()
        ctx.profile(ctx.PROF_EVALS)
        r = m.dataset.wiener_like_nodes(tab)
        _, _, ne = ctx.profile_read(reset=True)
        lists = ctx.profile_lists(reset=True)
        ctx.profile(0)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            m.dataset.wiener_like_nodes(tab)
        ctx.synchronize()
        el = (time.perf_counter() - t0) / a.reps
        out[tag] = {"call_ms": el * 1e3, "evals_per_trial": ne / m.n_trials, "lists": lists,
                    "finite_nodes": int(np.isfinite(r).sum()),
                    "logp_sum": float(np.sum(r[np.isfinite(r)]))}
        print(json.dumps({tag: out[tag]}), flush=True)
    print(json.dumps(out), flush=True)
    _lib  # noqa: B018


if __name__ == "__main__":
    main()
