"""Per-dataset timing of the stress set and C3 (run under rocprofv3 --kernel-trace
on the GPU box to attribute time to fast / deferred-trial / finalize kernels).

Stress set: 4 x 250k trials, parameters drawn from hddm/generate.py:38-46 ranges
(seed 20261016), RTs sampled from each model.

    python tools/stress_probe.py [--reps 10] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KN = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
FULL = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)


def stress_sets(wfpt, n=250_000):
    rng = np.random.default_rng(20261016)
    np.random.seed(20261016)
    out = []
    for _ in range(4):
        p = (rng.uniform(-4, 4), rng.uniform(0, 2.5), rng.uniform(0.5, 2), rng.uniform(0.4, 0.6),
             rng.uniform(0, 0.4), rng.uniform(0.2, 0.5), rng.uniform(0, 0.35))
        out.append((wfpt.gen_rts_from_cdf(*p, samples=n, dt=1e-3), p))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--engine-only", action="store_true",
                    help="only the stress sets whose steady-state call runs engine_kernel, no C3 "
                         "set (the PMC passes behind profiles/traffic_stress.json: every "
                         "engine launch of the run is one of bench.py's engine sets)")
    a = ap.parse_args()
    from hddm_amd import _lib, wfpt
    ctx = _lib.context(0)
    rows = []
    sets = stress_sets(wfpt)
    if a.engine_only:
        # bench.py's stress line: sets 0, 1, 3 take the engine, set 2 the lean
        # pass (checked below: each kept set's calls run the engine)
        sets = [sets[k] for k in (0, 1, 3)]
    else:
        np.random.seed(20261015)
        sets.append((wfpt.gen_rts_from_cdf(*FULL, samples=1_000_000, dt=1e-3), FULL))
    for x, p in sets:
        ds = wfpt.Dataset(x)
        ds.wiener_like(*p, *KN)
        if a.engine_only:
            assert ctx.last_path() & _lib.PATH_ENGINE, "an --engine-only set took another path"
        ctx.profile(ctx.PROF_EVALS)
        ds.wiener_like(*p, *KN)
        _, _, ne = ctx.profile_read(reset=True)
        lists = ctx.profile_lists(reset=True)
        ctx.profile(0)
        for _ in range(3):
            ds.wiener_like(*p, *KN)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ds.wiener_like(*p, *KN)
        ctx.synchronize()
        el = (time.perf_counter() - t0) / a.reps
        ctx.profile(ctx.PROF_EVENTS)
        ctx.profile_read(reset=True)
        for _ in range(a.reps):
            ds.wiener_like(*p, *KN)
        k_ms, nl, _ = ctx.profile_read(reset=True)
        ctx.profile(0)
        ctx.profile_lists(reset=True)
        for _ in range(a.reps):
            ds.wiener_like(*p, *KN)
        ph = ctx.profile_lists(reset=True).get("phase_kcycles", [])
        lists["phase_kcycles_per_call"] = [round(v / a.reps) for v in ph]
        rows.append({"params": [round(float(v), 4) for v in p], "trials": x.size,
                     "evals_per_trial": ne / x.size, "call_ms": el * 1e3,
                     "fast_kernel_ms": k_ms / max(nl, 1), "lists": lists})
        print(json.dumps(rows[-1]), flush=True)
        del ds
    st = rows[:4]
    tot = sum(r["call_ms"] for r in st)
    print(json.dumps({"stress_call_ms_per_1M": tot, "stress_trials_per_s": 1e6 / (tot / 1e3),
                      "stress_fast_ms_per_1M": sum(r["fast_kernel_ms"] for r in st)}), flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
