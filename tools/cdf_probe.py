"""DMAT CDF probe (cdfdif_wrapper.dmat_cdf_array over
cdfdif.c:59-221): full DDM and simple-DDM CDFs of 100k signed RTs per call on
one GPU (dmat_cdf_kernel + cdf_wave_kernel), for rocprofv3 passes
(tools/gpu_profile_cmd.sh) and the CDF row's numbers.

    python tools/cdf_probe.py [--reps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FULL = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
SIMPLE = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--trials", type=int, default=100_000)
    a = ap.parse_args()
    from hddm_amd import _lib, cdfdif_wrapper, wfpt
    ctx = _lib.context(0)
    for name, p in (("full", FULL), ("simple", SIMPLE)):
        np.random.seed(20261015)
        x = wfpt.gen_rts_from_cdf(*p, samples=2 * a.trials, dt=1e-3)
        x = x[np.abs(x) < 4.99][:a.trials].copy()  # |rt| < 1/(2 w_outlier) (pyx:20-21)
        cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            y = cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
        el = (time.perf_counter() - t0) / a.reps
        ctx.profile(ctx.PROF_EVENTS)
        ctx.profile_read(reset=True)
        for _ in range(a.reps):
            cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
        k_ms, nl, _ = ctx.profile_read(reset=True)
        ctx.profile(0)
        print(json.dumps({"row": f"dmat_cdf_array {name}", "trials": x.size,
                          "call_ms": el * 1e3, "kernel_ms": k_ms / max(nl, 1),
                          "trials_per_s": x.size / el, "mean_cdf": float(np.mean(y))}),
              flush=True)


if __name__ == "__main__":
    main()
