"""Config 2 probe: simple DDM (v, a, t) Navarro-Fuss pdf over 10M resident
trials on one GPU (BASELINE.json configs[1]), HDDM knobs, p_outlier .05;
K timed wiener_like calls plus HIP-event kernel time of the level-0 pass
(fast_kernel<kDirect>). For rocprofv3 passes (tools/gpu_profile_cmd.sh).

    python tools/c2_probe.py [--reps 20] [--trials 10000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIMPLE = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)
KN = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--trials", type=int, default=10_000_000)
    a = ap.parse_args()
    from hddm_amd import _lib, wfpt
    ctx = _lib.context(0)
    np.random.seed(20261015)
    x = wfpt.gen_rts_from_cdf(*SIMPLE, samples=a.trials, dt=1e-3)
    ds = wfpt.Dataset(x)
    for _ in range(3):
        v = ds.wiener_like(*SIMPLE, *KN)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        v = ds.wiener_like(*SIMPLE, *KN)
    ctx.synchronize()
    el = (time.perf_counter() - t0) / a.reps
    ctx.profile(ctx.PROF_EVENTS)
    ctx.profile_read(reset=True)
    for _ in range(a.reps):
        ds.wiener_like(*SIMPLE, *KN)
    k_ms, nl, _ = ctx.profile_read(reset=True)
    ctx.profile(0)
    print(json.dumps({"row": "C2 simple DDM resident", "trials": a.trials, "call_ms": el * 1e3,
                      "kernel_ms": k_ms / max(nl, 1), "trials_per_s": a.trials / el,
                      "logp": v}), flush=True)


if __name__ == "__main__":
    main()
