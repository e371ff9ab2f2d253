"""Per-call overhead of a resident wiener_like (run via gpurun): a 64-trial
dataset (one chunk: kernel time ~ a few us) timed through the Python binding
and through a bare ctypes loop, plus the 1M C3 call, to separate the
kernel, launch and host parts of a step.

    python tools/call_overhead.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(fn, reps=2000):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    import bench
    from hddm_amd import _lib, wfpt
    ctx = _lib.context(0)
    out = {}
    args, kn = bench.args_tuple(), bench.knobs_tuple()
    for n in (64, 1_000_000):
        x = bench.make_rts(n, 20261015)
        ds = wfpt.Dataset(x)
        out[f"python_us_n{n}"] = per_call(lambda: ds.wiener_like(*args, *kn),
                                          reps=2000 if n == 64 else 300)
        P = _lib.make_params(*args, kn[5])
        K = _lib.make_knobs(kn[0], kn[1], kn[2], kn[3], kn[4], kn[6])
        res = ctypes.c_double()
        f = _lib.wfpt_wiener_like
        h, dh, pP, pK, pr = ctx.handle, ds.handle, ctypes.byref(P), ctypes.byref(K), ctypes.byref(res)
        out[f"ctypes_us_n{n}"] = per_call(lambda: f(h, dh, pP, pK, pr),
                                          reps=2000 if n == 64 else 300)
        ctx.profile(1)
        ctx.profile_read(reset=True)
        for _ in range(100):
            ds.wiener_like(*args, *kn)
        ms, nl, _ = ctx.profile_read(reset=True)
        ctx.profile(0)
        out[f"kernel_us_n{n}"] = ms / nl * 1e3
        del ds
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
