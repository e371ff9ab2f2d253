"""dmat_cdf_array timing on the GPU vs the reference extension (oracle/_ref)."""
import os, sys, time, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle
from hddm_amd import _lib, cdfdif_wrapper, wfpt
C = oracle.load_ref_cdfdif()
ctx = _lib.context(0)
for name, p in (("full", (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)), ("simple", (0.5, 0, 2.0, 0.5, 0, 0.3, 0))):
    np.random.seed(1)
    x = wfpt.gen_rts_from_cdf(*p, samples=200_000, dt=1e-3)
    x = x[np.abs(x) < 4.99][:100_000].copy()
    f = lambda: cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
    f()
    ctx.profile(1); ctx.profile_read(reset=True)
    t0 = time.perf_counter()
    for _ in range(5): y = f()
    el = (time.perf_counter() - t0) / 5
    ms, nl, _ = ctx.profile_read(reset=True); ctx.profile(0)
    s = x[:5000].copy()
    t0 = time.perf_counter(); r = C.dmat_cdf_array(s, *p, 0.05, 0.1); cpu = time.perf_counter() - t0
    print(json.dumps({"cdf": name, "n": x.size, "kernel_ms": ms / nl, "call_ms": el * 1e3,
                      "gpu_trials_per_s": x.size / el, "cpu_ref_trials_per_s": s.size / cpu,
                      "max_abs_diff_first5000": float(np.max(np.abs(y[:5000] - r)))}), flush=True)
