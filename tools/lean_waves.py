"""Per-wave clocks of lean_kernel on bench.py's C3 call (diagnostic build with
WFPT_PHASE_TIMING: `python tools/ab_variants.py build --names phase`, run with
WFPT_AMD_LIB=hddm_amd/lib/variants/libwfpt_phase.so).

Prints the launch's span, the wave-duration distribution by position in the
dataset (deciles of the chunk id: |rt| ascending within each boundary), the
number of waves in flight over time (the dispatch rounds and the tail) and
the per-XCD end times.

    WFPT_AMD_LIB=hddm_amd/lib/variants/libwfpt_phase.so python tools/lean_waves.py
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_PHASE = 16384  # wfpt_internal.h kPhaseWaves


def main():
    import bench
    from hddm_amd import _lib, wfpt
    ctx = _lib.context(0)
    x = bench.make_rts(1_000_000, 20261015)
    ds = wfpt.Dataset(x)
    args, kn = bench.args_tuple(), bench.knobs_tuple()
    for _ in range(3):
        ds.wiener_like(*args, *kn)
    ctx.synchronize()
    assert ctx.last_path() & _lib.PATH_LEAN
    buf = (ctypes.c_uint64 * (K_PHASE * 8))()
    _lib.check(_lib.wfpt_debug_waves(ctx.handle, buf, K_PHASE))
    r = np.frombuffer(buf, dtype=np.uint64).reshape(K_PHASE, 8).astype(np.int64)
    nw = (len(ds) + 63) // 64
    r = r[:nw]
    t0 = r[:, 0].min()
    st = (r[:, 0] - t0) / 100.0  # us (100 MHz)
    en = (r[:, 1] - t0) / 100.0
    du = en - st
    xcc = r[:, 3] & 0xf
    out = {"waves": int(nw), "span_us": float(en.max()),
           "dur_median_us": float(np.median(du)), "dur_p90_us": float(np.quantile(du, 0.9)),
           "dur_max_us": float(du.max())}
    dec = np.array_split(np.arange(nw), 10)
    out["dur_median_by_decile_us"] = [round(float(np.median(du[d])), 1) for d in dec]
    out["start_median_by_decile_us"] = [round(float(np.median(st[d])), 1) for d in dec]
    # waves in flight over time
    grid = np.arange(0.0, en.max() + 1.0, 1.0)
    live = np.array([int(((st <= t) & (en > t)).sum()) for t in grid])
    peak = int(live.max())
    out["in_flight_peak"] = peak
    out["in_flight_every_5us"] = [int(v) for v in live[::5]]
    half = np.flatnonzero(live >= peak / 2)
    out["time_below_half_peak_at_end_us"] = float(en.max() - grid[half[-1]]) if half.size else None
    out["mean_in_flight_over_span"] = float(live.mean())
    out["xcc_last_end_us"] = {int(k): round(float(en[xcc == k].max()), 1) for k in np.unique(xcc)}
    out["xcc_waves"] = {int(k): int((xcc == k).sum()) for k in np.unique(xcc)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
