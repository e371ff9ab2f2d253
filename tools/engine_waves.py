"""Per-wave clocks of engine_kernel on the stress sets (diagnostic build with
WFPT_PHASE_TIMING: `python -m hddm_amd.build --variants` makes
hddm_amd/lib/libwfpt_amd_phase.so; run with WFPT_AMD_LIB pointing at it).

For each engine set: the launch's span, the distribution of wave durations
of whole chunks and of split units, and the slowest waves with their chunk,
z-walk / t-task counts and phase cycles (level 0, tables, z rounds, t rounds,
tests + epilogue).

    WFPT_AMD_LIB=hddm_amd/lib/libwfpt_amd_phase.so python tools/engine_waves.py
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

K_PHASE = 16384  # wfpt_internal.h kPhaseWaves


def main():
    from hddm_amd import _lib, wfpt
    from stress_probe import KN, stress_sets
    ctx = _lib.context(0)
    sets = stress_sets(wfpt)
    buf = (ctypes.c_uint64 * (K_PHASE * 8))()
    for k in (0, 1, 3):
        x, p = sets[k]
        ds = wfpt.Dataset(x)
        for _ in range(3):
            ds.wiener_like(*p, *KN)
        ctx.synchronize()
        _lib.check(_lib.wfpt_debug_waves(ctx.handle, buf, K_PHASE))
        r = np.frombuffer(buf, dtype=np.uint64).reshape(K_PHASE, 8).astype(np.int64)
        end = r[:, 1].max()
        live = (r[:, 0] > 0) & (r[:, 0] > end - 25_000)  # this call (100 MHz clock: 250 us)
        t0 = r[live, 0].min()
        idx = np.flatnonzero(live)
        dur = (r[idx, 1] - r[idx, 0]) / 100.0  # us
        start = (r[idx, 0] - t0) / 100.0
        split = idx >= K_PHASE // 2
        out = {"set": k, "span_us": float((end - t0) / 100.0), "waves": int(idx.size),
               "split_units": int(split.sum())}
        for name, m in (("chunks", ~split), ("units", split)):
            if m.any():
                d = dur[m]
                out[name] = {"n": int(m.sum()), "median_us": float(np.median(d)),
                             "p90_us": float(np.quantile(d, 0.9)), "max_us": float(d.max()),
                             "last_end_us": float((start[m] + d).max())}
        top = np.argsort(-(start + dur))[:8]
        out["slowest"] = [{"rec": int(idx[j]), "start_us": float(start[j]), "dur_us": float(dur[j]),
                           "nz": int(r[idx[j], 7] & 0xffffffff), "nt": int(r[idx[j], 7] >> 32),
                           "phase_kcyc": [int(v // 1000) for v in r[idx[j], 2:7]]} for j in top]
        # whole-chunk durations by position in the dataset (deciles of chunk id)
        ch = idx[~split]
        if ch.size:
            dec = np.array_split(np.argsort(ch), 10)
            out["chunk_decile_median_us"] = [round(float(np.median(dur[~split][d])), 1) for d in dec]
        print(json.dumps(out), flush=True)
        del ds


if __name__ == "__main__":
    main()
