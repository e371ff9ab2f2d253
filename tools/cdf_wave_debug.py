"""Per deferred trial of tools/cdf_probe.py's full set: the wave kernel's
rounds (beyond-window series, 64 terms each) and elapsed time, from a
WFPT_CDF_DEBUG library (tools/ab_cdf.py builds it as variant `debug`).

    WFPT_AMD_LIB=hddm_amd/lib/variants/libwfpt_cdf_debug.so python tools/cdf_wave_debug.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from hddm_amd import cdfdif_wrapper, wfpt
    p = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    np.random.seed(20261015)
    x = wfpt.gen_rts_from_cdf(*p, samples=200_000, dt=1e-3)
    x = x[np.abs(x) < 4.99][:100_000].copy()
    for rep in range(3):
        y = np.asarray(cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1))
    d = np.flatnonzero(y < 0)
    raw = -y[d]  # the debug build stores the record in place of the value
    rounds = np.floor(raw / 1e12 + 1e-9)
    rest = raw - rounds * 1e12
    ser = np.floor(rest / 1e6 + 1e-9)
    ticks = rest - ser * 1e6
    t = np.abs(x[d])
    order = np.argsort(-ticks)
    print("deferred", d.size, "window", int((t <= 0.35 + 5e-11).sum()))
    print("us (100 MHz ticks / 100): median", np.median(ticks) / 100, "max", ticks.max() / 100)
    for k in order[:25]:
        print(f"  t {t[k]:.6f} x {x[d[k]]:+.6f} rounds {int(rounds[k])} us {ticks[k] / 100:.2f} window series us {ser[k] / 100:.2f}")


if __name__ == "__main__":
    main()
