"""Which trials of tools/cdf_probe.py's sets reach cdf_wave_kernel: the branch
of each trial (cdfdif.c:121-216: below / beyond / inside the Ter window) and the
distance to the window edge that sets its series length.

    python tools/cdf_defer_stats.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from hddm_amd import wfpt
    for name, p in (("full", (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)),
                    ("simple", (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0))):
        np.random.seed(20261015)
        x = wfpt.gen_rts_from_cdf(*p, samples=200_000, dt=1e-3)
        x = x[np.abs(x) < 4.99][:100_000].copy()
        t = np.abs(x)
        Ter, st = p[5], p[6] + 1e-10
        lower, upper = Ter - st / 2, Ter + st / 2
        live = (t - Ter) + st / 2 > 0.001
        beyond = live & (t > upper)
        window = live & ~(t > upper)
        tup = t[beyond] - upper
        tl = t[window] - lower
        print(name, "trials", t.size, "below", int((~live).sum()), "beyond", int(beyond.sum()),
              "window", int(window.sum()))
        for lim in (1e-6, 1e-4, 1e-3, 2e-3, 5e-3, 1e-2, 2.5e-2):
            print(f"   beyond with t_up < {lim:g}: {int((tup < lim).sum())}")
        if tl.size:
            print("   window tl quantiles", np.quantile(tl, [0, 0.01, 0.1, 0.5, 1]).round(5))
        print("   min t_up", tup.min() if tup.size else None, "distinct t near edge",
              np.unique(t[beyond & (t - upper < 0.01)])[:8])


if __name__ == "__main__":
    main()
