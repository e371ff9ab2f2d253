"""Per-wave latency of node_fast_kernel (config 4's level 0 of the batched node
call) at the generating parameters, from a WFPT_NODE_DEBUG_FAST library
(tools/ab_variants.py variant `fastdbg`): the slowest waves and their trials'
x - t range (tt = (x - t) / a^2 decides the series and its term count).

    WFPT_AMD_LIB=hddm_amd/lib/variants/libwfpt_fastdbg.so python tools/node_fast_debug.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from hddm_amd import _lib
    from hddm_amd.hierarchical import HDDM, gen_data
    _lib.context(0)
    for full in (True, False):
        inter = dict(sv=0.1, sz=0.1, st=0.1) if full else {}
        data, truth = gen_data(n_subj=200, n_trials=500, **inter)
        m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05)
        for name in ("truth", "start"):
            P = m.node_table().copy()
            if name == "truth":
                for j, (s, c) in enumerate(m.node_keys):
                    P[j, 0] = truth["v"][c][s]
                    P[j, 2] = truth["a"][s]
                    P[j, 5] = truth["t"][s]
                    for k, col in (("sv", 1), ("sz", 4), ("st", 6)):
                        P[j, col] = inter.get(k, 0.0)
            ds = m.dataset
            for _ in range(3):
                _, terms = ds.wiener_like_nodes(P, trials=True, **m.wp)
            order = np.asarray(ds.order()) if hasattr(ds, "order") else None
            w = np.flatnonzero(terms <= -1e6 + 1)
            us = (-terms[w] - 1e6) / 100
            print(f"full={full} {name}: waves {w.size} median {np.median(us):.2f} us, "
                  f"p90 {np.percentile(us, 90):.2f}, max {us.max():.2f}")
            x = data["rt"].to_numpy(dtype=np.float64)
            nd = data.groupby(["subj_idx", "cond"], sort=True).ngroup().to_numpy()
            top = list(np.argsort(-us)[:6]) + list(np.argsort(us)[:2])
            for k in top:
                t0 = int(w[k])
                q = P[nd[t0]]
                # the wave's 64 trials: the same node, consecutive in |rt| order
                same = np.flatnonzero(nd == nd[t0])
                ax = np.sort(np.abs(x[same]))
                r = np.searchsorted(ax, abs(x[t0]))
                lo, hi = ax[max(r - 2, 0)], ax[min(r + 62, ax.size - 1)]
                print(f"    {us[k]:6.2f} us  node {nd[t0]:3d} v {q[0]:+.2f} a {q[2]:.2f} t {q[5]:.3f}"
                      f" st {q[6]:.2f}  |x| ~[{lo:.3f}, {hi:.3f}]  tt_min {(lo - q[5] - q[6]/2) / q[2]**2:.4f}")


if __name__ == "__main__":
    main()
