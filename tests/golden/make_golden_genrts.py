"""Generate tests/golden/gen_rts.npz (run in the build container).

gen_rts_from_cdf (src/wfpt.pyx:323-354) is deterministic for a fixed NumPy
global seed: a density grid from the reference's own full_pdf (t = st = 0,
err = 1e-4, full_pdf's defaults n_st = n_sz = 2, adaptive, simps_err = 1e-3),
a sequential running sum (wfpt.pyx:333-335), normalisation by the last value
(:337), np.random.rand(samples) then, if st != 0, np.random.rand(samples) for
the delays (:340-343), np.searchsorted per sample (:345) and the
non-decision-time shift (:347-350). The grid densities come from the
REFERENCE's kernels (oracle/_ref, compiled from /root/reference/src by
oracle/build_ref.py); the ~20 lines of that loop are restated here because
wfpt.pyx itself cannot be imported (its line 16 imports hddm -> PyMC/kabuki).

Usage: python tests/golden/make_golden_genrts.py [--reference /root/reference]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# (v, sv, a, z, sz, t, st), samples, cdf_lb, cdf_ub, dt, seed
CASES = [
    ((0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1), 20000, -6.0, 6.0, 1e-3, 20261015),  # bench model
    ((0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0), 5000, -6.0, 6.0, 1e-2, 20261016),   # simple, default dt
    ((-1.2, 0.8, 1.4, 0.45, 0.25, 0.25, 0.0), 5000, -5.0, 5.0, 1e-3, 7),      # sz only, no st
    ((1.7, 2.0, 0.61, 0.54, 0.21, 0.36, 0.2), 5000, -6.0, 6.0, 1e-3, 11),     # stress set 4
]


def reference_gen_rts(R, v, sv, a, z, sz, t, st, samples, cdf_lb, cdf_ub, dt):
    x = np.arange(cdf_lb, cdf_ub, dt)
    size = x.shape[0]
    pdf = R.pdf_array(x[1:].copy(), v, sv, a, z, sz, 0.0, 0.0, 1e-4)  # full_pdf per point
    l_cdf = np.empty(size, dtype=np.double)
    l_cdf[0] = 0
    for i in range(1, size):
        l_cdf[i] = l_cdf[i - 1] + pdf[i - 1]
    l_cdf /= l_cdf[size - 1]
    f = np.random.rand(samples)
    if st != 0:
        delay = np.random.rand(samples) * st + (t - st / 2.)
    rts = np.empty(samples, dtype=np.double)
    for i in range(samples):
        idx = np.searchsorted(l_cdf, f[i])
        rt = x[idx]
        rts[i] = rt + np.sign(rt) * (t if st == 0 else delay[i])
    return rts


def main(reference):
    from oracle import build_ref
    import oracle
    build_ref.build(reference, quiet=True)
    R = oracle.load_ref()
    assert R is not None, "oracle/_ref did not build"
    out = {}
    for k, (p, n, lb, ub, dt, seed) in enumerate(CASES):
        np.random.seed(seed)
        out[f"rts_{k}"] = reference_gen_rts(R, *p, n, lb, ub, dt)
        out[f"args_{k}"] = np.array([*p, n, lb, ub, dt, seed], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "gen_rts.npz"), **out)
    print("wrote", os.path.join(HERE, "gen_rts.npz"), len(CASES), "cases")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    main(ap.parse_args().reference)
