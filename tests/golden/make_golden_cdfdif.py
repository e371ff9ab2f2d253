"""Generate tests/golden/cdfdif.npz (run in the build container).

Expected values come from the REFERENCE'S OWN `cdfdif_wrapper` extension
(src/cdfdif_wrapper.pyx + src/cdfdif.c compiled where they lie by
oracle/build_ref.build_cdfdif into oracle/_ref/), never from this repository.

Rows cover every branch of cdfdif (src/cdfdif.c): t below the Ter window
(:213-216), inside it with |xi| > eps (:153-184) and with every drift node ~ 0
(v = sv = 0, :185-207), beyond it (:121-149); both boundaries; x = 0; the
wrapper's sz = st = 0 substitution (cdfdif_wrapper.pyx:38-41, HDDM's default
model); the outlier mixture (:11-12, :51).

Usage: python tests/golden/make_golden_cdfdif.py [--reference /root/reference]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

M = 64  # trials per parameter row


def rows(rng):
    out = []
    # HDDM defaults: simple DDM (sv = sz = st = 0), outlier mixture on / off
    for v, a, z, t in [(0.5, 2.0, 0.5, 0.3), (-1.0, 1.2, 0.45, 0.25), (2.5, 0.8, 0.6, 0.4)]:
        out.append([v, 0, a, z, 0, t, 0, 0.0, 0.1])
        out.append([v, 0, a, z, 0, t, 0, 0.05, 0.1])
    # pinned full DDM (test_models.py:18,71)
    out.append([0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.0, 0.1])
    out.append([0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05, 0.1])
    # drift nodes ~ 0: v = 0 (sv = 0) -> the |gk| <= eps series (cdfdif.c:185-207)
    out.append([0.0, 0, 1.5, 0.5, 0.2, 0.3, 0.2, 0.0, 0.1])
    out.append([0.0, 0, 1.5, 0.5, 0.0, 0.3, 0.0, 0.0, 0.1])
    # wide Ter windows (many trials inside the window branch)
    out.append([1.0, 0.5, 1.5, 0.5, 0.3, 0.45, 0.35, 0.0, 0.1])
    out.append([-0.7, 1.0, 1.8, 0.4, 0.2, 0.35, 0.3, 0.1, 0.12])
    # random rows over hddm/generate.py:38-46 ranges
    for _ in range(12):
        sv = rng.choice([0.0, rng.uniform(0, 2.5)])
        sz = rng.choice([0.0, rng.uniform(0, 0.4)])
        st = rng.choice([0.0, rng.uniform(0, 0.35)])
        out.append([rng.uniform(-4, 4), sv, rng.uniform(0.5, 2.0), rng.uniform(0.4, 0.6), sz,
                    rng.uniform(0.2, 0.5), st, rng.choice([0.0, 0.05]), 0.1])
    return np.array(out, dtype=np.float64)


def x_vector(rng, p):
    t, st = p[5], p[6]
    lo, hi = t - st / 2, t + st / 2
    mag = np.concatenate([
        [0.0, max(lo - 0.01, 0.0), lo + 0.0005, lo + 0.002, hi, hi + 1e-4, hi + 0.01],
        rng.uniform(max(lo - 0.05, 0.0), hi + 0.05, 17),   # around / inside the window
        rng.uniform(hi, t + 3.0, M - 24),                  # the bulk of real RTs
    ])
    sign = rng.choice([-1.0, 1.0], mag.size)
    return sign * mag


def main(reference):
    from oracle import build_ref
    import oracle
    build_ref.build_cdfdif(reference, quiet=True)
    C = oracle.load_ref_cdfdif()
    assert C is not None, "oracle/_ref/cdfdif_wrapper did not build"
    rng = np.random.default_rng(20261018)
    P = rows(rng)
    X = np.array([x_vector(rng, p) for p in P])
    Y = np.array([C.dmat_cdf_array(x, *p) for x, p in zip(X, P)])
    np.savez_compressed(os.path.join(HERE, "cdfdif.npz"), params=P, x=X, y=Y,
                        keys=np.array(["v", "sv", "a", "z", "sz", "t", "st", "p_outlier",
                                       "w_outlier"]))
    print("wrote", os.path.join(HERE, "cdfdif.npz"), P.shape, X.shape)
    # random rows for the GPU tests (the reference never travels to the GPU box):
    # tests/test_cdfdif.py::test_random_cdfdif_vs_reference and the stochastic hook
    rng = np.random.default_rng(77)
    RP, RX, RY = [], [], []
    for _ in range(10):
        p = [rng.uniform(-3, 3), rng.choice([0.0, rng.uniform(0, 2)]), rng.uniform(0.6, 2.0),
             rng.uniform(0.4, 0.6), rng.choice([0.0, rng.uniform(0.05, 0.3)]),
             rng.uniform(0.2, 0.45), rng.choice([0.0, rng.uniform(0.05, 0.3)]),
             rng.choice([0.0, 0.05]), 0.1]
        x = rng.choice([-1.0, 1.0], 2000) * (p[5] - p[6] / 2 + rng.gamma(1.5, 0.5, 2000))
        x = np.clip(x, -4.9, 4.9)
        RP.append(p)
        RX.append(x)
        RY.append(C.dmat_cdf_array(x, *p))
    hook_p = np.array([0.7, 0.2, 1.8, 0.5, 0.1, 0.3, 0.1, 0.05, 0.1])
    hook_x = np.linspace(-3, 3, 101)
    np.savez_compressed(os.path.join(HERE, "cdfdif_random.npz"), params=np.array(RP),
                        x=np.array(RX), y=np.array(RY), hook_params=hook_p, hook_x=hook_x,
                        hook_y=C.dmat_cdf_array(hook_x, *hook_p))
    print("wrote", os.path.join(HERE, "cdfdif_random.npz"))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    main(ap.parse_args().reference)
