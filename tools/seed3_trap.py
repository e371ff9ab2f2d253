"""Config 4's seed-3 chain (tools/bench_hier.py --seed 3) kept its samples at
a 15.4, v 9.0 / 17.0, sv 16.9, sz 0.96, st 0.22 (truth: a 2.0, v 0.5 / 1.0,
sv 0.1, sz 0.1, st 0.1). Is that a likelihood error or a sampler trap?

The likelihood at those parameters is pinned per trial against the reference
(tests/test_parity_summing.py::test_seed3_burn_in_region_per_trial). This tool
evaluates the data log-likelihood (the 400-node wiener_like sum the sampler
sees, HDDM's knobs, p_outlier 0.05) on the CPU with the oracle (the
reference's algorithm, bit-exact) along
  * the joint line from the trapped node table to a truth-like one, and
  * one-coordinate moves from the trapped point (the moves a coordinate-wise
    slice sampler makes: sv, sz, st alone, all subjects' a alone, v alone),
and prints a JSON summary.

    python tools/seed3_trap.py tools/scratch/slow_seed3.npz
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KN = (1e-4, 2, 2, 1, 1e-3)


def main(path):
    import oracle
    d = np.load(path)
    rt = np.where(d["response"] == 0, -np.abs(d["rt"]), np.abs(d["rt"]))
    node = d["subj_idx"].astype(np.int64) * 2 + d["cond"].astype(np.int64)
    trap = d["params"].copy()
    groups = [np.ascontiguousarray(rt[node == j]) for j in range(trap.shape[0])]
    nth = len(os.sched_getaffinity(0))

    def loglik(P):
        tot = 0.0
        for j, x in enumerate(groups):
            v, sv, a, z, sz, t, st, po = P[j]
            lp = oracle.pdf_array(x, v, sv, a, z, sz, t, st, KN[0], 1, KN[1], KN[2], KN[3],
                                  KN[4], po, 0.1, n_threads=nth)
            tot += float(np.sum(lp))
        return tot

    truth = trap.copy()
    truth[:, 0] = np.where(np.arange(len(trap)) % 2, 1.0, 0.5)
    truth[:, 1], truth[:, 2], truth[:, 4], truth[:, 5], truth[:, 6] = 0.1, 2.0, 0.1, 0.3, 0.1
    out = {"trap": loglik(trap), "truth_like": loglik(truth)}
    lam = np.linspace(0.0, 1.0, 11)
    out["joint_line"] = [[float(l), loglik((1 - l) * trap + l * truth)] for l in lam]
    coord = {}
    for name, col, vals in (("sv", 1, [18.0, 12.0, 6.0, 2.0, 0.5, 0.1]),
                            ("sz", 4, [0.966, 0.8, 0.5, 0.2, 0.1]),
                            ("st", 6, [0.205, 0.15, 0.1, 0.05]),
                            ("a_scale", 2, [1.0, 0.8, 0.6, 0.4, 0.2, 0.13]),
                            ("v_scale", 0, [1.0, 0.8, 0.5, 0.2, 0.07])):
        rows = []
        for val in vals:
            P = trap.copy()
            if name.endswith("_scale"):
                P[:, col] = trap[:, col] * val
            else:
                P[:, col] = val
            rows.append([val, loglik(P)])
        coord[name] = rows
    out["one_coordinate"] = coord
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
