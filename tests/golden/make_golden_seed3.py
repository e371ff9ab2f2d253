"""Fixture of the parameter region config 4's seed-3 chain visited (VERDICT r03
"missing" 4): the 400-node parameter table of the slowest batched likelihood
call of `tools/bench_hier.py --seed 3 --slow-dump` (v 7-22, sv 18, a 12-23,
sz 0.97, st 0.2, p_outlier 0.05) and a truth-like table, over 8 trials of each
of the 400 (subject x condition) nodes of that run's data (the 3 shortest and 2
longest |rt| of the node and 3 random ones).

Expected values come from the REFERENCE'S OWN kernels (oracle/_ref/ref_shim:
src/pdf.pxi + src/integrate.pxi compiled by oracle/build_ref.py): per trial
the addend log(full_pdf * (1 - p_outlier) + w_outlier * p_outlier) of
wfpt.pyx:66-74 with libm's log (math.log), at HDDM's knobs
(hddm/likelihoods.py:52-55: err 1e-4, n_st = n_sz = 2, simps_err 1e-3,
w_outlier 0.1).

Usage (build container): python tests/golden/make_golden_seed3.py gpurun_out/hier/slow_seed3.npz
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
KNOBS = dict(err=1e-4, n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3, w_outlier=0.1)


def main(src):
    import oracle
    R = oracle.load_ref()
    assert R is not None, "oracle/_ref not built (python oracle/build_ref.py)"
    d = np.load(src)
    rt = np.where(d["response"] == 0, -np.abs(d["rt"]), np.abs(d["rt"]))
    node = d["subj_idx"].astype(np.int64) * 2 + d["cond"].astype(np.int64)
    trap = d["params"]
    n_nodes = trap.shape[0]
    assert n_nodes == 400 and node.max() == n_nodes - 1
    rng = np.random.default_rng(3)
    xs, ids = [], []
    for j in range(n_nodes):
        idx = np.flatnonzero(node == j)
        o = idx[np.argsort(np.abs(rt[idx]), kind="stable")]
        pick = list(o[:3]) + list(o[-2:]) + list(rng.choice(o[3:-2], 3, replace=False))
        xs.extend(rt[pick])
        ids.extend([j] * len(pick))
    x = np.array(xs)
    ids = np.array(ids, dtype=np.int32)
    truth = np.tile([0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05], (n_nodes, 1))
    truth[1::2, 0] = 1.0  # v(c1)
    out = {"x": x, "node": ids, "params_trap": trap, "params_truth": truth,
           "knobs": np.array([KNOBS[k] for k in ("err", "n_st", "n_sz", "use_adaptive",
                                                  "simps_err", "w_outlier")])}
    for name in ("trap", "truth"):
        P = out["params_" + name]
        terms = np.empty(x.size)
        for i, (xi, j) in enumerate(zip(x, ids)):
            v, sv, a, z, sz, t, st, po = P[j]
            p = R.full_pdf(xi, v, sv, a, z, sz, t, st, KNOBS["err"], KNOBS["n_st"], KNOBS["n_sz"],
                           KNOBS["use_adaptive"], KNOBS["simps_err"])
            m = p * (1 - po) + KNOBS["w_outlier"] * po
            terms[i] = math.log(m) if m > 0 else -math.inf
        out["terms_" + name] = terms
        out["nodes_" + name] = np.array([math.fsum(terms[ids == j]) for j in range(n_nodes)])
    np.savez_compressed(os.path.join(HERE, "seed3_nodes.npz"), **out)
    print("wrote", os.path.join(HERE, "seed3_nodes.npz"), x.size, "trials")


if __name__ == "__main__":
    main(sys.argv[1])
