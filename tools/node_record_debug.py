"""Phase times of config 4's deferred records (node_record_spec) at the
generating parameters, from a WFPT_NODE_DEBUG library (tools/ab_variants.py
builds it as variant `nodedbg`): tables, evaluations, z settlement, t tree.

    WFPT_AMD_LIB=hddm_amd/lib/variants/libwfpt_nodedbg.so python tools/node_record_debug.py
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
    inter = dict(sv=0.1, sz=0.1, st=0.1)
    data, truth = gen_data(n_subj=200, n_trials=500, **inter)
    m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05)
    P = m.node_table().copy()
    for j, (s, c) in enumerate(m.node_keys):
        P[j, 0] = truth["v"][c][s]
        P[j, 2] = truth["a"][s]
        P[j, 5] = truth["t"][s]
        for k, col in (("sv", 1), ("sz", 4), ("st", 6)):
            P[j, col] = inter[k]
    ds = m.dataset
    for rep in range(5):
        _, terms = ds.wiener_like_nodes(P, trials=True, **m.wp)
    d = np.flatnonzero(terms < -1e3)
    print("records", d.size)
    if os.environ.get("ENTRY"):  # WFPT_NODE_DEBUG_ENTRY build
        for k in d:
            v = -terms[k]
            e = np.floor(v / 1e8 + 1e-9)
            print("  trial", int(k), "kernel entry -> record start %.2f us, record %.2f us" %
                  (e / 100, (v - e * 1e8) / 100))
        return
    for k in d:
        v = -terms[k]
        f = []
        for sc in (1e12, 1e8, 1e4, 1):
            q = np.floor(v / sc + 1e-9)
            f.append(q)
            v -= q * sc
        print("  trial", int(k), "us: tables %.2f evals %.2f zsettle %.2f ttree %.2f" %
              tuple(x / 100 for x in f))


if __name__ == "__main__":
    main()
