"""Staleness check of the batched node call's publication (config 4's call).

The per-node sums of `Dataset.wiener_like_nodes` reach a mapped host slot
that the host reads as soon as the call's completion word appears
(wfpt_kernels.hip: segment_publish_kernel). If any sum could land after the
word, the host would read the previous call's value for that node. This
alternates two parameter tables A, B over config 4's 200 x 500 dataset and
counts calls whose sums differ from the table's own sums (computed once,
each by a call whose result was read after a full stream synchronisation).

    python tests/node_publication_check.py [--full] [--reps N]

prints one JSON line {calls, stale_calls, stale_nodes, first}. The GPU test
runs it in-process on the shipped library (stale_calls must be 0) and in a
child process on the WFPT_PUB_DIAG build (hddm_amd/lib/libwfpt_amd_pubdiag.so,
whose non-last blocks store their sums only after the completion word): there
it must report stale calls, i.e. the check can see the failure it guards
against.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def tables(full):
    from hddm_amd.hierarchical import HDDM, gen_data
    inter = dict(sv=0.1, sz=0.1, st=0.1) if full else {}
    data, truth = gen_data(n_subj=200, n_trials=500, **inter)
    m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05)
    A = m.node_table()
    B = A.copy()
    for j, (s, c) in enumerate(m.node_keys):
        B[j, 0] = truth["v"][c][s]
        B[j, 2] = truth["a"][s]
        B[j, 5] = truth["t"][s]
    return m, A, B


def reference_sums(m, T):
    """T's sums from a call read only after a full synchronisation: the
    per-trial variant (wfpt_wiener_like_nodes_ex) copies the terms back with
    a blocking copy after the published sums, so by then every kernel of the
    call has completed; its sums are re-derived from nothing but T."""
    ds = m.dataset
    ds.wiener_like_nodes(T, **m.wp)
    ds.ctx.synchronize()
    r1, _ = ds.wiener_like_nodes(T, trials=True, **m.wp)
    ds.ctx.synchronize()
    r2, _ = ds.wiener_like_nodes(T, trials=True, **m.wp)
    ds.ctx.synchronize()
    return r1.copy(), r2.copy()


def run(full=True, reps=150):
    m, A, B = tables(full)
    ds = m.dataset
    ra1, ra2 = reference_sums(m, A)
    rb1, rb2 = reference_sums(m, B)
    stale_calls, stale_nodes, first = 0, 0, None
    for k in range(reps):
        T, ref = (A, ra2) if k % 2 == 0 else (B, rb2)
        r = ds.wiener_like_nodes(T, **m.wp)
        bad = np.flatnonzero(r != ref)
        if bad.size:
            stale_calls += 1
            stale_nodes += int(bad.size)
            if first is None:
                j = int(bad[0])
                other = rb2 if k % 2 == 0 else ra2
                first = {"call": k, "node": j, "got": float(r[j]), "expected": float(ref[j]),
                         "previous_tables_value": float(other[j]), "n_bad": int(bad.size)}
    ds.ctx.synchronize()
    return {"full": bool(full), "calls": reps, "n_nodes": int(A.shape[0]),
            "tables_differ": bool(not np.array_equal(ra2, rb2)),
            "sync_reads_agree": bool(np.array_equal(ra1, ra2) and np.array_equal(rb1, rb2)),
            "stale_calls": stale_calls, "stale_nodes": stale_nodes, "first": first,
            "lib": os.path.basename(os.environ.get("WFPT_AMD_LIB", "libwfpt_amd.so"))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--reps", type=int, default=150)
    a = ap.parse_args()
    print(json.dumps(run(a.full, a.reps)), flush=True)


if __name__ == "__main__":
    main()
