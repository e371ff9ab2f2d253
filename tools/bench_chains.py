"""Config 4 with several chains: HDDMChains(200 subj x 500 trials,
depends_on v:cond, chains=C).sample(2000) on one MI355X, every slice
evaluation of every chain in one multi-table launch (hddm_amd.hierarchical).

    python tools/bench_chains.py [--chains 8] [--iters 2000] [--full] [--no-pair]

Prints one JSON line: seconds for the lockstep sample, chain-sweeps/s,
batched calls per sweep, likelihood us per call and per chain-call, R-hat.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=8)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--burn", type=int, default=20)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--no-pair", action="store_true")
    ap.add_argument("--seed", type=int, default=20261017)
    a = ap.parse_args()
    from hddm_amd.hierarchical import HDDMChains, gen_data
    inter = dict(sv=0.1, sz=0.1, st=0.1) if a.full else {}
    data, truth = gen_data(n_subj=200, n_trials=500, seed=a.seed, dt=1e-4, **inter)
    m = HDDMChains(data, chains=a.chains, depends_on={"v": "cond"}, include=tuple(inter),
                   p_outlier=0.05, seed=1, paired_probes=not a.no_pair)
    m.sample(a.burn)
    c0, s0 = m.likelihood_calls, m.likelihood_seconds
    d0, tb0 = getattr(m, "device_call_seconds", 0.0), getattr(m, "tables_evaluated", 0)
    m.call_stats = {}
    t0 = time.perf_counter()
    m.sample(a.iters)
    el = time.perf_counter() - t0
    calls = m.likelihood_calls - c0
    lik = m.likelihood_seconds - s0
    st = m.gen_stats()
    tables = m.tables_evaluated - tb0
    dev = m.device_call_seconds - d0
    out = {"workload": "C4 x %d chains: HDDMChains 200 subj x 500 trials, depends_on v:cond, "
                       "p_outlier .05, sample(%d) after %d burn-in, data dt 1e-4"
                       % (a.chains, a.iters, a.burn),
           "full_ddm": a.full, "chains": a.chains, "paired_probes": not a.no_pair,
           "seconds": el, "chain_sweeps_per_s": a.chains * a.iters / el,
           "batched_calls_per_sweep": calls / a.iters,
           "tables_per_call": tables / max(calls, 1),
           "likelihood_us_per_call": lik / max(calls, 1) * 1e6,
           "likelihood_us_per_table": lik / max(tables, 1) * 1e6,
           "likelihood_fraction_of_time": lik / el,
           "binding_call_us_per_call": dev / max(calls, 1) * 1e6,
           "binding_call_us_per_table": dev / max(tables, 1) * 1e6,
           "calls_by_update": {k: {"calls": c, "us_per_call": t / c * 1e6}
                               for k, (c, t) in sorted(m.call_stats.items())},
           "posterior": {k: st[k]["mean"] for k in st},
           "rhat": {k: st[k]["rhat"] for k in st}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
