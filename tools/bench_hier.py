"""Config-4 benchmark: hierarchical HDDM, 200 subjects x 500 trials,
depends_on={'v': 'cond'}, sampled on one MI355X (hddm_amd.hierarchical).

Prints one JSON line: sweeps/s (one sweep = every stochastic node updated
once, as one PyMC MCMC iteration), batched likelihood calls per sweep,
node-likelihood evaluations per second, and — for context — the reference's
CPU cost of the same node evaluations (oracle/_ref wiener_like on one
250-trial node x the node evaluations the sweep performed; the reference's
PyMC/kabuki sampler itself cannot run offline, so this is an estimate of its
likelihood time only, labelled as such).

    python tools/bench_hier.py [--subjects 200] [--trials 500] [--iters 200] [--full]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subjects", type=int, default=200)
    ap.add_argument("--trials", type=int, default=500)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--burn", type=int, default=20)
    ap.add_argument("--full", action="store_true", help="include sv, sz, st (full DDM)")
    ap.add_argument("--progress", type=int, default=0)
    ap.add_argument("--json", default=None, help="also write the JSON line here")
    ap.add_argument("--dt", type=float, default=1e-4,
                    help="RT grid of the data sampler (the reference's sampling_dt default "
                         "is 1e-4, hddm/likelihoods.py:30)")
    ap.add_argument("--seed", type=int, default=20261017)
    ap.add_argument("--sv", type=float, default=0.1, help="true sv with --full")
    ap.add_argument("--p-outlier", type=float, default=0.05,
                    help="the model's fixed p_outlier (HDDM's recommended 0.05; the data "
                         "carry no outliers, so 0 is the correctly specified model)")
    ap.add_argument("--slow-dump", default=None,
                    help="save the data and the parameter table of the slowest batched "
                         "likelihood call (npz) here")
    ap.add_argument("--no-pair", action="store_true",
                    help="one table per stepping-out probe (no paired two-table calls)")
    ap.add_argument("--watchdog", type=float, default=0.0,
                    help="dump every thread's stack and exit after this many seconds")
    a = ap.parse_args()
    if a.watchdog > 0:
        import faulthandler
        faulthandler.dump_traceback_later(a.watchdog, exit=True)
    from hddm_amd.hierarchical import HDDM, gen_data
    t0 = time.perf_counter()
    sv = sz = st = 0.0
    if a.full:
        sv, sz, st = a.sv, 0.1, 0.1
    data, truth = gen_data(n_subj=a.subjects, n_trials=a.trials, sv=sv, sz=sz, st=st,
                           seed=a.seed, dt=a.dt)
    t_gen = time.perf_counter() - t0
    if a.progress:
        print(f"data: {len(data)} trials in {t_gen:.1f}s", flush=True)
    m = HDDM(data, depends_on={"v": "cond"}, include=("sv", "sz", "st") if a.full else (),
             p_outlier=a.p_outlier, seed=1, paired_probes=not a.no_pair)
    if a.slow_dump:
        ds, inner, worst = m.dataset, m.dataset.wiener_like_nodes, [0.0]

        def timed(params, **kw):
            t = time.perf_counter()
            r = inner(params, **kw)
            el = time.perf_counter() - t
            if el > worst[0]:
                worst[0] = el
                np.savez(a.slow_dump, params=np.asarray(params), rt=data["rt"].to_numpy(),
                         response=data["response"].to_numpy(),
                         subj_idx=data["subj_idx"].to_numpy(),
                         cond=(data["cond"] == "c1").to_numpy(), seconds=el)
                if el > 1e-3:
                    print(f"slowest call so far: {el * 1e3:.2f} ms", flush=True)
            return r
        ds.wiener_like_nodes = timed
    m.sample(a.burn, progress=a.progress or None)  # burn-in (untimed)
    c0, s0 = m.likelihood_calls, m.likelihood_seconds
    m.call_stats = {}
    t0 = time.perf_counter()
    m.sample(a.iters, progress=a.progress or None)
    el = time.perf_counter() - t0
    calls = m.likelihood_calls - c0
    lik_s = m.likelihood_seconds - s0
    stats = m.gen_stats()
    node_evals = calls * m.n_nodes
    out = {
        "metric": "hierarchical HDDM sweeps/sec (200 subj x 500 trials, depends_on v:cond)",
        "value": a.iters / el, "unit": "sweeps/s",
        "config": {"subjects": a.subjects, "trials_per_subject": a.trials,
                   "nodes": m.n_nodes, "trials": m.n_trials, "full_ddm": a.full,
                   "iters": a.iters, "data_dt": a.dt, "seed": a.seed,
                   "p_outlier": a.p_outlier},
        "seconds": el, "extrapolated_sample_2000_s": 2000 * el / a.iters,
        "batched_likelihood_calls_per_sweep": calls / a.iters,
        "likelihood_fraction_of_time": lik_s / el,
        "node_evals_per_s": node_evals / el,
        "trial_evals_per_s": calls * m.n_trials / el,
        "data_generation_s": t_gen,
        "posterior": {k: stats[k]["mean"] for k in stats},
        "posterior_95": {k: [stats[k]["2.5q"], stats[k]["97.5q"]] for k in stats},
        "truth": {"a": float(np.mean(truth["a"])), "t": float(np.mean(truth["t"])),
                  "v(c0)": float(np.mean(truth["v"]["c0"])),
                  "v(c1)": float(np.mean(truth["v"]["c1"])), "sv": sv, "sz": sz, "st": st},
        "subject_recovery": {
            f: float(np.corrcoef(np.mean(m.trace_subj[f], axis=0)[::len(m.levels[f])],
                                 np.asarray(truth[f] if f != "v" else truth["v"]["c0"]))[0, 1])
            for f in ("a", "t", "v")},
        "burn": a.burn,
        "likelihood_calls_by_update": {k: {"calls": c, "us_per_call": t / c * 1e6}
                                       for k, (c, t) in sorted(m.call_stats.items())},
    }
    # the reference's CPU cost of the same node evaluations: the C restatement
    # of wiener_like (oracle/wfpt_oracle.c, calibrated 1.0x against the
    # reference's own kernels, profiles/r02/cpu_calibration.json), 1 thread
    import oracle
    node = data["rt"].to_numpy()[: a.trials // 2].copy()
    p = (1.0, sv, 2.0, 0.5, sz, 0.3, st)
    reps, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < 2.0:
        oracle.wiener_like(node, *p, 1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
        reps += 1
    per_node = (time.perf_counter() - t1) / reps
    out["cpu_port_estimate"] = {
        "per_node_call_s": per_node, "node_size": int(node.size), "kind": "port", "cores": 1,
        "likelihood_s_per_sweep": per_node * node_evals / a.iters,
        "note": "C restatement of the reference's wiener_like per node x the node evaluations "
                "of one sweep; excludes PyMC/kabuki overhead (not runnable offline)"}
    # device view of the node likelihood at the chain's final state: kernel
    # time per batched call (HIP events around the per-node kernels) and
    # pdf_sv evaluations per trial, for one slice update of each kind
    from hddm_amd import _lib
    ctx = _lib.context()
    dev = {}
    for kind in ("v", "a", "t", "sv", "sz", "st"):
        if kind in ("sv", "sz", "st") and kind not in m.include:
            continue
        over = {kind: m.subj[kind] if kind in m.FAMILIES else m.inter[kind]}
        ctx.profile(ctx.PROF_EVENTS)
        ctx.profile_read(reset=True)
        for _ in range(20):
            m.node_logp(over)
        k_ms, nl, _ = ctx.profile_read(reset=True)
        ctx.profile(ctx.PROF_EVALS)
        m.node_logp(over)
        _, _, ne = ctx.profile_read(reset=True)
        ctx.profile(0)
        dev[kind] = {"kernel_us": k_ms / max(nl, 1) * 1e3, "evals_per_trial": ne / m.n_trials}
    out["device_per_call"] = dev
    out["state"] = {k: float(v) for k, v in m.inter.items()}
    line = json.dumps(out)
    print(line, flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
