"""Per-row measurement of SURVEY.md §8 on one MI355X (run via gpurun).

One JSON line per row: GPU throughput (kernel time from HIP events on the
library's stream, and wall time of the whole call), the reference CPU path on
a bounded sample of the same inputs (oracle/_ref: the reference's own
kernels / cdfdif extension, 1 thread), and their ratio. bench.py stays the
headline (config 3); this file covers the other configs and the §8(f) rows.

    python tools/bench_rows.py [--quick] > gpurun_out/rows.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KN = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)  # HDDM knobs + p_outlier .05 (base.py:712-716)
SIMPLE = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)
FULL = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)


def timed(fn, min_s=0.5, min_reps=3):
    fn()
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if reps >= min_reps and el >= min_s:
            return el / reps


def gpu_kernel_ms(ctx, fn, reps=10):
    fn()
    ctx.profile(1)
    ctx.profile_read(reset=True)
    for _ in range(reps):
        fn()
    ms, nl, _ = ctx.profile_read(reset=True)
    ctx.profile(0)
    return ms / max(nl, 1)


def cpu_rate(fn, n, budget):
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget:
            return n * reps / el


def threads():
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else len(os.sched_getaffinity(0))


def emit(row):
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-seconds", type=float, default=2.0)
    a = ap.parse_args()
    import oracle
    from hddm_amd import _lib, cdfdif_wrapper, wfpt
    # CPU baselines: the C restatement of the reference's kernels (kind "port",
    # oracle/wfpt_oracle.c; calibrated 0.87-1.01x against the reference's own
    # compiled kernels in the build container, profiles/r02/cpu_calibration.json),
    # 1 thread. The reference's compiled cdfdif exists only in the build
    # container (oracle/_ref never travels); on the GPU box the CDF row's CPU
    # baseline is the C restatement oracle/cdfdif_oracle.c (bit-exact to the
    # reference's fixtures, tests/test_cdfdif.py).
    R = oracle
    C = oracle.load_ref_cdfdif()
    ctx = _lib.context(0)
    np.random.seed(20261015)
    x_full = wfpt.gen_rts_from_cdf(*FULL, samples=1_000_000, dt=1e-3)
    np.random.seed(20261015)
    x_simple = wfpt.gen_rts_from_cdf(*SIMPLE, samples=1_000_000, dt=1e-3)
    cs = a.cpu_seconds

    # C1: simple DDM, 10k trials, pdf_array (host array in, per-trial log density out)
    x = x_simple[:10_000].copy()
    wall = timed(lambda: wfpt.pdf_array(x, *SIMPLE, 1e-4, 1))
    ref = cpu_rate(lambda: R.pdf_array(x, *SIMPLE, 1e-4, 1), x.size, cs) if R else None
    emit({"row": "C1 pdf_array simple 10k (host in/out, PCIe incl.)", "trials": x.size,
          "gpu_call_us": wall * 1e6, "gpu_trials_per_s": x.size / wall,
          "cpu_port_trials_per_s": ref})

    # C2: simple DDM, 10M resident trials, wiener_like
    x10 = np.tile(x_simple, 10)
    ds = wfpt.Dataset(x10)
    k = gpu_kernel_ms(ctx, lambda: ds.wiener_like(*SIMPLE, *KN))
    wall = timed(lambda: ds.wiener_like(*SIMPLE, *KN))
    s = x_simple[:200_000].copy()
    ref = cpu_rate(lambda: R.wiener_like(s, *SIMPLE, *KN), s.size, cs) if R else None
    emit({"row": "C2 wiener_like simple 10M resident", "trials": x10.size, "kernel_ms": k,
          "call_ms": wall * 1e3, "gpu_trials_per_s": x10.size / wall,
          "cpu_port_trials_per_s": ref})
    del ds

    # C3: full DDM, 1M resident (the headline; also PCIe-inclusive host path)
    ds = wfpt.Dataset(x_full)
    k = gpu_kernel_ms(ctx, lambda: ds.wiener_like(*FULL, *KN))
    wall = timed(lambda: ds.wiener_like(*FULL, *KN))
    wall_h = timed(lambda: wfpt.wiener_like(x_full, *FULL, *KN))
    s = x_full[:20_000].copy()
    ref = cpu_rate(lambda: R.wiener_like(s, *FULL, *KN), s.size, cs) if R else None
    emit({"row": "C3 wiener_like full DDM 1M", "trials": x_full.size, "kernel_ms": k,
          "call_ms_resident": wall * 1e3, "call_ms_host_array": wall_h * 1e3,
          "gpu_trials_per_s": x_full.size / wall,
          "gpu_trials_per_s_pcie_incl": x_full.size / wall_h, "cpu_port_trials_per_s": ref})
    del ds

    # stress: random parameter sets (hddm/generate.py:38-46 ranges), 4 x 250k
    rng = np.random.default_rng(20261016)
    np.random.seed(20261016)
    sets = []
    for _ in range(4):
        p = (rng.uniform(-4, 4), rng.uniform(0, 2.5), rng.uniform(0.5, 2), rng.uniform(0.4, 0.6),
             rng.uniform(0, 0.4), rng.uniform(0.2, 0.5), rng.uniform(0, 0.35))
        sets.append((wfpt.Dataset(wfpt.gen_rts_from_cdf(*p, samples=250_000, dt=1e-3)), p))
    k = sum(gpu_kernel_ms(ctx, lambda d=d, p=p: d.wiener_like(*p, *KN), reps=5) for d, p in sets)
    wall = sum(timed(lambda d=d, p=p: d.wiener_like(*p, *KN)) for d, p in sets)
    emit({"row": "stress (random params, full DDM) 4 x 250k", "trials": 1_000_000,
          "fast_kernel_ms_per_1M": k, "call_ms_per_1M": wall * 1e3,
          "gpu_trials_per_s": 1e6 / wall})
    del sets

    # (f)1: batched per-node likelihood, 400 nodes x 250 trials (config 4 call)
    n_nodes = 400
    node = np.repeat(np.arange(n_nodes), 250)
    xn = x_simple[: node.size].copy()
    dsn = wfpt.Dataset(xn, node_id=node, n_nodes=n_nodes)
    P = np.tile(np.array([*SIMPLE, 0.05]), (n_nodes, 1))
    P[:, 0] += np.linspace(-0.2, 0.2, n_nodes)
    k = gpu_kernel_ms(ctx, lambda: dsn.wiener_like_nodes(P))
    wall = timed(lambda: dsn.wiener_like_nodes(P))
    xs = xn[:250].copy()
    ref_call = None
    if R:
        per = 1.0 / cpu_rate(lambda: R.wiener_like(xs, *SIMPLE, *KN), 1, min(cs, 1.0))
        ref_call = per * n_nodes
    emit({"row": "(f)1 wiener_like_nodes simple 400 nodes x 250 (one batched call)",
          "trials": node.size, "kernel_ms": k, "call_ms": wall * 1e3,
          "cpu_port_ms_for_400_node_calls": ref_call and ref_call * 1e3})
    Pf = P.copy()
    Pf[:, 1], Pf[:, 4], Pf[:, 6] = 0.1, 0.1, 0.1
    k = gpu_kernel_ms(ctx, lambda: dsn.wiener_like_nodes(Pf))
    wall = timed(lambda: dsn.wiener_like_nodes(Pf))
    if R:
        per = 1.0 / cpu_rate(lambda: R.wiener_like(xs, *FULL, *KN), 1, min(cs, 1.0))
        ref_call = per * n_nodes
    emit({"row": "(f)1 wiener_like_nodes full DDM 400 nodes x 250", "trials": node.size,
          "kernel_ms": k, "call_ms": wall * 1e3,
          "cpu_port_ms_for_400_node_calls": ref_call and ref_call * 1e3})
    del dsn

    # (f)2: wiener_like_multi, per-trial v and a, 1M (host arrays)
    xm = x_full.copy()
    vm = 0.5 + 0.2 * np.sin(np.arange(xm.size))
    am = 2.0 + 0.1 * np.cos(np.arange(xm.size))
    f = lambda: wfpt.wiener_like_multi(xm, vm, 0.1, am, 0.5, 0.1, 0.3, 0.1, 1e-4, multi=["v", "a"],
                                       n_st=2, n_sz=2, simps_err=1e-3, p_outlier=0.05,
                                       w_outlier=0.1)
    wall = timed(f)
    s = slice(0, 20_000)
    xs_, vs_, as_ = xm[s].copy(), vm[s].copy(), am[s].copy()
    # wfpt.pyx:244-274 is restated in the oracle (C, 1 thread): kind "port"
    ref = cpu_rate(lambda: oracle.wiener_like_multi(xs_, vs_, 0.1, as_, 0.5, 0.1, 0.3, 0.1, 1e-4,
                                                    multi=["v", "a"], n_st=2, n_sz=2,
                                                    simps_err=1e-3, p_outlier=0.05,
                                                    w_outlier=0.1), xs_.size, cs)
    emit({"row": "(f)2 wiener_like_multi full DDM 1M (v, a per trial; host arrays)",
          "trials": xm.size, "call_ms": wall * 1e3, "gpu_trials_per_s": xm.size / wall,
          "cpu_port_trials_per_s": ref})
    # resident RTs (input order), per-trial v and a uploaded per call
    dsm = wfpt.Dataset(xm, input_order=True)
    g = lambda: dsm.wiener_like_multi(vm, 0.1, am, 0.5, 0.1, 0.3, 0.1, 1e-4, ["v", "a"], n_st=2,
                                      n_sz=2, simps_err=1e-3, p_outlier=0.05, w_outlier=0.1)
    k = gpu_kernel_ms(ctx, g, reps=5)
    wall = timed(g)
    emit({"row": "(f)2 wiener_like_multi full DDM 1M (resident RTs, v and a per trial uploaded "
                 "per call)", "trials": xm.size, "kernel_ms": k, "call_ms": wall * 1e3,
          "gpu_trials_per_s": xm.size / wall, "cpu_port_trials_per_s": ref})
    del dsm

    # (f)3: gen_rts_from_cdf (density grid on GPU), 1M samples, dt 1e-3
    wall = timed(lambda: wfpt.gen_rts_from_cdf(*FULL, samples=1_000_000, dt=1e-3), min_reps=2)
    emit({"row": "(f)3 gen_rts_from_cdf full DDM 1M samples dt=1e-3", "call_ms": wall * 1e3})

    # (f)4: DMAT CDF, dmat_cdf_array, 50k trials (full DDM and simple): the
    # first 50k of the 1M-trial set with |rt| < 4.99
    for name, p in (("full", FULL), ("simple", SIMPLE)):
        # |rt| < 1/(2 w_outlier) = 5 s is required with p_outlier > 0 (cdfdif_wrapper.pyx:20-21)
        xc = (x_full if name == "full" else x_simple)[:100_000].copy()
        xc = xc[np.abs(xc) < 4.99][:50_000].copy()
        k = gpu_kernel_ms(ctx, lambda: cdfdif_wrapper.dmat_cdf_array(xc, *p, 0.05, 0.1), reps=5)
        wall = timed(lambda: cdfdif_wrapper.dmat_cdf_array(xc, *p, 0.05, 0.1))
        s = xc[:5_000].copy()
        ref = cpu_rate(lambda: C.dmat_cdf_array(s, *p, 0.05, 0.1), s.size, cs) if C else None
        # the C restatement of cdfdif (oracle/cdfdif_oracle.c, bit-exact to the
        # reference's fixtures): 1 thread, and all host threads (OpenMP)
        port1 = cpu_rate(lambda: R.dmat_cdf_array(s, *p, 0.05, 0.1), s.size, cs)
        nt = threads()
        portn = cpu_rate(lambda: R.dmat_cdf_array(xc, *p, 0.05, 0.1, n_threads=nt), xc.size, cs)
        emit({"row": f"(f)4 dmat_cdf_array {name} {xc.size // 1000}k", "trials": xc.size,
              "kernel_ms": k,
              "call_ms": wall * 1e3, "gpu_trials_per_s": xc.size / wall,
              "cpu_ref_trials_per_s": ref, "cpu_port_1thread_trials_per_s": port1,
              "cpu_port_threads": nt, "cpu_port_all_threads_trials_per_s": portn})


if __name__ == "__main__":
    main()
