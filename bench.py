#!/usr/bin/env python3
"""Headline benchmark: full-DDM trial-likelihood evaluations / s on MI355X.

Workloads (BASELINE.json configs):
  N = 1  C3: full DDM v=0.5 a=2 z=0.5 t=0.3 sv=sz=st=0.1 (reference
         test_models.py:18,71), 1M trials resident on the GPU.
  N > 1  C5: the same model, 100M trials in total sharded contiguously over the
         N ranks (100M/N per GPU: 12.5M at N = 8), one RCCL all-reduce of
         {sum log p, #zero trials, status} per call (scaling "strong").
Knobs are HDDM's: err=1e-4, n_st=n_sz=2, adaptive, simps_err=1e-3,
w_outlier=0.1, p_outlier=0.05 (base.py:688,713-716). RTs are sampled from the
model by this package's gen_rts_from_cdf (density grid on the GPU, dt=1e-3).

One step = one wiener_like call (wfpt.pyx:54-76 semantics) over the resident
shard. value = trials processed by all ranks / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W]

With --gpus N > 1 and no WORLD_SIZE in the environment this process launches
`torch.distributed.run` with N ranks itself (it never touches the GPU) and
exits with the launcher's code.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "trial-likelihood evals/sec (full DDM, sv/sz/st) at 1/2/4/8 GPUs"
PARAMS = dict(v=0.5, sv=0.1, a=2.0, z=0.5, sz=0.1, t=0.3, st=0.1)
KNOBS = dict(err=1e-4, n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3, w_outlier=0.1)
P_OUTLIER = 0.05
C3_TRIALS = 1_000_000
C5_TRIALS = 100_000_000
# fp64 VALU peak: 256 CU x 4 SIMD x 16 fp64 lanes/clk x 2.4 GHz = 39.3e12 lane-ops/s
# (the 78.6 TFLOP/s FMA-counted vector peak, MI355X_MICROARCH.md)
PEAK_LANE_OPS = 39.3e12


def args_tuple():
    p = PARAMS
    return (p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"])


def knobs_tuple(p_outlier=P_OUTLIER):
    k = KNOBS
    return (k["err"], k["n_st"], k["n_sz"], k["use_adaptive"], k["simps_err"], p_outlier,
            k["w_outlier"])


def make_rts(n, seed):
    from hddm_amd import wfpt
    np.random.seed(seed)
    p = PARAMS
    return wfpt.gen_rts_from_cdf(p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"],
                                 samples=n, dt=1e-3)


def host_threads():
    """Host cores this process may use (the GPU box exports OMP_NUM_THREADS=16,
    its CPU share per GPU; the machine has many more)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(x, budget_s):
    """The reference CPU path restated in C (oracle/wfpt_oracle.c, kind "port";
    calibrated against the reference's own kernels in the build container:
    profiles/r03/cpu_calibration.json), timed on this host's cores:
    1 thread = the reference's serial wiener_like loop (wfpt.pyx:66-76);
    all cores = the same per-trial full_pdf under OpenMP (the reference's
    prange in pdf_array, wfpt.pyx:40, built with -fopenmp)."""
    import oracle
    kn = knobs_tuple()
    one = x[:50_000].copy()
    done, t0 = 0, time.perf_counter()
    while True:
        oracle.wiener_like(one, *args_tuple(), *kn)
        done += one.size
        el1 = time.perf_counter() - t0
        if el1 >= budget_s / 2:
            break
    v1 = done / el1
    nt = host_threads()
    allc = x.copy()
    done, t0 = 0, time.perf_counter()
    while True:
        lp = oracle.pdf_array(allc, *args_tuple(), kn[0], 1, kn[1], kn[2], kn[3], kn[4], kn[5],
                              kn[6], n_threads=nt)
        float(np.sum(lp))
        done += allc.size
        eln = time.perf_counter() - t0
        if eln >= budget_s / 2:
            break
    vn = done / eln
    return {"value": vn, "unit": "trials/s", "cores": nt, "kind": "port",
            "value_1_thread": v1,
            "sample": f"C restatement of wfpt.wiener_like (oracle/wfpt_oracle.c; port/reference "
                      f"speed 1.03 on 1 thread, 1.26 on 8 OpenMP threads, measured in the build "
                      f"container, BASELINE.md 3a): all {nt} host threads over "
                      f"the {allc.size} benchmark trials x{done // allc.size} ({eln:.1f} s); "
                      f"1 thread over the first {one.size} trials ({el1:.1f} s, "
                      f"{v1:.3e} trials/s)"}


STRESS_TRIALS = 250_000  # per set


def stress_sets(n=STRESS_TRIALS):
    """The refining workload MCMC proposals hit: 4 full-DDM parameter sets drawn
    from HDDM's generator ranges (hddm/generate.py:38-46, seed 20261016; the
    same sets as tools/stress_probe.py), RTs sampled from each model."""
    from hddm_amd import wfpt
    rng = np.random.default_rng(20261016)
    np.random.seed(20261016)
    out = []
    for _ in range(4):
        p = (rng.uniform(-4, 4), rng.uniform(0, 2.5), rng.uniform(0.5, 2), rng.uniform(0.4, 0.6),
             rng.uniform(0, 0.4), rng.uniform(0.2, 0.5), rng.uniform(0, 0.35))
        out.append((wfpt.gen_rts_from_cdf(*p, samples=n, dt=1e-3), p))
    return out


def stress_line(ctx, steps, warmup, lib_path):
    """Secondary figure under the same clock (not the headline): resident
    wiener_like calls over the 4 stress sets, trials/s = 1M trials / the summed
    per-call times, and the in-wave engine kernel (the level-0 pass these sets
    take) per launch from HIP events, with its executed-work fraction when
    profiles/traffic_stress.json was measured on this build."""
    from hddm_amd import _lib, wfpt
    kn = knobs_tuple()
    call_s, evals, ntr = 0.0, 0, 0
    sets = []
    for si, (x, p) in enumerate(stress_sets()):
        ds = wfpt.Dataset(x)
        ctx.profile(ctx.PROF_EVALS)
        ds.wiener_like(*p, *kn)
        _, _, ne = ctx.profile_read(reset=True)
        ctx.profile(0)
        evals += ne
        ntr += x.size
        for _ in range(warmup):
            ds.wiener_like(*p, *kn)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ds.wiener_like(*p, *kn)
        ctx.synchronize()
        el = (time.perf_counter() - t0) / steps
        call_s += el
        # the set's steady-state kernels: the engine (refining data) or the
        # lean pass (a set whose waves settle at level 0)
        engine = bool(ctx.last_path() & _lib.PATH_ENGINE)
        ctx.profile(ctx.PROF_EVENTS)
        ctx.profile_read(reset=True)
        for _ in range(steps):
            ds.wiener_like(*p, *kn)
        ctx.synchronize()
        km, l, _ = ctx.profile_read(reset=True)
        ctx.profile(0)
        sets.append({"set": si, "call_ms": el * 1e3, "main_kernel": "engine" if engine else "lean",
                     "main_kernel_ms": km / max(l, 1), "pdf_sv_evals_per_trial": ne / x.size})
        ds.close()
    eng = [r for r in sets if r["main_kernel"] == "engine"]
    k_avg_s = sum(r["main_kernel_ms"] for r in eng) / max(len(eng), 1) / 1e3
    out = {"workload": "4 x 250k full-DDM trials, parameters from hddm/generate.py:38-46 "
                       "ranges (seed 20261016), one resident wiener_like call per set",
           "trials_per_s": ntr / call_s, "ms_per_1M_trials": call_s * 1e3 * 1e6 / ntr,
           "pdf_sv_evals_per_trial": evals / ntr, "sets": sets,
           "kernel": "wfpt::engine_kernel<3, false, 0> (in-wave adaptive engine), over the "
                     "sets whose steady-state call runs it (%s)" % [r["set"] for r in eng],
           "kernel_ms_avg": k_avg_s * 1e3, "frac": None}
    pmc = pmc_summary(lib_path, "traffic_stress.json")
    if pmc and pmc.get("matches_build") and eng:
        # fp64 lane-ops per trial averaged over the engine launches of the same
        # sets' steady-state calls (tools/stress_probe.py --engine-only under
        # rocprofv3): equal launches per set, so n * mean(w) / mean(t) is the
        # engine sets' total work over their total kernel time
        w = float(pmc["fp64_lane_ops_per_trial"])
        ach = STRESS_TRIALS * w / k_avg_s / 1e12
        tr = pmc.get("hbm_bytes_per_trial")
        out.update(achieved=ach, frac=ach / (PEAK_LANE_OPS / 1e12), fp64_lane_ops_per_trial=w,
                   valu_issue_utilisation=pmc.get("valu_issue_utilisation"),
                   traffic=tr * STRESS_TRIALS if tr is not None else None,
                   algorithmic_bytes=8.0 * STRESS_TRIALS, pmc_source=pmc.get("source"),
                   pmc_sets=pmc.get("sets"))
    return out


C2_TRIALS = 10_000_000
C2_PARAMS = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)  # simple DDM (v, a, t), z = .5


def c2_line(ctx, steps, warmup, lib_path):
    """BASELINE config 2 under the same clock: the simple DDM (Navarro-Fuss
    pdf, one pdf_sv per trial) over 10M resident trials, HDDM knobs,
    p_outlier .05 (the same dataset as tools/c2_probe.py, seed 20261015); the
    direct_kernel's per-launch time from HIP events and its executed-work
    fraction when profiles/traffic_c2.json was measured on this build."""
    from hddm_amd import wfpt
    np.random.seed(20261015)
    x = wfpt.gen_rts_from_cdf(*C2_PARAMS, samples=C2_TRIALS, dt=1e-3)
    ds = wfpt.Dataset(x)
    kn = knobs_tuple()
    for _ in range(warmup):
        v = ds.wiener_like(*C2_PARAMS, *kn)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        v = ds.wiener_like(*C2_PARAMS, *kn)
    ctx.synchronize()
    el = (time.perf_counter() - t0) / steps
    ctx.profile(ctx.PROF_EVENTS)
    ctx.profile_read(reset=True)
    for _ in range(steps):
        ds.wiener_like(*C2_PARAMS, *kn)
    ctx.synchronize()
    km, l, _ = ctx.profile_read(reset=True)
    ctx.profile(0)
    ds.close()
    k_s = km / max(l, 1) / 1e3
    out = {"workload": "C2: simple DDM (v=.5 a=2 z=.5 t=.3), 10M resident trials, one "
                       "wiener_like call per step", "trials": C2_TRIALS,
           "ms_per_step": el * 1e3, "trials_per_s": C2_TRIALS / el, "logp": v,
           "kernel": "wfpt::direct_kernel<false>", "kernel_ms_avg": k_s * 1e3, "frac": None}
    pmc = pmc_summary(lib_path, "traffic_c2.json")
    if pmc and pmc.get("matches_build"):
        w = float(pmc["fp64_lane_ops_per_trial"])
        ach = C2_TRIALS * w / k_s / 1e12
        tr = pmc.get("hbm_bytes_per_trial")
        out.update(achieved=ach, frac=ach / (PEAK_LANE_OPS / 1e12), fp64_lane_ops_per_trial=w,
                   valu_lane_ops_per_trial=pmc.get("valu_lane_ops_per_trial"),
                   valu_issue_utilisation=pmc.get("valu_issue_utilisation"),
                   traffic=tr * C2_TRIALS if tr is not None else None,
                   algorithmic_bytes=8.0 * C2_TRIALS, pmc_source=pmc.get("source"))
    return out


C5_BLOCK = 12_500_000  # C5's 100M trials as 8 blocks (seed 20261015 + block)


def c5_rts(lo, hi):
    """Trials [lo, hi) of config 5's 100M: block b (12.5M trials) is sampled
    with seed 20261015 + b, so every world size shards the same 100M trials
    (rank r of N = 8 holds block r) and N = 1 holds all of them."""
    parts = []
    for b in range(lo // C5_BLOCK, (hi - 1) // C5_BLOCK + 1):
        blk = make_rts(C5_BLOCK, 20261015 + b)
        s, e = max(lo, b * C5_BLOCK), min(hi, (b + 1) * C5_BLOCK)
        parts.append(blk[s - b * C5_BLOCK:e - b * C5_BLOCK])
    return np.concatenate(parts)


def c5_n1_line(ctx, steps, warmup):
    """Config 5's whole workload on ONE GPU: the 100M trials every world size
    shards (c5_rts), resident, through wiener_like_allreduce on a world-1 RCCL
    communicator -- the N = 1 point of the 1/2/4/8-GPU curve on the same
    workload and path as the N > 1 lines (value(N) / value_c5_n1 is the
    speed-up)."""
    from hddm_amd import dist as hdist
    from hddm_amd import wfpt
    t0 = time.perf_counter()
    x = c5_rts(0, C5_TRIALS)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    ds = wfpt.Dataset(x)
    t_ds = time.perf_counter() - t0
    del x
    hdist.init_comm(ctx, 0, 1)
    step = lambda: ds.wiener_like_allreduce(*args_tuple(), *knobs_tuple())
    for _ in range(warmup):
        v = step()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        v = step()
    ctx.synchronize()
    el = (time.perf_counter() - t0) / steps
    ds.close()
    return {"workload": "C5 on 1 GPU: the same 100M full-DDM trials the N > 1 lines shard "
                        "(12.5M blocks, seed 20261015 + block), one wiener_like_allreduce "
                        "per step on a world-1 RCCL communicator",
            "trials": C5_TRIALS, "ms_per_step": el * 1e3, "value": C5_TRIALS / el,
            "unit": "trials/s", "logp": v, "data_generation_s": t_gen,
            "dataset_create_s": t_ds}


def c4_line(cpu_seconds=2.0):
    """BASELINE config 4 under the same clock: HDDM(200 subjects x 500
    trials, depends_on={'v': 'cond'}).sample(2000) on one GPU (after 20 burn-in
    sweeps, hddm_amd.hierarchical), full DDM (sv, sz, st) and simple; beside
    it the reference-port CPU likelihood time of one sweep's node evaluations
    (oracle/wfpt_oracle.c wiener_like per 250-trial node, 1 thread, x the
    sweep's node evaluations; the reference's PyMC sampler cannot run
    offline)."""
    import oracle
    from hddm_amd.hierarchical import HDDM, gen_data
    out = {"workload": "C4: HDDM 200 subj x 500 trials, depends_on v:cond, p_outlier .05, "
                       "sample(2000) after 20 burn-in sweeps, data at dt 1e-4"}
    for full in (True, False):
        inter = dict(sv=0.1, sz=0.1, st=0.1) if full else {}
        data, _ = gen_data(n_subj=200, n_trials=500, dt=1e-4, **inter)
        m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05, seed=1)
        m.sample(20)
        c0, s0 = m.likelihood_calls, m.likelihood_seconds
        t0 = time.perf_counter()
        m.sample(2000)
        el = time.perf_counter() - t0
        calls = m.likelihood_calls - c0
        node = data["rt"].to_numpy()[:250].copy()
        p = (1.0, *((0.1,) if full else (0.0,)), 2.0, 0.5, *((0.1,) if full else (0.0,)), 0.3,
             *((0.1,) if full else (0.0,)))
        reps, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < cpu_seconds:
            oracle.wiener_like(node, *p, 1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
            reps += 1
        per_node = (time.perf_counter() - t1) / reps
        out["full" if full else "simple"] = {
            "sample_2000_s": el, "sweeps_per_s": 2000 / el,
            "batched_likelihood_calls_per_sweep": calls / 2000,
            "likelihood_us_per_call": (m.likelihood_seconds - s0) / max(calls, 1) * 1e6,
            "likelihood_fraction_of_time": (m.likelihood_seconds - s0) / el,
            "cpu_port_likelihood_s_per_sweep": per_node * calls * m.n_nodes / 2000,
            "cpu_port": {"kind": "port", "cores": 1, "per_node_call_s": per_node,
                         "sample": f"{reps} wiener_like calls on one 250-trial node"}}
        m.dataset.close()
    # HDDM's multi-chain usage (docs/source/howto.rst:267-291): 8 chains of the
    # full model in lockstep, every slice evaluation of every chain in one
    # multi-table launch (hddm_amd.hierarchical.HDDMChains)
    from hddm_amd.hierarchical import HDDMChains
    data, _ = gen_data(n_subj=200, n_trials=500, dt=1e-4, sv=0.1, sz=0.1, st=0.1)
    m = HDDMChains(data, chains=8, depends_on={"v": "cond"}, include=("sv", "sz", "st"),
                   p_outlier=0.05, seed=1)
    m.sample(20)
    c0, s0 = m.likelihood_calls, m.likelihood_seconds
    tb0 = m.tables_evaluated
    t0 = time.perf_counter()
    m.sample(2000)
    el = time.perf_counter() - t0
    calls = m.likelihood_calls - c0
    rh = m.gelman_rubin()
    out["full_8_chains"] = {
        "sample_2000_s": el, "chain_sweeps_per_s": 8 * 2000 / el,
        "batched_likelihood_calls_per_sweep": calls / 2000,
        "tables_per_call": (m.tables_evaluated - tb0) / max(calls, 1),
        "likelihood_us_per_call": (m.likelihood_seconds - s0) / max(calls, 1) * 1e6,
        "likelihood_fraction_of_time": (m.likelihood_seconds - s0) / el,
        "rhat_max_group_nodes": max(rh[k] for k in ("a", "t", "v(c0)", "v(c1)", "sv", "sz", "st")),
        "vs_8_single_chain_runs": 8 * out["full"]["sample_2000_s"] / el}
    m.dataset.close()
    return out


def pmc_summary(lib_path, name="traffic.json"):
    """Executed-work figures of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/traffic.json, written by tools/summarize_profile.py),
    used only if it was measured on a library built from the same sources and
    flags as the one loaded (hddm_amd.build.source_digest, recorded at build
    time next to the .so). Per-trial figures: the C3 and C5 datasets are
    samples of the same model."""
    from hddm_amd import build as hb
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as fh:
            t = json.load(fh)
    except Exception:
        return None
    digest = hb.built_digest(lib_path)
    t["matches_build"] = digest is not None and t.get("src_sha1") == digest
    return t


def launch_ranks(a):
    """--gpus N > 1 without a torch.distributed environment: run this script
    under torch.distributed.run with N ranks (one process per GPU)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--trials", type=int, default=None,
                    help="trials per GPU (default: C3 1M at N=1, C5 100M/N at N>1)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stress", action="store_true",
                    help="skip the secondary stress-set figure (N = 1 only)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the C2 and C5-on-one-GPU figures (N = 1 only)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the config-4 sample(2000) figures (N = 1 only)")
    a = ap.parse_args()

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={a.gpus}", file=sys.stderr)
    os.environ.setdefault("WFPT_DEVICE", str(local))
    from hddm_amd import _lib, wfpt

    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist.group.WORLD
    ctx = _lib.context(local)

    c5 = world > 1
    total = C5_TRIALS if c5 else C3_TRIALS
    if a.trials is not None:
        n = a.trials
    else:
        lo, hi = _lib.shard_range(total, world, rank)
        n = hi - lo
    if c5 and a.trials is None:
        x = c5_rts(lo, hi)  # the 100M trials' shard: the same data at every world size
    else:
        x = make_rts(n, 20261015 + rank)
    ds = wfpt.Dataset(x, device=local)
    if world > 1:
        from hddm_amd import dist as hdist
        hdist.init_comm(ctx, rank, world)  # the library's TCP rendezvous (no torch)
        step = lambda: ds.wiener_like_allreduce(*args_tuple(), *knobs_tuple())
    else:
        step = lambda: ds.wiener_like(*args_tuple(), *knobs_tuple())

    # untimed pass: count pdf_sv evaluations on this dataset
    ctx.profile(ctx.PROF_EVALS)
    val = step()
    _, _, n_evals = ctx.profile_read(reset=True)
    ctx.profile(0)
    for _ in range(a.warmup):
        step()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    # timed region: K plain calls (no per-launch instrumentation in the way)
    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        val = step()
    ctx.synchronize()
    el = time.perf_counter() - t0
    barrier()
    # the same K calls again with HIP events recorded on the library's stream
    # around the dominant kernel (the level-0 pass): its per-launch duration
    ctx.profile(ctx.PROF_EVENTS)
    ctx.profile_read(reset=True)
    for _ in range(a.steps):
        step()
    ctx.synchronize()
    k_ms, launches, _ = ctx.profile_read(reset=True)
    ctx.profile(0)
    if world > 1:
        import torch
        import torch.distributed as dist
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    glob = n * world
    value = glob * a.steps / el
    k_avg_s = (k_ms / 1e3) / max(launches, 1)
    pmc = pmc_summary(_lib.LIB_PATH)
    roof = {"bound": "valu-fp64", "peak": PEAK_LANE_OPS / 1e12, "unit": "T fp64-lane-ops/s",
            "achieved": None, "frac": None, "traffic": None,
            "kernel": "wfpt::lean_kernel<3, false, 0> (level-0 pass)",
            "kernel_ms_avg": k_avg_s * 1e3, "kernel_launches": launches}
    if pmc and pmc.get("matches_build"):
        # executed fp64 VALU lane-ops per trial of this kernel (rocprofv3
        # SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 x 64 lanes, same build and dataset)
        # over its live per-launch time
        w = float(pmc["fp64_lane_ops_per_trial"])
        achieved = n * w / k_avg_s / 1e12
        traffic = pmc.get("hbm_bytes_per_trial")
        roof.update(achieved=achieved, frac=achieved / (PEAK_LANE_OPS / 1e12),
                    traffic=traffic * n if traffic is not None else None,
                    fp64_lane_ops_per_trial=w,
                    valu_issue_utilisation=pmc.get("valu_issue_utilisation"),
                    algorithmic_bytes=8.0 * n, pmc_source=pmc.get("source"))
    else:
        roof["note"] = ("profiles/traffic.json was not measured on this library build / size; "
                        "run tools/gpu_profile.sh + tools/summarize_profile.py")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "trials/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if c5 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (RTs sampled from the DDM by hddm_amd.wfpt.gen_rts_from_cdf, "
                "seed 20261015+rank)",
        "config": {"workload": ("C5: full DDM 100M trials sharded over %d GPUs + RCCL "
                                "all-reduce" % world) if c5 else
                               "C3: full DDM 1M trials on 1 GPU",
                   "params": "sv=sz=st=0.1 v=.5 a=2 z=.5 t=.3, HDDM knobs (err 1e-4, "
                             "n_st=n_sz=2, adaptive, simps_err 1e-3), p_outlier .05; one "
                             "wiener_like call per step",
                   "trials_per_gpu": n, "global_trials": glob,
                   "parallelism": f"trial-shard x{world}" + (" + RCCL all-reduce"
                                                              if world > 1 else ""),
                   "pdf_sv_evals_per_trial": n_evals / n,
                   "logp": val},
        "roofline": roof,
    }
    if world == 1 and not a.no_stress:
        out["stress"] = stress_line(ctx, a.steps, a.warmup, _lib.LIB_PATH)
    if world == 1 and not a.no_extra:
        ds.close()
        out["c2"] = c2_line(ctx, a.steps, a.warmup, _lib.LIB_PATH)
        out["c5_n1"] = c5_n1_line(ctx, a.steps, a.warmup)
        out["config"]["c5_n1_speedup_basis"] = (
            "value at N > 1 / c5_n1.value = the speed-up on config 5's one 100M workload")
    if world == 1 and not a.no_c4:
        out["c4"] = c4_line()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(x, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
