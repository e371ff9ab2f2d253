#!/usr/bin/env python3
"""Headline benchmark: full-DDM trial-likelihood evaluations / s on MI355X.

Workload (BASELINE.json configs[2], the metric's single-GPU config): full DDM
v=0.5 a=2 z=0.5 t=0.3 sv=sz=st=0.1 (reference test_models.py:18,71), HDDM's
knobs err=1e-4 n_st=n_sz=2 adaptive simps_err=1e-3 w_outlier=0.1, p_outlier=0.05
(base.py:688,713-716); 1M synthetic RTs per GPU sampled from the model with
this package's gen_rts_from_cdf (density grid on the GPU, dt=1e-3).

One step = one wiener_like call (wfpt.pyx:54-76 semantics) over the resident
dataset: trial kernel + finalize + 16-byte result to the host; with N>1 ranks
each rank owns 1M trials and the per-call exchange is one RCCL all-reduce
(weak scaling). value = trials processed by all ranks / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "trial-likelihood evals/sec (full DDM, sv/sz/st) at 1/2/4/8 GPUs"
PARAMS = dict(v=0.5, sv=0.1, a=2.0, z=0.5, sz=0.1, t=0.3, st=0.1)
KNOBS = dict(err=1e-4, n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3, w_outlier=0.1)
P_OUTLIER = 0.05
W_EVAL = 970.0   # FP64 VALU lane-ops per pdf_sv evaluation
W_EPI = 99.0     # per-trial mixture + log + sum
PEAK_LANE_OPS = 39.3e12  # 256 CU x 4 SIMD x 16 fp64 lanes/clk x 2.4 GHz (= 78.6 TFLOP/s FMA)


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


def cpu_baseline(x, budget_s):
    """Reference CPU path on the host: oracle/_ref (the reference's own kernels
    in its serial wiener_like loop) if present, else the C restatement."""
    import oracle
    ref = oracle.load_ref()
    kind = "reference" if ref is not None else "port"
    fn = ref.wiener_like if ref is not None else oracle.wiener_like
    sample = x[:50_000].copy()
    done, t0 = 0, time.perf_counter()
    while True:
        fn(sample, *args_tuple(), *knobs_tuple())
        done += sample.size
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": done / el, "unit": "trials/s", "cores": 1, "kind": kind,
            "sample": f"wiener_like over the first {sample.size} trials of the benchmark "
                      f"dataset, repeated {done // sample.size}x ({el:.1f} s, 1 thread)"}


def load_traffic(n_trials):
    """HBM bytes per launch and VALU issue utilisation of the main kernel from
    the committed rocprofv3 PMC summary (profiles/traffic.json), if present."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None, None, None
    try:
        with open(path) as fh:
            t = json.load(fh)
        if int(t.get("n_trials", -1)) == int(n_trials):
            return (float(t["hbm_bytes_per_launch"]), t.get("valu_issue_utilisation"),
                    t.get("fp64_lane_ops_per_trial"))
    except Exception:
        return None, None, None
    return None, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--trials", type=int, default=1_000_000, help="trials per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus={a.gpus}", file=sys.stderr)
    os.environ.setdefault("WFPT_DEVICE", str(local))
    from hddm_amd import _lib, wfpt

    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist.group.WORLD
    ctx = _lib.context(local)

    n = a.trials
    x = make_rts(n, 20261015 + rank)
    ds = wfpt.Dataset(x, device=local)
    if world > 1:
        from hddm_amd import dist as hdist
        hdist.init_comm(ctx, rank, world, pg)
        step = lambda: ds.wiener_like_allreduce(*args_tuple(), *knobs_tuple())
    else:
        step = lambda: ds.wiener_like(*args_tuple(), *knobs_tuple())

    # untimed pass: count pdf_sv evaluations on this dataset (feeds W_trial)
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
    # each rank's clock stops when its own K calls are done (every call ends in
    # the all-reduce, so ranks finish together); the closing barrier aligns the
    # ranks for the next phase and the max over ranks below is the job time
    el = time.perf_counter() - t0
    barrier()
    # the same K calls again with HIP events recorded on the library's stream
    # around the likelihood kernels of every call: per-launch kernel time
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

    total_trials = n * world * a.steps
    value = total_trials / el
    evals_per_trial = n_evals / n
    w_trial = evals_per_trial * W_EVAL + W_EPI
    k_avg_s = (k_ms / 1e3) / max(launches, 1)
    achieved = n * w_trial / k_avg_s / 1e12
    traffic, valu_util, f64_per_trial = load_traffic(n)
    # hardware view: fp64 VALU lane-ops the kernel actually executes per trial
    # (rocprofv3 SQ_INSTS_VALU_*_F64 x 64, profiles/traffic.json) over its time
    exec_tops = n * f64_per_trial / k_avg_s / 1e12 if f64_per_trial else None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "trials/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (RTs sampled from the DDM by hddm_amd.wfpt.gen_rts_from_cdf, "
                "seed 20261015+rank)",
        "config": {"workload": "full DDM sv=sz=st=0.1 v=.5 a=2 z=.5 t=.3, HDDM knobs "
                               "(err 1e-4, n_st=n_sz=2, adaptive, simps_err 1e-3), "
                               "p_outlier .05; one wiener_like call per step",
                   "trials_per_gpu": n, "global_trials": n * world,
                   "parallelism": f"trial-shard x{world}" + (" + RCCL all-reduce"
                                                              if world > 1 else ""),
                   "pdf_sv_evals_per_trial": evals_per_trial,
                   "logp": val},
        "roofline": {"bound": "valu-fp64", "achieved": achieved, "peak": PEAK_LANE_OPS / 1e12,
                     "unit": "T fp64-lane-ops/s", "frac": achieved / (PEAK_LANE_OPS / 1e12),
                     "traffic": traffic,
                     "kernel_ms_avg": k_avg_s * 1e3, "kernel_launches": launches,
                     "w_trial_lane_ops": w_trial,
                     # hardware view (rocprofv3 PMC, profiles/traffic.json): share of SIMD
                     # cycles issuing VALU (4 cycles per wave64 fp64 op, 2 otherwise)
                     "valu_issue_utilisation": valu_util,
                     # frac above is algorithmic (the reference's op count, SURVEY.md
                     # 8d); this is executed fp64 work over the same peak
                     "executed_fp64": exec_tops,
                     "executed_frac": exec_tops / (PEAK_LANE_OPS / 1e12) if exec_tops else None},
    }
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
