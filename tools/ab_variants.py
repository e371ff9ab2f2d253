"""A/B timing of library build variants on one GPU (run via gpurun).

    python tools/ab_variants.py build            # here: compile the variants
    python tools/ab_variants.py run [--reps 5]   # GPU box: time each variant

Each variant is timed in its own subprocess (WFPT_AMD_LIB points at it), on
the bench workloads (full DDM pinned, stress, simple), with HIP-event kernel
time per call; variants are interleaved rep by rep (MI355X guide rule 24).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {
    "default": [],
    "exptab": ["WFPT_EXP_TABLE=1"],
    "exptab_lds": ["WFPT_EXP_TABLE=2"],
    "nodedbg": ["WFPT_NODE_DEBUG"],
    "nodedbg_solo": ["WFPT_NODE_DEBUG", "WFPT_NODE_REC_TEAM=0"],
    "nodedbg_entry": ["WFPT_NODE_DEBUG", "WFPT_NODE_DEBUG_ENTRY"],
    "stamps_noout": ["WFPT_NODE_DEBUG", "WFPT_NODE_DEBUG_NOOUT"],
    "recfence": ["WFPT_REC_FENCES=1"],
    "syncfence": ["WFPT_SYNC_FENCE=1"],
    "pub_diag": ["WFPT_PUB_DIAG=1"],
    "fastdbg": ["WFPT_NODE_DEBUG_FAST"],
    "ilp": ["-mllvm -amdgpu-sched-strategy=max-ilp"],
    "occbias": ["-mllvm -amdgpu-schedule-metric-bias=100"],
    "memclause": ["-mllvm -amdgpu-sched-strategy=max-memory-clause"],
    "wavepri": ["-mllvm -amdgpu-set-wave-priority"],
    "latbias": ["-mllvm -amdgpu-schedule-metric-bias=0"],
    "rec_solo": ["WFPT_NODE_REC_TEAM=0"],
    "direct_off": ["WFPT_DIRECT_ARGS=0"],
    "lb64": ["WFPT_LEAN_BLOCK=64"],
    "lb128": ["WFPT_LEAN_BLOCK=128"],
    "phase": ["WFPT_PHASE_TIMING"],
    "htot0": ["WFPT_HEAVY_TOTAL=0"],
    "split16": ["WFPT_SPLIT=16"],
    "split4": ["WFPT_SPLIT=4"],
    "pubnodes1": ["WFPT_PUB_NODES=1"],
}
LIBDIR = os.path.join(ROOT, "hddm_amd", "lib", "variants")

CHILD = r'''
import os, sys, json, time
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from hddm_amd import _lib, wfpt
import bench
ctx = _lib.context(0)
res = {}
rng = np.random.default_rng(5)
sets = {
  "full": (bench.make_rts(1_000_000, 20261015), bench.args_tuple()),
  "simple": (bench.make_rts(1_000_000, 20261015), (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)),
}
# stress: random params from generate.py:38-46 ranges, RTs sampled from each
np.random.seed(20261016)
xs, ps = [], []
for k in range(4):
    p = (rng.uniform(-4, 4), rng.uniform(0, 2.5), rng.uniform(0.5, 2), rng.uniform(0.4, 0.6),
         rng.uniform(0, 0.4), rng.uniform(0.2, 0.5), rng.uniform(0, 0.35))
    xs.append(wfpt.gen_rts_from_cdf(p[0], p[1], p[2], p[3], p[4], p[5], p[6], samples=250_000, dt=1e-3))
    ps.append(p)
kn = bench.knobs_tuple()
for name, (x, args) in sets.items():
    ds = wfpt.Dataset(x)
    ds.wiener_like(*args, *kn)
    ctx.profile(1); ctx.profile_read(reset=True)
    for _ in range(10): v = ds.wiener_like(*args, *kn)
    ms, nl, _ = ctx.profile_read(reset=True); ctx.profile(0)
    res[name] = {"kernel_ms": ms / nl, "logp": v}
tot = 0.0; val = 0.0
dss = [wfpt.Dataset(x) for x in xs]
for d, p in zip(dss, ps): d.wiener_like(*p, *kn)
t0 = time.perf_counter()
for _ in range(5):
    for d, p in zip(dss, ps): val += d.wiener_like(*p, *kn)
el = (time.perf_counter() - t0) / 5
# wall time per 1M trials (fast + slow passes + finalize + host)
res["stress"] = {"kernel_ms_per_1M": el * 1e3, "logp": val / 5}
print("RESULT " + json.dumps(res))
'''


def build(names=None):
    from hddm_amd import build as hb
    os.makedirs(LIBDIR, exist_ok=True)
    for name, d in VARIANTS.items():
        if names and name not in names:
            continue
        hb.build(force=True, defines=d, out=os.path.join(LIBDIR, f"libwfpt_{name}.so"))
        print("built", name, flush=True)


def run(reps, names=None):
    names = names or list(VARIANTS)
    out = {k: [] for k in names}
    for r in range(reps):
        for name in names:
            lib = os.path.join(LIBDIR, f"libwfpt_{name}.so")
            if not os.path.exists(lib):  # hddm_amd.build variants: lib_<name>.so
                lib = os.path.join(LIBDIR, f"lib_{name}.so")
            if name == "default" and not os.path.exists(lib):
                lib = os.path.join(ROOT, "hddm_amd", "lib", "libwfpt_amd.so")
            env = dict(os.environ, WFPT_AMD_LIB=lib, ROOT=ROOT)
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True,
                               text=True, timeout=600)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(name, "FAILED", p.returncode, p.stderr[-2000:], flush=True)
                return 1
            res = json.loads(line[0][7:])
            out[name].append(res)
            print(r, name, json.dumps(res), flush=True)
    summ = {}
    for name, rs in out.items():
        summ[name] = {k: min(x[k]["kernel_ms" if "kernel_ms" in x[k] else "kernel_ms_per_1M"]
                             for x in rs) for k in rs[0]}
    print("SUMMARY " + json.dumps(summ), flush=True)
    return 0


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[sys.argv.index("--names") + 1].split(",") if "--names" in sys.argv else None)
    else:
        reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
        # --names a,b: time already-built hddm_amd/lib/variants/libwfpt_<name>.so
        names = (sys.argv[sys.argv.index("--names") + 1].split(",") if "--names" in sys.argv
                 else None)
        sys.exit(run(reps, names))
