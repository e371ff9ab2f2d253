"""A/B timing of CDF build variants (cdfdif_kernels.hip knobs) on one GPU.

    python tools/ab_cdf.py build            # here: compile the variants
    python tools/ab_cdf.py run [--reps 3]   # GPU box (via gpurun)

Each variant runs in its own subprocess (WFPT_AMD_LIB points at it) on
tools/cdf_probe.py's 100k full-DDM and simple sets; variants are interleaved
rep by rep. Per call: the kernels' HIP-event time and the wall time. Every
variant's outputs are compared with the first variant's (bit-equal expected:
the knobs change the schedule, not the arithmetic).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {
    "base": ["WFPT_CDF_CHUNK=1", "WFPT_CDF_BEY=0", "WFPT_CDF_READLANE=0"],
    "chunk8": ["WFPT_CDF_BEY=0"],
    "bey": ["WFPT_CDF_CHUNK=1", "WFPT_CDF_READLANE=0"],
    "new": [],
    "new_w16k": ["WFPT_CDF_WAVES=16384"],
    "new_c4": ["WFPT_CDF_CHUNK=4"],
    "debug": ["WFPT_CDF_DEBUG", "WFPT_CDF_CHUNK=1", "WFPT_CDF_READLANE=0"],
    "debug_rl": ["WFPT_CDF_DEBUG"],
    "rl": [],
    "stage": [],
    "debug_stage": ["WFPT_CDF_DEBUG"],
    "nodpp": ["WFPT_CDF_DPP=0"],
    "dpp": [],
    "dpp_c1": ["WFPT_CDF_CHUNK=1"],
    "dpp_c4": ["WFPT_CDF_CHUNK=4"],
}
LIBDIR = os.path.join(ROOT, "hddm_amd", "lib", "variants")

CHILD = r'''
import os, sys, json, time, hashlib
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from hddm_amd import _lib, cdfdif_wrapper, wfpt
ctx = _lib.context(0)
res = {}
for name, p in (("full", (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)),
                ("simple", (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0))):
    np.random.seed(20261015)
    x = wfpt.gen_rts_from_cdf(*p, samples=200_000, dt=1e-3)
    x = x[np.abs(x) < 4.99][:100_000].copy()
    y = cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
    el = (time.perf_counter() - t0) / 10
    ctx.profile(ctx.PROF_EVENTS); ctx.profile_read(reset=True)
    for _ in range(10):
        cdfdif_wrapper.dmat_cdf_array(x, *p, 0.05, 0.1)
    ms, nl, _ = ctx.profile_read(reset=True); ctx.profile(0)
    res[name] = {"kernel_ms": ms / max(nl, 1), "call_ms": el * 1e3,
                 "digest": hashlib.sha1(np.ascontiguousarray(y).tobytes()).hexdigest()[:12]}
print("RESULT " + json.dumps(res))
'''


def build(names=None):
    from hddm_amd import build as hb
    os.makedirs(LIBDIR, exist_ok=True)
    for name, d in VARIANTS.items():
        if names and name not in names:
            continue
        hb.build(force=True, defines=d, out=os.path.join(LIBDIR, f"libwfpt_cdf_{name}.so"))
        print("built", name, flush=True)


def run(reps, names=None):
    names = names or list(VARIANTS)
    out = {k: [] for k in names}
    for r in range(reps):
        for name in names:
            env = dict(os.environ, ROOT=ROOT,
                       WFPT_AMD_LIB=os.path.join(LIBDIR, f"libwfpt_cdf_{name}.so"))
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True,
                               text=True, timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(name, "FAILED", p.returncode, p.stderr[-2000:], flush=True)
                sys.exit(1)
            res = json.loads(line[0][7:])
            out[name].append(res)
            print(r, name, json.dumps(res), flush=True)
    ref = out[names[0]][0]
    summary = {}
    for name in names:
        summary[name] = {
            s: {"kernel_ms_min": min(x[s]["kernel_ms"] for x in out[name]),
                "call_ms_min": min(x[s]["call_ms"] for x in out[name]),
                "same_as_" + names[0]: all(x[s]["digest"] == ref[s]["digest"] for x in out[name])}
            for s in ("full", "simple")}
    print("SUMMARY " + json.dumps(summary, indent=1), flush=True)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--names", nargs="*")
    a = ap.parse_args()
    build(a.names) if a.cmd == "build" else run(a.reps, a.names)
