"""Level-0 kernel time vs dataset size on the bench distribution (fixed cost
and tail effects of the lean pass): n = 125k ... 4M, HIP-event kernel time.

    python tools/size_probe.py [--reps 10]     (WFPT_AMD_LIB selects a variant)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import bench
    from hddm_amd import _lib, wfpt
    ctx = _lib.context(0)
    x = bench.make_rts(4_000_000, 20261015)
    args, kn = bench.args_tuple(), bench.knobs_tuple()
    out = {}
    for n in (125_000, 250_000, 500_000, 1_000_000, 2_000_000, 4_000_000):
        ds = wfpt.Dataset(x[:n].copy())
        ds.wiener_like(*args, *kn)
        ds.wiener_like(*args, *kn)
        ctx.profile(1)
        ctx.profile_read(reset=True)
        for _ in range(a.reps):
            ds.wiener_like(*args, *kn)
        ms, nl, _ = ctx.profile_read(reset=True)
        ctx.profile(0)
        out[n] = ms / max(nl, 1)
        print(json.dumps({"n": n, "kernel_ms": out[n], "ns_per_trial": out[n] * 1e6 / n}), flush=True)
        del ds


if __name__ == "__main__":
    main()
