"""World-1 RCCL timing of the sharded call on one C5 shard (12.5M trials):
wiener_like vs wiener_like_allreduce per call, with HIP-event time of the
level-0 kernel (run via gpurun; WFPT_LEAN=0/1 to compare sequences).

    python tools/allreduce_probe.py [--trials 12500000] [--steps 20]
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
    ap.add_argument("--trials", type=int, default=12_500_000)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from hddm_amd import _lib, wfpt
    from hddm_amd import dist as hdist
    ctx = _lib.context(0)
    hdist.init_comm(ctx, 0, 1)
    x = bench.make_rts(a.trials, 20261015 + 3)
    ds = wfpt.Dataset(x)
    args, kn = bench.args_tuple(), bench.knobs_tuple()
    out = {"trials": a.trials, "lean": os.environ.get("WFPT_LEAN", "1")}
    for name, fn in (("local", lambda: ds.wiener_like(*args, *kn)),
                     ("allreduce", lambda: ds.wiener_like_allreduce(*args, *kn))):
        for _ in range(3):
            v = fn()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            v = fn()
        ctx.synchronize()
        out[name + "_ms"] = (time.perf_counter() - t0) / a.steps * 1e3
        out[name + "_logp"] = v
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
