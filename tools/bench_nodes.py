"""wiener_like_nodes kernel time, 400 nodes x 250 trials, for several parameter
regimes (run twice: default two-pass path and WFPT_NODES=generic)."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hddm_amd import _lib, wfpt
ctx = _lib.context(0)
np.random.seed(3)
n_nodes = 400
x = wfpt.gen_rts_from_cdf(0.7, 0.3, 2.0, 0.5, 0.2, 0.3, 0.1, samples=100_000, dt=1e-3)
node = np.repeat(np.arange(n_nodes), 250)
ds = wfpt.Dataset(x, node_id=node, n_nodes=n_nodes)
for name, (sv, sz, st) in {"simple": (0, 0, 0), "pinned": (0.1, 0.1, 0.1),
                           "mid": (0.5, 0.3, 0.15), "wide": (1.6, 0.8, 0.24)}.items():
    P = np.zeros((n_nodes, 8))
    P[:, 0] = np.linspace(0.3, 1.1, n_nodes); P[:, 1] = sv; P[:, 2] = 2.0; P[:, 3] = 0.5
    P[:, 4] = sz; P[:, 5] = 0.22; P[:, 6] = st; P[:, 7] = 0.05
    ds.wiener_like_nodes(P)
    ctx.profile(1); ctx.profile_read(reset=True)
    t0 = time.perf_counter()
    for _ in range(10): r = ds.wiener_like_nodes(P)
    el = (time.perf_counter() - t0) / 10
    ms, nl, _ = ctx.profile_read(reset=True); ctx.profile(0)
    print(json.dumps({"regime": name, "mode": os.environ.get("WFPT_NODES", "two-pass"),
                      "kernel_ms": ms / nl, "call_ms": el * 1e3, "sum": float(np.sum(r))}), flush=True)
