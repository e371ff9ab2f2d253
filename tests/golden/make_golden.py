"""Generate the golden fixtures under tests/golden/ (run in the build container).

Expected values come from the REFERENCE'S OWN kernels (oracle/_ref/ref_shim, the
reference src/pdf.pxi + src/integrate.pxi compiled by oracle/build_ref.py),
never from this repository's code. The MATLAB tuples are read as data from the
reference's hddm/tests/matlab_values.py with ast.literal_eval (no code executed).

Outputs (all small, numpy .npz without pickles, or JSON):
  matlab_values.json   20 Navarro-Fuss tuples (v,t,a,z,z_nonorm,rt,err,wfpt)
  full_pdf_grid.npz    branch-covering per-trial full_pdf values
  wiener_like.npz      summed log-likelihoods (wfpt.pyx:54-76 semantics)
  pdf_array.npz        per-trial mixture density / log density
  datasets.npz         model-sampled RT datasets (pinned, stress) + totals

Usage: python tests/golden/make_golden.py [--reference /root/reference]
"""
import argparse
import ast
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

PKEYS = ["v", "sv", "a", "z", "sz", "t", "st", "err", "n_st", "n_sz", "use_adaptive",
         "simps_err"]


def stress_params(rng, fam):
    """Ranges of hddm/generate.py:38-46 (gen_single_params_set)."""
    p = dict(v=rng.uniform(-4, 4), a=rng.uniform(0.5, 2.0), t=rng.uniform(0.2, 0.5),
             z=rng.uniform(0.4, 0.6), sv=0.0, sz=0.0, st=0.0)
    if "sv" in fam:
        p["sv"] = rng.uniform(0, 2.5)
    if "sz" in fam:
        p["sz"] = rng.uniform(0, 0.4)
    if "st" in fam:
        p["st"] = rng.uniform(0, 0.35)
    return p


def x_vector(rng, p, m):
    lo = p["t"] - p["st"] / 2.0
    mag = np.concatenate([
        rng.uniform(max(lo - 0.05, 0.0), lo + 0.05, m // 4),      # at/below the support edge
        rng.uniform(lo, p["t"] + 3.0, m - m // 4 - 4),
        [0.0, lo, lo + 1e-9, lo + 1e-6],
    ])
    sign = rng.choice([-1.0, 1.0], mag.size)
    return (sign * mag)[:m]


def gen_rts_restated(R, rng, p, samples, cdf_lb=-6.0, cdf_ub=6.0, dt=1e-3):
    """Restatement of wfpt.pyx:323-354 (gen_rts_from_cdf) around the reference full_pdf."""
    x = np.arange(cdf_lb, cdf_ub, dt)
    pdf = np.array([R.full_pdf(xi, p["v"], p["sv"], p["a"], p["z"], p["sz"], 0, 0, 1e-4)
                    for xi in x[1:]])
    l_cdf = np.concatenate([[0.0], np.cumsum(pdf)])
    l_cdf /= l_cdf[-1]
    f = rng.random(samples)
    idx = np.searchsorted(l_cdf, f)
    rt = x[idx]
    if p["st"] != 0:
        delay = rng.random(samples) * p["st"] + (p["t"] - p["st"] / 2.0)
        return rt + np.sign(rt) * delay
    return rt + np.sign(rt) * p["t"]


def main(reference):
    import oracle
    from oracle import build_ref
    build_ref.build(reference, quiet=True)
    R = oracle.load_ref()
    assert R is not None, "oracle/_ref did not build"
    rng = np.random.default_rng(20261015)

    # 1. MATLAB tuples (data only)
    src = open(os.path.join(reference, "hddm/tests/matlab_values.py")).read()
    tree = ast.parse(src)
    vals = None
    for node in tree.body:
        if isinstance(node, ast.Assign) and node.targets[0].id == "vals":
            vals = ast.literal_eval(node.value)
    assert vals is not None and len(vals) == 20
    with open(os.path.join(HERE, "matlab_values.json"), "w") as fh:
        json.dump({"source": "hddm/tests/matlab_values.py:3-162 (Navarro-Fuss wfpt.m)",
                   "fields": ["v", "t", "a", "z", "z_nonorm", "rt", "err", "matlab_wfpt"],
                   "reference_full_pdf": [R.full_pdf(-rt, v, 0, a, z, 0, t, 0, err, 0)
                                          for v, t, a, z, _, rt, err, _ in vals],
                   "vals": [list(map(float, v)) for v in vals]}, fh, indent=1)

    # 2. branch-covering full_pdf grid
    M = 48
    fams = ["simple", "sv", "sz", "st", "sz_st", "sv_sz_st"]
    errs = [1e-10, 1e-8, 1e-6, 1e-4, 1e-4, 1e-4, 1e-3, 1e-2, 0.1, 1.0]
    rows, xs = [], []
    for fam in fams:
        for k in range(24):
            p = stress_params(rng, fam.replace("sz_st", "sz st"))
            knob = dict(err=errs[k % len(errs)], n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3)
            if k % 6 == 5:
                knob.update(n_st=int(rng.integers(0, 6)), n_sz=int(rng.integers(0, 6)),
                            simps_err=float(10 ** rng.uniform(-8, -2)))
            if k % 8 == 7:
                knob.update(use_adaptive=0, n_st=2 * int(rng.integers(1, 6)),
                            n_sz=2 * int(rng.integers(1, 6)))
            rows.append([p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"],
                         knob["err"], knob["n_st"], knob["n_sz"], knob["use_adaptive"],
                         knob["simps_err"]])
            xs.append(x_vector(rng, p, M))
    # edge parameter sets (invalid / boundary semantics, pdf.pxi:111-125)
    base = dict(v=1.0, sv=1.0, a=1.5, z=0.5, sz=0.2, t=0.2, st=0.1)
    edges = [dict(z=1.1), dict(z=-0.1), dict(z=0.1, sz=0.25), dict(a=-0.1), dict(a=0.0),
             dict(t=0.7, st=0.0), dict(t=-0.3), dict(t=0.1, st=0.3), dict(sv=-0.5), dict(sz=-0.1),
             dict(st=-0.1), dict(sz=1.5), dict(st=5e-4), dict(sz=5e-4), dict(st=5e-4, sz=5e-4),
             dict(v=0.0), dict(v=12.0), dict(v=-12.0), dict(a=0.05), dict(a=6.0), dict(sv=0.0),
             dict(z=0.1, sz=0.2), dict(z=0.9, sz=0.2), dict(t=0.05, st=0.1)]
    for e in edges:
        p = dict(base, **e)
        rows.append([p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"], 1e-4, 2, 2, 1,
                     1e-3])
        xs.append(np.concatenate([[0.6, -0.6, 0.0], x_vector(rng, dict(p, st=abs(p["st"]),
                                                                       t=abs(p["t"])), M - 3)]))
    params = np.array(rows, dtype=np.float64)
    X = np.array(xs, dtype=np.float64)
    Y = np.empty_like(X)
    for i, r in enumerate(params):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se = r
        for j, x in enumerate(X[i]):
            Y[i, j] = R.full_pdf(x, v, sv, a, z, sz, t, st, err, int(n_st), int(n_sz), int(ua), se)
    np.savez_compressed(os.path.join(HERE, "full_pdf_grid.npz"), params=params, x=X, y=Y,
                        keys=np.array(PKEYS))

    # 3. wiener_like totals + 4. pdf_array (mixture, logp) on the same sets
    wl_rows, wl_x, wl_y = [], [], []
    pa_rows, pa_y = [], []
    for i in range(0, params.shape[0], 3):
        r = params[i]
        for p_out, w_out in [(0.0, 0.1), (0.05, 0.1), (0.2, 0.5), (1.2, 0.1), (-0.1, 0.1)]:
            v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se = r
            tot = R.wiener_like(X[i], v, sv, a, z, sz, t, st, err, int(n_st), int(n_sz), int(ua),
                                se, p_out, w_out)
            wl_rows.append(list(r) + [p_out, w_out])
            wl_x.append(X[i])
            wl_y.append(tot)
        for logp, p_out, w_out in [(0, 0.05, 0.1), (1, 0.05, 0.1), (1, 0.0, 0.0)]:
            v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se = r
            y = R.pdf_array(X[i], v, sv, a, z, sz, t, st, err, logp, int(n_st), int(n_sz),
                            int(ua), se, p_out, w_out)
            pa_rows.append(list(r) + [p_out, w_out, logp, i])
            pa_y.append(y)
    np.savez_compressed(os.path.join(HERE, "wiener_like.npz"), params=np.array(wl_rows),
                        x=np.array(wl_x), y=np.array(wl_y),
                        keys=np.array(PKEYS + ["p_outlier", "w_outlier"]))
    np.savez_compressed(os.path.join(HERE, "pdf_array.npz"), params=np.array(pa_rows),
                        y=np.array(pa_y),
                        keys=np.array(PKEYS + ["p_outlier", "w_outlier", "logp", "grid_row"]))

    # 5. model-sampled datasets: pinned (test_models.py:18,71) and stress
    ds = {}
    pinned = dict(v=0.5, a=2.0, z=0.5, t=0.3, sv=0.1, sz=0.1, st=0.1)
    rng5 = np.random.default_rng(20261015)
    x_p = gen_rts_restated(R, rng5, pinned, 4096)
    ds["pinned_x"] = x_p
    ds["pinned_params"] = np.array([pinned[k] for k in ["v", "sv", "a", "z", "sz", "t", "st"]])
    ds["pinned_logp"] = R.pdf_array(x_p, pinned["v"], pinned["sv"], pinned["a"], pinned["z"],
                                    pinned["sz"], pinned["t"], pinned["st"], 1e-4, 1, 2, 2, 1,
                                    1e-3, 0.05, 0.1)
    ds["pinned_total"] = np.array(R.wiener_like(x_p, pinned["v"], pinned["sv"], pinned["a"],
                                                pinned["z"], pinned["sz"], pinned["t"],
                                                pinned["st"], 1e-4, 2, 2, 1, 1e-3, 0.05, 0.1))
    rng6 = np.random.default_rng(20261016)
    sx, sp, sl = [], [], []
    for k in range(8):
        p = stress_params(rng6, "sv sz st")
        x = gen_rts_restated(R, rng6, p, 512)
        sx.append(x)
        sp.append([p[kk] for kk in ["v", "sv", "a", "z", "sz", "t", "st"]])
        sl.append(R.pdf_array(x, p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"],
                              1e-4, 1, 2, 2, 1, 1e-3, 0.05, 0.1))
    ds["stress_x"] = np.array(sx)
    ds["stress_params"] = np.array(sp)
    ds["stress_logp"] = np.array(sl)
    np.savez_compressed(os.path.join(HERE, "datasets.npz"), **ds)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    main(ap.parse_args().reference)
