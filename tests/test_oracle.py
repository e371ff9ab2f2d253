"""The oracle is pinned before it is trusted (CPU, no GPU needed).

1. The C restatement is bit-exact against the reference's own kernels
   (oracle/_ref, built from /root/reference/src/pdf.pxi + integrate.pxi) on the
   committed golden vectors, which were generated from oracle/_ref.
2. Both reproduce the 20 Navarro-Fuss MATLAB tuples (matlab_values.py) to 1e-9.
"""
import numpy as np
import pytest


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.array_equal(a, b) or np.array_equal(np.isnan(a), np.isnan(b)) and \
        np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)])


def test_matlab_values(oracle_lib, golden):
    m = golden["matlab"]
    for (v, t, a, z, _zn, rt, err, matlab), ref_val in zip(m["vals"], m["reference_full_pdf"]):
        mine = oracle_lib.full_pdf(-rt, v, 0, a, z, 0, t, 0, err, 0)
        assert abs(mine - matlab) < 1e-9
        assert mine == ref_val  # bit-exact with the reference kernels


def test_full_pdf_grid_bit_exact(oracle_lib, golden):
    g = golden["full_pdf_grid"]
    for i, r in enumerate(g["params"]):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se = r
        got = [oracle_lib.full_pdf(x, v, sv, a, z, sz, t, st, err, int(n_st), int(n_sz), int(ua),
                                   se) for x in g["x"][i]]
        assert _same(got, g["y"][i]), f"row {i}"


def test_wiener_like_bit_exact(oracle_lib, golden):
    g = golden["wiener_like"]
    for r, x, y in zip(g["params"], g["x"], g["y"]):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se, p_out, w_out = r
        got = oracle_lib.wiener_like(x, v, sv, a, z, sz, t, st, err, int(n_st), int(n_sz),
                                     int(ua), se, p_out, w_out)
        assert _same(got, y)


def test_pdf_array_bit_exact(oracle_lib, golden):
    g, grid = golden["pdf_array"], golden["full_pdf_grid"]
    for r, y in zip(g["params"], g["y"]):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se, p_out, w_out, logp, row = r
        with np.errstate(divide="ignore"):
            got = oracle_lib.pdf_array(grid["x"][int(row)], v, sv, a, z, sz, t, st, err,
                                       int(logp), int(n_st), int(n_sz), int(ua), se, p_out, w_out)
        assert _same(got, y)


def test_datasets_bit_exact(oracle_lib, golden):
    d = golden["datasets"]
    v, sv, a, z, sz, t, st = d["pinned_params"]
    got = oracle_lib.pdf_array(d["pinned_x"], v, sv, a, z, sz, t, st, 1e-4, 1, 2, 2, 1, 1e-3,
                               0.05, 0.1)
    assert _same(got, d["pinned_logp"])
    tot = oracle_lib.wiener_like(d["pinned_x"], v, sv, a, z, sz, t, st, 1e-4, 2, 2, 1, 1e-3,
                                 0.05, 0.1)
    assert tot == float(d["pinned_total"])
    for x, p, lp in zip(d["stress_x"], d["stress_params"], d["stress_logp"]):
        got = oracle_lib.pdf_array(x, *p, 1e-4, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
        assert _same(got, lp)


def test_oracle_vs_reference_random(oracle_lib, ref):
    """Fresh random draws, every branch family and knob, against oracle/_ref."""
    rng = np.random.default_rng(99)
    for _ in range(1500):
        v, a, t, z = rng.uniform(-5, 5), rng.uniform(0.3, 2.5), rng.uniform(0.1, 0.5), \
            rng.uniform(0.2, 0.8)
        sv = rng.choice([0.0, rng.uniform(0, 3)])
        sz = rng.choice([0.0, 5e-4, rng.uniform(0, 0.4)])
        st = rng.choice([0.0, 5e-4, rng.uniform(0, 0.4)])
        err = 10 ** rng.uniform(-12, 0)
        n = int(rng.integers(0, 7))
        ua = int(rng.integers(0, 2))
        if ua == 0 and n == 0:
            n = 2
        se = 10 ** rng.uniform(-8, -1)
        x = rng.choice([-1, 1]) * rng.uniform(0, 3)
        a1 = ref.full_pdf(x, v, sv, a, z, sz, t, st, err, n, n, ua, se)
        a2 = oracle_lib.full_pdf(x, v, sv, a, z, sz, t, st, err, n, n, ua, se)
        assert _same(a1, a2), (x, v, sv, a, z, sz, t, st, err, n, ua, se)


def test_multi_restatement(oracle_lib, ref):
    """wiener_like_multi restated (wfpt.pyx:244-274) vs per-trial reference full_pdf."""
    rng = np.random.default_rng(3)
    n = 300
    x = rng.choice([-1.0, 1.0], n) * rng.uniform(0.4, 2.5, n)
    x[::37] = 999.0
    x[::41] = -999.0
    v = rng.uniform(-2, 2, n)
    got = oracle_lib.wiener_like_multi(x, v, 0.2, 1.5, 0.5, 0.1, 0.3, 0.1, 1e-4, multi=["v"],
                                       n_st=2, n_sz=2, p_outlier=0.05, w_outlier=0.1)
    s = 0.0
    for i in range(n):
        if abs(x[i]) != 999.0:
            p = ref.full_pdf(x[i], v[i], 0.2, 1.5, 0.5, 0.1, 0.3, 0.1, 1e-4, 2, 2, 1, 1e-3)
            p = p * (1 - 0.05) + 0.1 * 0.05
        elif x[i] == 999.0:
            p = ref.ref_prob_ub(v[i], 1.5, 0.5)
        else:
            p = 1 - ref.ref_prob_ub(v[i], 1.5, 0.5)
        s += np.log(p)
    assert got == s
