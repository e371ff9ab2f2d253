"""Parity of the MI355X kernels (through the C ABI) with the reference.

Bar (BASELINE.json north_star): |log p_gpu - log p_ref| < 1e-6 per trial.
Exact zeros and NaNs must match exactly (they are decisions, not roundings).
Totals are compared against math.fsum of the reference's per-trial values with
a relative tolerance, because the reference sums sequentially and the GPU sums
by a fixed tree (SURVEY.md §7 hard part 5).
"""
import math
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOGP_TOL = 1e-6     # per trial, absolute, on log densities (north_star)
TOTAL_RTOL = 1e-11  # totals, relative to sum |log p|


def assert_density_parity(gpu, ref, what=""):
    """Per-trial densities: |log p_gpu - log p_ref| < 1e-6 for every positive
    reference density, subnormal ones included (no relaxation); zeros, NaNs
    and signs match exactly; negative densities (the large-time series can
    dip below zero) agree in log|p| to the same bar."""
    gpu = np.asarray(gpu, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert gpu.shape == ref.shape
    nan_r, nan_g = np.isnan(ref), np.isnan(gpu)
    assert np.array_equal(nan_r, nan_g), f"{what}: NaN pattern differs at {np.flatnonzero(nan_r != nan_g)[:10]}"
    zr, zg = ref == 0, gpu == 0
    bad = np.flatnonzero(zr != zg)
    assert bad.size == 0, f"{what}: zero pattern differs at {bad[:10]} ref={ref[bad[:5]]} " \
                          f"gpu={gpu[bad[:5]]}"
    nz = ~nan_r & ~zr
    assert np.array_equal(np.sign(gpu[nz]), np.sign(ref[nz])), f"{what}: sign differs"
    with np.errstate(divide="ignore"):
        d = np.abs(np.log(np.abs(gpu[nz])) - np.log(np.abs(ref[nz])))
    if d.size:
        k = int(np.argmax(d))
        assert d[k] < LOGP_TOL, f"{what}: max |dlogp| = {d[k]:.3e} (ref {ref[nz][k]:.6e}, " \
                                f"gpu {gpu[nz][k]:.6e})"


def assert_logp_parity(gpu, ref, what=""):
    """|dlogp| < 1e-6 per trial, everywhere (log densities of subnormal
    densities included); NaN and -inf patterns exact."""
    gpu = np.asarray(gpu, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert np.array_equal(np.isnan(gpu), np.isnan(ref)), f"{what}: NaN pattern"
    assert np.array_equal(np.isneginf(gpu), np.isneginf(ref)), f"{what}: -inf pattern"
    fin = np.isfinite(ref)
    d = np.abs(gpu[fin] - ref[fin])
    if d.size:
        k = int(np.argmax(d))
        assert d[k] < LOGP_TOL, f"{what}: max |dlogp| = {d[k]:.3e} (ref {ref[fin][k]:.6e})"


def assert_total(gpu, ref_terms, what=""):
    ref_terms = np.asarray(ref_terms)
    if np.isnan(ref_terms).any():
        assert np.isnan(gpu), what
        return
    if np.isneginf(ref_terms).any():
        assert gpu == -np.inf, what
        return
    ref = math.fsum(ref_terms)
    scale = max(math.fsum(np.abs(ref_terms)), 1.0)
    assert abs(gpu - ref) <= TOTAL_RTOL * scale + 1e-9, f"{what}: {gpu} vs {ref}"


# --------------------------------------------------------------------------- fixtures

def test_golden_full_pdf_grid(gpu, golden):
    g = golden["full_pdf_grid"]
    for i, r in enumerate(g["params"]):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se = r
        got = np.array([gpu.full_pdf(x, v, sv, a, z, sz, t, st, err, int(n_st), int(n_sz),
                                     int(ua), se) for x in g["x"][i]])
        assert_density_parity(got, g["y"][i], f"grid row {i} params={r}")


def test_golden_pdf_array(gpu, golden):
    g, grid = golden["pdf_array"], golden["full_pdf_grid"]
    for r, y in zip(g["params"], g["y"]):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se, p_out, w_out, logp, row = r
        x = grid["x"][int(row)]
        got = gpu.pdf_array(x, v, sv, a, z, sz, t, st, err, int(logp), int(n_st), int(n_sz),
                            int(ua), se, p_out, w_out)
        if int(logp):
            assert_logp_parity(got, y, f"pdf_array logp row {row}")
        else:
            assert_density_parity(got, y, f"pdf_array row {row}")


def test_golden_wiener_like(gpu, golden):
    g = golden["wiener_like"]
    for r, x, y in zip(g["params"], g["x"], g["y"]):
        v, sv, a, z, sz, t, st, err, n_st, n_sz, ua, se, p_out, w_out = r
        got = gpu.wiener_like(x, v, sv, a, z, sz, t, st, err, int(n_st), int(n_sz), int(ua), se,
                              p_out, w_out)
        if np.isnan(y):
            assert np.isnan(got)
        elif np.isinf(y):
            assert got == y
        else:
            assert abs(got - y) <= 1e-11 * max(abs(y), 1.0), (r, got, y)


def test_golden_datasets(gpu, golden):
    d = golden["datasets"]
    v, sv, a, z, sz, t, st = d["pinned_params"]
    got = gpu.pdf_array(d["pinned_x"], v, sv, a, z, sz, t, st, 1e-4, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
    assert_logp_parity(got, d["pinned_logp"], "pinned")
    tot = gpu.wiener_like(d["pinned_x"], v, sv, a, z, sz, t, st, 1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    assert_total(tot, d["pinned_logp"], "pinned total")
    assert abs(tot - float(d["pinned_total"])) < 1e-9 * abs(float(d["pinned_total"]))
    for x, p, lp in zip(d["stress_x"], d["stress_params"], d["stress_logp"]):
        v, sv, a, z, sz, t, st = p
        got = gpu.pdf_array(x, v, sv, a, z, sz, t, st, 1e-4, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
        assert_logp_parity(got, lp, f"stress {p}")
        ds = gpu.Dataset(x)
        tot = ds.wiener_like(v, sv, a, z, sz, t, st, 1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
        assert_total(tot, lp, "stress dataset total")


# --------------------------------------------------------------------------- oracle, random

FAMILIES = {
    "simple": dict(sv=0, sz=0, st=0),
    "sv": dict(sz=0, st=0),
    "sz": dict(sv=0, st=0),
    "st": dict(sv=0, sz=0),
    "sz_st": dict(sv=0),
    "full": dict(),
}


@pytest.mark.parametrize("fam", list(FAMILIES))
def test_oracle_random_families(gpu, oracle_lib, fam):
    rng = np.random.default_rng(zlib.crc32(fam.encode()))
    for rep in range(6):
        p = dict(v=rng.uniform(-4, 4), a=rng.uniform(0.5, 2), t=rng.uniform(0.2, 0.5),
                 z=rng.uniform(0.4, 0.6), sv=rng.uniform(0, 2.5), sz=rng.uniform(0, 0.4),
                 st=rng.uniform(0, 0.35))
        p.update(FAMILIES[fam])
        n = 4000
        x = rng.choice([-1.0, 1.0], n) * rng.uniform(0.0, 4.0, n)
        args = (p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"])
        for knobs in [(1e-4, 2, 2, 1, 1e-3), (1e-8, 4, 4, 1, 1e-6), (1e-4, 6, 6, 0, 1e-3)]:
            err, n_st, n_sz, ua, se = knobs
            ref = oracle_lib.pdf_array(x, *args, err, 0, n_st, n_sz, ua, se, 0, 0)
            got = gpu.pdf_array(x, *args, err, 0, n_st, n_sz, ua, se, 0, 0)
            assert_density_parity(got, ref, f"{fam} {p} {knobs}")
            ref_l = oracle_lib.pdf_array(x, *args, err, 1, n_st, n_sz, ua, se, 0.05, 0.1)
            tot = gpu.wiener_like(x, *args, err, n_st, n_sz, ua, se, 0.05, 0.1)
            assert_total(tot, ref_l, f"{fam} total")


def test_pinned_full_ddm_large(gpu, oracle_lib):
    """Config-3 parameters (test_models.py:18,71), 200k model-shaped RTs."""
    rng = np.random.default_rng(20261015)
    n = 200_000
    x = np.sign(rng.uniform(-0.27, 0.73, n)) * (0.3 + rng.gamma(2.0, 0.45, n))
    args = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    ref = oracle_lib.pdf_array(x, *args, 1e-4, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
    got = gpu.pdf_array(x, *args, 1e-4, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
    assert_logp_parity(got, ref, "pinned 200k")
    ds = gpu.Dataset(x)
    assert_total(ds.wiener_like(*args, 1e-4, 2, 2, 1, 1e-3, 0.05, 0.1), ref, "pinned dataset")


# --------------------------------------------------------------------------- semantics

def test_edge_semantics(gpu):
    args = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)
    assert gpu.wiener_like(np.array([], dtype=np.float64), *args, 1e-4) == 0.0
    x = np.array([0.8, -0.9, 1.2])
    assert gpu.wiener_like(x, *args, 1e-4, p_outlier=1.5) == -np.inf
    assert gpu.wiener_like(x, *args, 1e-4, p_outlier=-0.1) == -np.inf
    assert gpu.wiener_like(np.array([0.8, 0.1]), *args, 1e-4) == -np.inf  # rt < t
    # zero density dominates a NaN elsewhere? (a == 0 gives NaN everywhere)
    assert np.isnan(gpu.wiener_like(x, 0.5, 0.0, 0.0, 0.5, 0.0, 0.3, 0.0, 1e-4))
    # with outliers a zero-density trial is finite
    assert np.isfinite(gpu.wiener_like(np.array([0.8, 0.1]), *args, 1e-4, p_outlier=0.05))
    with pytest.raises(TypeError):
        gpu.wiener_like([0.8, 0.9], *args, 1e-4)
    with pytest.raises(ValueError):
        gpu.wiener_like(np.array([0.8, 0.9], dtype=np.float32), *args, 1e-4)
    with pytest.raises(ValueError):
        gpu.wiener_like(np.ones((2, 2)), *args, 1e-4)


def test_depth_overflow_fails_loudly(gpu):
    x = np.array([0.35, 0.9, -1.3])
    # simps_err=0 refines every interval: the leftmost path hits the stack cap
    # at once and the call must fail, not hang and not return a number.
    with pytest.raises(NotImplementedError):
        gpu.wiener_like(x, 0.5, 0.3, 2.0, 0.5, 0.3, 0.3, 0.0, 1e-10, n_st=40, n_sz=40,
                        simps_err=0.0)
    with pytest.raises(NotImplementedError):
        gpu.wiener_like(x, 0.5, 0.3, 2.0, 0.5, 0.3, 0.3, 0.3, 1e-10, n_st=40, n_sz=40,
                        simps_err=0.0)
    # legal but heavy: the reference's own test_pdf_integrate_to_one knobs
    assert np.isfinite(gpu.wiener_like(x, 0.5, 0.3, 2.0, 0.5, 0.3, 0.3, 0.3, 1e-8))


def test_dataset_order_invariance_and_additivity(gpu, oracle_lib):
    rng = np.random.default_rng(7)
    n = 300_000
    x = rng.choice([-1.0, 1.0], n) * (0.3 + rng.gamma(2.0, 0.45, n))
    args = (0.8, 0.3, 1.6, 0.45, 0.0, 0.25, 0.0)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    full = gpu.Dataset(x).wiener_like(*args, *kn)
    perm = gpu.Dataset(x[rng.permutation(n)]).wiener_like(*args, *kn)
    parts = sum(gpu.Dataset(c).wiener_like(*args, *kn) for c in np.array_split(x, 7))
    host = gpu.wiener_like(x, *args, *kn)
    ref = oracle_lib.pdf_array(x, *args, kn[0], 1, kn[1], kn[2], kn[3], kn[4], kn[5], kn[6])
    for val in (full, perm, parts, host):
        assert_total(val, ref, "order/additivity")


@pytest.mark.parametrize("n", [1000, 70_000, 300_000])
def test_stored_order_is_the_stable_comparator_order(gpu, n):
    """wfpt_dataset_create's stored order (radix sort above 64k trials, the
    comparator sort below) is the stable sort by (boundary, |rt|, NaN last),
    ties in input order; node datasets: by node, then |rt|. Inputs carry ties,
    +-0, +-inf and NaNs (several payloads)."""
    rng = np.random.default_rng(n)
    x = np.round(rng.choice([-1.0, 1.0], n) * (0.3 + rng.gamma(2.0, 0.45, n)), 3)
    k = max(n // 50, 4)
    pos = rng.choice(n, 4 * k, replace=False)
    x[pos[:k]] = np.nan
    x[pos[k:k + 4]] = [0.0, -0.0, np.inf, -np.inf]
    bits = x.view(np.uint64)
    bits[pos[k + 4:2 * k]] |= 0x8000000000000000  # negative zero / sign flips
    x[pos[2 * k:2 * k + 8]] = np.frombuffer(np.array(
        [0x7ff8000000000001 + j for j in range(8)], dtype=np.uint64).tobytes(), dtype=np.float64)
    nan = np.isnan(x)
    ab = np.where(nan, 0.0, np.abs(x))
    want = np.lexsort((np.arange(n), ab, nan, x > 0))
    assert np.array_equal(gpu.Dataset(x).order(), want)
    node = rng.integers(0, 97, n).astype(np.int32)
    want_n = np.lexsort((np.arange(n), ab, nan, node))
    assert np.array_equal(gpu.Dataset(x, node_id=node, n_nodes=97).order(), want_n)


def test_nodes_match_per_node_wiener_like(gpu, oracle_lib):
    rng = np.random.default_rng(11)
    n_nodes = 37
    sizes = rng.integers(0, 400, n_nodes)
    node = np.repeat(np.arange(n_nodes), sizes)
    rng.shuffle(node)
    x = rng.choice([-1.0, 1.0], node.size) * (0.35 + rng.gamma(2.0, 0.4, node.size))
    P = np.zeros((n_nodes, 8))
    P[:, 0] = rng.uniform(-2, 2, n_nodes)
    P[:, 1] = rng.choice([0.0, 0.4], n_nodes)
    P[:, 2] = rng.uniform(0.8, 2.0, n_nodes)
    P[:, 3] = rng.uniform(0.4, 0.6, n_nodes)
    P[:, 4] = rng.choice([0.0, 0.1], n_nodes)
    P[:, 5] = rng.uniform(0.2, 0.33, n_nodes)
    P[:, 6] = rng.choice([0.0, 0.1], n_nodes)
    P[:, 7] = 0.05
    P[3, 7] = 1.5  # out-of-range p_outlier => -inf for that node
    ds = gpu.Dataset(x, node_id=node, n_nodes=n_nodes)
    got = ds.wiener_like_nodes(P, 1e-4, 2, 2, 1, 1e-3, 0.1)
    for j in range(n_nodes):
        xj = x[node == j]
        v, sv, a, z, sz, t, st, po = P[j]
        ref = oracle_lib.wiener_like(xj, v, sv, a, z, sz, t, st, 1e-4, 2, 2, 1, 1e-3, po, 0.1)
        if not np.isfinite(ref):
            assert got[j] == ref
        else:
            terms = oracle_lib.pdf_array(xj, v, sv, a, z, sz, t, st, 1e-4, 1, 2, 2, 1, 1e-3, po,
                                         0.1)
            assert_total(got[j], terms, f"node {j}")


def test_wiener_like_multi(gpu, oracle_lib):
    rng = np.random.default_rng(13)
    n = 5000
    x = rng.choice([-1.0, 1.0], n) * (0.4 + rng.gamma(2.0, 0.4, n))
    x[::97] = 999.0
    x[::89] = -999.0
    v = rng.uniform(-1, 1, n)
    a = rng.uniform(1.0, 2.0, n)
    for kw in [dict(multi=["v", "a"]), dict(multi=["v"])]:
        aa = a if "a" in kw["multi"] else 1.5
        ref = oracle_lib.wiener_like_multi(x, v, 0.2, aa, 0.5, 0.1, 0.3, 0.1, 1e-4,
                                           multi=kw["multi"], n_st=2, n_sz=2, p_outlier=0.05,
                                           w_outlier=0.1)
        got = gpu.wiener_like_multi(x, v, 0.2, aa, 0.5, 0.1, 0.3, 0.1, 1e-4, multi=kw["multi"],
                                    n_st=2, n_sz=2, p_outlier=0.05, w_outlier=0.1)
        assert abs(got - ref) < 1e-9 * abs(ref)


@pytest.mark.parametrize("case", ["adapt_tz", "direct", "adapt_t", "adapt_z", "generic_sz",
                                  "heavy"])
def test_wiener_like_multi_families(gpu, oracle_lib, case):
    """wiener_like_multi's level-0 fast path for every uniform family (sz, st
    scalar) incl. a refinement-heavy parameter set (deferred records), and the
    generic per-trial kernel (sz per trial); host and resident datasets; the
    +-999 missing responses. Total vs the reference restated (oracle, pinned to
    the reference's kernels), relative 1e-10."""
    rng = np.random.default_rng(17)
    n = 20000
    x = rng.choice([-1.0, 1.0], n) * (0.3 + rng.gamma(2.0, 0.4, n))
    x[::101] = 999.0
    x[::103] = -999.0
    v = rng.uniform(-1.5, 1.5, n)
    a = rng.uniform(0.8, 2.2, n)
    z = rng.uniform(0.4, 0.6, n)
    sz_arr = rng.uniform(0.0, 0.3, n)
    base = dict(v=v, sv=0.3, a=a, z=0.5, sz=0.1, t=0.25, st=0.1)
    multi = ["v", "a"]
    kn = dict(n_st=2, n_sz=2, simps_err=1e-3, p_outlier=0.05, w_outlier=0.1)
    if case == "direct":
        base.update(sz=0.0, st=0.0, sv=0.0)
    elif case == "adapt_t":
        base.update(sz=0.0)
    elif case == "adapt_z":
        base.update(st=0.0, z=z)
        multi = ["v", "a", "z"]
    elif case == "generic_sz":
        base.update(sz=sz_arr)
        multi = ["v", "a", "sz"]
    elif case == "heavy":
        base.update(sv=2.0, sz=0.35, st=0.3)
        kn.update(simps_err=1e-6, n_st=4, n_sz=4)
        x = np.where(np.abs(x) < 998, np.sign(x) * (0.16 + 0.3 * rng.random(n)), x)
    args = [base[k] for k in ("v", "sv", "a", "z", "sz", "t", "st")]
    ref = oracle_lib.wiener_like_multi(x, *args, 1e-4, multi=multi, **kn)
    tol = 1e-10 * abs(ref)  # every term is negative: |sum| = sum |terms|
    got = gpu.wiener_like_multi(x, *args, 1e-4, multi=multi, **kn)
    assert np.isfinite(ref) and abs(got - ref) <= tol, (case, got, ref)
    ds = gpu.Dataset(x, input_order=True)
    got2 = ds.wiener_like_multi(*args, 1e-4, multi, **kn)
    assert got2 == got, (got2, got)
    with pytest.raises(ValueError):
        gpu.Dataset(x).wiener_like_multi(*args, 1e-4, multi, **kn)


def test_gen_rts_from_cdf(gpu):
    np.random.seed(5)
    rts = gpu.gen_rts_from_cdf(0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, samples=20000, dt=1e-3)
    assert rts.shape == (20000,)
    assert np.all(np.abs(rts) >= 0.25)
    # P(upper) = prob_ub (pdf.pxi:67-72) = 0.731 for v=.5, a=2, z=.5
    assert abs(np.mean(rts > 0) - gpu.prob_ub(0.5, 2.0, 0.5)) < 0.02


@pytest.mark.parametrize("family", ["full", "simple", "sz_only", "st_only"])
def test_nodes_uniform_family_fast_path(gpu, oracle_lib, family):
    """Every node selects the same integration family (the HDDM case: sv/sz/st
    are group-level), so wfpt_wiener_like_nodes takes the two-pass per-node
    fast path; per-node sums must match the reference per node."""
    rng = np.random.default_rng(29)
    n_nodes = 53
    sizes = rng.integers(1, 300, n_nodes)
    sizes[7] = 0  # an empty node between non-empty ones
    node = np.repeat(np.arange(n_nodes), sizes)
    rng.shuffle(node)
    x = rng.choice([-1.0, 1.0], node.size) * (0.25 + rng.gamma(2.0, 0.4, node.size))
    P = np.zeros((n_nodes, 8))
    P[:, 0] = rng.uniform(-2, 2, n_nodes)
    P[:, 2] = rng.uniform(0.8, 2.0, n_nodes)
    P[:, 3] = rng.uniform(0.4, 0.6, n_nodes)
    P[:, 5] = rng.uniform(0.2, 0.33, n_nodes)
    P[:, 7] = 0.05
    if family == "full":
        P[:, 1], P[:, 4], P[:, 6] = 0.6, 0.25, 0.2  # wide sz/st: some trials refine (slow pass)
    elif family == "sz_only":
        P[:, 4] = 0.3
    elif family == "st_only":
        P[:, 6] = 0.25
    P[3, 7] = 1.5    # out-of-range p_outlier => -inf for that node
    P[5, 7] = 0.0    # no outliers: trials below t - st/2 give -inf
    ds = gpu.Dataset(x, node_id=node, n_nodes=n_nodes)
    got = ds.wiener_like_nodes(P, 1e-4, 2, 2, 1, 1e-3, 0.1)
    for j in range(n_nodes):
        xj = x[node == j]
        v, sv, a, z, sz, t, st, po = P[j]
        ref = oracle_lib.wiener_like(xj, v, sv, a, z, sz, t, st, 1e-4, 2, 2, 1, 1e-3, po, 0.1)
        if not np.isfinite(ref):
            assert got[j] == ref, (j, got[j], ref)
        else:
            terms = oracle_lib.pdf_array(xj, v, sv, a, z, sz, t, st, 1e-4, 1, 2, 2, 1, 1e-3, po,
                                         0.1)
            assert_total(got[j], terms, f"{family} node {j}")


# --------------------------------------------------------------------------- resident sizes

def test_resident_sizes_and_repeats(gpu, oracle_lib):
    """Resident wiener_like across sizes that straddle the 64-trial chunk, the
    256-trial block and the finalize stride; repeated and interleaved calls
    must return bit-identical totals (workspace words are zero at rest)."""
    rng = np.random.default_rng(20261016)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    pinned = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    stress = (-2.5, 2.2, 0.6, 0.45, 0.35, 0.25, 0.3)  # deep adaptive refinement
    sets = []
    for n in (1, 63, 64, 65, 255, 257, 16_383, 16_384, 16_385, 1_048_577, 1_100_001):
        x = rng.choice([-1.0, 1.0], n) * (0.3 + rng.gamma(2.0, 0.45, n))
        sets.append((gpu.Dataset(x), x))
    for args in (pinned, stress, (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0),
                 (0.7, 0.4, 1.5, 0.5, 0.0, 0.3, 0.0)):
        want = {}
        for ds, x in sets:
            host = gpu.wiener_like(x, *args, *kn)
            got = ds.wiener_like(*args, *kn)
            if ds.n < 100_000:  # the big sizes: vs the (parity-tested) host path
                ref = oracle_lib.pdf_array(x, *args, kn[0], 1, *kn[1:5], kn[5], kn[6])
                assert_total(got, ref, f"resident n={ds.n} {args}")
            assert abs(got - host) <= 1e-11 * max(abs(host), 1.0), (ds.n, got, host)
            want[ds.n] = got
        for rep in range(40):
            ds, _ = sets[rep % len(sets)]
            assert ds.wiener_like(*args, *kn) == want[ds.n], (rep, ds.n)
    # semantics: a zero-density trial, NaN parameters (a == 0)
    ds = gpu.Dataset(np.array([0.8, 0.1, -0.9] * 5000))
    assert ds.wiener_like(0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0, 1e-4) == -np.inf
    assert np.isfinite(ds.wiener_like(0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0, 1e-4, p_outlier=0.05))
    assert ds.wiener_like(0.5, 0.0, 0.0, 0.5, 0.0, 0.3, 0.0, 1e-4) == -np.inf  # zero beats NaN
    assert np.isnan(gpu.Dataset(np.array([0.8, -0.9] * 5000)).wiener_like(
        0.5, 0.0, 0.0, 0.5, 0.0, 0.3, 0.0, 1e-4))


def test_resident_fast_only_prediction(gpu, oracle_lib):
    """A resident dataset whose last call deferred no trial runs the level-0 pass
    + finalize only (run_sum_fast in wfpt_capi.cpp); when that prediction is
    wrong the slow pass runs after all. Alternating deferring / non-deferring
    parameters on one dataset exercises both transitions; every result must
    equal the host-array path (always the full sequence) and the oracle."""
    rng = np.random.default_rng(20261018)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    pinned = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    stress = (-2.5, 2.2, 0.6, 0.45, 0.35, 0.25, 0.3)
    st_only = (0.8, 0.0, 1.6, 0.45, 0.0, 0.25, 0.2)
    sz_only = (0.8, 0.0, 1.6, 0.45, 0.3, 0.25, 0.0)
    for n in (65, 20_000, 300_001):
        x = rng.choice([-1.0, 1.0], n) * (0.3 + rng.gamma(2.0, 0.45, n))
        ds = gpu.Dataset(x)
        seq = [pinned, pinned, stress, stress, pinned, pinned, st_only, sz_only, stress, pinned]
        for args in seq:
            got = ds.wiener_like(*args, *kn)
            host = gpu.wiener_like(x, *args, *kn)
            assert abs(got - host) <= 1e-11 * max(abs(host), 1.0), (n, args, got, host)
            if n <= 20_000:
                ref = oracle_lib.pdf_array(x, *args, kn[0], 1, *kn[1:5], kn[5], kn[6])
                assert_total(got, ref, f"fast-only n={n} {args}")
    # a Simpson-stack overflow in a mispredicted call still fails loudly
    ds = gpu.Dataset(np.array([0.35, 0.9, -1.3]))
    assert np.isfinite(ds.wiener_like(0.5, 0.3, 2.0, 0.5, 0.3, 0.3, 0.3, 1e-8, n_st=2, n_sz=2,
                                      simps_err=1.0))
    with pytest.raises(NotImplementedError):
        ds.wiener_like(0.5, 0.3, 2.0, 0.5, 0.3, 0.3, 0.3, 1e-10, n_st=40, n_sz=40, simps_err=0.0)
