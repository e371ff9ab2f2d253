"""Per-trial parity wherever a total is claimed, and the series decisions at
their boundaries (VERDICT r02 "do this" #1).

* Per-node (wfpt_wiener_like_nodes_ex) and per-trial-parameter
  (wfpt_wiener_like_multi_ex) paths return each trial's log term; every term
  must be within |dlogp| < 1e-6 of the reference's (north_star bar), with
  -inf / NaN patterns exact — including the refinement-heavy families and
  config 4's own 200 x 500, 400-node dataset.
* The decisions of ftt_01w (src/pdf.pxi:36-60) — the small-time term count
  ks hitting an integer, the large-time kl hitting an integer, the
  small/large switch ks ~ kl, the clamps ks = max(ks, sqrt(tt) + 1) and
  kl = max(kl, 1/(pi sqrt(tt))) — with err placed within a few ulps of each
  boundary (found by bisection on the reference's own expressions, restated
  below with Python's libm, which is the reference's), checked at
  |dlogp| < 1e-12: a flipped decision moves the value by a whole series term.
  The 2-D family places the boundary on an interior t node, and a t grid
  straddling the peak of ks(tt) (args = 2 sqrt(2 pi tt) err = e^-1/2, err ~
  0.12, tt ~ 1) exercises the shared-decision shortcut (l0_hints).
"""
import math

import numpy as np
import pytest

from test_gpu_parity import assert_logp_parity

pytestmark = pytest.mark.gpu

KN = (1e-4, 2, 2, 1, 1e-3, 0.1)  # err, n_st, n_sz, use_adaptive, simps_err, w_outlier


def node_terms_ref(oracle_lib, x, node, P, kn=KN):
    """The reference's per-trial term of each node's wfpt_like (wfpt.pyx:63-72
    per node): log of the mixture, -inf for a zero density or a p_outlier
    outside [0, 1]."""
    out = np.empty(x.size)
    for j in range(P.shape[0]):
        m = node == j
        if not m.any():
            continue
        v, sv, a, z, sz, t, st, po = P[j]
        if not (0 <= po <= 1):
            out[m] = -np.inf
            continue
        out[m] = oracle_lib.pdf_array(x[m], v, sv, a, z, sz, t, st, kn[0], 1, kn[1], kn[2],
                                      kn[3], kn[4], po, kn[5])
    return out


def _node_dataset(rng, n_nodes, family, max_size=300):
    sizes = rng.integers(1, max_size, n_nodes)
    sizes[min(7, n_nodes - 1)] = 0
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
        P[:, 1], P[:, 4], P[:, 6] = 0.6, 0.25, 0.2
    elif family == "heavy":  # the engine records on most trials
        P[:, 1], P[:, 4], P[:, 6] = 2.0, 0.35, 0.3
        x = np.sign(x) * (0.2 + 0.3 * rng.random(node.size))
    elif family == "sz_only":
        P[:, 4] = 0.3
    elif family == "st_only":
        P[:, 6] = 0.25
    elif family == "mixed":
        P[:, 1] = rng.choice([0.0, 0.4], n_nodes)
        P[:, 4] = rng.choice([0.0, 0.1], n_nodes)
        P[:, 6] = rng.choice([0.0, 0.1], n_nodes)
    P[min(3, n_nodes - 1), 7] = 1.5  # out-of-range p_outlier => -inf terms
    P[min(5, n_nodes - 1), 7] = 0.0  # no outliers: trials below t - st/2 give -inf
    return x, node, P


@pytest.mark.parametrize("family", ["full", "heavy", "simple", "sz_only", "st_only", "mixed"])
def test_node_terms_per_trial(gpu, oracle_lib, family):
    rng = np.random.default_rng({"full": 1, "heavy": 2, "simple": 3, "sz_only": 4,
                                 "st_only": 5, "mixed": 6}[family])
    x, node, P = _node_dataset(rng, 41, family)
    ds = gpu.Dataset(x, node_id=node, n_nodes=P.shape[0])
    sums, terms = ds.wiener_like_nodes(P, *KN, trials=True)
    ref = node_terms_ref(oracle_lib, x, node, P)
    assert_logp_parity(terms, ref, f"{family} per-trial node terms")
    # the per-node sums are the sums of those terms (segment_sum_kernel)
    for j in range(P.shape[0]):
        tj = terms[node == j]
        if np.isneginf(tj).any():
            assert sums[j] == -np.inf
        elif tj.size:
            assert abs(sums[j] - math.fsum(tj)) <= 1e-12 * math.fsum(np.abs(tj)) + 1e-12
        else:
            assert sums[j] == 0.0
    # the same call without per-trial output gives the same sums, bit for bit
    assert np.array_equal(ds.wiener_like_nodes(P, *KN), sums, equal_nan=True)


def _ctx_env(env):
    import os
    from hddm_amd import _lib
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return _lib.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def node_variant_ctxs(gpu):
    """Contexts on the other node-path variants: the t-node split level 0
    (WFPT_NODE_SPLIT=1) and the breadth-first rounds for sparse deferred
    trials instead of the speculative records (WFPT_NODE_SPEC=0)."""
    ctxs = {"split": _ctx_env({"WFPT_NODE_SPLIT": "1"}),
            "rounds": _ctx_env({"WFPT_NODE_SPEC": "0"})}
    yield ctxs
    for c in ctxs.values():
        c.close()


@pytest.mark.parametrize("family", ["full", "heavy", "st_only", "c4_full"])
def test_node_path_variants_bit_identical(gpu, oracle_lib, node_variant_ctxs, family):
    """The batched node call's variants give every trial the same bits: the
    default (one lane per trial at level 0, sparse deferred trials as
    speculative records: node_record_spec evaluates every tree point in two
    rounds and keeps the flags of the points the recursion reads), the t-node
    split level 0 (node_split_kernel, five lanes per trial) and the
    breadth-first records (node_records); per trial against the reference at
    1e-6. The split context takes the split path (WFPT_PATH_NODE_SPLIT)."""
    from hddm_amd import _lib
    if family == "c4_full":
        from hddm_amd.hierarchical import HDDM, gen_data
        data, _ = gen_data(n_subj=200, n_trials=500, sv=0.1, sz=0.1, st=0.1)
        m = HDDM(data, depends_on={"v": "cond"}, include=("sv", "sz", "st"), p_outlier=0.05)
        x = data["rt"].to_numpy(dtype=np.float64)
        node = data.groupby(["subj_idx", "cond"], sort=True).ngroup().to_numpy()
        P = m.node_table()
        kn = (m.wp["err"], m.wp["n_st"], m.wp["n_sz"], m.wp["use_adaptive"], m.wp["simps_err"],
              m.wp["w_outlier"])
    else:
        rng = np.random.default_rng({"full": 11, "heavy": 12, "st_only": 13}[family])
        x, node, P = _node_dataset(rng, 57, family)
        kn = KN
    out = {}
    for name, ctx in (("default", _lib.context()), ("split", node_variant_ctxs["split"]),
                      ("rounds", node_variant_ctxs["rounds"])):
        ds = gpu.Dataset(x, node_id=node, n_nodes=P.shape[0], ctx=ctx)
        sums, terms = ds.wiener_like_nodes(P, *kn, trials=True)
        assert bool(ctx.last_path() & _lib.PATH_NODE_SPLIT) == (name == "split"), (name, family)
        assert np.array_equal(ds.wiener_like_nodes(P, *kn), sums, equal_nan=True)
        out[name] = (sums, terms)
        ds.close()
    for name in ("split", "rounds"):
        assert np.array_equal(out["default"][1], out[name][1], equal_nan=True), (family, name)
        assert np.array_equal(out["default"][0], out[name][0], equal_nan=True), (family, name)
    ref = node_terms_ref(oracle_lib, x, node, P, kn)
    assert_logp_parity(out["default"][1], ref, f"node path {family}")


@pytest.mark.parametrize("case", ["adapt_tz", "direct", "adapt_t", "adapt_z", "generic_sz",
                                  "heavy"])
def test_multi_terms_per_trial(gpu, oracle_lib, case):
    """wiener_like_multi per trial (wfpt.pyx:261-272) for every family the
    level-0 fast path serves, the refinement-heavy set (deferred records) and
    the generic per-trial kernel; host and resident inputs; +-999 trials."""
    rng = np.random.default_rng(17)
    n = 20000
    x = rng.choice([-1.0, 1.0], n) * (0.3 + rng.gamma(2.0, 0.4, n))
    x[::101] = 999.0
    x[::103] = -999.0
    v = rng.uniform(-1.5, 1.5, n)
    a = rng.uniform(0.8, 2.2, n)
    z = rng.uniform(0.4, 0.6, n)
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
        base.update(sz=rng.uniform(0.0, 0.3, n))
        multi = ["v", "a", "sz"]
    elif case == "heavy":
        base.update(sv=2.0, sz=0.35, st=0.3)
        kn.update(simps_err=1e-6, n_st=4, n_sz=4)
        x = np.where(np.abs(x) < 998, np.sign(x) * (0.16 + 0.3 * rng.random(n)), x)
    args = [base[k] for k in ("v", "sv", "a", "z", "sz", "t", "st")]
    ref_tot, ref = oracle_lib.wiener_like_multi(x, *args, 1e-4, multi=multi, terms=True, **kn)
    tot, terms = gpu.wiener_like_multi_terms(x, *args, 1e-4, multi, **kn)
    assert_logp_parity(terms, ref, f"multi {case}")
    assert abs(tot - ref_tot) <= 1e-10 * abs(ref_tot)
    ds = gpu.Dataset(x, input_order=True)
    tot2, terms2 = ds.wiener_like_multi(*args, 1e-4, multi, trials=True, **kn)
    assert tot2 == tot and np.array_equal(terms2, terms)


@pytest.mark.parametrize("full", [False, True])
def test_config4_dataset_per_node_and_per_trial(gpu, oracle_lib, full):
    """Config 4's own data: 200 subjects x 500 trials, depends_on v by two
    conditions = 400 nodes of 250 trials (hddm_amd.hierarchical.gen_data,
    seed 20261017), HDDM's knobs and p_outlier = .05; per trial at 1e-6 and
    per node against math.fsum of the reference's terms, at the generating
    parameters and at HDDM's starting values (hddm_info.py:121-140)."""
    from hddm_amd.hierarchical import HDDM, gen_data
    inter = dict(sv=0.1, sz=0.1, st=0.1) if full else {}
    data, truth = gen_data(n_subj=200, n_trials=500, **inter)
    m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05)
    assert m.n_nodes == 400 and m.n_trials == 100_000
    x = data["rt"].to_numpy(dtype=np.float64)
    # the model's node of each trial: one per (subject, condition) cell
    node = data.groupby(["subj_idx", "cond"], sort=True).ngroup().to_numpy()
    tables = [m.node_table()]  # HDDM's starting values
    P = m.node_table().copy()
    for j, (s, c) in enumerate(m.node_keys):
        P[j, 0] = truth["v"][c][s]
        P[j, 2] = truth["a"][s]
        P[j, 5] = truth["t"][s]
        for k, col in (("sv", 1), ("sz", 4), ("st", 6)):
            P[j, col] = inter.get(k, 0.0)
    tables.append(P)
    for T in tables:
        sums, terms = m.dataset.wiener_like_nodes(T, **m.wp, trials=True)
        ref = node_terms_ref(oracle_lib, x, node, T, (m.wp["err"], m.wp["n_st"], m.wp["n_sz"],
                                                      m.wp["use_adaptive"], m.wp["simps_err"],
                                                      m.wp["w_outlier"]))
        assert_logp_parity(terms, ref, f"C4 full={full}")
        for j in range(400):
            rj = ref[node == j]
            if np.isneginf(rj).any():
                assert sums[j] == -np.inf
            else:
                assert abs(sums[j] - math.fsum(rj)) <= 1e-11 * math.fsum(np.abs(rj)), j


# --------------------------------------------------------------------------- decisions

def ref_decision(tt, err):
    """(small, K, ks, kl, ks_raw, kl_raw) of ftt_01w (src/pdf.pxi:36-60), with
    the reference's operations and libm."""
    pi = math.pi
    if pi * tt * err < 1:
        kl_raw = math.sqrt(-2 * math.log(pi * tt * err) / (pi ** 2 * tt))
        kl = max(kl_raw, 1. / (pi * math.sqrt(tt)))
    else:
        kl_raw = kl = 1. / (pi * math.sqrt(tt))
    if 2 * math.sqrt(2 * pi * tt) * err < 1:
        ks_raw = 2 + math.sqrt(-2 * tt * math.log(2 * math.sqrt(2 * pi * tt) * err))
        ks = max(ks_raw, math.sqrt(tt) + 1)
    else:
        ks_raw = ks = 2
    small = ks < kl
    return small, int(math.ceil(ks if small else kl)), ks, kl, ks_raw, kl_raw


def _bisect_err(q, lo, hi, iters=200):
    """err in [lo, hi] (geometric) where the sign of q(err) changes, to the
    last bit: returns the err on the upper side of the change."""
    qlo = q(lo) > 0
    if (q(hi) > 0) == qlo:
        return None
    for _ in range(iters):
        mid = math.sqrt(lo * hi)
        if mid in (lo, hi):
            break
        if (q(mid) > 0) == qlo:
            lo = mid
        else:
            hi = mid
        if math.nextafter(lo, math.inf) >= hi:
            break
    return hi


def _nudges(val, k=6):
    out, lo, hi = [val], val, val
    for _ in range(k):
        lo, hi = math.nextafter(lo, -math.inf), math.nextafter(hi, math.inf)
        out += [lo, hi]
    return out


BOUNDARIES = {
    # quantity whose sign change is the boundary; branch the quantity decides
    "ks_integer": [(lambda tt, K: (lambda e: ref_decision(tt, e)[4] - K)), (3, 4, 5)],
    "kl_integer": [(lambda tt, K: (lambda e: ref_decision(tt, e)[5] - K)), (1, 2, 3)],
    "switch": [(lambda tt, K: (lambda e: ref_decision(tt, e)[2] - ref_decision(tt, e)[3])), (0,)],
    "ks_clamp": [(lambda tt, K: (lambda e: ref_decision(tt, e)[4] - (math.sqrt(tt) + 1))), (0,)],
    "kl_clamp": [(lambda tt, K: (lambda e: ref_decision(tt, e)[5] -
                                 1. / (math.pi * math.sqrt(tt)))), (0,)],
}


def _boundary_points(kind):
    """(tt, err) pairs within ulps of the `kind` boundary, over a tt grid."""
    mk, Ks = BOUNDARIES[kind]
    pts = []
    for tt0 in (0.004, 0.01, 0.03, 0.06, 0.1, 0.2, 0.35, 0.6, 1.0, 2.0, 4.0):
        # tt as the kernel forms it: |x| - t with t = 0.25, a = 1 (pdf.pxi:98)
        t = 0.25
        x = t + tt0
        tt = x - t
        for K in Ks:
            e = _bisect_err(mk(tt, K), 1e-14, 50.0)
            if e is None:
                continue
            for err in _nudges(e):
                pts.append((x, tt, err))
    return pts


@pytest.mark.parametrize("kind", sorted(BOUNDARIES))
@pytest.mark.parametrize("sv", [0.0, 0.6])
def test_series_decision_boundaries(gpu, oracle_lib, kind, sv):
    """Direct family (one pdf_sv per trial): err within 6 ulps of each decision
    boundary of ftt_01w; the library must take the reference's decision (fp32
    estimate ambiguous -> fp64 operations -> exact path within 1e-12)."""
    pts = _boundary_points(kind)
    assert len(pts) >= 13, (kind, len(pts))
    flips = 0
    for x, tt, err in pts:
        for w in (0.3, 0.5, 0.7):
            args = (0.4, sv, 1.0, w, 0.0, 0.25, 0.0, err)
            want = oracle_lib.full_pdf(-x, *args)
            got = gpu.full_pdf(-x, *args)
            if want == 0 or not np.isfinite(want):
                assert got == want or (np.isnan(got) and np.isnan(want)), (kind, tt, err, w)
            else:
                assert np.sign(got) == np.sign(want)
                assert abs(math.log(abs(got)) - math.log(abs(want))) < 1e-12, \
                    (kind, tt, err, w, got, want)
    # the nudged sets straddle the boundary: the decision (branch, K) changes
    by_tt = {}
    for x, tt, err in pts:
        by_tt.setdefault(tt, set()).add(ref_decision(tt, err)[:2])
    flips = sum(len(s) > 1 for s in by_tt.values())
    if kind in ("ks_integer", "kl_integer", "switch"):
        assert flips >= 2, (kind, by_tt)


def test_decision_boundary_on_interior_t_node(gpu, oracle_lib):
    """2-D family (sz, st): err at a decision boundary of the middle t node
    (c) of a trial's root t grid while its ends decide differently (no shared
    decision), both boundaries of the response."""
    checked = 0
    t, st, a = 0.3, 0.2, 1.0
    for tt_c in (0.02, 0.05, 0.1, 0.3, 0.8):
        x = t + tt_c  # |x| - c = tt_c at the centre node c = t
        for kind in ("ks_integer", "kl_integer", "switch"):
            mk, Ks = BOUNDARIES[kind]
            for K in Ks:
                e = _bisect_err(mk(x - t, K), 1e-14, 50.0)
                if e is None:
                    continue
                for err in _nudges(e, 3):
                    for sgn in (-1.0, 1.0):
                        args = (0.4, 0.3, a, 0.5, 0.1, t, st, err, 2, 2, 1, 1e-3)
                        want = oracle_lib.full_pdf(sgn * x, *args)
                        got = gpu.full_pdf(sgn * x, *args)
                        if want == 0:
                            assert got == 0
                        else:
                            assert abs(math.log(abs(got)) - math.log(abs(want))) < 1e-12, \
                                (kind, tt_c, err, sgn)
                        checked += 1
    assert checked >= 60


def test_shared_decision_grid_straddling_ks_peak(gpu, oracle_lib):
    """ks(tt) peaks where 2 sqrt(2 pi tt) err = e^-1/2; the level-0 pass shares
    one decision over a trial's 5 t nodes only when both ends agree and the
    grid lies left of that peak (l0_hints: args0 < 0.5). t grids straddling
    the peak (err ~ 0.12, tt ~ 1) for the 2-D and t-only families, per trial
    at 1e-12 on both boundaries."""
    t, st = 0.6, 1.0
    xs = t + np.linspace(0.3, 2.2, 191)
    x = np.concatenate([xs, -xs])
    for err in (0.09, 0.1, 0.121, 0.13, 0.15):
        peak_tt = (math.exp(-0.5) / (2 * err)) ** 2 / (2 * math.pi)
        assert 0.3 < peak_tt < 2.5
        for sz in (0.0, 0.1):
            args = (0.4, 0.3, 1.0, 0.5, sz, t, st, err)
            ref = oracle_lib.pdf_array(x, *args, 0, 2, 2, 1, 1e-3, 0, 0)
            got = gpu.pdf_array(x, *args, 0, 2, 2, 1, 1e-3, 0, 0)
            ok = ref > 0
            assert np.array_equal(got > 0, ok)
            d = np.abs(np.log(got[ok]) - np.log(ref[ok]))
            assert d.max() < 1e-12, (err, sz, d.max())
            # and through a resident dataset (the lean level-0 pass)
            ds = gpu.Dataset(x)
            tot = ds.wiener_like(*args, 2, 2, 1, 1e-3, 0.05, 0.1)
            tot = ds.wiener_like(*args, 2, 2, 1, 1e-3, 0.05, 0.1)
            terms = oracle_lib.pdf_array(x, *args, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
            assert abs(tot - math.fsum(terms)) <= 1e-11 * math.fsum(np.abs(terms))


@pytest.mark.parametrize("p", [
    (1e160, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0), (-1e160, 0.5, 2.0, 0.5, 0.1, 0.3, 0.1),
    (3e77, 0.3, 2.0, 0.5, 0.1, 0.3, 0.1), (0.5, 1e160, 2.0, 0.5, 0.1, 0.3, 0.1),
    (0.5, 0.1, 1e160, 0.5, 0.1, 0.3, 0.1), (0.5, 0.1, 1e-160, 0.5, 0.1, 0.3, 0.1),
    (40.0, 2.5, 0.5, 0.5, 0.1, 0.3, 0.1), (-40.0, 0.0, 0.5, 0.5, 0.0, 0.3, 0.0)])
def test_extreme_parameters_match_reference(gpu, oracle_lib, p):
    """Parameters that overflow / underflow the series and drift exponents
    (-inf arguments of the fitted exp): per-trial densities and
    log mixtures with and without outliers, and resident totals, follow the
    reference's semantics (0, -inf, NaN exactly where it gives them)."""
    from test_gpu_parity import assert_density_parity
    rng = np.random.default_rng(41)
    x = rng.choice([-1.0, 1.0], 512) * (0.3 + rng.gamma(2.0, 0.4, 512))
    x[:8] = [0.30001, -0.30001, 0.3 + 1e-9, 0.0, 1e-300, 5.0, -5.0, 0.25]
    for po, w in ((0.0, 0.0), (0.05, 0.1)):
        ref = oracle_lib.pdf_array(x, *p, 1e-4, 0, 2, 2, 1, 1e-3, po, w)
        got = gpu.pdf_array(x, *p, 1e-4, 0, 2, 2, 1, 1e-3, po, w)
        assert_density_parity(got, ref, f"{p} po={po}")
        ds = gpu.Dataset(x)
        want = oracle_lib.wiener_like(x, *p, 1e-4, 2, 2, 1, 1e-3, po, w)
        for _ in range(2):  # full sequence, then the predicted (lean) one
            tot = ds.wiener_like(*p, 1e-4, 2, 2, 1, 1e-3, po, w)
            if np.isnan(want) or np.isinf(want):
                assert (np.isnan(tot) and np.isnan(want)) or tot == want, (p, po, tot, want)
            else:
                terms = oracle_lib.pdf_array(x, *p, 1e-4, 1, 2, 2, 1, 1e-3, po, w)
                assert abs(tot - math.fsum(terms)) <= 1e-11 * math.fsum(np.abs(terms)), (p, po)


@pytest.mark.parametrize("case", ["tiny_tt", "many_terms", "big_drift", "sz_wide", "a_small"])
def test_small_time_table_paths(gpu, oracle_lib, case):
    """The small-time grid's 2-D recurrence (wfpt_device.hpp: small_grid2d)
    and its node-by-node fallback: short decision times (8|m| beyond the
    table's exponent bound: the fallback), small err (K up to 8 and past it),
    large drift exponents (sv, v), wide z intervals and small a; per trial
    |dlogp| < 1e-6 against the reference through pdf_array, and the resident
    total (full sequence, then the predicted lean one) against its fsum."""
    rng = np.random.default_rng(97)
    n = 2048
    args = {"tiny_tt": (0.8, 0.3, 1.5, 0.5, 0.2, 0.3, 0.05),
            "many_terms": (0.5, 0.2, 2.0, 0.5, 0.1, 0.3, 0.1),
            "big_drift": (3.5, 2.5, 2.5, 0.45, 0.1, 0.3, 0.1),
            "sz_wide": (-1.0, 0.8, 1.8, 0.5, 0.9, 0.3, 0.1),
            "a_small": (1.0, 0.5, 0.45, 0.5, 0.2, 0.2, 0.05)}[case]
    err = 1e-12 if case == "many_terms" else 1e-4
    t = args[5]
    x = rng.choice([-1.0, 1.0], n) * (t + rng.gamma(1.5, 0.08 if case == "tiny_tt" else 0.35, n))
    x[:4] = [t + 1e-4, -(t + 1e-3), t + 0.01, -(t + 0.02)]
    ref = oracle_lib.pdf_array(x, *args, err, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
    got = gpu.pdf_array(x, *args, err, 1, 2, 2, 1, 1e-3, 0.05, 0.1)
    assert_logp_parity(got, ref, case)
    ds = gpu.Dataset(x)
    want = math.fsum(ref)
    for _ in range(2):  # full sequence, then the predicted one
        tot = ds.wiener_like(*args, err, 2, 2, 1, 1e-3, 0.05, 0.1)
        assert abs(tot - want) <= 1e-11 * math.fsum(np.abs(ref)), (case, tot, want)


@pytest.mark.gpu
@pytest.mark.parametrize("family", ["simple", "full"])
def test_node_dataset_with_nan_rts(gpu, oracle_lib, family):
    """NaN RTs in a node dataset: the per-node |rt| sort puts them
    last within their node (a strict weak order), the per-trial terms come
    back in the caller's order with NaN exactly where the reference has it
    (its full_pdf of NaN is NaN, wfpt.pyx:66-74), and a node holding a NaN
    sums to NaN while the others keep their sums."""
    rng = np.random.default_rng(31 if family == "simple" else 32)
    x, node, P = _node_dataset(rng, 9, family)
    P[:, 7] = 0.05  # every node in range: NaN must come from the RTs alone
    bad = rng.choice(x.size, 12, replace=False)
    x = x.copy()
    x[bad] = np.where(rng.random(bad.size) < 0.5, np.nan, -np.nan)
    ds = gpu.Dataset(x, node_id=node, n_nodes=P.shape[0])
    sums, terms = ds.wiener_like_nodes(P, *KN, trials=True)
    ref = node_terms_ref(oracle_lib, x, node, P)
    assert np.array_equal(np.isnan(ref), np.isnan(x))  # the reference's own semantics
    assert_logp_parity(terms, ref, f"{family} node terms with NaN RTs")
    for j in range(P.shape[0]):
        tj = ref[node == j]
        if np.isnan(tj).any():
            assert np.isnan(sums[j]), j
        elif tj.size:
            assert abs(sums[j] - math.fsum(tj)) <= 1e-12 * math.fsum(np.abs(tj)) + 1e-12, j


@pytest.mark.gpu
@pytest.mark.parametrize("full", [False, True])
def test_node_sums_never_stale(gpu, full):
    """The batched node call's per-node sums reach the mapped result slot
    before its completion word (segment_publish_kernel: agent-scope sum
    stores, an acq_rel ticket, a system-scope release of the word, the host's
    acquire poll). Alternating two parameter tables over config 4's dataset,
    every call must return exactly its own table's sums. That this loop can
    see a late publication is shown by the next test, on a build whose sums
    land after the word."""
    import node_publication_check as npc
    r = npc.run(full=full, reps=150 if full else 400)
    assert r["tables_differ"] and r["sync_reads_agree"], r
    assert r["stale_calls"] == 0, r


@pytest.mark.gpu
def test_stale_check_detects_late_publication(gpu):
    """Sensitivity of test_node_sums_never_stale: the same loop in a child
    process on the WFPT_PUB_DIAG build (built by __graft_entry__.build next to
    the shipped library), whose non-last blocks store their nodes' sums ~70 us
    after the completion word, must report stale calls -- the r05 failure
    (a node sum of the previous call) made deterministic."""
    import json
    import os
    import subprocess
    import sys
    from hddm_amd import build as hb
    lib = os.path.join(hb.LIBDIR, "libwfpt_amd_pubdiag.so")
    assert os.path.exists(lib), "diagnostic build missing: run __graft_entry__.build()"
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, WFPT_AMD_LIB=lib)
    p = subprocess.run([sys.executable, os.path.join(here, "node_publication_check.py"),
                        "--full", "--reps", "20"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    print("diagnostic build:", r)
    assert r["lib"] == "libwfpt_amd_pubdiag.so", r
    assert r["tables_differ"] and r["sync_reads_agree"], r
    assert r["stale_calls"] >= r["calls"] // 2, r
