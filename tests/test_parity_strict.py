"""Parity at the north_star bar on the configs' own data, near-ties and
bit-for-bit call-sequence determinism (VERDICT r01 "do this" items 1, 6 and
ADVICE r01 #1).

Every comparison is against the oracle (oracle/wfpt_oracle.c, pinned bit-exact
to the reference's own kernels by tests/test_oracle.py) or against fixtures
generated from the reference's kernels (tests/golden/). Tolerances:
  * per trial |log p_gpu - log p_ref| < 1e-6 (north_star), no relaxation;
  * totals vs math.fsum of the reference's per-trial values, relative 1e-11
    (the reference sums sequentially, the GPU in a fixed tree);
  * near-ties / guard bands: |dlogp| < 1e-12 — a flipped decision there moves
    the value by far more (one series term or one Simpson refinement), so this
    checks the decision itself, not just the 1e-6 bar.
"""
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KN = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
PINNED = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
SIMPLE = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)


def threads():
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else len(os.sched_getaffinity(0))


def ref_logp(oracle_lib, x, args, kn=KN):
    """Per-trial log mixture density of the reference, all host threads."""
    return oracle_lib.pdf_array(x, *args, kn[0], 1, kn[1], kn[2], kn[3], kn[4], kn[5], kn[6],
                                n_threads=threads())


def assert_total(got, terms, what):
    terms = np.asarray(terms)
    assert np.all(np.isfinite(terms)), what
    ref = math.fsum(terms)
    scale = math.fsum(np.abs(terms))
    assert abs(got - ref) <= 1e-11 * scale, f"{what}: {got} vs {ref} (scale {scale})"


# --------------------------------------------------------------------------- CPU

def test_gen_rts_sampling_matches_reference_fixture(oracle_lib, monkeypatch):
    """hddm_amd.wfpt.gen_rts_from_cdf's host logic (running sum, normalisation,
    draws, searchsorted, delays) reproduces the reference's loop bit for bit
    when fed the reference's grid densities (the oracle's, bit-exact)."""
    from hddm_amd import wfpt
    monkeypatch.setattr(wfpt, "pdf_array", oracle_lib.pdf_array)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "gen_rts.npz")))
    k = 0
    while f"rts_{k}" in g:
        v, sv, a, z, sz, t, st, n, lb, ub, dt, seed = g[f"args_{k}"]
        np.random.seed(int(seed))
        got = wfpt.gen_rts_from_cdf(v, sv, a, z, sz, t, st, samples=int(n), cdf_lb=lb, cdf_ub=ub,
                                    dt=dt)
        np.testing.assert_array_equal(got, g[f"rts_{k}"])
        k += 1
    assert k == 4


# --------------------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_gen_rts_matches_reference_fixture(gpu):
    """GPU density grid: identical samples to the reference's gen_rts_from_cdf
    (wfpt.pyx:323-354) for the fixture's seeds. A sample can only differ where
    its uniform draw falls between the two versions of one normalised CDF value
    (|dF| ~ 1e-15): at most 1 in 10^4 samples is allowed to sit on the
    adjacent grid point."""
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "gen_rts.npz")))
    for k in range(4):
        v, sv, a, z, sz, t, st, n, lb, ub, dt, seed = g[f"args_{k}"]
        np.random.seed(int(seed))
        got = gpu.gen_rts_from_cdf(v, sv, a, z, sz, t, st, samples=int(n), cdf_lb=lb, cdf_ub=ub,
                                   dt=dt)
        want = g[f"rts_{k}"]
        diff = np.flatnonzero(got != want)
        assert diff.size <= max(1, int(n) // 10_000), (k, diff[:10], got[diff[:5]], want[diff[:5]])
        if diff.size:  # adjacent grid point only
            assert np.all(np.abs(np.abs(got[diff]) - np.abs(want[diff])) <= dt * 1.000001 + 1e-12)


@pytest.mark.gpu
def test_bench_dataset_per_trial(gpu, oracle_lib):
    """bench.py's own C3 dataset (1M RTs sampled from the model by
    gen_rts_from_cdf, seed 20261015): per-trial log p at 1e-6 and the resident
    total against fsum of the reference's per-trial values."""
    np.random.seed(20261015)
    x = gpu.gen_rts_from_cdf(*PINNED, samples=1_000_000, dt=1e-3)
    ref = ref_logp(oracle_lib, x, PINNED)
    got = gpu.pdf_array(x, *PINNED, KN[0], 1, *KN[1:])
    d = np.abs(got - ref)
    assert np.all(np.isfinite(got)) and d.max() < 1e-6, d.max()
    assert_total(gpu.Dataset(x).wiener_like(*PINNED, *KN), ref, "bench dataset")


@pytest.mark.gpu
def test_c2_simple_10m_resident_total(gpu, oracle_lib):
    """C2: simple DDM, 10M resident trials; total vs fsum of the reference."""
    np.random.seed(20261015)
    x = gpu.gen_rts_from_cdf(*SIMPLE, samples=10_000_000, dt=1e-3)
    ref = ref_logp(oracle_lib, x, SIMPLE)
    ds = gpu.Dataset(x)
    assert_total(ds.wiener_like(*SIMPLE, *KN), ref, "C2 10M")
    assert_total(ds.wiener_like(*SIMPLE, *KN), ref, "C2 10M (fast-only call)")


@pytest.mark.gpu
def test_c5_shard_12_5m_resident_total(gpu, oracle_lib):
    """C5's per-GPU shard: 12.5M full-DDM trials resident; total vs fsum."""
    from hddm_amd import _lib
    lo, hi = _lib.shard_range(100_000_000, 8, 3)
    assert hi - lo == 12_500_000
    np.random.seed(20261015 + 3)
    x = gpu.gen_rts_from_cdf(*PINNED, samples=hi - lo, dt=1e-3)
    ref = ref_logp(oracle_lib, x, PINNED)
    ds = gpu.Dataset(x)
    assert_total(ds.wiener_like(*PINNED, *KN), ref, "C5 shard")


STRESS = [(-1.2388, 1.3918, 1.4387, 0.4995, 0.2891, 0.277, 0.0698),
          (1.7431, 2.0137, 0.6119, 0.5386, 0.2108, 0.3567, 0.1981),
          (0.8, 0.0, 1.6, 0.45, 0.0, 0.25, 0.2),      # st only
          (0.8, 0.7, 1.6, 0.45, 0.3, 0.25, 0.0),      # sz only
          (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)]        # direct


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", [(1e-4, 2, 2, 1, 1e-3), (1e-6, 3, 3, 1, 1e-5),
                                   (1e-4, 4, 4, 1, 1e-4)])
def test_evaluation_counts_equal_reference(gpu, oracle_lib, knobs):
    """The quadrature trees are the reference's: the number of pdf_sv
    evaluations the library performs (level-0 pass + breadth-first levels +
    inner refinements, or the exact / per-lane path from scratch) equals the
    reference's count on the same data, exactly. Knob sets cover trees within
    the breadth-first levels (depth 2) and deeper ones (per-lane walk)."""
    from hddm_amd import _lib
    ctx = _lib.context()
    err, n_st, n_sz, ua, se = knobs
    for k, p in enumerate(STRESS):
        np.random.seed(100 + k)
        x = gpu.gen_rts_from_cdf(*p, samples=20_000, dt=1e-3)
        ds = gpu.Dataset(x)
        ctx.profile(ctx.PROF_EVALS)
        ds.wiener_like(*p, err, n_st, n_sz, ua, se, 0.05, 0.1)
        _, _, ne = ctx.profile_read(reset=True)
        ctx.profile(0)
        assert ne == oracle_lib.count_evals(x, *p, err, n_st, n_sz, ua, se), (p, knobs)


@pytest.mark.gpu
def test_call_sequence_determinism(gpu):
    """a likelihood does not depend on the call history. The
    same parameters on the same dataset give bit-identical totals whether the
    call ran the full sequence (level-0 + deferred pass), the predicted
    fast-only sequence, or a mispredicted one that finished the deferred pass
    after a round trip."""
    np.random.seed(3)
    x = gpu.gen_rts_from_cdf(*STRESS[1], samples=300_000, dt=1e-3)
    ds = gpu.Dataset(x)
    kn = KN
    defer, nodefer = STRESS[1], PINNED
    a1 = ds.wiener_like(*nodefer, *kn)      # first call: full sequence
    a2 = ds.wiener_like(*nodefer, *kn)      # predicted fast-only
    b1 = ds.wiener_like(*defer, *kn)        # mispredicted: fast, round trip, deferred
    b2 = ds.wiener_like(*defer, *kn)        # full sequence
    a3 = ds.wiener_like(*nodefer, *kn)      # full sequence (last call deferred)
    a4 = ds.wiener_like(*nodefer, *kn)      # fast-only again
    assert a1 == a2 == a3 == a4, (a1, a2, a3, a4)
    assert b1 == b2, (b1, b2)
    # host-array path (full sequence) on the dataset's own trial order (a
    # Dataset orders trials by boundary, then |rt|; the chunk partials, and so
    # the last bit of the total, follow the order)
    xs = x[np.lexsort((np.abs(x), x > 0))]
    host = gpu.wiener_like(xs, *defer, *kn)
    assert host == b1


@pytest.mark.gpu
def test_call_sequence_determinism_multiblock_finalize(gpu, oracle_lib):
    """The same bitwise call-history independence when the finalize runs as
    several blocks (> 16k chunk partials: 1.5M trials, 23.4k chunks): the
    full, predicted (lean / fast-only) and mispredicted sequences and the
    host-array path give identical totals, and the total equals the
    reference's per-trial fsum to 1e-11 relative."""
    np.random.seed(11)
    x = gpu.gen_rts_from_cdf(*PINNED, samples=1_500_000, dt=1e-3)
    ds = gpu.Dataset(x)
    kn = KN
    defer = STRESS[1]
    a = [ds.wiener_like(*PINNED, *kn) for _ in range(3)]
    b1 = ds.wiener_like(*defer, *kn)  # mispredicted after the lean calls
    b2 = ds.wiener_like(*defer, *kn)
    a.append(ds.wiener_like(*PINNED, *kn))
    assert a[0] == a[1] == a[2] == a[3], a
    assert b1 == b2, (b1, b2)
    xs = x[np.lexsort((np.abs(x), x > 0))]
    assert gpu.wiener_like(xs, *PINNED, *kn) == a[0]
    terms = oracle_lib.pdf_array(x[:200_000], *PINNED, kn[0], 1, *kn[1:])
    ref_head = math.fsum(terms)
    got_head = gpu.Dataset(x[:200_000]).wiener_like(*PINNED, *kn)
    assert abs(got_head - ref_head) <= 1e-11 * math.fsum(np.abs(terms))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 200, 250, 256])
def test_one_block_calls_match_two_launch_sequence(gpu, oracle_lib, n):
    """Datasets of <= 256 trials (an HDDM node) run level 0 and the finalize
    in one launch once the call sequence is predicted (small_kernel): the
    totals are bit for bit those of the first call's full two-launch
    sequence, for the direct and the adaptive families, and after a
    misprediction (a parameter set that defers, then one that does not)."""
    rng = np.random.default_rng(n)
    x = rng.choice([-1.0, 1.0], n) * (0.32 + rng.gamma(2.0, 0.4, n))
    simple = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)
    for args in (simple, PINNED, STRESS[3]):
        ds = gpu.Dataset(x)
        first = ds.wiener_like(*args, *KN)   # full sequence (two launches)
        again = [ds.wiener_like(*args, *KN) for _ in range(3)]  # predicted: one launch
        assert all(v == first for v in again), (n, args, first, again)
        terms = oracle_lib.pdf_array(x, *args, KN[0], 1, *KN[1:])
        ref = math.fsum(terms)
        assert abs(first - ref) <= 1e-11 * math.fsum(np.abs(terms)) + 1e-300, (n, args)
    ds = gpu.Dataset(x)
    a0 = ds.wiener_like(*PINNED, *KN)
    b = [ds.wiener_like(*STRESS[1], *KN) for _ in range(2)]  # mispredicted, then full
    a1 = ds.wiener_like(*PINNED, *KN)
    a2 = ds.wiener_like(*PINNED, *KN)
    assert b[0] == b[1] and a0 == a1 == a2, (a0, a1, a2, b)


def _flip(x, v, z):
    return (abs(x), -v, 1 - z) if x > 0 else (abs(x), v, z)


def _root_S(f, lb, ub):
    """S and S2 of an adaptive Simpson root (integrate.pxi:114-141, 72-112),
    f = (f(lb), f(d), f(c), f(e), f(ub)) already divided by the width."""
    h = ub - lb
    S = (h / 6) * ((f[0] + (4 * f[2])) + f[4])
    Sl = (h / 12) * ((f[0] + (4 * f[1])) + f[2])
    Sr = (h / 12) * ((f[2] + (4 * f[3])) + f[4])
    return S, Sl + Sr


def _nudges(val, k=4):
    out, lo, hi = [val], val, val
    for _ in range(k):
        lo, hi = np.nextafter(lo, -np.inf), np.nextafter(hi, np.inf)
        out += [lo, hi]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["t", "z"])
def test_near_tie_stop_test(gpu, oracle_lib, mode):
    """simps_err placed so that |S2 - S| of the root interval sits within 0-4
    ulps of 15 * simps_err (integrate.pxi:105): the library must take the
    reference's branch (it routes such trials to the exact path)."""
    rng = np.random.default_rng(21)
    checked = 0
    for _ in range(12):
        v, sv, a = rng.uniform(-2, 2), rng.uniform(0, 1.5), rng.uniform(0.8, 2.0)
        z, t = rng.uniform(0.4, 0.6), rng.uniform(0.25, 0.4)
        sz, st = (0.0, rng.uniform(0.1, 0.3)) if mode == "t" else (rng.uniform(0.1, 0.3), 0.0)
        x = rng.choice([-1.0, 1.0]) * (t + st / 2 + rng.uniform(0.05, 0.6))
        xa, vv, zz = _flip(x, v, z)
        err = 1e-4
        if mode == "t":
            lb, ub = t - st / 2., t + st / 2.
            ZT = ub - lb
            c = (ub + lb) / 2.
            pts = [lb, (lb + c) / 2., c, (c + ub) / 2., ub]
            f = [oracle_lib.pdf_sv(xa - q, vv, sv, a, zz, err) / ZT for q in pts]
        else:
            lb, ub = zz - sz / 2., zz + sz / 2.
            ZT = ub - lb
            c = (ub + lb) / 2.
            pts = [lb, (lb + c) / 2., c, (c + ub) / 2., ub]
            f = [oracle_lib.pdf_sv(xa - t, vv, sv, a, q, err) / ZT for q in pts]
        S, S2 = _root_S(f, lb, ub)
        if not abs(S2 - S) > 0:
            continue
        for se in _nudges(abs(S2 - S) / 15):
            args = (v, sv, a, z, sz, t, st, err, 2, 2, 1, se)
            want = oracle_lib.full_pdf(x, *args)
            got = gpu.full_pdf(x, *args)
            assert abs(math.log(got) - math.log(want)) < 1e-12, (args, got, want)
            checked += 1
    assert checked >= 60


@pytest.mark.gpu
def test_series_decision_guard_band(gpu, oracle_lib):
    """err placed so that the large-time term count kl (pdf.pxi:36-40) sits
    within a few ulps of an integer (K = ceil(kl) flips there), with err large
    enough that one series term changes the density by ~1e-3: the library must
    use the reference's K (fp32 estimate ambiguous -> fp64 decision ->
    exact path within 1e-12 of the threshold)."""
    checked = 0
    for tt in (0.2, 0.3, 0.45):
        for K in (1, 2):
            err0 = math.exp(-(K * K) * math.pi ** 2 * tt / 2) / (math.pi * tt)
            for err in _nudges(err0, 6):
                a, t = 1.0, 0.3
                for w in (0.3, 0.5, 0.7):
                    x = -(t + tt * a * a)  # lower boundary: z = w unflipped
                    args = (0.4, 0.0, a, w, 0.0, t, 0.0, err)
                    want = oracle_lib.full_pdf(x, *args)
                    got = gpu.full_pdf(x, *args)
                    if want == 0:
                        assert got == 0
                    else:
                        assert abs(math.log(abs(got)) - math.log(abs(want))) < 1e-12, (tt, K, err, w)
                    checked += 1
    assert checked == 3 * 2 * 13 * 3


@pytest.mark.gpu
def test_subnormal_and_zero_densities(gpu, oracle_lib):
    """Trials a hair above t: densities from normal down through the subnormal
    range to exact zeros, per trial at the 1e-6 log bar (exact path), for the
    direct, 1-D and 2-D families, both boundaries."""
    from test_gpu_parity import assert_density_parity
    t = 0.3
    xx = np.concatenate([np.linspace(2e-4, 2e-3, 400), np.geomspace(1e-5, 2e-4, 100)])
    x = np.concatenate([t + xx, -(t + xx)])
    n_sub = 0
    for p in [(0.5, 0.0, 2.0, 0.5, 0.0, t, 0.0), (0.5, 1.0, 2.0, 0.5, 0.0, t, 0.0),
              (-1.0, 0.5, 2.0, 0.45, 0.2, t, 0.0), (0.5, 0.0, 2.0, 0.5, 0.0, t + 0.001, 0.002)]:
        ref = oracle_lib.pdf_array(x, *p, 1e-4, 0, 2, 2, 1, 1e-3, 0, 0)
        got = gpu.pdf_array(x, *p, 1e-4, 0, 2, 2, 1, 1e-3, 0, 0)
        assert_density_parity(got, ref, f"near-t {p}")
        n_sub += int(np.sum((ref > 0) & (ref < np.finfo(float).tiny)))
    assert n_sub >= 20  # the grid does reach the subnormal range
