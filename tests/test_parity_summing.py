"""Per-trial parity of the kernels the bench and HDDM actually time (VERDICT r03
"do this" 1): the lean level-0 pass (lean_kernel, OUT_SUM), the one-launch
node-sized path (small_kernel) and the engine / redo / fold sequences.

Those kernels only write 64-trial chunk partials. Two checks pin them to the
reference trial by trial:
  * wfpt_wiener_like_trials runs the same predicted call sequence with the
    same kernel templates built with one extra store per trial (OUT_BOTH).
    Its chunk partials and total must equal the summing call's BIT FOR BIT,
    so its per-trial terms are the terms the timed kernels add. Each term must
    match the reference's addend log(p (1 - p_outlier) + w_outlier p_outlier)
    (src/wfpt.pyx:66-74) to |dlogp| < 1e-6 (north_star), with -inf exactly
    where the reference has a zero mixture density.
  * The timed kernel's own chunk partials (wfpt_debug_partials after a plain
    wiener_like) must equal math.fsum of the reference's 64 terms of that
    chunk to 1e-12 relative to the sum of their magnitudes (+1e-12 absolute:
    a relative error of p is an absolute error of log p, so chunks of terms
    near log p = 0 get that floor), and the zero-count word must equal the
    reference's count of -inf terms.
The reference terms come from the oracle (oracle/wfpt_oracle.c, bit-exact to
the reference's compiled pdf.pxi / integrate.pxi, tests/test_oracle.py) with
libm's log, as wfpt.pyx:70 takes it.
"""
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KN = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)  # HDDM's knobs (likelihoods.py:52-55) + p_outlier
PINNED = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
SIMPLE = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)
ST_ONLY = (0.8, 0.0, 1.6, 0.45, 0.0, 0.25, 0.2)
SZ_ONLY = (0.8, 0.7, 1.6, 0.45, 0.3, 0.25, 0.0)
# tests/test_parity_strict.py STRESS[0:2] (random full-DDM sets that refine)
STRESS = [(-1.2388, 1.3918, 1.4387, 0.4995, 0.2891, 0.277, 0.0698),
          (1.7431, 2.0137, 0.6119, 0.5386, 0.2108, 0.3567, 0.1981), ST_ONLY, SZ_ONLY]


def threads():
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else len(os.sched_getaffinity(0))


def ref_terms(oracle_lib, x, args, kn=KN):
    """The reference's per-trial addends of wiener_like (libm log of the
    mixture; -inf for a zero mixture density)."""
    return oracle_lib.pdf_array(x, *args, kn[0], 1, kn[1], kn[2], kn[3], kn[4], kn[5], kn[6],
                                n_threads=threads())


def assert_terms(got, ref, what):
    got, ref = np.asarray(got), np.asarray(ref)
    zr, zg = np.isneginf(ref), np.isneginf(got)
    assert np.array_equal(zr, zg), (what, np.flatnonzero(zr != zg)[:10])
    fin = ~zr
    assert np.all(np.isfinite(got[fin])), (what, np.flatnonzero(~np.isfinite(got[fin]))[:10])
    d = np.abs(got[fin] - ref[fin])
    assert d.size == 0 or d.max() < 1e-6, (what, d.max(), np.argmax(d))
    return float(d.max()) if d.size else 0.0


def assert_chunks(ctx, ds, ref, what):
    """The timed call's chunk partials vs fsum of the reference's 64 terms."""
    n = len(ds)
    nb = (n + 63) // 64
    part, zero = ctx.partials(nb)
    r = ref[ds.order()]
    worst = 0.0
    for c in range(nb):
        seg = r[64 * c:64 * c + 64]
        fin = seg[np.isfinite(seg)]
        nz = int(np.isneginf(seg).sum())
        assert (int(zero[c]) & 0xFFFF) == nz, (what, c, zero[c], nz)
        want = math.fsum(fin)
        scale = math.fsum(np.abs(fin))
        err = abs(part[c] - want)
        assert err <= 1e-12 * scale + 1e-12, (what, c, part[c], want, scale)
        worst = max(worst, err / (scale + 1.0))
    return worst


def path_names(bits):
    from hddm_amd import _lib
    names = {_lib.PATH_LEAN: "lean", _lib.PATH_ENGINE: "engine", _lib.PATH_SMALL: "small",
             _lib.PATH_REDO: "redo", _lib.PATH_FOLD: "fold", _lib.PATH_DIRECT: "direct",
             _lib.PATH_FIXED: "fixed", _lib.PATH_SPLIT: "split",
             _lib.PATH_SMALL_SPLIT: "small_split"}
    return {v for k, v in names.items() if bits & k}


def summing_vs_trials(ctx, ds, args, kn=KN):
    """A plain wiener_like (the timed kernels), its chunk partials, then the
    per-trial build on the same prediction: path, partials and total equal."""
    tot = ds.wiener_like(*args, *kn)
    path = ctx.last_path()
    nb = (len(ds) + 63) // 64
    part, zero = ctx.partials(nb)
    tot2, terms = ds.wiener_like_trials(*args, *kn)
    assert ctx.last_path() == path, (path_names(path), path_names(ctx.last_path()))
    part2, zero2 = ctx.partials(nb)
    assert tot2 == tot or (math.isnan(tot) and math.isnan(tot2)), (tot, tot2)
    assert np.array_equal(part.view(np.int64), part2.view(np.int64))
    assert np.array_equal(zero, zero2)
    return tot, terms, path


@pytest.mark.gpu
def test_lean_kernel_per_trial_on_bench_dataset(gpu, oracle_lib):
    """bench.py's C3 dataset (1M RTs, seed 20261015): the call bench.py times
    is lean_kernel -> finalize; its per-trial terms and every chunk partial
    match the reference."""
    from hddm_amd import _lib
    ctx = _lib.context()
    np.random.seed(20261015)
    x = gpu.gen_rts_from_cdf(*PINNED, samples=1_000_000, dt=1e-3)
    ref = ref_terms(oracle_lib, x, PINNED)
    ds = gpu.Dataset(x)
    first = ds.wiener_like(*PINNED, *KN)  # nothing predicted yet: the state sequence
    assert path_names(ctx.last_path()) & {"engine", "state"}, path_names(ctx.last_path())
    tot, terms, path = summing_vs_trials(ctx, ds, PINNED)
    assert path_names(path) == {"lean"}, path_names(path)
    assert tot == first
    dmax = assert_terms(terms, ref, "bench C3 1M")
    assert_chunks(ctx, ds, ref, "bench C3 1M")
    assert dmax < 1e-9  # observed ~1e-14: far inside the bar


@pytest.mark.gpu
def test_c2_direct_kernel_per_trial_10m(gpu, oracle_lib):
    """C2's timed kernel at dataset scale: the 10M simple-DDM resident dataset
    (tests/test_parity_strict.py's C2 data) through fast_kernel<kDirect>'s
    OUT_BOTH build. Its chunk partials and total are bitwise the plain call's,
    each term is within 1e-6 of the reference's addend (src/wfpt.pyx:66-74),
    and every one of the plain call's 156,250 chunk partials is within 1e-12
    of fsum of the reference's 64 terms."""
    np.random.seed(20261015)
    x = gpu.gen_rts_from_cdf(*SIMPLE, samples=10_000_000, dt=1e-3)
    ref = ref_terms(oracle_lib, x, SIMPLE)
    from hddm_amd import _lib
    ctx = _lib.context()
    ds = gpu.Dataset(x)
    ds.wiener_like(*SIMPLE, *KN)
    tot, terms, path = summing_vs_trials(ctx, ds, SIMPLE)
    assert path_names(path) == {"direct"}, path_names(path)
    dmax = assert_terms(terms, ref, "C2 10M")
    assert dmax < 1e-9
    assert_chunks_fast(ctx, ds, ref, "C2 10M")
    ds.close()


def assert_chunks_fast(ctx, ds, ref, what):
    """assert_chunks for millions of chunks: exact (fsum) sums only where the
    float64 pairwise sum is not already far inside the bound."""
    n = len(ds)
    nb = (n + 63) // 64
    part, zero = ctx.partials(nb)
    r = ref[ds.order()]
    pad = np.full(nb * 64, np.nan)
    pad[:n] = r
    seg = pad.reshape(nb, 64)
    real = ~np.isnan(seg)
    fin = np.isfinite(seg)
    nz = (np.isneginf(seg) & real).sum(axis=1)
    assert np.array_equal(zero & 0xFFFF, nz), what
    vals = np.where(fin, seg, 0.0)
    want = vals.sum(axis=1)
    scale = np.abs(vals).sum(axis=1)
    err = np.abs(part - want)
    bound = 1e-12 * scale + 1e-12
    # numpy's float64 row sums are within ~64 ulp of scale of the exact sum:
    # recheck with fsum wherever that could matter
    close = err > 0.5 * bound
    for c in np.flatnonzero(close):
        w = math.fsum(vals[c])
        assert abs(part[c] - w) <= bound[c], (what, c, part[c], w, scale[c])
    return int(close.sum())


def _ctx_with(env):
    """A fresh context opened under the given WFPT_* settings (read at open)."""
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


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(4))
def test_stress_sets_per_trial_every_sequence(gpu, oracle_lib, k):
    """The stress sets (parameters that refine) per trial and per chunk along
    every call sequence a refining dataset can take: the chunk engine (the
    default once refinement is predicted: in-wave rounds, heavy-chunk split
    units from the third call, fold), and the lean pass + the engine's redo of
    the flagged chunks (WFPT_LEAN_TREE=1). Their totals are bitwise equal."""
    from hddm_amd import _lib
    p = STRESS[k]
    np.random.seed(100 + k)
    x = gpu.gen_rts_from_cdf(*p, samples=250_000, dt=1e-3)
    ref = ref_terms(oracle_lib, x, p)
    tots = {}
    for name, env, need in (("engine", None, "engine"), ("lean+redo", {"WFPT_LEAN_TREE": "1.0"},
                                                         "lean")):
        ctx = _lib.context() if env is None else _ctx_with(env)
        ds = gpu.Dataset(x, ctx=ctx)
        ds.wiener_like(*p, *KN)
        ds.wiener_like(*p, *KN)  # the engine records heavy chunks for the next call's split
        tot, terms, path = summing_vs_trials(ctx, ds, p)
        if need:
            assert need in path_names(path), (name, path_names(path))
        assert_terms(terms, ref, f"stress {k} {name} {path_names(path)}")
        assert_chunks(ctx, ds, ref, f"stress {k} {name}")
        tots[name] = tot
        ds.close()
        if env is not None:
            ctx.close()
    assert len(set(tots.values())) == 1, tots


@pytest.mark.gpu
def test_dataset_outliving_its_context(gpu):
    """Closing a context detaches its datasets (their device memory is
    released with it); destroying one afterwards frees only its host part and
    leaves no error behind for the next call, and using it fails loudly."""
    ctx = _ctx_with({})
    x = np.linspace(0.4, 2.0, 1000) * np.where(np.arange(1000) % 2, 1, -1)
    ds = gpu.Dataset(x, ctx=ctx)
    ds.wiener_like(*PINNED, *KN)
    ctx.close()
    with pytest.raises(ValueError):
        ds.wiener_like(*PINNED, *KN)
    ds.close()
    assert np.isfinite(gpu.Dataset(x).wiener_like(*PINNED, *KN))


@pytest.fixture(scope="module")
def lean_ctx(gpu):
    """A second context whose resident calls always take the lean level-0
    pass (WFPT_LEAN_TREE=1: chunks that refine go to the engine's redo pass),
    so the lean / small kernels run on data that would otherwise predict the
    engine."""
    from hddm_amd import _lib
    old = os.environ.get("WFPT_LEAN_TREE")
    os.environ["WFPT_LEAN_TREE"] = "1.0"
    try:
        ctx = _lib.Context(0)
    finally:
        if old is None:
            del os.environ["WFPT_LEAN_TREE"]
        else:
            os.environ["WFPT_LEAN_TREE"] = old
    yield ctx
    ctx.close()


def one_launch_path(args):
    """The kernels of a predicted level-0-only call of <= 256 trials: the
    one-block launch (small_kernel; the full DDM's small_split_kernel)."""
    sz, st = args[4], args[6]
    if sz == 0 and st == 0:
        return {"small", "direct"}
    if sz > 0 and st > 0:
        return {"small", "lean", "small_split"}
    return {"small", "lean"}


def check_one_launch(path, args, n, what):
    """A node-sized call that neither refined nor deferred took the one-block
    kernel of its family (not level 0 + a separate finalize)."""
    names = path_names(path)
    if n <= 256 and not names & {"engine", "redo", "fold"}:
        assert names == one_launch_path(args), (what, names)
        return True
    return False


def _both_contexts(gpu, lean_ctx, x, args, what, oracle_lib, need):
    """Per trial and per chunk on the default context's predicted path and on
    the forced-lean one (which must include a kernel of `need`); the two
    totals are bitwise equal. A predicted level-0-only call of <= 256 trials
    must be the one-block launch of its family."""
    from hddm_amd import _lib
    ref = ref_terms(oracle_lib, x, args)
    tots = []
    for ctx in (_lib.context(), lean_ctx):
        ds = gpu.Dataset(x, ctx=ctx)
        ds.wiener_like(*args, *KN)
        tot, terms, path = summing_vs_trials(ctx, ds, args)
        check_one_launch(path, args, len(x), what)
        if ctx is lean_ctx:
            assert path_names(path) & need, (what, path_names(path))
        assert_terms(terms, ref, f"{what} {path_names(path)}")
        assert_chunks(ctx, ds, ref, f"{what} {path_names(path)}")
        tots.append(tot)
        ds.close()
    assert tots[0] == tots[1], (what, tots)


@pytest.mark.gpu
@pytest.mark.parametrize("n_lower,n", [(37, 1000), (100, 3000), (64, 200), (1, 130)])
def test_mixed_boundary_wave_per_trial(gpu, oracle_lib, lean_ctx, n_lower, n):
    """The wave where the dataset's boundary-ordered trials switch from the
    lower to the upper boundary runs the lean level 0 at two call sites (the
    scalar root grid of each boundary): per trial and per chunk, for the
    2-D, 1-D (t, z) families."""
    rng = np.random.default_rng(n_lower * 7 + n)
    mag = 0.33 + rng.gamma(2.0, 0.35, n)
    x = np.where(np.arange(n) < n_lower, -mag, mag)
    rng.shuffle(x)
    for args in (PINNED, ST_ONLY, SZ_ONLY):
        _both_contexts(gpu, lean_ctx, x, args, f"mixed wave {n_lower}/{n} {args}", oracle_lib,
                       {"lean", "small"})


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 17, 63, 64, 65, 128, 200, 250, 256])
def test_node_sized_one_launch_per_trial(gpu, oracle_lib, lean_ctx, n):
    """Datasets of <= 256 trials (one HDDM node: what the install()ed
    wfpt_like runs per node per logp) take small_kernel once the lean pass is
    predicted: per trial and per chunk against the reference, every family."""
    rng = np.random.default_rng(1000 + n)
    x = rng.choice([-1.0, 1.0], n) * (0.32 + rng.gamma(2.0, 0.4, n))
    for args in (SIMPLE, PINNED, ST_ONLY, SZ_ONLY):
        # refining data: the lean pass + the engine's redo (a refining call
        # is never predicted level-0-only, so small_kernel is not taken)
        _both_contexts(gpu, lean_ctx, x, args, f"node-sized {n} {args}", oracle_lib,
                       {"small", "lean"})


NODE_FAMILIES = (SIMPLE, PINNED, (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.1),
                 (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.0))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 17, 64, 65, 200, 250, 256])
def test_node_sized_calls_take_the_one_block_kernel(gpu, oracle_lib, n):
    """What an install()ed HDDM node call runs (hddm/likelihoods.py:52-55 per
    node): data on which no trial refines (the oracle's evaluation count is
    the root level's, so the reference's trees stop at level 0) is predicted
    level-0-only after one call, and that call must be ONE launch of the
    family's one-block kernel: small_kernel (direct / 1-D families) or
    small_split_kernel (the full DDM). A regression back to level 0 + a
    separate finalize fails here. Per trial and per chunk against the
    reference on the same calls."""
    from hddm_amd import _lib
    rng = np.random.default_rng(5000 + n)
    x = rng.choice([-1.0, 1.0], n) * (0.5 + rng.gamma(2.0, 0.3, n))
    ctx = _lib.context()
    for args in NODE_FAMILIES:
        root = 1 if (args[4] == 0 and args[6] == 0) else (25 if args[4] > 0 and args[6] > 0 else 5)
        assert oracle_lib.count_evals(x, *args, *KN[:5]) == n * root, "data refines"
        ref = ref_terms(oracle_lib, x, args)
        ds = gpu.Dataset(x, ctx=ctx)
        ds.wiener_like(*args, *KN)
        tot, terms, path = summing_vs_trials(ctx, ds, args)
        assert path_names(path) == one_launch_path(args), (n, args, path_names(path))
        assert_terms(terms, ref, f"one-block {n} {args}")
        assert_chunks(ctx, ds, ref, f"one-block {n} {args}")
        assert ds.wiener_like(*args, *KN) == tot
        assert path_names(ctx.last_path()) == one_launch_path(args)
        ds.close()


def _seed3():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "seed3_nodes.npz"),
                        allow_pickle=False))


def test_oracle_matches_seed3_fixture(oracle_lib):
    """CPU: the oracle reproduces the reference's terms on config 4's seed-3
    burn-in region (tests/golden/seed3_nodes.npz, made from oracle/_ref) bit
    for bit."""
    g = _seed3()
    x, ids = g["x"], g["node"]
    err, n_st, n_sz, ua, se, w = g["knobs"]
    for name in ("trap", "truth"):
        P = g["params_" + name]
        got = np.array([math.log(oracle_lib.full_pdf(xi, *P[j][:7], err, int(n_st), int(n_sz),
                                                     int(ua), se) * (1 - P[j][7]) + w * P[j][7])
                        for xi, j in zip(x, ids)])
        assert np.array_equal(got, g["terms_" + name]), name


@pytest.mark.gpu
def test_seed3_burn_in_region_per_trial(gpu):
    """The batched node path (wiener_like_nodes, what the config-4 sampler
    calls) at the parameters config 4's seed-3 chain sat at (a 12-23, v 7-22,
    sv 18, sz 0.97, st 0.2) and at truth-like ones: per trial at 1e-6 and per
    node against the reference's fsum."""
    g = _seed3()
    x, ids = g["x"], g["node"]
    err, n_st, n_sz, ua, se, w = g["knobs"]
    ds = gpu.Dataset(x, node_id=ids, n_nodes=400)
    for name in ("trap", "truth", "trap"):
        sums, terms = ds.wiener_like_nodes(g["params_" + name], err, int(n_st), int(n_sz),
                                           int(ua), se, w, trials=True)
        assert_terms(terms, g["terms_" + name], f"seed3 {name}")
        ref = g["nodes_" + name]
        scale = np.array([math.fsum(np.abs(g["terms_" + name][ids == j])) for j in range(400)])
        assert np.all(np.abs(sums - ref) <= 1e-12 * scale + 1e-12), name
