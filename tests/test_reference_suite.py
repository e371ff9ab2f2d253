"""The reference's own likelihood tests (hddm/tests/test_likelihoods.py), restated.

Each test runs twice: against the oracle (CPU restatement, pinned to the
reference) and against the MI355X kernels through the drop-in `hddm_amd.wfpt`
module (marked gpu). Tolerances are the reference's own decimals.
"""
import numpy as np
import pytest
from scipy import integrate
from scipy.stats import norm


def _impl_oracle():
    import oracle
    oracle.build()
    return oracle


def _impl_gpu():
    from hddm_amd import _lib, wfpt
    assert _lib.device_count() >= 1, "gpu test without a visible HIP device"
    return wfpt


IMPLS = [pytest.param(_impl_oracle, id="oracle"),
         pytest.param(_impl_gpu, id="mi355x", marks=pytest.mark.gpu)]


@pytest.fixture(params=IMPLS)
def W(request):
    return request.param()


def test_pdf_no_matlab(W, golden):
    """test_likelihoods.py:49-56 — Navarro-Fuss MATLAB values to 9 decimals."""
    for v, t, a, z, z_nonorm, rt, err, matlab in golden["matlab"]["vals"]:
        mine = W.full_pdf(-rt, v, 0, a, z, 0, t, 0, err, 0)
        np.testing.assert_array_almost_equal(matlab, mine, 9)


def test_summed_logp(W):
    """test_likelihoods.py:79-97 — sum(pdf_array(logp)) vs wiener_like; -inf on rt=0."""
    rng = np.random.RandomState(123)
    p = dict(sv=2.5 * rng.rand(), sz=rng.rand() * 0.4, st=rng.rand() * 0.35,
             z=0.5, v=(rng.rand() - .5) * 8, t=0.2 + rng.rand() * 0.3, a=0.5 + rng.rand() * 1.5)
    rts = p["t"] + p["st"] + rng.rand(50) * 2
    lp = W.pdf_array(rts, p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"], 1e-4,
                     logp=True)
    like = W.wiener_like(rts, p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"], 1e-4)
    np.testing.assert_almost_equal(np.sum(lp), like, 2)
    assert W.wiener_like(np.array([1., 2., 3., 0.]), 1, 0, 2, .5, 0, 0, 0, 1e-4) == -np.inf


def test_pdf_sv(W):
    """test_likelihoods.py:99-114 — analytic sv integral vs quad over N(v, sv)."""
    rng = np.random.RandomState(3123)
    for _ in range(20):
        sv = rng.rand() * 0.4 + 0.1
        v = (rng.rand() - .5) * 4
        t = rng.rand() * .5
        a = 1.5 + rng.rand()
        z = .5 * rng.rand()
        rt = rng.rand() * 4 + t
        err = 10 ** (-3 - np.ceil(rng.rand() * 12))
        f = lambda v_i: W.full_pdf(rt, v_i, 0, a, z, 0, 0, 0, err) * norm.pdf(v_i, v, sv)
        ref = integrate.quad(f, -np.inf, np.inf, epsrel=1e-10, epsabs=1e-10)[0]
        mine = W.full_pdf(rt, v, sv, a, z, 0, 0, 0, err)
        np.testing.assert_array_almost_equal(mine, ref)


def test_adaptive(W):
    """test_likelihoods.py:117-144 — adaptive (n=5) vs fixed Simpson (n=60), 3 decimals."""
    rng = np.random.RandomState(3124)
    for _ in range(20):
        v = (rng.rand() - .5) * 4
        st = rng.rand() * 0.3
        t = rng.rand() * .5 + (st / 2)
        a = 1.5 + rng.rand()
        rt = (rng.rand() * 4 + t) * np.sign(rng.rand())
        sz = rng.rand() * 0.3
        z = .5 * rng.rand() + sz / 2
        mine = W.full_pdf(rt, v, 0, a, z, 0, t, st, 1e-9, n_st=5, n_sz=5, use_adaptive=1)
        ref = W.full_pdf(rt, v, 0, a, z, 0, t, st, 1e-9, n_st=60, n_sz=60, use_adaptive=0)
        assert not np.isnan(mine) and not np.isnan(ref)
        np.testing.assert_array_almost_equal(mine, ref, 3)


def test_pdf_integrate_to_one(W):
    """test_likelihoods.py:147-161 — exp(wiener_like) integrates to 1 over [-5, 5]."""
    rng = np.random.RandomState(123)
    for _ in range(2):
        sv = rng.rand() * 0.4 + 0.1
        v = (rng.rand() - .5) * 4
        st = rng.rand() * 0.3
        t = rng.rand() * .5 + (st / 2)
        a = 1.5 + rng.rand()
        sz = rng.rand() * 0.3
        z = .5 * rng.rand() + sz / 2
        f = lambda x: np.exp(W.wiener_like(np.array([x]), v, sv, a, z, sz, t, st, 1e-8))
        integ, _ = integrate.quad(f, a=-5, b=5, limit=100)
        np.testing.assert_almost_equal(integ, 1, 2)


def test_wiener_like_full_single(W):
    """test_likelihoods.py:163-222 — sv/sz/st integrals vs composite Simpson grids."""
    rng = np.random.RandomState(3125)
    n = 60
    for _ in range(5):
        sv = rng.rand() * 0.4 + 0.1
        v = (rng.rand() - .5) * 4
        st = rng.rand() * 0.3
        t = rng.rand() * .5 + (st / 2)
        a = 1.5 + rng.rand()
        rt = (rng.rand() * 4 + t) * np.sign(rng.rand())
        sz = rng.rand() * 0.3
        z = .5 * rng.rand() + sz / 2
        for svv in (0, sv):
            mine = W.full_pdf(rt, v, svv, a, z, sz, t, st, 1e-8, n_st=n, n_sz=n)
            zs = z - sz / 2. + sz / n * np.arange(n + 1)
            ts = t - st / 2. + st / n * np.arange(n + 1)
            grid = np.array([[W.full_pdf(rt, v, svv, a, zz, 0, tt, 0, 1e-8, 0, 0) / sz / st
                              for zz in zs] for tt in ts])
            inner = integrate.simpson(grid, dx=sz / n, axis=1)
            ref = integrate.simpson(inner, dx=st / n)
            np.testing.assert_array_almost_equal(mine, ref, 2)


def test_failure_mode(W):
    """test_likelihoods.py:225-262 — invalid parameters give exactly 0."""
    for rt in (-0.6, 0.6):
        base = dict(v=1, sv=1, a=1.5, z=0.5, sz=0.2, t=0.2, st=0.1)
        bad = [dict(z=1.1), dict(z=-0.1), dict(z=0.1, sz=0.25), dict(a=-0.1),
               dict(t=0.7, st=0), dict(t=-0.3), dict(t=0.1, st=0.3)]
        for b in bad:
            p = dict(base, **b)
            assert W.full_pdf(rt, p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"],
                              1e-10, n_st=10, n_sz=10) == 0
