"""The PyMC-facing stochastic (hddm/likelihoods.py:30-105): `random` and the
resident-data cache behind `wfpt_like`."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_random_matches_reference_gen_rts(oracle_lib, monkeypatch):
    """node.random() (likelihoods.py:76-81) = flip_errors(gen_rts(method='cdf',
    structured=True)): a DataFrame of the reference's samples with signed 'rt'
    and 'response' 1/0. Fed the reference's grid densities (the oracle's,
    bit-exact), the samples equal the committed gen_rts fixture bit for bit."""
    from hddm_amd import likelihoods, wfpt
    monkeypatch.setattr(wfpt, "pdf_array", oracle_lib.pdf_array)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "gen_rts.npz")))
    cls = likelihoods.generate_wfpt_stochastic_class()
    for k in range(4):
        v, sv, a, z, sz, t, st, n, lb, ub, dt, seed = g[f"args_{k}"]
        cls = likelihoods.generate_wfpt_stochastic_class(cdf_range=(lb, ub), sampling_dt=dt)
        node = cls("wfpt", np.zeros(int(n)), v=v, sv=sv, a=a, z=z, sz=sz, t=t, st=st,
                   p_outlier=0.0)
        np.random.seed(int(seed))
        df = node.random()
        assert list(df.columns) == ["rt", "response"] and len(df) == int(n)
        np.testing.assert_array_equal(df["rt"].to_numpy(), g[f"rts_{k}"])
        np.testing.assert_array_equal(df["response"].to_numpy(),
                                      (g[f"rts_{k}"] >= 0).astype(float))


def test_random_size_conventions(oracle_lib, monkeypatch):
    """generate.py:180-184: PyMC shapes () -> 1 sample, (n,) -> n samples."""
    from hddm_amd import likelihoods, wfpt
    monkeypatch.setattr(wfpt, "pdf_array", oracle_lib.pdf_array)
    p = dict(v=0.5, a=2.0, t=0.3)
    assert len(likelihoods.gen_random(p, (), "cdf", (-5, 5), 1e-2)) == 1
    assert len(likelihoods.gen_random(p, (37,), "cdf", (-5, 5), 1e-2)) == 37


@pytest.mark.gpu
def test_resident_cache_identity_and_staleness(gpu, oracle_lib):
    """wfpt_like serves repeated calls on the same node value from one
    resident upload without an O(n) host pass, and an in-place rewrite of the
    value is not served stale."""
    import pandas as pd
    from hddm_amd import likelihoods
    likelihoods._cache.clear()
    rng = np.random.default_rng(9)
    x = rng.choice([-1.0, 1.0], 5000) * (0.35 + rng.gamma(2.0, 0.4, 5000))
    df = pd.DataFrame({"rt": x.copy()})
    like = likelihoods.make_wfpt_like()
    args = (0.7, 0.2, 1.8, 0.5, 0.1, 0.3, 0.1)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    a = like(df, *args, p_outlier=0.05)
    assert len(likelihoods._cache._by_bytes) == 1
    b = like(df, *args, p_outlier=0.05)
    assert a == b and len(likelihoods._cache._by_bytes) == 1
    ref = oracle_lib.wiener_like(df["rt"].to_numpy(), *args, *kn)
    assert abs(a - ref) < 1e-9 * abs(ref)
    # in-place rewrite of sampled positions: a new upload, the new value
    col = df["rt"].to_numpy()
    col[::100] *= 1.1
    df["rt"] = col
    c = like(df, *args, p_outlier=0.05)
    ref2 = oracle_lib.wiener_like(df["rt"].to_numpy(), *args, *kn)
    assert abs(c - ref2) < 1e-9 * abs(ref2) and c != a
    # one element that no sample would cover (the column is below EXACT_MAX:
    # the whole column is compared on every hit)
    col = df["rt"].to_numpy()
    col[57] = col[57] * 1.05
    df["rt"] = col
    d = like(df, *args, p_outlier=0.05)
    ref3 = oracle_lib.wiener_like(df["rt"].to_numpy(), *args, *kn)
    assert abs(d - ref3) < 1e-9 * abs(ref3) and d != c
    # a second node holding equal data shares the upload
    n0 = len(likelihoods._cache._by_bytes)
    like(pd.DataFrame({"rt": df["rt"].to_numpy().copy()}), *args, p_outlier=0.05)
    assert len(likelihoods._cache._by_bytes) == n0


def test_install_patches_hot_path_only():
    """install() rebinds the hot-path attributes of the
    reference's `wfpt` / `cdfdif_wrapper` module objects (hddm_rl.py:8 and
    rl.py:8 hold the same objects and keep wiener_like_rl*), and restores
    them on uninstall; with no reference module, ours is registered."""
    import sys
    import types
    from hddm_amd import cdfdif_wrapper as amd_cdf, integration, wfpt as amd
    ref = types.ModuleType("wfpt")
    for n in integration.HOT_PATH + ("wiener_like_rl", "wiener_like_rlddm", "split_cdf"):
        setattr(ref, n, lambda *a, _n=n: _n)
    cdf = types.ModuleType("cdfdif_wrapper")
    cdf.dmat_cdf_array = lambda *a: "ref"
    lk = types.ModuleType("hddm.likelihoods")
    lk.generate_wfpt_stochastic_class = lambda *a, **k: "ref-class"
    lk.Wfpt = "ref-Wfpt"
    held_by_rl = ref                      # `import wfpt` in hddm/models/hddm_rl.py
    from hddm_amd import likelihoods as amd_lk
    inst = integration.install(ref, cdf, lk)
    assert lk.generate_wfpt_stochastic_class is amd_lk.generate_wfpt_stochastic_class
    assert lk.Wfpt != "ref-Wfpt"
    for n in integration.HOT_PATH:
        assert getattr(held_by_rl, n) is getattr(amd, n)
    assert held_by_rl.wiener_like_rl() == "wiener_like_rl"
    assert held_by_rl.split_cdf() == "split_cdf"
    assert cdf.dmat_cdf_array is amd_cdf.dmat_cdf_array
    inst.uninstall()
    assert ref.wiener_like() == "wiener_like" and cdf.dmat_cdf_array() == "ref"
    assert lk.generate_wfpt_stochastic_class() == "ref-class" and lk.Wfpt == "ref-Wfpt"
    # no reference extension importable here: ours under the module names
    had = {k: sys.modules.get(k) for k in ("wfpt", "cdfdif_wrapper")}
    inst = integration.install()
    try:
        if had["wfpt"] is None:
            assert sys.modules["wfpt"] is amd
        if had["cdfdif_wrapper"] is None:
            assert sys.modules["cdfdif_wrapper"] is amd_cdf
    finally:
        inst.uninstall()
    for k, v in had.items():
        assert sys.modules.get(k) is v
