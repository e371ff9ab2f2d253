"""Several parameter tables per node launch (wfpt_wiener_like_nodes_multi):
config 4's chains in lockstep and the slice step's paired probes.

Each table's sums must be bit-identical to a one-table wiener_like_nodes call
on that table (same kernels' operations per trial: level 0, speculative
records or the chunk engine, the fixed segment order), and per trial within
1e-6 of the reference (the oracle pinned to oracle/_ref) on config 4's own
dataset and on the seed-3 burn-in fixture, whose tables defer thousands of
trials to the records / chunk engine.
"""
import math
import os

import numpy as np
import pytest

from test_parity_summing import _seed3, assert_terms
from test_parity_trials import KN, node_terms_ref

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c4(full):
    from hddm_amd.hierarchical import HDDM, gen_data
    inter = dict(sv=0.1, sz=0.1, st=0.1) if full else {}
    data, truth = gen_data(n_subj=200, n_trials=500, **inter)
    m = HDDM(data, depends_on={"v": "cond"}, include=tuple(inter), p_outlier=0.05)
    start = m.node_table().copy()
    P = start.copy()
    for j, (s, c) in enumerate(m.node_keys):
        P[j, 0] = truth["v"][c][s]
        P[j, 2] = truth["a"][s]
        P[j, 5] = truth["t"][s]
        for k, col in (("sv", 1), ("sz", 4), ("st", 6)):
            P[j, col] = inter.get(k, 0.0)
    return m, data, start, P


def _chain_tables(rng, P, T, full):
    """T tables around P as T chains' states: subject-level v, a, t moved
    independently per table (and the group-level sv, sz, st per table in the
    full model)."""
    out = np.repeat(P[None], T, axis=0)
    m = P.shape[0]
    out[:, :, 0] += rng.normal(0, 0.3, (T, m))
    out[:, :, 2] *= np.exp(rng.normal(0, 0.08, (T, m)))
    out[:, :, 5] = np.maximum(out[:, :, 5] + rng.normal(0, 0.02, (T, m)), 0.05)
    if full:
        for col, sd in ((1, 0.3), (4, 0.05), (6, 0.03)):
            out[:, :, col] = np.abs(P[0, col] + rng.normal(0, sd, (T, 1)))
    return out


@pytest.mark.parametrize("full", [False, True])
def test_multi_tables_bitwise_equal_single_calls(gpu, full):
    m, _, start, P = _c4(full)
    ds = m.dataset
    rng = np.random.default_rng(20261018 + full)
    for T in (1, 2, 8, 17):
        tabs = _chain_tables(rng, P, T, full)
        if T >= 2:
            tabs[0] = start  # HDDM's starting values (a 1, t .001: mostly settled at level 0)
            tabs[1] = P      # the generating parameters (sparse records)
        got = ds.wiener_like_nodes_multi(tabs, **m.wp)
        assert got.shape == (T, m.n_nodes)
        for t in range(T):
            one = ds.wiener_like_nodes(tabs[t], **m.wp)
            bad = np.flatnonzero(got[t] != one)
            assert bad.size == 0, (T, t, bad[:5], got[t][bad[:5]], one[bad[:5]])


@pytest.mark.parametrize("full", [False, True])
def test_multi_tables_per_trial_config4(gpu, oracle_lib, full):
    """Per trial at 1e-6 against the reference for every table of a 3-table
    call on config 4's dataset, and the per-node sums against fsum."""
    m, data, start, P = _c4(full)
    x = data["rt"].to_numpy(dtype=np.float64)
    node = data.groupby(["subj_idx", "cond"], sort=True).ngroup().to_numpy()
    tabs = np.stack([start, P, _chain_tables(np.random.default_rng(5), P, 1, full)[0]])
    sums, terms = m.dataset.wiener_like_nodes_multi(tabs, **m.wp, trials=True)
    kn = (m.wp["err"], m.wp["n_st"], m.wp["n_sz"], m.wp["use_adaptive"], m.wp["simps_err"],
          m.wp["w_outlier"])
    for t in range(3):
        ref = node_terms_ref(oracle_lib, x, node, tabs[t], kn)
        assert_terms(terms[t], ref, f"C4 full={full} table {t}")
        for j in range(m.n_nodes):
            rj = ref[node == j]
            if np.isneginf(rj).any():
                assert sums[t, j] == -np.inf
            else:
                assert abs(sums[t, j] - math.fsum(rj)) <= 1e-11 * math.fsum(np.abs(rj)), (t, j)


def test_multi_tables_seed3_fixture(gpu):
    """The seed-3 burn-in tables (52,875 of 100k trials leave level 0: the
    chunk engine) next to the truth-like table (sparse records) in one call:
    per trial against the fixture's reference terms, per node against fsum,
    and each table bit-equal to its own one-table call."""
    g = _seed3()
    x, ids = g["x"], g["node"]
    err, n_st, n_sz, ua, se, w = g["knobs"]
    kn = (err, int(n_st), int(n_sz), int(ua), se, w)
    ds = gpu.Dataset(x, node_id=ids, n_nodes=400)
    names = ("trap", "truth", "trap", "truth")
    tabs = np.stack([g["params_" + nm] for nm in names])
    sums, terms = ds.wiener_like_nodes_multi(tabs, *kn, trials=True)
    for t, nm in enumerate(names):
        assert_terms(terms[t], g["terms_" + nm], f"seed3 {nm} table {t}")
        ref = g["nodes_" + nm]
        scale = np.array([math.fsum(np.abs(g["terms_" + nm][ids == j])) for j in range(400)])
        assert np.all(np.abs(sums[t] - ref) <= 1e-12 * scale + 1e-12), (t, nm)
        assert np.array_equal(sums[t], ds.wiener_like_nodes(tabs[t], *kn)), (t, nm)


def test_multi_tables_mixed_families_and_errors(gpu):
    """Tables whose nodes select different integration families take the
    generic kernel once per table (still bit-equal to the one-table call);
    shapes are checked before the call."""
    rng = np.random.default_rng(3)
    n_nodes = 23
    sizes = rng.integers(0, 300, n_nodes)
    node = np.repeat(np.arange(n_nodes), sizes)
    rng.shuffle(node)
    x = rng.choice([-1.0, 1.0], node.size) * (0.35 + rng.gamma(2.0, 0.4, node.size))
    ds = gpu.Dataset(x, node_id=node, n_nodes=n_nodes)
    tabs = np.zeros((3, n_nodes, 8))
    tabs[:, :, 0] = rng.uniform(-2, 2, (3, n_nodes))
    tabs[:, :, 1] = rng.choice([0.0, 0.4], (3, n_nodes))
    tabs[:, :, 2] = rng.uniform(0.8, 2.0, (3, n_nodes))
    tabs[:, :, 3] = 0.5
    tabs[:, :, 4] = rng.choice([0.0, 0.1], (3, n_nodes))
    tabs[:, :, 5] = rng.uniform(0.2, 0.3, (3, n_nodes))
    tabs[:, :, 6] = rng.choice([0.0, 0.1], (3, n_nodes))
    tabs[:, :, 7] = 0.05
    got = ds.wiener_like_nodes_multi(tabs)
    for t in range(3):
        assert np.array_equal(got[t], ds.wiener_like_nodes(tabs[t])), t
    with pytest.raises(ValueError):
        ds.wiener_like_nodes_multi(tabs[0])
    with pytest.raises(ValueError):
        ds.wiener_like_nodes_multi(tabs[:, :-1])
    with pytest.raises(ValueError):
        gpu.Dataset(x).wiener_like_nodes_multi(tabs)


@pytest.mark.parametrize("family", ["simple", "full", "st_only"])
def test_rare_trials_settled_and_republished(gpu, oracle_lib, family):
    """Trials the node kernels cannot settle -- densities below kExactBelow
    without an outlier mixture to absorb them (RTs a hair above t, p_outlier
    = 0), i.e. the exact path -- go to the rare list; the publication reports
    the call pending, node_rare_kernel settles them and the sums are published
    again (WFPT_PATH_NODE_RARE). Per trial against the reference, per node
    against fsum, one- and multi-table calls bit-equal, and the next call
    (no rare trial) is not pending."""
    from hddm_amd import _lib
    rng = np.random.default_rng({"simple": 21, "full": 22, "st_only": 23}[family])
    n_nodes = 12
    sizes = rng.integers(40, 120, n_nodes)
    node = np.repeat(np.arange(n_nodes), sizes)
    rng.shuffle(node)
    t = 0.3
    x = rng.choice([-1.0, 1.0], node.size) * (t + 0.4 + rng.gamma(2.0, 0.3, node.size))
    close = rng.random(node.size) < 0.08  # a hair above t: tiny densities
    x[close] = np.sign(x[close]) * (t + rng.uniform(2e-4, 2e-3, close.sum()))
    P = np.zeros((n_nodes, 8))
    P[:, 0] = rng.uniform(-1.5, 1.5, n_nodes)
    P[:, 2] = rng.uniform(1.5, 2.5, n_nodes)
    P[:, 3] = 0.5
    P[:, 5] = t
    if family == "full":
        P[:, 1], P[:, 4], P[:, 6] = 0.3, 0.1, 1e-4
    elif family == "st_only":
        P[:, 6] = 1e-4
    P[:, 7] = np.where(np.arange(n_nodes) % 2 == 0, 0.0, 0.05)  # no mixture on even nodes
    ds = gpu.Dataset(x, node_id=node, n_nodes=n_nodes)
    ctx = _lib.context()
    sums, terms = ds.wiener_like_nodes(P, *KN, trials=True)
    assert ctx.last_path() & _lib.PATH_NODE_RARE, "no rare trial reached the rare list"
    ref = node_terms_ref(oracle_lib, x, node, P)
    assert_terms(terms, ref, f"rare {family}")
    for j in range(n_nodes):
        rj = ref[node == j]
        if np.isneginf(rj).any():
            assert sums[j] == -np.inf
        else:
            assert abs(sums[j] - math.fsum(rj)) <= 1e-11 * math.fsum(np.abs(rj)) + 1e-12, j
    assert np.array_equal(ds.wiener_like_nodes(P, *KN), sums)
    multi = ds.wiener_like_nodes_multi(np.stack([P, P]), *KN)
    assert np.array_equal(multi[0], sums) and np.array_equal(multi[1], sums)
    P2 = P.copy()
    P2[:, 5] = 0.1  # every RT well above t: no tiny density, nothing rare
    s2 = ds.wiener_like_nodes(P2, *KN)
    assert not ctx.last_path() & _lib.PATH_NODE_RARE
    assert np.all(np.isfinite(s2))
