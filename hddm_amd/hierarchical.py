"""Hierarchical DDM sampler that scores every observed node in one launch.

The reference builds the model with kabuki + PyMC 2 (hddm/models/base.py,
hddm_info.py) and samples node by node: each slice step of one subject
parameter calls `wfpt_like` on that subject's nodes (likelihoods.py:52-73),
i.e. thousands of tiny CPU likelihood calls per sweep. Neither kabuki nor
PyMC is available here, so this module restates the model and its step
methods around the batched GPU likelihood:

* model (informative HDDM, hddm_info.py:121-140; families base.py:578-690):
    a_subj ~ Gamma(mean=a, sd=a_std),  a ~ Gamma(mean 1.5, sd 0.75), a_std ~ HalfNormal(sd 2)
    v_subj ~ Normal(v, v_std),         v ~ Normal(2, sd 3),          v_std ~ HalfNormal(sd 2)
    t_subj ~ Gamma(mean=t, sd=t_std),  t ~ Gamma(mean .4, sd .2),    t_std ~ HalfNormal(sd 1)
    sv ~ HalfNormal(sd 2), sz ~ Beta(1, 3), st ~ HalfNormal(sd .3)   (group only, if included)
    z = 0.5, p_outlier = 0.05 (base.py:687-752)
  `depends_on={'v': 'cond'}` splits a family per condition level (kabuki), with
  one shared std node (std_depends=False, base.py:614).
* step methods (hddm_info.py:163-175): the group mean of a Normal family with
  Normal children is Gibbs-updated (kNormalNormal); everything else is
  slice-sampled (stepping out + shrinkage, Neal 2003) with the reference's
  slice widths (hddm_info.py:103-105).
* batching: subject-level parameters of one kind are conditionally
  independent given the group level, so all of them take their slice step
  together (a block Gibbs update with the same stationary distribution as the
  reference's one-at-a-time sweep); each evaluation of the slice is ONE call
  of `Dataset.wiener_like_nodes` over all (subject x condition) nodes.

Model-level parity with the reference sampler is unpinned (PyMC/kabuki are
absent); the per-node log-likelihood it uses is pinned to the reference via
tests/test_hierarchical.py.
"""
import math
import time

import numpy as np
from scipy import special

from . import wfpt as _wfpt

SLICE_WIDTHS = {"a": 1, "t": 0.01, "a_std": 1, "t_std": 0.15, "sz": 1.1, "v": 1.5, "st": 0.1,
                "sv": 3, "v_std": 1}  # hddm_info.py:103-105
WIENER_PARAMS = {"err": 1e-4, "n_st": 2, "n_sz": 2, "use_adaptive": 1, "simps_err": 1e-3,
                 "w_outlier": 0.1}  # base.py:712-716


# ---------------------------------------------------------------- log densities

def gamma_logpdf_mean_sd(x, mean, sd):
    """pm.Gamma(alpha=mean^2/sd^2, beta=mean/sd^2) (base.py:642-667); -inf for
    x <= 0. It runs once per slice evaluation next to a ~20 us likelihood call,
    so the common case (scalar parameters, every x > 0) avoids NumPy's error
    state machinery and array-valued special functions."""
    x = np.asarray(x, dtype=np.float64)
    if isinstance(mean, float) and isinstance(sd, float) and mean > 0 and sd > 0:
        shape = mean * mean / (sd * sd)
        rate = mean / (sd * sd)
        if x.min(initial=np.inf) > 0:
            return (shape * math.log(rate) - math.lgamma(shape)) + (shape - 1) * np.log(x) - rate * x
    shape = mean ** 2 / sd ** 2
    rate = mean / sd ** 2
    with np.errstate(divide="ignore", invalid="ignore"):
        out = shape * np.log(rate) - special.gammaln(shape) + (shape - 1) * np.log(x) - rate * x
    return np.where(x > 0, out, -np.inf)


def normal_logpdf(x, mu, sd):
    return -0.5 * np.log(2 * np.pi * sd ** 2) - 0.5 * ((x - mu) / sd) ** 2


def halfnormal_logpdf(x, sd):
    x = np.asarray(x, dtype=np.float64)
    out = 0.5 * np.log(2 / (np.pi * sd ** 2)) - 0.5 * (x / sd) ** 2
    return np.where(x >= 0, out, -np.inf)


def beta_logpdf(x, a, b):
    x = np.asarray(x, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        out = (a - 1) * np.log(x) + (b - 1) * np.log1p(-x) - special.betaln(a, b)
    return np.where((x > 0) & (x < 1), out, -np.inf)


# ---------------------------------------------------------------- slice sampler

def slice_step(x0, logp, w, rng, lower=None, max_steps=50, max_shrink=200, logp_pair=None,
               masked=False):
    """Vectorised univariate slice sampling (stepping out + shrinkage).

    x0: (n,) current values of n conditionally independent coordinates;
    logp(x) -> (n,) log conditional of each coordinate evaluated at x (one
    batched likelihood call). Returns the new values and the number of logp
    calls used.

    logp_pair(xl, xr) -> (f(xl), f(xr)) (optional: both probes in ONE batched
    call, wfpt_wiener_like_nodes_multi with two tables): the left and right
    stepping-out run side by side. Given y and the initial interval the two
    sides are independent (Neal 2003, fig. 3), so L, R -- and with the same
    random numbers the whole step -- are those of the side-by-side-free loop;
    only the number of calls drops (max of the two sides' steps instead of
    their sum).

    masked=True: logp(x, active) and logp_pair(xl, xr, act_l, act_r) also get
    the coordinates whose value the step will read; the others' results are
    never used (a caller may skip evaluating them -- HDDMChains drops settled
    chains' tables from the launch).
    """
    x0 = np.asarray(x0, dtype=np.float64)
    n = x0.size
    calls = 1
    y = logp(x0) - rng.exponential(size=n)
    L = x0 - w * rng.uniform(size=n)
    R = L + w
    if lower is not None:
        L = np.maximum(L, lower)

    def grow_left(active, f):
        nonlocal L
        grow = active & (f > y)
        L = np.where(grow, L - w, L)
        if lower is not None:
            L = np.maximum(L, lower)
            grow &= L > lower
        return grow

    def grow_right(active, f):
        nonlocal R
        grow = active & (f > y)
        R = np.where(grow, R + w, R)
        return grow

    def f1(x, act):
        return logp(x, act) if masked else logp(x)

    if logp_pair is not None:
        act_l = np.ones(n, dtype=bool)
        act_r = np.ones(n, dtype=bool)
        steps_l = steps_r = 0
        while True:
            do_l = steps_l < max_steps and act_l.any()
            do_r = steps_r < max_steps and act_r.any()
            if do_l and do_r:
                pl, pr = np.where(act_l, L, x0), np.where(act_r, R, x0)
                fl, fr = logp_pair(pl, pr, act_l, act_r) if masked else logp_pair(pl, pr)
            elif do_l:
                fl = f1(np.where(act_l, L, x0), act_l)
            elif do_r:
                fr = f1(np.where(act_r, R, x0), act_r)
            else:
                break
            calls += 1
            if do_l:
                act_l = grow_left(act_l, fl)
                steps_l += 1
            if do_r:
                act_r = grow_right(act_r, fr)
                steps_r += 1
    else:
        for side in (0, 1):
            active = np.ones(n, dtype=bool)
            for _ in range(max_steps):
                probe = np.where(active, L if side == 0 else R, x0)
                f = f1(probe, active)
                calls += 1
                grow = grow_left(active, f) if side == 0 else grow_right(active, f)
                if not grow.any():
                    break
                active = grow
    x1 = x0.copy()
    done = np.zeros(n, dtype=bool)
    for _ in range(max_shrink):
        cand = np.where(done, x1, L + rng.uniform(size=n) * (R - L))
        f = f1(cand, ~done)
        calls += 1
        acc = ~done & (f > y)
        x1 = np.where(acc, cand, x1)
        done |= acc
        if done.all():
            break
        lo = ~done & (cand < x0)
        L = np.where(lo, cand, L)
        R = np.where(~done & ~lo, cand, R)
    return x1, calls


# ---------------------------------------------------------------- the model

class HDDM:
    """HDDM(data, depends_on={'v': 'cond'}).sample(n) on one MI355X.

    data: pandas DataFrame with columns rt (seconds), response (1 upper / 0
    lower; optional when rt is already signed), subj_idx and the condition
    columns named in depends_on.
    """

    FAMILIES = ("a", "v", "t")

    def __init__(self, data, depends_on=None, include=(), p_outlier=0.05, wiener_params=None,
                 seed=None, device=None, paired_probes=True):
        import pandas as pd
        # both stepping-out probes of a slice step in one two-table call
        # (slice_step's logp_pair): the same chain, fewer likelihood calls
        self.paired_probes = bool(paired_probes)
        self.data = data = pd.DataFrame(data).reset_index(drop=True)
        self.depends = {k: ([v] if isinstance(v, str) else list(v))
                        for k, v in (depends_on or {}).items()}
        for k in self.depends:
            if k not in self.FAMILIES + ("sv", "sz", "st"):
                raise NotImplementedError(f"depends_on for '{k}' is not supported")
        self.include = set(include) | {"a", "v", "t"}
        unsupported = self.include - {"a", "v", "t", "sv", "sz", "st"}
        if unsupported:
            raise NotImplementedError(f"include {sorted(unsupported)} is not supported")
        self.p_outlier = float(p_outlier)
        self.wp = dict(WIENER_PARAMS if wiener_params is None else wiener_params)
        self.rng = np.random.default_rng(seed)

        rt = data["rt"].to_numpy(dtype=np.float64)
        if "response" in data and not np.any(rt < 0):
            rt = np.where(data["response"].to_numpy() == 0, -np.abs(rt), np.abs(rt))  # flip_errors
        subj_levels = np.sort(data["subj_idx"].unique())
        self.n_subj = len(subj_levels)
        cond_cols = sorted({c for cs in self.depends.values() for c in cs})
        keys = ["subj_idx"] + cond_cols
        grp = data.groupby(keys, sort=True)
        node_codes = grp.ngroup().to_numpy()
        node_frame = grp.size().reset_index()[keys]
        self.node_keys = [tuple(r) for r in node_frame.itertuples(index=False)]
        self.n_nodes = len(node_frame)
        self.node_subj = np.searchsorted(subj_levels, node_frame["subj_idx"].to_numpy())
        # per family: condition level of each node and (subject, level) unit of each node
        self.levels, self.node_level, self.node_unit, self.n_units = {}, {}, {}, {}
        for fam in self.FAMILIES:
            cols = self.depends.get(fam, [])
            if cols:
                g = node_frame.groupby(cols, sort=True)
                lv_codes = g.ngroup().to_numpy()
                self.levels[fam] = [tuple(r) for r in g.size().reset_index()[cols]
                                    .itertuples(index=False)]
            else:
                lv_codes = np.zeros(self.n_nodes, dtype=np.int64)
                self.levels[fam] = [()]
            n_lv = len(self.levels[fam])
            self.node_level[fam] = lv_codes
            self.node_unit[fam] = self.node_subj * n_lv + lv_codes
            self.n_units[fam] = self.n_subj * n_lv
        self.dataset = _wfpt.Dataset(rt, node_id=node_codes, n_nodes=self.n_nodes, device=device)
        self.n_trials = rt.size
        self.likelihood_calls = 0
        self.likelihood_seconds = 0.0
        self.call_stats = {}  # updated parameter -> [calls, seconds]
        self._init_values()

    # -- state ---------------------------------------------------------------
    def _init_values(self):
        """Starting values of hddm_info.py:121-140."""
        nl = {f: len(self.levels[f]) for f in self.FAMILIES}
        self.group = {"a": np.full(nl["a"], 1.5), "v": np.full(nl["v"], 2.0),
                      "t": np.full(nl["t"], 0.4)}
        self.std = {"a": 0.1, "v": 0.1, "t": 0.2}
        self.subj = {"a": np.full(self.n_units["a"], 1.0), "v": np.full(self.n_units["v"], 2.0),
                     "t": np.full(self.n_units["t"], 0.001)}
        self.inter = {"sv": 1.0 if "sv" in self.include else 0.0,
                      "sz": 0.01 if "sz" in self.include else 0.0,
                      "st": 0.001 if "st" in self.include else 0.0}

    _COL = {"v": 0, "sv": 1, "a": 2, "sz": 4, "t": 5, "st": 6}

    def node_table(self, over=None):
        """(n_nodes, 8) parameter table v, sv, a, z, sz, t, st, p_outlier. The
        table at the current values is kept and only the columns in `over`
        (the one parameter a slice step moves) are rewritten."""
        key = (self.subj["v"].tobytes(), self.subj["a"].tobytes(), self.subj["t"].tobytes(),
               self.inter["sv"], self.inter["sz"], self.inter["st"])
        if getattr(self, "_table_key", None) != key:
            P = np.empty((self.n_nodes, 8))
            P[:, 0] = self.subj["v"][self.node_unit["v"]]
            P[:, 1] = self.inter["sv"]
            P[:, 2] = self.subj["a"][self.node_unit["a"]]
            P[:, 3] = 0.5
            P[:, 4] = self.inter["sz"]
            P[:, 5] = self.subj["t"][self.node_unit["t"]]
            P[:, 6] = self.inter["st"]
            P[:, 7] = self.p_outlier
            self._table, self._table_key = P, key
        if not over:
            return self._table
        P = self._table.copy()
        for name, val in over.items():
            col = self._COL[name]
            P[:, col] = val[self.node_unit[name]] if name in self.FAMILIES else val
        return P

    def node_logp(self, over=None):
        t0 = time.perf_counter()
        out = self.dataset.wiener_like_nodes(self.node_table(over), **self.wp)
        dt = time.perf_counter() - t0
        self.likelihood_seconds += dt
        self.likelihood_calls += 1
        key = ",".join(sorted(over)) if over else "-"
        st = self.call_stats.setdefault(key, [0, 0.0])
        st[0] += 1
        st[1] += dt
        return out

    def node_logp_multi(self, overs):
        """node_logp for several overrides in ONE launch (list of `over` dicts
        -> (len(overs), n_nodes)): wfpt_wiener_like_nodes_multi, each row bit
        for bit the one-table call's."""
        t0 = time.perf_counter()
        out = self.dataset.wiener_like_nodes_multi(np.stack([self.node_table(o) for o in overs]),
                                                   **self.wp)
        dt = time.perf_counter() - t0
        self.likelihood_seconds += dt
        self.likelihood_calls += 1
        key = ",".join(sorted(overs[0])) + f" x{len(overs)}"
        st = self.call_stats.setdefault(key, [0, 0.0])
        st[0] += 1
        st[1] += dt
        return out

    def _unit_group(self, fam):
        """Group mean of each unit of `fam` (a float when the family has one
        level: the scalar fast path of the prior densities)."""
        if len(self.levels[fam]) == 1:
            return float(self.group[fam][0])
        return self.group[fam][np.arange(self.n_units[fam]) % len(self.levels[fam])]

    def subj_prior(self, fam, x):
        g = self._unit_group(fam)
        if fam == "v":
            return normal_logpdf(x, g, self.std["v"])
        return gamma_logpdf_mean_sd(x, g, self.std[fam])

    def logp(self):
        """Joint log density of the model at the current values."""
        lp = float(np.sum(self.node_logp()))
        for fam in self.FAMILIES:
            lp += float(np.sum(self.subj_prior(fam, self.subj[fam])))
        lp += float(np.sum(self._group_prior("a", self.group["a"])))
        lp += float(np.sum(self._group_prior("t", self.group["t"])))
        lp += float(np.sum(normal_logpdf(self.group["v"], 2.0, 3.0)))
        lp += float(np.sum([halfnormal_logpdf(self.std[f], s)
                            for f, s in (("a", 2.0), ("v", 2.0), ("t", 1.0))]))
        return lp

    @staticmethod
    def _group_prior(fam, x):
        return gamma_logpdf_mean_sd(x, 1.5, 0.75) if fam == "a" else gamma_logpdf_mean_sd(x, .4, .2)

    # -- updates ---------------------------------------------------------------
    def _update_subject(self, fam):
        unit = self.node_unit[fam]
        nu = self.n_units[fam]

        def logp(x):
            ll = np.bincount(unit, weights=self.node_logp({fam: x}), minlength=nu)
            return ll + self.subj_prior(fam, x)

        def logp_pair(xl, xr):
            r = self.node_logp_multi([{fam: xl}, {fam: xr}])
            return (np.bincount(unit, weights=r[0], minlength=nu) + self.subj_prior(fam, xl),
                    np.bincount(unit, weights=r[1], minlength=nu) + self.subj_prior(fam, xr))

        lower = 0.0 if fam in ("a", "t") else None
        self.subj[fam], _ = slice_step(self.subj[fam], logp, SLICE_WIDTHS[fam], self.rng,
                                       lower=lower,
                                       logp_pair=logp_pair if self.paired_probes else None)

    def _update_group(self, fam):
        nl = len(self.levels[fam])
        lv = np.arange(self.n_units[fam]) % nl
        if fam == "v":  # kNormalNormal: conjugate Normal mean (hddm_info.py:167-168)
            tau0, mu0 = 3.0 ** -2, 2.0
            tau = self.std["v"] ** -2
            for k in range(nl):
                xs = self.subj["v"][lv == k]
                prec = tau0 + tau * xs.size
                mean = (tau0 * mu0 + tau * xs.sum()) / prec
                self.group["v"][k] = self.rng.normal(mean, prec ** -0.5)
        else:
            def logp(g):
                out = self._group_prior(fam, g)
                for k in range(nl):
                    out[k] += np.sum(gamma_logpdf_mean_sd(self.subj[fam][lv == k], g[k],
                                                          self.std[fam]))
                return out
            self.group[fam], _ = slice_step(self.group[fam], logp, SLICE_WIDTHS[fam], self.rng,
                                            lower=0.0)
        std_sd = {"a": 2.0, "v": 2.0, "t": 1.0}[fam]

        def logp_std(s):
            s = float(s[0])
            if s <= 0:
                return np.array([-np.inf])
            g = self._unit_group(fam)
            x = self.subj[fam]
            ll = normal_logpdf(x, g, s) if fam == "v" else gamma_logpdf_mean_sd(x, g, s)
            return np.array([float(halfnormal_logpdf(s, std_sd)) + float(np.sum(ll))])

        new, _ = slice_step(np.array([self.std[fam]]), logp_std, SLICE_WIDTHS[fam + "_std"],
                            self.rng, lower=0.0)
        self.std[fam] = float(new[0])

    def _update_inter(self, name):
        prior = {"sv": lambda x: halfnormal_logpdf(x, 2.0), "sz": lambda x: beta_logpdf(x, 1, 3),
                 "st": lambda x: halfnormal_logpdf(x, 0.3)}[name]

        def logp(x):
            val = float(x[0])
            pr = float(prior(val))
            if not np.isfinite(pr):
                return np.array([-np.inf])
            return np.array([pr + float(np.sum(self.node_logp({name: val})))])

        def logp_pair(xl, xr):
            vals = (float(xl[0]), float(xr[0]))
            prs = [float(prior(v)) for v in vals]
            live = [v for v, pr in zip(vals, prs) if np.isfinite(pr)]
            if len(live) < 2:  # a probe outside the prior's support: no likelihood needed
                return logp(xl), logp(xr)
            r = self.node_logp_multi([{name: vals[0]}, {name: vals[1]}])
            return (np.array([prs[0] + float(np.sum(r[0]))]),
                    np.array([prs[1] + float(np.sum(r[1]))]))

        new, _ = slice_step(np.array([self.inter[name]]), logp, SLICE_WIDTHS[name], self.rng,
                            lower=0.0, logp_pair=logp_pair if self.paired_probes else None)
        self.inter[name] = float(new[0])

    def sweep(self):
        """One MCMC iteration: every stochastic updated once."""
        for fam in self.FAMILIES:
            self._update_group(fam)
            self._update_subject(fam)
        for name in ("sv", "sz", "st"):
            if name in self.include:
                self._update_inter(name)

    def sample(self, iter, burn=0, thin=1, progress=None):
        """Run `iter` sweeps; keep every `thin`-th after `burn`. Returns traces
        of the group-level nodes (dict name -> array)."""
        trace = {}
        names = []
        for fam in self.FAMILIES:
            for k, lv in enumerate(self.levels[fam]):
                names.append((f"{fam}" + (f"({','.join(map(str, lv))})" if lv else ""), fam, k))
        self.trace_subj = {f: [] for f in self.FAMILIES}
        for name, _, _ in names:
            trace[name] = []
        for fam in self.FAMILIES:
            trace[f"{fam}_std"] = []
        for name in ("sv", "sz", "st"):
            if name in self.include:
                trace[name] = []
        t0 = time.perf_counter()
        for it in range(iter):
            self.sweep()
            if it >= burn and (it - burn) % thin == 0:
                for name, fam, k in names:
                    trace[name].append(self.group[fam][k])
                for fam in self.FAMILIES:
                    trace[f"{fam}_std"].append(self.std[fam])
                    self.trace_subj[fam].append(self.subj[fam].copy())
                for name in ("sv", "sz", "st"):
                    if name in self.include:
                        trace[name].append(self.inter[name])
            if progress and (it + 1) % progress == 0:
                el = time.perf_counter() - t0
                print(f"  [{it + 1}/{iter}] {el:.1f}s, {self.likelihood_calls} batched "
                      f"likelihood calls", flush=True)
        self.trace = {k: np.asarray(v) for k, v in trace.items()}
        self.trace_subj = {k: np.asarray(v) for k, v in self.trace_subj.items()}
        self.sample_seconds = time.perf_counter() - t0
        return self.trace

    def gen_stats(self):
        out = {}
        for k, v in self.trace.items():
            out[k] = {"mean": float(np.mean(v)), "std": float(np.std(v)),
                      "2.5q": float(np.quantile(v, .025)), "97.5q": float(np.quantile(v, .975))}
        return out


class HDDMChains(HDDM):
    """`chains` independent chains of HDDM(...) sampled in lockstep on one GPU.

    HDDM's documented usage runs several chains (docs/source/howto.rst:267-291:
    one model per chain, then kabuki's Gelman-Rubin R-hat) -- there, C
    separate processes each making thousands of small likelihood calls. Here
    the chains share the resident dataset and step together: every slice
    evaluation of every chain is ONE wfpt_wiener_like_nodes_multi launch over
    C parameter tables (2C for the paired stepping-out probes), so a launch
    carries C x 100k trials of config 4 instead of 100k (one chain's call is
    one wave round on the chip: DESIGN.md §10 "Launch-size floor").

    The chains are independent Markov chains of the same model and step
    methods as HDDM (each has its own coordinates and random numbers; a chain
    whose slice is settled keeps evaluating its current point, whose value is
    ignored). State arrays carry a leading chain axis: group[f] (C, levels),
    std[f] (C,), subj[f] (C, units), inter[n] (C,); traces (kept, C).
    """

    def __init__(self, data, chains=4, **kw):
        self.C = int(chains)
        if self.C < 1:
            raise ValueError("chains must be >= 1")
        super().__init__(data, **kw)

    def _init_values(self):
        super()._init_values()  # HDDM's starting values (hddm_info.py:121-140), every chain
        C = self.C
        self.group = {k: np.tile(v, (C, 1)) for k, v in self.group.items()}
        self.std = {k: np.full(C, float(v)) for k, v in self.std.items()}
        self.subj = {k: np.tile(v, (C, 1)) for k, v in self.subj.items()}
        self.inter = {k: np.full(C, float(v)) for k, v in self.inter.items()}

    def node_tables(self, over=None, idx=None):
        """(C, n_nodes, 8) parameter tables of the chains at their current
        values, the columns in `over` replaced ((C, units) per family, (C,)
        for sv / sz / st); idx: only these chains' tables (len(idx), n_nodes, 8)."""
        key = tuple(self.subj[f].tobytes() for f in self.FAMILIES) + tuple(
            self.inter[k].tobytes() for k in ("sv", "sz", "st"))
        if getattr(self, "_tables_key", None) != key:
            P = np.empty((self.C, self.n_nodes, 8))
            P[:, :, 0] = self.subj["v"][:, self.node_unit["v"]]
            P[:, :, 1] = self.inter["sv"][:, None]
            P[:, :, 2] = self.subj["a"][:, self.node_unit["a"]]
            P[:, :, 3] = 0.5
            P[:, :, 4] = self.inter["sz"][:, None]
            P[:, :, 5] = self.subj["t"][:, self.node_unit["t"]]
            P[:, :, 6] = self.inter["st"][:, None]
            P[:, :, 7] = self.p_outlier
            self._tables, self._tables_key = P, key
        if idx is None and not over:
            return self._tables
        P = self._tables.copy() if idx is None else self._tables[idx]
        for name, val in (over or {}).items():
            col = self._COL[name]
            val = np.asarray(val, dtype=np.float64)
            if idx is not None:
                val = val[idx]
            P[:, :, col] = val[:, self.node_unit[name]] if name in self.FAMILIES else val[:, None]
        return P

    def node_logp_chains(self, overs, chains=None):
        """Per-node log-likelihoods of every chain for each override in
        `overs`, one launch: (len(overs), C, n_nodes). chains (bool (C,),
        optional): only these chains' tables go into the launch (a slice
        step's settled chains are not evaluated; their rows are 0, unread)."""
        t0 = time.perf_counter()
        C, m = self.C, self.n_nodes
        idx = None if chains is None or chains.all() else np.flatnonzero(chains)
        out = np.zeros((len(overs), C, m))
        if idx is not None and idx.size == 0:
            return out
        tabs = np.concatenate([self.node_tables(o, idx) for o in overs])
        t1 = time.perf_counter()
        # one launch per integration family: a table whose sz or st is 0 (a
        # probe at the slice's lower bound) selects another family, and a
        # launch over tables of several families takes the generic per-trial
        # kernel (wfpt_capi.cpp: nodes_launch)
        fam = (tabs[:, 0, 4] > 0).astype(np.int8) * 2 + (tabs[:, 0, 6] > 0)
        if (fam == fam[0]).all():
            r = self.dataset.wiener_like_nodes_multi(tabs, **self.wp)
        else:
            r = np.empty((tabs.shape[0], m))
            for f in np.unique(fam):
                sel = np.flatnonzero(fam == f)
                r[sel] = self.dataset.wiener_like_nodes_multi(tabs[sel], **self.wp)
        t2 = time.perf_counter()
        if idx is None:
            out = r.reshape(len(overs), C, m)
        else:
            out[:, idx] = r.reshape(len(overs), idx.size, m)
        dt = time.perf_counter() - t0
        self.likelihood_seconds += dt
        self.device_call_seconds = getattr(self, "device_call_seconds", 0.0) + (t2 - t1)
        self.likelihood_calls += 1
        self.tables_evaluated = getattr(self, "tables_evaluated", 0) + tabs.shape[0]
        key = ",".join(sorted(overs[0])) + f" x{len(overs)}"
        st = self.call_stats.setdefault(key, [0, 0.0])
        st[0] += 1
        st[1] += dt
        return out

    def node_logp(self, over=None):
        return self.node_logp_chains([over or {}])[0]

    def node_table(self, over=None):
        raise NotImplementedError("HDDMChains: node_tables() holds one table per chain")

    def _unit_group_c(self, fam):
        """(C, units) group mean of each unit's level, per chain."""
        nl = len(self.levels[fam])
        return self.group[fam][:, np.arange(self.n_units[fam]) % nl]

    def subj_prior_c(self, fam, x):
        g = self._unit_group_c(fam)
        sd = self.std[fam][:, None]
        if fam == "v":
            return normal_logpdf(x, g, sd)
        return gamma_logpdf_mean_sd(x, g, sd)

    def logp(self):
        """Joint log density of the model at each chain's values: (C,)."""
        lp = np.sum(self.node_logp(), axis=1)
        for fam in self.FAMILIES:
            lp = lp + np.sum(self.subj_prior_c(fam, self.subj[fam]), axis=1)
        lp = lp + np.sum(self._group_prior("a", self.group["a"]), axis=1)
        lp = lp + np.sum(self._group_prior("t", self.group["t"]), axis=1)
        lp = lp + np.sum(normal_logpdf(self.group["v"], 2.0, 3.0), axis=1)
        for f, s in (("a", 2.0), ("v", 2.0), ("t", 1.0)):
            lp = lp + halfnormal_logpdf(self.std[f], s)
        return lp

    def _update_subject(self, fam):
        C, nu = self.C, self.n_units[fam]
        unit = self.node_unit[fam]
        bins = (np.arange(C)[:, None] * nu + unit[None, :]).ravel()  # (chain, node) -> coordinate

        def ll(rows):
            return np.bincount(bins, weights=rows.ravel(), minlength=C * nu)

        def prior(x):
            return self.subj_prior_c(fam, x.reshape(C, nu)).ravel()

        def chains_of(act):
            return act.reshape(C, nu).any(axis=1)

        def logp(x, act=None):
            r = self.node_logp_chains([{fam: x.reshape(C, nu)}],
                                      None if act is None else chains_of(act))
            return ll(r[0]) + prior(x)

        def logp_pair(xl, xr, act_l=None, act_r=None):
            ch = None if act_l is None else chains_of(act_l) | chains_of(act_r)
            r = self.node_logp_chains([{fam: xl.reshape(C, nu)}, {fam: xr.reshape(C, nu)}], ch)
            return ll(r[0]) + prior(xl), ll(r[1]) + prior(xr)

        lower = 0.0 if fam in ("a", "t") else None
        new, _ = slice_step(self.subj[fam].ravel(), logp, SLICE_WIDTHS[fam], self.rng,
                            lower=lower, logp_pair=logp_pair if self.paired_probes else None,
                            masked=True)
        self.subj[fam] = new.reshape(C, nu)

    def _update_group(self, fam):
        C, nl = self.C, len(self.levels[fam])
        lv = np.arange(self.n_units[fam]) % nl
        if fam == "v":  # kNormalNormal per chain and level (hddm_info.py:167-168)
            tau0, mu0 = 3.0 ** -2, 2.0
            tau = self.std["v"] ** -2
            for k in range(nl):
                xs = self.subj["v"][:, lv == k]
                prec = tau0 + tau * xs.shape[1]
                mean = (tau0 * mu0 + tau * xs.sum(axis=1)) / prec
                self.group["v"][:, k] = self.rng.normal(mean, prec ** -0.5)
        else:
            def logp(g):
                g = g.reshape(C, nl)
                out = self._group_prior(fam, g)
                for k in range(nl):
                    xs = self.subj[fam][:, lv == k]
                    out[:, k] = out[:, k] + np.sum(
                        gamma_logpdf_mean_sd(xs, g[:, k:k + 1], self.std[fam][:, None]), axis=1)
                return out.ravel()
            new, _ = slice_step(self.group[fam].ravel(), logp, SLICE_WIDTHS[fam], self.rng,
                                lower=0.0)
            self.group[fam] = new.reshape(C, nl)
        std_sd = {"a": 2.0, "v": 2.0, "t": 1.0}[fam]

        def logp_std(s):
            ok = s > 0
            ss = np.where(ok, s, 1.0)[:, None]
            g = self._unit_group_c(fam)
            x = self.subj[fam]
            ll = normal_logpdf(x, g, ss) if fam == "v" else gamma_logpdf_mean_sd(x, g, ss)
            val = halfnormal_logpdf(np.where(ok, s, 1.0), std_sd) + np.sum(ll, axis=1)
            return np.where(ok, val, -np.inf)

        self.std[fam], _ = slice_step(self.std[fam].copy(), logp_std, SLICE_WIDTHS[fam + "_std"],
                                      self.rng, lower=0.0)

    def _update_inter(self, name):
        prior = {"sv": lambda x: halfnormal_logpdf(x, 2.0), "sz": lambda x: beta_logpdf(x, 1, 3),
                 "st": lambda x: halfnormal_logpdf(x, 0.3)}[name]
        cur = self.inter[name]

        def masked(x):
            pr = prior(x)
            ok = np.isfinite(pr)
            # a probe outside the prior's support is not evaluated: the table
            # keeps the chain's current value there and the result is -inf
            return pr, ok, np.where(ok, x, cur)

        def logp(x, act=None):
            pr, ok, xv = masked(x)
            ch = ok if act is None else ok & act
            r = self.node_logp_chains([{name: xv}], ch)[0]
            return np.where(ok, pr + np.sum(r, axis=1), -np.inf)

        def logp_pair(xl, xr, act_l=None, act_r=None):
            (pl, okl, vl), (pr_, okr, vr) = masked(xl), masked(xr)
            ch = (okl | okr) if act_l is None else (okl & act_l) | (okr & act_r)
            r = self.node_logp_chains([{name: vl}, {name: vr}], ch)
            return (np.where(okl, pl + np.sum(r[0], axis=1), -np.inf),
                    np.where(okr, pr_ + np.sum(r[1], axis=1), -np.inf))

        self.inter[name], _ = slice_step(cur.copy(), logp, SLICE_WIDTHS[name], self.rng,
                                         lower=0.0,
                                         logp_pair=logp_pair if self.paired_probes else None,
                                         masked=True)

    def sample(self, iter, burn=0, thin=1, progress=None):
        """Run `iter` lockstep sweeps of every chain; keep every `thin`-th
        after `burn`. Returns traces (dict name -> (kept, C))."""
        names = []
        for fam in self.FAMILIES:
            for k, lv in enumerate(self.levels[fam]):
                names.append((f"{fam}" + (f"({','.join(map(str, lv))})" if lv else ""), fam, k))
        trace = {nm: [] for nm, _, _ in names}
        for fam in self.FAMILIES:
            trace[f"{fam}_std"] = []
        inter = [nm for nm in ("sv", "sz", "st") if nm in self.include]
        for nm in inter:
            trace[nm] = []
        self.trace_subj = {f: [] for f in self.FAMILIES}
        t0 = time.perf_counter()
        for it in range(iter):
            self.sweep()
            if it >= burn and (it - burn) % thin == 0:
                for nm, fam, k in names:
                    trace[nm].append(self.group[fam][:, k].copy())
                for fam in self.FAMILIES:
                    trace[f"{fam}_std"].append(self.std[fam].copy())
                    self.trace_subj[fam].append(self.subj[fam].copy())
                for nm in inter:
                    trace[nm].append(self.inter[nm].copy())
            if progress and (it + 1) % progress == 0:
                el = time.perf_counter() - t0
                print(f"  [{it + 1}/{iter}] {el:.1f}s, {self.likelihood_calls} batched "
                      f"likelihood calls ({self.C} chains)", flush=True)
        self.trace = {k: np.asarray(v).reshape(-1, self.C) for k, v in trace.items()}
        self.trace_subj = {k: np.asarray(v) for k, v in self.trace_subj.items()}
        self.sample_seconds = time.perf_counter() - t0
        return self.trace

    def gen_stats(self):
        """Posterior summaries pooled over the chains, with the Gelman-Rubin
        R-hat of each node (kabuki.analyze.gelman_rubin's statistic)."""
        out = {}
        rh = self.gelman_rubin()
        for k, v in self.trace.items():
            flat = v.ravel()
            out[k] = {"mean": float(np.mean(flat)), "std": float(np.std(flat)),
                      "2.5q": float(np.quantile(flat, .025)),
                      "97.5q": float(np.quantile(flat, .975)), "rhat": rh[k]}
        return out

    def gelman_rubin(self):
        """R-hat per traced node: sqrt(((n - 1)/n W + B/n) / W) with W the mean
        within-chain variance and B/n the variance of the chain means."""
        out = {}
        for k, v in self.trace.items():
            n, C = v.shape
            if C < 2 or n < 2:
                out[k] = float("nan")
                continue
            W = float(np.mean(np.var(v, axis=0, ddof=1)))
            Bn = float(np.var(np.mean(v, axis=0), ddof=1))
            out[k] = float(np.sqrt(((n - 1) / n * W + Bn) / W)) if W > 0 else float("nan")
        return out


def gen_data(n_subj=200, n_trials=500, conds=None, a=2.0, t=0.3, sv=0.0, sz=0.0, st=0.0,
             jitter=0.1, seed=20261017, dt=1e-3):
    """Synthetic hierarchical data set: per subject,
    parameters jittered by +-`jitter` (relative), RTs drawn with the GPU
    inverse-CDF sampler (wfpt.gen_rts_from_cdf, wfpt.pyx:323-354). Returns a
    DataFrame with rt (signed: lower-boundary responses negative), response,
    subj_idx, cond, plus the true subject parameters as a dict."""
    import pandas as pd
    conds = conds or {"c0": 0.5, "c1": 1.0}
    rng = np.random.default_rng(seed)
    np.random.seed(seed)
    rows = []
    truth = {"a": [], "t": [], "v": {c: [] for c in conds}}
    per = n_trials // len(conds)
    for s in range(n_subj):
        a_s = a * (1 + jitter * rng.uniform(-1, 1))
        t_s = t * (1 + jitter * rng.uniform(-1, 1))
        truth["a"].append(a_s)
        truth["t"].append(t_s)
        for c, v in conds.items():
            v_s = v * (1 + jitter * rng.uniform(-1, 1))
            truth["v"][c].append(v_s)
            x = _wfpt.gen_rts_from_cdf(v_s, sv, a_s, 0.5, sz, t_s, st, samples=per, dt=dt)
            rows.append(pd.DataFrame({"rt": x, "response": (x > 0).astype(float),
                                      "subj_idx": s, "cond": c}))
    return pd.concat(rows, ignore_index=True), truth
