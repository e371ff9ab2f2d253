"""PyMC-facing likelihood of the observed RT node, on MI355X.

Restates hddm/likelihoods.py:30-105 (`generate_wfpt_stochastic_class`,
`wfpt_like`) over `hddm_amd.wfpt`:

* `wfpt_like(x, v, sv, a, z, sz, t, st, p_outlier=0)` keeps the reference's
  logp signature, its `abs(rt).max() < 998` dispatch and the missing-response
  branch (|rt| >= 999 scored by a binomial on P(upper), likelihoods.py:56-73).
* The observed data of a node never changes during sampling, so the RT
  column is uploaded once per node and kept resident (`Dataset`), keyed by the
  identity of the node's value (contents hashed only on a miss); the
  reference re-reads host memory on every logp call.
* `generate_wfpt_stochastic_class` returns the same PyMC class as the
  reference when kabuki is importable (kabuki.utils.stochastic_from_dist);
  otherwise a light `WfptNode` with `.value`, `.parents`, `.logp`, `.pdf`,
  `.cdf`, `.random` so hierarchical samplers (hddm_amd.hierarchical) can drive it.
  `.cdf` is the DMAT CDF (likelihoods.py:90-91 -> cdfdif_wrapper.dmat_cdf_array).
"""

import numpy as np
from scipy import stats

from . import cdfdif_wrapper as _cdfdif
from . import wfpt as _wfpt

DEFAULT_WIENER_PARAMS = {"err": 1e-4, "n_st": 2, "n_sz": 2, "use_adaptive": 1,
                         "simps_err": 1e-3, "w_outlier": 0.1}  # base.py:711-716


_F64 = np.dtype(np.float64)


def _rt_column(x):
    """`x['rt']` of a pandas slice, or a plain signed-RT array, as a contiguous
    float64 array (a view when the column already is one: `Series.to_numpy`
    costs ~3 us where `np.asarray(series, dtype)` costs ~12 us)."""
    if hasattr(x, "columns"):
        rt = x["rt"].to_numpy()
    elif hasattr(x, "dtype") and getattr(x.dtype, "names", None):
        rt = x["rt"]
    else:
        rt = x
    if not (type(rt) is np.ndarray and rt.dtype is _F64 and rt.flags.c_contiguous):
        rt = np.ascontiguousarray(rt, dtype=np.float64)
    return rt


class _ResidentCache:
    """Device-resident copies of node data (a node's RT column never changes
    during sampling; changed data is a new entry).

    Lookups are keyed on the identity of the node's value object, which the
    entry keeps alive so its id cannot be recycled while the entry exists.
    Contents are hashed only on a miss (nodes holding equal data share one
    upload). A hit re-checks the column against the entry: exactly (every
    byte) for columns of up to EXACT_MAX trials — HDDM's nodes, where the
    compare is well under a microsecond — so an in-place rewrite of a node's
    value is never served stale; larger columns, whose full compare would cost
    more than their kernel, are re-checked on a 256-element sample only (an
    in-place rewrite missing every sampled element is not detected: pass a new
    array instead of rewriting one).
    Each entry also caches max|rt| for wfpt_like's `< 998` dispatch."""

    EXACT_MAX = 16384

    def __init__(self, maxsize=4096):
        self._by_id = {}
        self._by_bytes = {}
        self.maxsize = maxsize

    @classmethod
    def _probe(cls, rt):
        if rt.size <= cls.EXACT_MAX:
            return rt.tobytes()
        return rt[:: max(1, rt.size // 256)][:256].tobytes()

    def get(self, rt, src):
        """(Dataset or None, max|rt|) for the contiguous column `rt` of `src`.
        The Dataset is None when the column holds missing responses."""
        hit = self._by_id.get(id(src))
        if hit is not None and hit[0] is src and hit[1] == self._probe(rt):
            return hit[2], hit[3]
        if len(self._by_id) >= self.maxsize:
            self._by_id.clear()
            self._by_bytes.clear()
        bkey = rt.tobytes()
        ent = self._by_bytes.get(bkey)
        if ent is None:
            amax = float(np.abs(rt).max(initial=0.0))
            ent = (_wfpt.Dataset(rt) if rt.size and amax < 998 else None, amax)
            self._by_bytes[bkey] = ent
        self._by_id[id(src)] = (src, self._probe(rt)) + ent
        return ent

    def clear(self):
        self._by_id.clear()
        self._by_bytes.clear()


_cache = _ResidentCache()


def make_wfpt_like(wiener_params=None, resident=True):
    """The logp closure of generate_wfpt_stochastic_class (likelihoods.py:52-73)."""
    wp = dict(DEFAULT_WIENER_PARAMS if wiener_params is None else wiener_params)

    def wfpt_like(x, v, sv, a, z, sz, t, st, p_outlier=0):
        rt = _rt_column(x)
        if resident:
            ds, amax = _cache.get(rt, x)
        else:
            ds, amax = None, float(np.abs(rt).max(initial=0.0))
        if amax < 998:
            if ds is not None:
                return ds.wiener_like(v, sv, a, z, sz, t, st, p_outlier=p_outlier, **wp)
            return _wfpt.wiener_like(rt, v, sv, a, z, sz, t, st, p_outlier=p_outlier, **wp)
        # missing responses (currently undocumented in the reference)
        noresponse = np.abs(rt) >= 999
        resp = np.ascontiguousarray(rt[~noresponse])
        logp_resp = _wfpt.wiener_like(resp, v, sv, a, z, sz, t, st, p_outlier=p_outlier, **wp)
        n_noresponse = int(noresponse.sum())
        k_upper = int((rt[noresponse] > 0).sum())
        if v == 0:
            p_upper = z
        else:
            p_upper = (np.exp(-2 * a * z * v) - 1) / (np.exp(-2 * a * v) - 1)
        logp_noresp = stats.binom.logpmf(k_upper, n_noresponse, p_upper)
        return logp_resp + logp_noresp

    wfpt_like.wiener_params = wp
    return wfpt_like


def gen_random(parents, size, sampling_method="cdf", cdf_range=(-5, 5), sampling_dt=1e-4):
    """The class's `random` (likelihoods.py:76-81): hddm.generate.gen_rts
    (generate.py:134-205, structured=True) followed by hddm.utils.flip_errors
    (utils.py:15-37), i.e. a DataFrame with signed 'rt' and 'response'
    (1 upper / 0 lower). method 'cdf' samples on the MI355X density grid
    (gen_rts_from_cdf); the host-only simulators ('drift', 'cdf_py') are the
    reference's own and are delegated to it when it is importable."""
    import pandas as pd
    p = {k: parents[k] for k in ("v", "sv", "a", "z", "sz", "t", "st") if k in parents}
    for k in ("sv", "sz", "st"):        # generate.py:169-177 defaults
        p.setdefault(k, 0)
    p.setdefault("z", .5)
    if isinstance(size, tuple):         # generate.py:180-184 (PyMC shapes)
        size = 1 if size == () else size[0]
    if sampling_method != "cdf":
        import hddm  # reference simulators (not on the accelerated path)
        return hddm.utils.flip_errors(hddm.generate.gen_rts(
            method=sampling_method, size=size, dt=sampling_dt, range_=cdf_range,
            structured=True, **parents))
    rts = _wfpt.gen_rts_from_cdf(p["v"], p["sv"], p["a"], p["z"], p["sz"], p["t"], p["st"],
                                 size, cdf_range[0], cdf_range[1], sampling_dt)
    # generate.py:200-203 then utils.py:27-35: |rt| with response, lower flipped back
    response = np.where(rts < 0, 0.0, 1.0)
    rt = np.abs(rts)
    rt = np.where(response == 0, -rt, rt)
    return pd.DataFrame({"rt": rt, "response": response})


class WfptNode:
    """Observed RT node with the attributes the reference's Wfpt class carries
    (value, parents, logp, pdf, random). Parents may be floats or objects
    exposing `.value` (stochastic parents)."""

    PARENTS = ("v", "sv", "a", "z", "sz", "t", "st", "p_outlier")

    def __init__(self, name, value, wfpt_like, sampling_method="cdf", cdf_range=(-5, 5),
                 sampling_dt=1e-4, **parents):
        self.__name__ = name
        self.value = value
        self._like = wfpt_like
        self.sampling_method = sampling_method
        self.cdf_range = cdf_range
        self.sampling_dt = sampling_dt
        self.parents = {k: parents.get(k, 0.0 if k != "z" else 0.5) for k in self.PARENTS}

    def parent_values(self):
        return {k: (p.value if hasattr(p, "value") else p) for k, p in self.parents.items()}

    @property
    def logp(self):
        return self._like(self.value, **self.parent_values())

    def pdf(self, x):
        pv = self.parent_values()
        return _wfpt.pdf_array(np.ascontiguousarray(x, dtype=np.float64), pv["v"], pv["sv"],
                               pv["a"], pv["z"], pv["sz"], pv["t"], pv["st"],
                               p_outlier=pv["p_outlier"])

    def cdf(self, x):
        """likelihoods.py:90-91: DMAT CDF with the class's w_outlier."""
        pv = self.parent_values()
        return _cdfdif.dmat_cdf_array(np.ascontiguousarray(x, dtype=np.float64),
                                      w_outlier=self._like.wiener_params["w_outlier"], **pv)

    @property
    def shape(self):
        return np.shape(_rt_column(self.value))

    def random(self):
        """likelihoods.py:76-81: a DataFrame of len(value) signed RTs + responses."""
        return gen_random(self.parent_values(), self.shape, self.sampling_method,
                          self.cdf_range, self.sampling_dt)


def generate_wfpt_stochastic_class(wiener_params=None, sampling_method="cdf",
                                   cdf_range=(-5, 5), sampling_dt=1e-4):
    """likelihoods.py:30-105. With kabuki available this is the reference's
    PyMC stochastic built on the MI355X `wfpt_like`; without it, a factory of
    `WfptNode`s."""
    wfpt_like = make_wfpt_like(wiener_params)
    try:
        from kabuki.utils import stochastic_from_dist  # noqa: F401  (absent offline)
    except ImportError:
        def factory(name, value, **parents):
            return WfptNode(name, value, wfpt_like, sampling_method, cdf_range, sampling_dt,
                            **parents)
        factory.wfpt_like = wfpt_like
        factory.pdf = lambda self, x: self.pdf(x)
        return factory
    wfpt_cls = stochastic_from_dist("wfpt", wfpt_like)

    def pdf(self, x):
        return _wfpt.pdf_array(x, **self.parents)

    def cdf(self, x):
        return _cdfdif.dmat_cdf_array(x, w_outlier=wfpt_like.wiener_params["w_outlier"],
                                      **self.parents)

    def random(self):
        return gen_random(self.parents.value, self.shape, sampling_method, cdf_range,
                          sampling_dt)

    wfpt_cls.pdf = pdf
    wfpt_cls.cdf = cdf
    wfpt_cls.random = random
    # likelihoods.py:98,103: cdf_vec over the reference's gen_cdf_using_pdf (not
    # on the accelerated path) and the quantile methods, when HDDM is loaded
    try:
        import hddm
        wp = wfpt_like.wiener_params
        wfpt_cls.cdf_vec = lambda self: hddm.wfpt.gen_cdf_using_pdf(
            time=cdf_range[1], **dict(list(self.parents.items()) + list(wp.items())))
        hddm.likelihoods.add_quantiles_functions_to_pymc_class(wfpt_cls)
    except (ImportError, AttributeError):
        pass
    return wfpt_cls
