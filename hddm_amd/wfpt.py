"""Drop-in for the reference's `wfpt` extension module (src/wfpt.pyx), on MI355X.

Same names, positional order, defaults and return conventions as the Cython
module that `hddm/__init__.py:16` imports as `hddm.wfpt`:

    pdf_array   src/wfpt.pyx:32-48    (defaults err=1e-4, n_st=n_sz=2, simps_err=1e-3, w_outlier=0)
    wiener_like src/wfpt.pyx:54-76    (defaults n_st=n_sz=10, simps_err=1e-8, w_outlier=0.1)
    full_pdf    src/pdf.pxi:104-146   (cpdef; defaults n_st=n_sz=2, simps_err=1e-3)
    wiener_like_multi  src/wfpt.pyx:244-274
    gen_rts_from_cdf   src/wfpt.pyx:323-354 (density grid on the GPU, sampling in NumPy)

Every density is computed by the HIP kernels of libwfpt_amd.so; there is no
CPU path. Argument checking mirrors Cython's buffer protocol: `x` must be a
1-D float64 ndarray (TypeError otherwise; ValueError for dtype / ndim).

Additions for resident data (the reference re-reads host memory every call):
`Dataset(rt)` uploads RTs once; `Dataset.wiener_like(...)` has wiener_like's
signature minus `x`. `Dataset(rt, node_id=...)` + `wiener_like_nodes` scores
many PyMC nodes in one launch.
"""
import ctypes

import numpy as np

from . import _lib

__all__ = ["pdf_array", "wiener_like", "full_pdf", "wiener_like_multi", "gen_rts_from_cdf",
           "Dataset", "prob_ub"]


def _check_x(x, name="x"):
    """Cython `np.ndarray[double, ndim=1]` argument semantics."""
    if not isinstance(x, np.ndarray):
        raise TypeError(f"Argument '{name}' has incorrect type (expected numpy.ndarray, got "
                        f"{type(x).__name__})")
    if x.dtype != np.float64:
        raise ValueError(f"Buffer dtype mismatch, expected 'double' but got {x.dtype}")
    if x.ndim != 1:
        raise ValueError(f"Buffer has wrong number of dimensions (expected 1, got {x.ndim})")
    return np.ascontiguousarray(x)


def pdf_array(x, v, sv, a, z, sz, t, st, err=1e-4, logp=0, n_st=2, n_sz=2, use_adaptive=1,
              simps_err=1e-3, p_outlier=0, w_outlier=0):
    x = _check_x(x)
    out = np.empty(x.shape[0], dtype=np.float64)
    c = _lib.context()
    P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
    K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
    _lib.check(_lib.wfpt_pdf_array(c.handle, _lib.dptr(x), x.shape[0], ctypes.byref(P),
                                   ctypes.byref(K), 1 if logp else 0, _lib.dptr(out)))
    return out


def wiener_like(x, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10, use_adaptive=1,
                simps_err=1e-8, p_outlier=0, w_outlier=0.1):
    x = _check_x(x)
    c = _lib.context()
    P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
    K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
    out = ctypes.c_double()
    _lib.check(_lib.wfpt_wiener_like_host(c.handle, _lib.dptr(x), x.shape[0], ctypes.byref(P),
                                          ctypes.byref(K), ctypes.byref(out)))
    return out.value


def full_pdf(x, v, sv, a, z, sz, t, st, err, n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3):
    x = float(x)
    c = _lib.context()
    P = _lib.make_params(v, sv, a, z, sz, t, st, 0.0)
    K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, 0.0)
    out = ctypes.c_double()
    _lib.check(_lib.wfpt_full_pdf(c.handle, x, ctypes.byref(P), ctypes.byref(K),
                                  ctypes.byref(out)))
    return out.value


def prob_ub(v, a, z):
    """P(upper boundary), pdf.pxi:67-72 (host scalar helper, as in likelihoods.py:64-67)."""
    if v == 0:
        return z
    return (np.exp(-2 * a * z * v) - 1) / (np.exp(-2 * a * v) - 1)


def _multi_args(n, v, sv, a, z, sz, t, st, multi):
    """Per-trial arrays (pointer table, kept alive) and scalars of a
    wiener_like_multi call (wfpt.pyx:257-260: names in `multi` are indexed per
    trial, the others are scalars)."""
    names = ("v", "sv", "a", "z", "sz", "t", "st")
    vals = (v, sv, a, z, sz, t, st)
    multi = set(multi)
    keep = []
    ptrs = (_lib._PD * 7)()
    scal = np.zeros(7)
    for j, (nm, val) in enumerate(zip(names, vals)):
        if nm in multi:
            arr = np.ascontiguousarray(np.asarray(val, dtype=np.float64))
            if arr.shape != (n,):
                raise ValueError(f"parameter {nm} must have one value per trial")
            keep.append(arr)
            ptrs[j] = _lib.dptr(arr)
        else:
            ptrs[j] = _lib._PD()
            scal[j] = float(val)
    return ptrs, scal, keep


def wiener_like_multi(x, v, sv, a, z, sz, t, st, err, multi=None, n_st=10, n_sz=10,
                      use_adaptive=1, simps_err=1e-3, p_outlier=0, w_outlier=0):
    x = _check_x(x)
    if multi is None:
        return full_pdf(x, v, sv, a, z, sz, t, st, err)  # wfpt.pyx:255-256 (TypeError for arrays)
    n = x.shape[0]
    ptrs, scal, keep = _multi_args(n, v, sv, a, z, sz, t, st, multi)
    c = _lib.context()
    K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
    out = ctypes.c_double()
    _lib.check(_lib.wfpt_wiener_like_multi(c.handle, _lib.dptr(x), n, ptrs, _lib.dptr(scal),
                                           ctypes.byref(K), float(p_outlier), ctypes.byref(out)))
    del keep
    return out.value


def wiener_like_multi_terms(x, v, sv, a, z, sz, t, st, err, multi, n_st=10, n_sz=10,
                            use_adaptive=1, simps_err=1e-3, p_outlier=0, w_outlier=0):
    """wiener_like_multi (wfpt.pyx:244-274) returning (sum, per-trial terms):
    terms[i] is trial i's addend log p_i (wfpt.pyx:261-272)."""
    x = _check_x(x)
    n = x.shape[0]
    ptrs, scal, keep = _multi_args(n, v, sv, a, z, sz, t, st, multi)
    c = _lib.context()
    K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
    out = ctypes.c_double()
    terms = np.empty(n, dtype=np.float64)
    _lib.check(_lib.wfpt_wiener_like_multi_ex(c.handle, _lib.dptr(x), n, ptrs, _lib.dptr(scal),
                                              ctypes.byref(K), float(p_outlier),
                                              ctypes.byref(out), _lib.dptr(terms)))
    del keep
    return out.value, terms


def gen_rts_from_cdf(v, sv, a, z, sz, t, st, samples=1000, cdf_lb=-6, cdf_ub=6, dt=1e-2):
    """wfpt.pyx:323-354: inverse-CDF sampling from the density on a dt grid.

    The grid density (full_pdf with t = st = 0, err = 1e-4) runs on the GPU;
    the running sum, normalisation, searchsorted and the non-decision-time
    delays follow the reference step for step and draw from NumPy's global
    RNG in the same order.
    """
    x = np.arange(cdf_lb, cdf_ub, dt)
    pdf = pdf_array(x[1:].copy(), v, sv, a, z, sz, 0, 0, 1e-4)
    l_cdf = np.empty(x.shape[0], dtype=np.float64)
    l_cdf[0] = 0
    l_cdf[1:] = np.cumsum(pdf)
    l_cdf /= l_cdf[x.shape[0] - 1]
    f = np.random.rand(samples)
    if st != 0:
        delay = np.random.rand(samples) * st + (t - st / 2.)
    idx = np.searchsorted(l_cdf, f)
    rt = x[idx]
    if st == 0:
        return rt + np.sign(rt) * t
    return rt + np.sign(rt) * delay


class Dataset:
    """RTs resident in HBM for repeated likelihood calls (MCMC: data fixed,
    parameters change per proposal). Optional `node_id` groups trials into
    `n_nodes` likelihood nodes scored together by `wiener_like_nodes`."""

    def __init__(self, rt, node_id=None, n_nodes=None, device=None, ctx=None, input_order=False):
        rt = np.ascontiguousarray(np.asarray(rt, dtype=np.float64).ravel())
        self.ctx = ctx if ctx is not None else _lib.context(device)
        self.n = rt.shape[0]
        self.input_order = bool(input_order)
        flags = _lib.WFPT_DS_INPUT_ORDER if input_order else 0
        h = _lib._VP()
        if node_id is not None:
            node = np.ascontiguousarray(np.asarray(node_id, dtype=np.int32).ravel())
            if node.shape != rt.shape:
                raise ValueError("node_id must have one entry per trial")
            self.n_nodes = int(n_nodes if n_nodes is not None else (node.max() + 1 if node.size
                                                                    else 0))
            _lib.check(_lib.wfpt_dataset_create_ex(
                self.ctx.handle, _lib.dptr(rt), self.n,
                node.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), self.n_nodes, flags,
                ctypes.byref(h)))
        else:
            self.n_nodes = 0
            _lib.check(_lib.wfpt_dataset_create_ex(self.ctx.handle, _lib.dptr(rt), self.n, None,
                                                   0, flags, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            _lib.wfpt_dataset_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.n

    def _knobs(self, err, n_st, n_sz, use_adaptive, simps_err, w_outlier):
        """The knobs struct, rebuilt only when the knobs change (they are fixed
        across an MCMC run; per-call Python work sits in front of the kernel)."""
        key = (err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        kc = getattr(self, "_kc", None)
        if kc is None or kc[0] != key:
            K = _lib.make_knobs(*key)
            kc = self._kc = (key, K, ctypes.addressof(K))
        return kc[1]

    def _knobs_addr(self, err, n_st, n_sz, use_adaptive, simps_err, w_outlier):
        """(knobs struct, its address). The caller keeps the struct in a local
        until the raw call returns: another thread may replace self._kc (other
        knobs) meanwhile, and the address must not outlive its struct."""
        self._knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        kc = self._kc
        return kc[1], kc[2]

    def wiener_like(self, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10, use_adaptive=1,
                    simps_err=1e-8, p_outlier=0, w_outlier=0.1):
        P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
        K, kaddr = self._knobs_addr(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = ctypes.c_double()
        c, h = self.ctx.handle, self.handle
        if not c or not h:  # closed: the C ABI's own argument error
            _lib.check(_lib.wfpt_wiener_like(c, h, ctypes.byref(P), ctypes.byref(K),
                                             ctypes.byref(out)))
        rc = _lib.raw_wiener_like(c.value, h.value, ctypes.addressof(P), kaddr,
                                  ctypes.addressof(out))
        if rc:
            _lib.check(rc)
        return out.value

    def wiener_like_trials(self, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10, use_adaptive=1,
                           simps_err=1e-8, p_outlier=0, w_outlier=0.1):
        """wiener_like plus each trial's addend (wfpt.pyx:66-74), in the order the
        trials were given: (total, terms). Same call sequence and kernels as
        wiener_like (with one more store per trial): the per-trial check of the
        summing path."""
        P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
        K = self._knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = ctypes.c_double()
        terms = np.empty(self.n, dtype=np.float64)
        _lib.check(_lib.wfpt_wiener_like_trials(self.ctx.handle, self.handle, ctypes.byref(P),
                                                ctypes.byref(K), ctypes.byref(out),
                                                _lib.dptr(terms)))
        return out.value, terms

    def order(self):
        """order()[i] = the caller's index of stored trial i (chunk c holds
        stored trials 64c .. 64c + 63)."""
        perm = np.empty(self.n, dtype=np.int64)
        _lib.check(_lib.wfpt_dataset_order(self.handle,
                                           perm.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        return perm

    def local_triple(self, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10, use_adaptive=1,
                     simps_err=1e-8, p_outlier=0, w_outlier=0.1):
        """This shard's {sum log p, #zero trials, encoded errors}: what
        wiener_like_allreduce contributes to its all-reduce."""
        P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
        K = self._knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        r = (ctypes.c_double * 3)()
        _lib.check(_lib.wfpt_wiener_like_local(self.ctx.handle, self.handle, ctypes.byref(P),
                                               ctypes.byref(K), r))
        return [r[0], r[1], r[2]]

    def wiener_like_allreduce(self, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10,
                              use_adaptive=1, simps_err=1e-8, p_outlier=0, w_outlier=0.1):
        """Global sum over every rank's shard (requires hddm_amd.dist.init_comm; torch-free)."""
        P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
        K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = ctypes.c_double()
        _lib.check(_lib.wfpt_wiener_like_allreduce(self.ctx.handle, self.handle,
                                                   ctypes.byref(P), ctypes.byref(K),
                                                   ctypes.byref(out)))
        return out.value

    def wiener_like_multi(self, v, sv, a, z, sz, t, st, err, multi, n_st=10, n_sz=10,
                          use_adaptive=1, simps_err=1e-3, p_outlier=0, w_outlier=0,
                          trials=False):
        """wiener_like_multi (wfpt.pyx:244-274) over this resident dataset
        (created with input_order=True): only the per-trial parameter arrays
        go to the device per call. trials=True: (sum, per-trial terms)."""
        ptrs, scal, keep = _multi_args(self.n, v, sv, a, z, sz, t, st, multi)
        K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = ctypes.c_double()
        terms = np.empty(self.n, dtype=np.float64) if trials else None
        _lib.check(_lib.wfpt_wiener_like_multi_resident_ex(
            self.ctx.handle, self.handle, ptrs, _lib.dptr(scal), ctypes.byref(K),
            float(p_outlier), ctypes.byref(out), _lib.dptr(terms) if trials else None))
        del keep
        return (out.value, terms) if trials else out.value

    def _node_table(self, params):
        """The (n_nodes, 8) parameter table as a wfpt_params pointer, zero-copy
        (wfpt_params is 8 doubles, the row layout of a C-contiguous float64
        array); returns (pointer, the array that owns the memory)."""
        if self.n_nodes == 0:
            raise ValueError("dataset was created without node ids")
        pm = np.ascontiguousarray(params, dtype=np.float64)
        if pm.shape != (self.n_nodes, 8):
            raise ValueError(f"params must have shape ({self.n_nodes}, 8)")
        return pm.ctypes.data_as(_lib._PP), pm

    def wiener_like_nodes_local(self, params, err=1e-4, n_st=2, n_sz=2, use_adaptive=1,
                                simps_err=1e-3, w_outlier=0.1):
        """This shard's per-node partial sums and its encoded error count
        (n_nodes + 1 values): what wiener_like_nodes_allreduce sums over ranks."""
        table, keep = self._node_table(params)
        K = self._knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = np.empty(self.n_nodes + 1, dtype=np.float64)
        _lib.check(_lib.wfpt_wiener_like_nodes_local(self.ctx.handle, self.handle, table,
                                                     ctypes.byref(K), _lib.dptr(out)))
        del keep
        return out

    def wiener_like_nodes_allreduce(self, params, err=1e-4, n_st=2, n_sz=2, use_adaptive=1,
                                    simps_err=1e-3, w_outlier=0.1):
        """Per-node sums over every rank's shard (hddm_amd.dist.init_comm):
        one all-reduce of n_nodes + 1 doubles per call.

        The exchange's count is the table's row count, which every rank
        shares; whether this rank's dataset matches it (node ids present,
        n_nodes rows) is checked by the library *inside* the collective, so a
        rank with a bad dataset enters the all-reduce poisoned instead of
        leaving its peers blocked in it."""
        pm = np.ascontiguousarray(params, dtype=np.float64)
        if pm.ndim != 2 or pm.shape[1] != 8:  # the table itself: the same on every rank
            raise ValueError("params must have shape (n_nodes, 8)")
        K = self._knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        m = pm.shape[0]
        out = np.empty(m, dtype=np.float64)
        _lib.check(_lib.wfpt_wiener_like_nodes_allreduce(self.ctx.handle, self.handle,
                                                         pm.ctypes.data_as(_lib._PP), m,
                                                         ctypes.byref(K), _lib.dptr(out)))
        return out

    def wiener_like_nodes_multi(self, tables, err=1e-4, n_st=2, n_sz=2, use_adaptive=1,
                                simps_err=1e-3, w_outlier=0.1, trials=False):
        """T parameter tables in ONE launch: tables (T, n_nodes, 8) -> per-node
        sums (T, n_nodes); row t equals wiener_like_nodes(tables[t]) bit for bit
        (several MCMC chains in lockstep, or both stepping-out probes of a slice
        step). trials=True: (sums, per-trial terms (T, n) in the caller's trial
        order)."""
        tb = np.ascontiguousarray(tables, dtype=np.float64)
        if self.n_nodes == 0:
            raise ValueError("dataset was created without node ids")
        if tb.ndim != 3 or tb.shape[1:] != (self.n_nodes, 8) or tb.shape[0] < 1:
            raise ValueError(f"tables must have shape (T, {self.n_nodes}, 8), T >= 1")
        T = tb.shape[0]
        K, kaddr = self._knobs_addr(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = np.empty((T, self.n_nodes), dtype=np.float64)
        c, h = self.ctx.handle, self.handle
        if trials:
            terms = np.empty((T, self.n), dtype=np.float64)
            _lib.check(_lib.wfpt_wiener_like_nodes_multi_ex(
                c, h, tb.ctypes.data_as(_lib._PP), T, ctypes.byref(K), _lib.dptr(out),
                _lib.dptr(terms)))
            return out, terms
        if not c or not h:  # closed: the C ABI's own argument error
            _lib.check(_lib.wfpt_wiener_like_nodes_multi(c, h, tb.ctypes.data_as(_lib._PP), T,
                                                         ctypes.byref(K), _lib.dptr(out)))
        rc = _lib.raw_wiener_like_nodes_multi(c.value, h.value, tb.ctypes.data, T, kaddr,
                                              out.ctypes.data)
        if rc:
            _lib.check(rc)
        return out

    def wiener_like_nodes(self, params, err=1e-4, n_st=2, n_sz=2, use_adaptive=1,
                          simps_err=1e-3, w_outlier=0.1, trials=False):
        """params: array (n_nodes, 8) of v, sv, a, z, sz, t, st, p_outlier.
        Returns the per-node summed log-likelihoods (float64[n_nodes]);
        trials=True: (per-node sums, per-trial log terms in the order the
        trials were given to the Dataset)."""
        if not trials:
            # the per-step MCMC call: plain addresses through the raw prototype
            pm = np.ascontiguousarray(params, dtype=np.float64)
            if self.n_nodes == 0:
                raise ValueError("dataset was created without node ids")
            if pm.shape != (self.n_nodes, 8):
                raise ValueError(f"params must have shape ({self.n_nodes}, 8)")
            K, kaddr = self._knobs_addr(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
            out = np.empty(self.n_nodes, dtype=np.float64)
            c, h = self.ctx.handle, self.handle
            if c and h:
                rc = _lib.raw_wiener_like_nodes(c.value, h.value, pm.ctypes.data, kaddr,
                                                out.ctypes.data)
                if rc:
                    _lib.check(rc)
                return out
        table, keep = self._node_table(params)
        K = self._knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = np.empty(self.n_nodes, dtype=np.float64)
        if trials:
            terms = np.empty(self.n, dtype=np.float64)
            _lib.check(_lib.wfpt_wiener_like_nodes_ex(self.ctx.handle, self.handle, table,
                                                      ctypes.byref(K), _lib.dptr(out),
                                                      _lib.dptr(terms)))
            return out, terms
        _lib.check(_lib.wfpt_wiener_like_nodes(self.ctx.handle, self.handle, table,
                                               ctypes.byref(K), _lib.dptr(out)))
        del keep
        return out
