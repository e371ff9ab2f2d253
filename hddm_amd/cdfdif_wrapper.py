"""Drop-in for the reference's `cdfdif_wrapper` extension module, on MI355X.

`hddm/__init__.py:11,19` imports it as `hddm.cdfdif`; its one function

    dmat_cdf_array(x, v, sv, a, z, sz, t, st, p_outlier, w_outlier)
                                              src/cdfdif_wrapper.pyx:16-53

returns the per-trial DMAT / Tuerlinckx (2004) CDF of signed RTs with the
outlier mixture: F(|x|, boundary) from cdfdif (src/cdfdif.c:59-221), folded as
(1 - P(upper)) + sign(x) * F, then y (1 - p_out) + (x + 1/(2 w_out)) w_out p_out.
Callers: the stochastic's `cdf` (hddm/likelihoods.py:90-91) and the quantile /
chi-square optimisers built on it (likelihoods.py:200-239, base.py:249-264).

The series run in the HIP kernel of libwfpt_amd.so (cdfdif_kernels.hip);
argument checks and their exceptions are the reference's.
"""
import ctypes

import numpy as np

from . import _lib
from .wfpt import _check_x

__all__ = ["dmat_cdf_array"]


def dmat_cdf_array(x, v, sv, a, z, sz, t, st, p_outlier, w_outlier):
    x = _check_x(x)
    # cdfdif_wrapper.pyx:20-21 (np.max of an empty array raises, as there)
    if p_outlier > 0:
        assert np.max(np.abs(x)) < (1. / (2 * w_outlier)), \
            ValueError('1. / (2*w_outlier) must be smaller than RT')
    # cdfdif_wrapper.pyx:23-25
    if (sv < 0) or (a <= 0) or (z < 0) or (z > 1) or (sz < 0) or (sz > 1) or \
            (z + sz / 2. > 1) or (z - sz / 2. < 0) or (t - st / 2. < 0) or (t < 0) or \
            (st < 0) or not ((p_outlier >= 0) & (p_outlier <= 1)):
        raise ValueError("at least one of the parameters is out of the support")
    n = x.shape[0]
    # add_outlier_cdf (cdfdif_wrapper.pyx:11-12) divides by 2*w_outlier in
    # Python semantics for every trial: a zero raises on the first one.
    if n > 0 and float(w_outlier) == 0.0:
        raise ZeroDivisionError("float division")
    out = np.empty(n, dtype=np.float64)
    if n == 0:
        return out
    c = _lib.context()
    P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
    _lib.check(_lib.wfpt_dmat_cdf_array(c.handle, _lib.dptr(x), n, ctypes.byref(P),
                                        float(w_outlier), _lib.dptr(out)))
    return out
