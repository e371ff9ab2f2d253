"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes bindings to oracle/wfpt_oracle.c, the plain-C CPU restatement of the
reference WFPT path (src/pdf.pxi, src/integrate.pxi, src/wfpt.pyx:32-76,244-274).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker or the timed CPU baseline. The product
package (hddm_amd) never imports it; it fails loudly without its HIP library.

Parity pins (tests/test_oracle.py): bit-exact vs oracle/_ref (the reference's
own kernels compiled by oracle/build_ref.py) on branch-covering vectors, and the
20 Navarro-Fuss MATLAB tuples of hddm/tests/matlab_values.py to 1e-9.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "liboracle_wfpt.so")
SRC = os.path.join(HERE, "wfpt_oracle.c")
SRC_CDF = os.path.join(HERE, "cdfdif_oracle.c")

_D = ctypes.c_double
_I = ctypes.c_int
_I64 = ctypes.c_int64
_PD = ctypes.POINTER(ctypes.c_double)


def build(force=False):
    """gcc -O2 -ffp-contract=off (the reference's setup.py:4-7 uses -O2, no FMA)."""
    os.makedirs(LIBDIR, exist_ok=True)
    hdr = os.path.join(HERE, "wfpt_oracle.h")
    if (not force and os.path.exists(LIB)
            and all(os.path.getmtime(LIB) > os.path.getmtime(f) for f in (SRC, SRC_CDF, hdr))):
        return LIB
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC",
                    "-shared", "-o", LIB, SRC, SRC_CDF, "-lm"], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_ftt_01w.restype = _D
        L.oracle_ftt_01w.argtypes = [_D, _D, _D]
        L.oracle_prob_ub.restype = _D
        L.oracle_prob_ub.argtypes = [_D, _D, _D]
        L.oracle_pdf_sv.restype = _D
        L.oracle_pdf_sv.argtypes = [_D] * 6
        L.oracle_full_pdf.restype = _D
        L.oracle_full_pdf.argtypes = [_D] * 9 + [_I, _I, _I, _D, ctypes.POINTER(_I64)]
        L.oracle_wiener_like.restype = _D
        L.oracle_wiener_like.argtypes = [_PD, _I64] + [_D] * 8 + [_I, _I, _I, _D, _D, _D]
        L.oracle_pdf_array.restype = None
        L.oracle_pdf_array.argtypes = [_PD, _I64] + [_D] * 8 + [_I, _I, _I, _I, _D, _D, _D, _PD]
        L.oracle_pdf_array_omp.restype = _I
        L.oracle_pdf_array_omp.argtypes = [_PD, _I64] + [_D] * 8 + [_I, _I, _I, _I, _D, _D, _D,
                                                                    _PD, _I]
        L.oracle_wiener_like_multi.restype = _D
        L.oracle_wiener_like_multi.argtypes = [_PD, _I64, ctypes.POINTER(_PD), _PD, _D, _I, _I,
                                               _I, _D, _D, _D]
        L.oracle_count_evals.restype = _I64
        L.oracle_wiener_like_multi_terms.restype = _D
        L.oracle_wiener_like_multi_terms.argtypes = [_PD, _I64, ctypes.POINTER(_PD), _PD, _D, _I,
                                                     _I, _I, _D, _D, _D, _PD]
        L.oracle_count_evals.argtypes = [_PD, _I64] + [_D] * 8 + [_I, _I, _I, _D]
        L.oracle_dmat_cdf_array.restype = _I
        L.oracle_dmat_cdf_array.argtypes = [_PD, _I64] + [_D] * 9 + [_PD]
        L.oracle_dmat_cdf_array_omp.restype = _I
        L.oracle_dmat_cdf_array_omp.argtypes = [_PD, _I64] + [_D] * 9 + [_PD, _I]
        _lib = L
    return _lib


def _arr(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return x, x.ctypes.data_as(_PD)


def ftt_01w(tt, w, err):
    return lib().oracle_ftt_01w(tt, w, err)


def prob_ub(v, a, z):
    return lib().oracle_prob_ub(v, a, z)


def pdf_sv(x, v, sv, a, z, err):
    return lib().oracle_pdf_sv(x, v, sv, a, z, err)


def full_pdf(x, v, sv, a, z, sz, t, st, err, n_st=2, n_sz=2, use_adaptive=1, simps_err=1e-3):
    return lib().oracle_full_pdf(x, v, sv, a, z, sz, t, st, err, n_st, n_sz, int(use_adaptive),
                                 simps_err, None)


def wiener_like(x, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10, use_adaptive=1,
                simps_err=1e-8, p_outlier=0, w_outlier=0.1):
    x, px = _arr(x)
    return lib().oracle_wiener_like(px, x.size, v, sv, a, z, sz, t, st, err, n_st, n_sz,
                                    int(use_adaptive), simps_err, p_outlier, w_outlier)


def pdf_array(x, v, sv, a, z, sz, t, st, err=1e-4, logp=0, n_st=2, n_sz=2, use_adaptive=1,
              simps_err=1e-3, p_outlier=0, w_outlier=0, n_threads=None):
    x, px = _arr(x)
    out = np.empty_like(x)
    if n_threads is None:
        # the reference applies np.log to the mixture array (wfpt.pyx:45-46); NumPy's log
        # differs from libm's by <= 1 ulp, so the log is taken here, in NumPy, too.
        lib().oracle_pdf_array(px, x.size, v, sv, a, z, sz, t, st, err, 0, n_st, n_sz,
                               int(use_adaptive), simps_err, p_outlier, w_outlier,
                               out.ctypes.data_as(_PD))
        if logp == 1:
            with np.errstate(divide="ignore", invalid="ignore"):
                out = np.log(out)
    else:
        lib().oracle_pdf_array_omp(px, x.size, v, sv, a, z, sz, t, st, err, int(logp), n_st,
                                   n_sz, int(use_adaptive), simps_err, p_outlier, w_outlier,
                                   out.ctypes.data_as(_PD), int(n_threads))
    return out


def wiener_like_multi(x, v, sv, a, z, sz, t, st, err, multi=None, n_st=10, n_sz=10,
                      use_adaptive=1, simps_err=1e-3, p_outlier=0, w_outlier=0, terms=False):
    """The reference's wiener_like_multi (wfpt.pyx:244-274); terms=True:
    (sum, per-trial terms)."""
    x, px = _arr(x)
    vals = [v, sv, a, z, sz, t, st]
    names = ["v", "sv", "a", "z", "sz", "t", "st"]
    multi = set(multi or ())
    keep = []
    ptrs = (_PD * 7)()
    scal = (_D * 7)()
    for j, (nm, val) in enumerate(zip(names, vals)):
        if nm in multi:
            arr, p = _arr(val)
            keep.append(arr)
            ptrs[j] = p
            scal[j] = 0.0
        else:
            ptrs[j] = _PD()
            scal[j] = float(val)
    out = np.empty(x.size) if terms else None
    tot = lib().oracle_wiener_like_multi_terms(px, x.size, ptrs, scal, err, n_st, n_sz,
                                               int(use_adaptive), simps_err, p_outlier,
                                               w_outlier,
                                               out.ctypes.data_as(_PD) if terms else None)
    return (tot, out) if terms else tot


def dmat_cdf_array(x, v, sv, a, z, sz, t, st, p_outlier, w_outlier, n_threads=None):
    """The reference's cdfdif_wrapper.dmat_cdf_array (cdfdif_wrapper.pyx:16-53
    over cdfdif.c:59-221) restated in C (oracle/cdfdif_oracle.c)."""
    x, px = _arr(x)
    out = np.empty_like(x)
    if n_threads is None:
        rc = lib().oracle_dmat_cdf_array(px, x.size, v, sv, a, z, sz, t, st, p_outlier,
                                         w_outlier, out.ctypes.data_as(_PD))
    else:
        rc = lib().oracle_dmat_cdf_array_omp(px, x.size, v, sv, a, z, sz, t, st, p_outlier,
                                             w_outlier, out.ctypes.data_as(_PD), int(n_threads))
    if rc < 0:
        raise ValueError("at least one of the parameters is out of the support")
    return out


def count_evals(x, v, sv, a, z, sz, t, st, err=1e-4, n_st=2, n_sz=2, use_adaptive=1,
                simps_err=1e-3):
    x, px = _arr(x)
    return lib().oracle_count_evals(px, x.size, v, sv, a, z, sz, t, st, err, n_st, n_sz,
                                    int(use_adaptive), simps_err)


def _load_ref_module(name):
    import importlib
    import sys
    d = os.path.join(HERE, "_ref")
    if not os.path.isdir(d):
        return None
    if d not in sys.path:
        sys.path.insert(0, d)
    try:
        return importlib.import_module(name)
    except ImportError:
        return None


def load_ref():
    """Import oracle/_ref/ref_shim (the reference's own kernels) or return None."""
    return _load_ref_module("ref_shim")


def load_ref_cdfdif():
    """Import oracle/_ref/cdfdif_wrapper (the reference's own cdfdif_wrapper
    extension, src/cdfdif_wrapper.pyx + src/cdfdif.c) or return None."""
    return _load_ref_module("cdfdif_wrapper")
