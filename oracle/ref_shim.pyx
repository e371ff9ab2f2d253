# cython: language_level=2
# cython: cdivision=True
# cython: wraparound=False
# cython: boundscheck=False
# distutils: language = c++
#
# ORACLE — TEST INFRASTRUCTURE ONLY.
#
# Thin Cython module that compiles the reference's OWN numeric kernels
# (/root/reference/src/integrate.pxi, which includes pdf.pxi) where they lie,
# via Cython's include path (see oracle/build_ref.py). No reference source is
# copied into this repository.
#
# Why not build src/wfpt.pyx itself: wfpt.pyx:16 executes `import hddm`, whose
# package needs PyMC 2 + kabuki (absent offline); making it importable would
# need a stand-in module, which this build does not use. Everything that
# computes (ftt_01w, pdf, pdf_sv, full_pdf, the Simpson integrators) comes from
# the reference unchanged; only the two ~15-line Python loops of
# wfpt.pyx:32-48 (pdf_array) and wfpt.pyx:54-76 (wiener_like) are restated
# below around the reference's `full_pdf`.

include "integrate.pxi"

def ref_ftt_01w(double tt, double w, double err):
    return ftt_01w(tt, w, err)

def ref_pdf_sv(double x, double v, double sv, double a, double z, double err):
    return pdf_sv(x, v, sv, a, z, err)

def ref_prob_ub(double v, double a, double z):
    return prob_ub(v, a, z)

# restatement of wfpt.pyx:32-48 around the reference full_pdf
def pdf_array(np.ndarray[double, ndim=1] x, double v, double sv, double a, double z, double sz,
              double t, double st, double err=1e-4, bint logp=0, int n_st=2, int n_sz=2, bint use_adaptive=1,
              double simps_err=1e-3, double p_outlier=0, double w_outlier=0):
    cdef Py_ssize_t size = x.shape[0]
    cdef Py_ssize_t i
    cdef np.ndarray[double, ndim=1] y = np.empty(size, dtype=np.double)
    for i in range(size):
        y[i] = full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive, simps_err)
    y = y * (1 - p_outlier) + (w_outlier * p_outlier)
    if logp == 1:
        return np.log(y)
    return y

# wfpt.pyx:32-42's prange loop around the reference full_pdf, for the
# all-threads CPU calibration only: oracle/build_ref.py compiles this module
# with -fopenmp so the prange runs in parallel (the reference's own setup.py
# has no -fopenmp, so its pdf_array runs serially). Densities only (no
# mixture / log epilogue): the same loop shape as oracle_pdf_array_omp.
from cython.parallel import prange

def pdf_array_prange(np.ndarray[double, ndim=1] x, double v, double sv, double a, double z,
                     double sz, double t, double st, double err=1e-4, int n_st=2, int n_sz=2,
                     bint use_adaptive=1, double simps_err=1e-3, int n_threads=1):
    cdef Py_ssize_t size = x.shape[0]
    cdef Py_ssize_t i
    cdef np.ndarray[double, ndim=1] y = np.empty(size, dtype=np.double)
    cdef double[::1] yv = y
    cdef double[::1] xv = x
    for i in prange(size, nogil=True, num_threads=n_threads, schedule='static'):
        yv[i] = full_pdf(xv[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive, simps_err)
    return y

# restatement of wfpt.pyx:54-76 around the reference full_pdf
def wiener_like(np.ndarray[double, ndim=1] x, double v, double sv, double a, double z, double sz, double t,
                double st, double err, int n_st=10, int n_sz=10, bint use_adaptive=1, double simps_err=1e-8,
                double p_outlier=0, double w_outlier=0.1):
    cdef Py_ssize_t size = x.shape[0]
    cdef Py_ssize_t i
    cdef double p
    cdef double sum_logp = 0
    cdef double wp_outlier = w_outlier * p_outlier
    if not ((p_outlier >= 0) & (p_outlier <= 1)):
        return -np.inf
    for i in range(size):
        p = full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive, simps_err)
        p = p * (1 - p_outlier) + wp_outlier
        if p == 0:
            return -np.inf
        sum_logp += log(p)
    return sum_logp
