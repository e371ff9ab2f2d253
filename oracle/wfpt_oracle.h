/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference WFPT likelihood path
 * (/root/reference/src/pdf.pxi, integrate.pxi, wfpt.pyx:32-76).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.
 * The product path (hddm_amd) never links or calls it.
 *
 * Parity pinning: bit-exact against oracle/_ref (the reference's own
 * pdf.pxi/integrate.pxi compiled by oracle/build_ref.py) and against the
 * Navarro-Fuss MATLAB golden tuples of hddm/tests/matlab_values.py
 * (tests/golden/matlab_values.json).
 */
#ifndef WFPT_ORACLE_H
#define WFPT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* f(t|0,1,w), pdf.pxi:28-65 */
double oracle_ftt_01w(double tt, double w, double err);
/* pdf.pxi:67-72 */
double oracle_prob_ub(double v, double a, double z);
/* pdf.pxi:74-85 */
double oracle_pdf(double x, double v, double a, double w, double err);
/* pdf.pxi:87-102 */
double oracle_pdf_sv(double x, double v, double sv, double a, double z, double err);
/* pdf.pxi:104-146 ; n_eval (nullable) is incremented by the number of pdf_sv calls */
double oracle_full_pdf(double x, double v, double sv, double a, double z, double sz,
                       double t, double st, double err, int n_st, int n_sz,
                       int use_adaptive, double simps_err, int64_t *n_eval);
/* wfpt.pyx:54-76 (sequential sum, early -inf) */
double oracle_wiener_like(const double *x, int64_t n, double v, double sv, double a,
                          double z, double sz, double t, double st, double err,
                          int n_st, int n_sz, int use_adaptive, double simps_err,
                          double p_outlier, double w_outlier);
/* wfpt.pyx:32-48 (per-trial mixture density or its log) */
void oracle_pdf_array(const double *x, int64_t n, double v, double sv, double a, double z,
                      double sz, double t, double st, double err, int logp, int n_st,
                      int n_sz, int use_adaptive, double simps_err, double p_outlier,
                      double w_outlier, double *out);
/* pdf_array with OpenMP over trials (not the reference's build: setup.py:6 has
 * no -fopenmp); used only for the multi-core CPU baseline. Returns the thread
 * count used. */
int oracle_pdf_array_omp(const double *x, int64_t n, double v, double sv, double a, double z,
                         double sz, double t, double st, double err, int logp, int n_st,
                         int n_sz, int use_adaptive, double simps_err, double p_outlier,
                         double w_outlier, double *out, int n_threads);
/* wfpt.pyx:244-274 wiener_like_multi restated with per-trial parameter arrays
 * (any of v..st may be NULL => the scalar in `scalars` [v,sv,a,z,sz,t,st] is used). */
double oracle_wiener_like_multi_terms(const double *x, int64_t n, const double *const arrays[7],
                                      const double scalars[7], double err, int n_st, int n_sz,
                                      int use_adaptive, double simps_err, double p_outlier,
                                      double w_outlier, double *terms);
double oracle_wiener_like_multi(const double *x, int64_t n, const double *const arrays[7],
                                const double scalars[7], double err, int n_st, int n_sz,
                                int use_adaptive, double simps_err, double p_outlier,
                                double w_outlier);
/* total pdf_sv evaluations of full_pdf over x (feeds the roofline's W_trial) */
int64_t oracle_count_evals(const double *x, int64_t n, double v, double sv, double a,
                           double z, double sz, double t, double st, double err, int n_st,
                           int n_sz, int use_adaptive, double simps_err);

#ifdef __cplusplus
}
#endif
#endif
