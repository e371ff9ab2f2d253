/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see wfpt_oracle.h).
 *
 * CPU restatement of the reference WFPT path, expression-for-expression in the
 * order the reference's generated C evaluates them, so that it is bit-exact
 * against the reference built with the same compiler and libm
 * (tests/test_oracle.py checks this against oracle/_ref).
 *
 * Build: gcc -O2 -ffp-contract=off (x86-64 without FMA, as the reference's
 * setup.py:4-13 build). `pow(x,2.)` is written x*x (gcc folds it the same way
 * at -O2); pow(tt,3.) stays a libm pow call like the reference.
 */
#include "wfpt_oracle.h"

#include <math.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static inline double dmax(double a, double b) { return (a < b) ? b : a; } /* std::max */

/* pdf.pxi:28-65 — Navarro & Fuss (2009) f(t|0,1,w) */
double oracle_ftt_01w(double tt, double w, double err)
{
    double kl, ks, p;
    int k, K, lower, upper;
    const double pi2 = M_PI * M_PI; /* M_PI**2, folded to a constant */

    /* number of terms for large t (pdf.pxi:36-40) */
    if ((M_PI * tt) * err < 1.0) {
        kl = sqrt((-2.0 * log((M_PI * tt) * err)) / (pi2 * tt));
        kl = dmax(kl, 1. / (M_PI * sqrt(tt)));
    } else {
        kl = 1. / (M_PI * sqrt(tt));
    }
    /* number of terms for small t (pdf.pxi:43-47) */
    if ((2.0 * sqrt((2.0 * M_PI) * tt)) * err < 1.0) {
        ks = 2.0 + sqrt((-2.0 * tt) * log((2.0 * sqrt((2.0 * M_PI) * tt)) * err));
        ks = dmax(ks, sqrt(tt) + 1.0);
    } else {
        ks = 2.0;
    }

    p = 0.0;
    if (ks < kl) { /* small-t series (pdf.pxi:51-57) */
        K = (int)ceil(ks);
        lower = (int)(-floor((K - 1) / 2.));
        upper = (int)ceil((K - 1) / 2.);
        for (k = lower; k <= upper; k++) {
            double wk = w + (double)(2 * k);
            p = p + wk * exp(((-(wk * wk)) / 2.0) / tt);
        }
        p = p / sqrt((2.0 * M_PI) * pow(tt, 3.0));
    } else { /* large-t series (pdf.pxi:59-63) */
        K = (int)ceil(kl);
        for (k = 1; k <= K; k++) {
            double dk = (double)k;
            p = p + (dk * exp((((-(dk * dk)) * pi2) * tt) / 2.0)) * sin((dk * M_PI) * w);
        }
        p = p * M_PI;
    }
    return p;
}

/* pdf.pxi:67-72 */
double oracle_prob_ub(double v, double a, double z)
{
    if (v == 0) return z;
    return (exp(((-2.0 * a) * z) * v) - 1.0) / (exp((-2.0 * a) * v) - 1.0);
}

/* pdf.pxi:74-85 */
double oracle_pdf(double x, double v, double a, double w, double err)
{
    if (x <= 0) return 0.0;
    double tt = x / (a * a);
    double p = oracle_ftt_01w(tt, w, err);
    return (p * exp((((-v) * a) * w) - (((v * v) * x) / 2.))) / (a * a);
}

/* pdf.pxi:87-102 */
double oracle_pdf_sv(double x, double v, double sv, double a, double z, double err)
{
    if (x <= 0) return 0.0;
    if (sv == 0) return oracle_pdf(x, v, a, z, err);
    double tt = x / (a * a);
    double p = oracle_ftt_01w(tt, z, err);
    double azsv = (a * z) * sv;
    return (exp(log(p) + ((((azsv * azsv) - (((2.0 * a) * v) * z)) - ((v * v) * x)) /
                          (((2.0 * (sv * sv)) * x) + 2.0))) /
            sqrt(((sv * sv) * x) + 1.0)) / (a * a);
}

/* evaluation counter threaded through the integrators */
typedef struct { int64_t *n; } cnt_t;
static inline double pdf_sv_c(double x, double v, double sv, double a, double z, double err,
                              cnt_t c)
{
    if (c.n) (*c.n)++;
    return oracle_pdf_sv(x, v, sv, a, z, err);
}

/* integrate.pxi:12-45 (fixed composite Simpson, 1-D) */
static double simpson_1D(double x, double v, double sv, double a, double z, double t, double err,
                         double lb_z, double ub_z, int n_sz, double lb_t, double ub_t, int n_st,
                         cnt_t c)
{
    double ht, hz;
    int n = (n_st < n_sz) ? n_sz : n_st;
    if (n_st == 0) {
        hz = (ub_z - lb_z) / n;
        ht = 0;
        lb_t = t;
        ub_t = t;
    } else {
        hz = 0;
        ht = (ub_t - lb_t) / n;
        lb_z = z;
        ub_z = z;
    }
    double S = pdf_sv_c(x - lb_t, v, sv, a, lb_z, err, c);
    double z_tag, t_tag;
    double y = 0.0; /* reference leaves y uninitialised when n == 0 (UB there) */
    int i;
    for (i = 1; i <= n; i++) {
        z_tag = lb_z + hz * i;
        t_tag = lb_t + ht * i;
        y = pdf_sv_c(x - t_tag, v, sv, a, z_tag, err, c);
        if (i & 1) S += (4 * y);
        else S += (2 * y);
    }
    S = S - y;
    S = S / ((ub_t - lb_t) + (ub_z - lb_z));
    return ((ht + hz) * S) / 3;
}

/* integrate.pxi:47-70 (fixed composite Simpson, 2-D) */
static double simpson_2D(double x, double v, double sv, double a, double z, double t, double err,
                         double lb_z, double ub_z, int n_sz, double lb_t, double ub_t, int n_st,
                         cnt_t c)
{
    double ht = (ub_t - lb_t) / n_st;
    double S = simpson_1D(x, v, sv, a, z, lb_t, err, lb_z, ub_z, n_sz, 0, 0, 0, c);
    double t_tag, y = 0.0;
    int i_t;
    for (i_t = 1; i_t <= n_st; i_t++) {
        t_tag = lb_t + ht * i_t;
        y = simpson_1D(x, v, sv, a, z, t_tag, err, lb_z, ub_z, n_sz, 0, 0, 0, c);
        if (i_t & 1) S += (4 * y);
        else S += (2 * y);
    }
    S = S - y;
    S = S / (ub_t - lb_t);
    return (ht * S) / 3;
}

/* integrate.pxi:72-112 */
static double adaptiveSimpsonsAux(double x, double v, double sv, double a, double z, double t,
                                  double pdf_err, double lb_z, double ub_z, double lb_t,
                                  double ub_t, double ZT, double simps_err, double S,
                                  double f_beg, double f_end, double f_mid, int bottom, cnt_t c)
{
    double z_c, z_d, z_e, t_c, t_d, t_e, h;
    if ((ub_t - lb_t) == 0) { /* integration over sz */
        h = ub_z - lb_z;
        z_c = (ub_z + lb_z) / 2.;
        z_d = (lb_z + z_c) / 2.;
        z_e = (z_c + ub_z) / 2.;
        t_c = t;
        t_d = t;
        t_e = t;
    } else { /* integration over t */
        h = ub_t - lb_t;
        t_c = (ub_t + lb_t) / 2.;
        t_d = (lb_t + t_c) / 2.;
        t_e = (t_c + ub_t) / 2.;
        z_c = z;
        z_d = z;
        z_e = z;
    }
    double fd = pdf_sv_c(x - t_d, v, sv, a, z_d, pdf_err, c) / ZT;
    double fe = pdf_sv_c(x - t_e, v, sv, a, z_e, pdf_err, c) / ZT;
    double Sleft = (h / 12) * ((f_beg + (4 * fd)) + f_mid);
    double Sright = (h / 12) * ((f_mid + (4 * fe)) + f_end);
    double S2 = Sleft + Sright;
    if (bottom <= 0 || fabs(S2 - S) <= 15 * simps_err) return S2 + (S2 - S) / 15;
    double left = adaptiveSimpsonsAux(x, v, sv, a, z, t, pdf_err, lb_z, z_c, lb_t, t_c, ZT,
                                      simps_err / 2, Sleft, f_beg, f_mid, fd, bottom - 1, c);
    double right = adaptiveSimpsonsAux(x, v, sv, a, z, t, pdf_err, z_c, ub_z, t_c, ub_t, ZT,
                                       simps_err / 2, Sright, f_mid, f_end, fe, bottom - 1, c);
    return left + right;
}

/* integrate.pxi:114-141 */
static double adaptiveSimpsons_1D(double x, double v, double sv, double a, double z, double t,
                                  double pdf_err, double lb_z, double ub_z, double lb_t,
                                  double ub_t, double simps_err, int maxRecursionDepth, cnt_t c)
{
    double h;
    if ((ub_t - lb_t) == 0) { /* integration over z */
        lb_t = t;
        ub_t = t;
        h = ub_z - lb_z;
    } else { /* integration over t */
        h = (ub_t - lb_t);
        lb_z = z;
        ub_z = z;
    }
    double ZT = h;
    double c_t = (lb_t + ub_t) / 2.;
    double c_z = (lb_z + ub_z) / 2.;
    double f_beg = pdf_sv_c(x - lb_t, v, sv, a, lb_z, pdf_err, c) / ZT;
    double f_end = pdf_sv_c(x - ub_t, v, sv, a, ub_z, pdf_err, c) / ZT;
    double f_mid = pdf_sv_c(x - c_t, v, sv, a, c_z, pdf_err, c) / ZT;
    double S = (h / 6) * ((f_beg + (4 * f_mid)) + f_end);
    return adaptiveSimpsonsAux(x, v, sv, a, z, t, pdf_err, lb_z, ub_z, lb_t, ub_t, ZT, simps_err,
                               S, f_beg, f_end, f_mid, maxRecursionDepth, c);
}

/* integrate.pxi:143-178 */
static double adaptiveSimpsonsAux_2D(double x, double v, double sv, double a, double z, double t,
                                     double pdf_err, double err_1d, double lb_z, double ub_z,
                                     double lb_t, double ub_t, double st, double err_2d, double S,
                                     double f_beg, double f_end, double f_mid,
                                     int maxRecursionDepth_sz, int bottom, cnt_t c)
{
    double t_c = (ub_t + lb_t) / 2.;
    double t_d = (lb_t + t_c) / 2.;
    double t_e = (t_c + ub_t) / 2.;
    double h = ub_t - lb_t;
    double fd = adaptiveSimpsons_1D(x, v, sv, a, z, t_d, pdf_err, lb_z, ub_z, 0, 0, err_1d,
                                    maxRecursionDepth_sz, c) / st;
    double fe = adaptiveSimpsons_1D(x, v, sv, a, z, t_e, pdf_err, lb_z, ub_z, 0, 0, err_1d,
                                    maxRecursionDepth_sz, c) / st;
    double Sleft = (h / 12) * ((f_beg + (4 * fd)) + f_mid);
    double Sright = (h / 12) * ((f_mid + (4 * fe)) + f_end);
    double S2 = Sleft + Sright;
    if (bottom <= 0 || fabs(S2 - S) <= 15 * err_2d) return S2 + (S2 - S) / 15;
    double left = adaptiveSimpsonsAux_2D(x, v, sv, a, z, t, pdf_err, err_1d, lb_z, ub_z, lb_t,
                                         t_c, st, err_2d / 2, Sleft, f_beg, f_mid, fd,
                                         maxRecursionDepth_sz, bottom - 1, c);
    double right = adaptiveSimpsonsAux_2D(x, v, sv, a, z, t, pdf_err, err_1d, lb_z, ub_z, t_c,
                                          ub_t, st, err_2d / 2, Sright, f_mid, f_end, fe,
                                          maxRecursionDepth_sz, bottom - 1, c);
    return left + right;
}

/* integrate.pxi:181-206 */
static double adaptiveSimpsons_2D(double x, double v, double sv, double a, double z, double t,
                                  double pdf_err, double lb_z, double ub_z, double lb_t,
                                  double ub_t, double simps_err, int maxRecursionDepth_sz,
                                  int maxRecursionDepth_st, cnt_t c)
{
    double h = (ub_t - lb_t);
    double st = (ub_t - lb_t);
    double err_1d = simps_err;
    double err_2d = simps_err;
    double f_beg = adaptiveSimpsons_1D(x, v, sv, a, z, lb_t, pdf_err, lb_z, ub_z, 0, 0, err_1d,
                                       maxRecursionDepth_sz, c) / st;
    double f_end = adaptiveSimpsons_1D(x, v, sv, a, z, ub_t, pdf_err, lb_z, ub_z, 0, 0, err_1d,
                                       maxRecursionDepth_sz, c) / st;
    double f_mid = adaptiveSimpsons_1D(x, v, sv, a, z, (lb_t + ub_t) / 2, pdf_err, lb_z, ub_z, 0,
                                       0, err_1d, maxRecursionDepth_sz, c) / st;
    double S = (h / 6) * ((f_beg + (4 * f_mid)) + f_end);
    return adaptiveSimpsonsAux_2D(x, v, sv, a, z, t, pdf_err, err_1d, lb_z, ub_z, lb_t, ub_t, st,
                                  err_2d, S, f_beg, f_end, f_mid, maxRecursionDepth_sz,
                                  maxRecursionDepth_st, c);
}

/* pdf.pxi:104-146 */
double oracle_full_pdf(double x, double v, double sv, double a, double z, double sz, double t,
                       double st, double err, int n_st, int n_sz, int use_adaptive,
                       double simps_err, int64_t *n_eval)
{
    cnt_t c = {n_eval};
    if ((z < 0) || (z > 1) || (a < 0) || (t < 0) || (st < 0) || (sv < 0) || (sz < 0) ||
        (sz > 1) || ((fabs(x) - (t - st / 2.)) < 0) || (z + sz / 2. > 1) || (z - sz / 2. < 0) ||
        (t - st / 2. < 0))
        return 0;
    if (x > 0) { /* upper-boundary response */
        v = -v;
        z = 1. - z;
    }
    x = fabs(x);
    if (st < 1e-3) st = 0;
    if (sz < 1e-3) sz = 0;

    if (sz == 0) {
        if (st == 0) return pdf_sv_c(x - t, v, sv, a, z, err, c);
        if (use_adaptive > 0)
            return adaptiveSimpsons_1D(x, v, sv, a, z, t, err, z, z, t - st / 2., t + st / 2.,
                                       simps_err, n_st, c);
        return simpson_1D(x, v, sv, a, z, t, err, z, z, 0, t - st / 2., t + st / 2., n_st, c);
    }
    if (st == 0) {
        if (use_adaptive)
            return adaptiveSimpsons_1D(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., t, t,
                                       simps_err, n_sz, c);
        return simpson_1D(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., n_sz, t, t, 0, c);
    }
    if (use_adaptive)
        return adaptiveSimpsons_2D(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., t - st / 2.,
                                   t + st / 2., simps_err, n_sz, n_st, c);
    return simpson_2D(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., n_sz, t - st / 2.,
                      t + st / 2., n_st, c);
}

/* wfpt.pyx:54-76 */
double oracle_wiener_like(const double *x, int64_t n, double v, double sv, double a, double z,
                          double sz, double t, double st, double err, int n_st, int n_sz,
                          int use_adaptive, double simps_err, double p_outlier,
                          double w_outlier)
{
    double sum_logp = 0;
    double wp_outlier = w_outlier * p_outlier;
    if (!((p_outlier >= 0) & (p_outlier <= 1))) return -INFINITY;
    for (int64_t i = 0; i < n; i++) {
        double p = oracle_full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive,
                                   simps_err, NULL);
        p = p * (1 - p_outlier) + wp_outlier;
        if (p == 0) return -INFINITY;
        sum_logp += log(p);
    }
    return sum_logp;
}

/* wfpt.pyx:32-48 */
void oracle_pdf_array(const double *x, int64_t n, double v, double sv, double a, double z,
                      double sz, double t, double st, double err, int logp, int n_st, int n_sz,
                      int use_adaptive, double simps_err, double p_outlier, double w_outlier,
                      double *out)
{
    for (int64_t i = 0; i < n; i++) {
        double y = oracle_full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive,
                                   simps_err, NULL);
        y = y * (1 - p_outlier) + (w_outlier * p_outlier);
        out[i] = (logp == 1) ? log(y) : y;
    }
}

int oracle_pdf_array_omp(const double *x, int64_t n, double v, double sv, double a, double z,
                         double sz, double t, double st, double err, int logp, int n_st,
                         int n_sz, int use_adaptive, double simps_err, double p_outlier,
                         double w_outlier, double *out, int n_threads)
{
    int used = 1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
    }
#pragma omp parallel for schedule(dynamic, 1024)
#endif
    for (int64_t i = 0; i < n; i++) {
        double y = oracle_full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive,
                                   simps_err, NULL);
        y = y * (1 - p_outlier) + (w_outlier * p_outlier);
        out[i] = (logp == 1) ? log(y) : y;
    }
    (void)n_threads;
    return used;
}

/* wfpt.pyx:244-274 */
/* wiener_like_multi with each trial's term of the sum in terms[i] (nullable) */
double oracle_wiener_like_multi_terms(const double *x, int64_t n, const double *const arrays[7],
                                      const double scalars[7], double err, int n_st, int n_sz,
                                      int use_adaptive, double simps_err, double p_outlier,
                                      double w_outlier, double *terms)
{
    double sum_logp = 0;
    double wp_outlier = w_outlier * p_outlier;
    for (int64_t i = 0; i < n; i++) {
        double q[7];
        for (int j = 0; j < 7; j++) q[j] = arrays[j] ? arrays[j][i] : scalars[j];
        /* q = v, sv, a, z, sz, t, st */
        double p;
        if (fabs(x[i]) != 999.) {
            p = oracle_full_pdf(x[i], q[0], q[1], q[2], q[3], q[4], q[5], q[6], err, n_st, n_sz,
                                use_adaptive, simps_err, NULL);
            p = p * (1 - p_outlier) + wp_outlier;
        } else if (x[i] == 999.) {
            p = oracle_prob_ub(q[0], q[2], q[3]);
        } else {
            p = 1 - oracle_prob_ub(q[0], q[2], q[3]);
        }
        if (terms) terms[i] = log(p);
        sum_logp += log(p);
    }
    return sum_logp;
}

double oracle_wiener_like_multi(const double *x, int64_t n, const double *const arrays[7],
                                const double scalars[7], double err, int n_st, int n_sz,
                                int use_adaptive, double simps_err, double p_outlier,
                                double w_outlier)
{
    return oracle_wiener_like_multi_terms(x, n, arrays, scalars, err, n_st, n_sz, use_adaptive,
                                          simps_err, p_outlier, w_outlier, NULL);
}

int64_t oracle_count_evals(const double *x, int64_t n, double v, double sv, double a, double z,
                           double sz, double t, double st, double err, int n_st, int n_sz,
                           int use_adaptive, double simps_err)
{
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; i++)
        (void)oracle_full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive,
                              simps_err, &cnt);
    return cnt;
}
