/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's DMAT / Tuerlinckx (2004) CDF:
 * cdfdif (/root/reference/src/cdfdif.c:59-221) and its array wrapper
 * dmat_cdf_array (/root/reference/src/cdfdif_wrapper.pyx:16-53), written as
 * separate steps (quadrature set-up, boundary probability, the two series)
 * with each expression in the reference's operation order, so that it gives
 * the reference's doubles. Used only by tests/ (pinned to the reference's
 * outputs in tests/golden/cdfdif*.npz) and as the timed CPU baseline of the
 * CDF row (tools/bench_rows.py); the product path (hddm_amd) never loads it.
 */
#include <math.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define CD_PI 3.1415926535897932384626433832795028841971693993751

/* 6-point Gauss-Hermite (drift) and Gauss-Legendre (start point) rules,
 * cdfdif.c:78-81 */
static const double GH_X[6] = {-2.3506049736744922818, -1.3358490740136970132,
                               -.43607741192761650950, .43607741192761650950,
                               1.3358490740136970132, 2.3506049736744922818};
static const double GH_W[6] = {.45300099055088421593e-2, .15706732032114842368,
                               .72462959522439207571, .72462959522439207571,
                               .15706732032114842368, .45300099055088421593e-2};
static const double GL_X[6] = {-.93246951420315193904, -.66120938646626381541,
                               -.23861918608319693247, .23861918608319712676,
                               .66120938646626459256, .93246951420315160597};
static const double GL_W[6] = {.17132449237917049545, .36076157304813916138,
                               .46791393457269092604, .46791393457269092604,
                               .36076157304813843973, .17132449237917132812};

typedef struct {
    double a, ter, eta, z, sz, st, nu, a2;
    double gk[6], wgh[6], gz[6];
} cd_model;

static void cd_setup(cd_model *M, const double *par)
{
    M->a = par[0];
    M->ter = par[1];
    M->eta = par[2];
    M->z = par[3];
    M->sz = par[4];
    M->st = par[5];
    M->nu = par[6];
    M->a2 = M->a * M->a;
    for (int m = 0; m < 6; m++) {
        M->gk[m] = 1.41421356237309505 * GH_X[m] * M->eta + M->nu; /* drift nodes */
        M->wgh[m] = GH_W[m] / 1.772453850905515882;
    }
    for (int i = 0; i < 6; i++) M->gz[i] = (.5 * M->sz * GL_X[i]) + M->z; /* start nodes */
}

/* P(absorbed at the lower boundary), averaged over drift and start point
 * (cdfdif.c:91-109) */
static double cd_prob(const cd_model *M)
{
    double tot = 0;
    for (int i = 0; i < 6; i++) {
        double acc = 0;
        for (int m = 0; m < 6; m++) {
            if (fabs(M->gk[m]) > 1e-7)
                acc += (exp(-200 * M->gz[i] * M->gk[m]) - 1) / (exp(-200 * M->a * M->gk[m]) - 1) *
                       M->wgh[m];
            else
                acc += M->gz[i] / M->a * M->wgh[m];
        }
        tot += acc * GL_W[i] / 2;
    }
    return tot;
}

/* The partial-sum stop rule shared by every series (cdfdif.c:139-141 etc.) */
static int cd_converged(const double h[3])
{
    return (fabs(h[0] - h[1]) < 1e-29) && (fabs(h[1] - h[2]) < 1e-29) && (h[2] > 0);
}

/* t beyond the Ter window (cdfdif.c:120-145): the series over v with the
 * drift integral inside each term */
static double cd_series_beyond(const cd_model *M, double t, int x, double zu, double zl,
                               double up, double lo)
{
    double h[3] = {0, 0, 0};
    const double sgn = 2 * x - 1;
    for (int v = 0; v < 5000; v++) {
        h[0] = h[1];
        h[1] = h[2];
        double acc = 0;
        const double sifa = CD_PI * v / M->a;
        for (int m = 0; m < 6; m++) {
            const double g = M->gk[m];
            const double den = (100 * g * g + (CD_PI * CD_PI) * (v * v) / (100 * M->a2));
            const double eu = exp(sgn * zu * g * 100 - 3 * log(den) + log(M->wgh[m]) - 2 * log(100));
            const double el = exp(sgn * zl * g * 100 - 3 * log(den) + log(M->wgh[m]) - 2 * log(100));
            const double f = eu * (sgn * g * sin(sifa * zu) * 100 - sifa * cos(sifa * zu)) -
                             el * (sgn * g * sin(sifa * zl) * 100 - sifa * cos(sifa * zl));
            const double ed = exp((-.5 * den * (t - up)) + log(1 - exp(-.5 * den * (up - lo))));
            acc += f * ed;
        }
        h[2] = h[1] + v * acc;
        if (cd_converged(h)) break;
    }
    return h[2];
}

/* t inside the Ter window, drift node m away from zero (cdfdif.c:152-177) */
static double cd_window_node(const cd_model *M, double t, int x, double lo, int m)
{
    const double g = M->gk[m];
    const double a = M->a, a2 = M->a2;
    double tot = 0;
    for (int i = 0; i < 6; i++) {
        const double zz = (a - M->gz[i]) * x + M->gz[i] * (1 - x);
        const double sh = sinh((1 - 2 * x) * g * a / .01);
        const double ser = -((a * a2) / ((1 - 2 * x) * g * CD_PI * .01)) *
                               sinh(zz * (1 - 2 * x) * g / .01) / (sh * sh) +
                           (zz * a2) / ((1 - 2 * x) * g * CD_PI * .01) *
                               cosh((a - zz) * (1 - 2 * x) * g / .01) / sh;
        double h[3] = {0, 0, 0};
        for (int v = 0; v < 5000; v++) {
            h[0] = h[1];
            h[1] = h[2];
            const double sifa = CD_PI * v / a;
            const double den = (g * g * 100 + (CD_PI * v) * (CD_PI * v) / (a2 * 100));
            h[2] = h[1] + v * sin(sifa * zz) * exp(-.5 * den * (t - lo) - 2 * log(den));
            if (cd_converged(h)) break;
        }
        tot += .5 * GL_W[i] * (ser - 4 * h[2]) * (CD_PI / 100) / (a2 * M->st) *
               exp((2 * x - 1) * zz * g * 100);
    }
    return tot;
}

/* t inside the Ter window, drift node at zero (cdfdif.c:179-197) */
static double cd_window_zero(const cd_model *M, double t, double zu, double zl, double lo)
{
    const double a = M->a, a2 = M->a2;
    double h[3] = {0, 0, 0};
    const double su = -(zu * zu) / (12 * a2) + (zu * zu * zu) / (12 * a * a2) -
                      (zu * zu * zu * zu) / (48 * a2 * a2);
    const double sl = -(zl * zl) / (12 * a2) + (zl * zl * zl) / (12 * a * a2) -
                      (zl * zl * zl * zl) / (48 * a2 * a2);
    for (int v = 1; v < 5000; v++) {
        h[0] = h[1];
        h[1] = h[2];
        const double sifa = CD_PI * v / a;
        const double den = (CD_PI * v) * (CD_PI * v) / (a2 * 100);
        h[2] = h[1] + 1 / (CD_PI * CD_PI * CD_PI * CD_PI * v * v * v * v) *
                          (cos(sifa * zl) - cos(sifa * zu)) * exp(-.5 * den * (t - lo));
        if (cd_converged(h)) break;
    }
    return 400 * a2 * a * (sl - su - h[2]) / (M->st * M->sz);
}

/* cdfdif(t, x, par, &prob) (cdfdif.c:59-221) */
double oracle_cdfdif(double t, int x, const double *par, double *prob)
{
    cd_model M;
    cd_setup(&M, par);
    const double zu = (1 - x) * M.z + x * (M.a - M.z) + M.sz / 2;
    const double zl = (1 - x) * M.z + x * (M.a - M.z) - M.sz / 2;
    const double lo = M.ter - M.st / 2;
    double F = 0;
    *prob = cd_prob(&M);
    if (t - M.ter + M.st / 2 > 0.001) {
        const double up = t < M.ter + M.st / 2 ? t : M.ter + M.st / 2;
        const double p1 = *prob * (up - lo) / M.st;
        const double p0 = (1 - *prob) * (up - lo) / M.st;
        if (t > M.ter + M.st / 2) {
            const double s = cd_series_beyond(&M, t, x, zu, zl, up, lo);
            F = (p0 * (1 - x) + p1 * x) - s * 4 * CD_PI / (M.a2 * M.sz * M.st);
        } else if (t <= M.ter + M.st / 2) {
            double acc = 0;
            for (int m = 0; m < 6; m++) {
                const double part = fabs(M.gk[m]) > 1e-7 ? cd_window_node(&M, t, x, lo, m)
                                                         : cd_window_zero(&M, t, zu, zl, lo);
                acc += part * M.wgh[m];
            }
            F = (p0 * (1 - x) + p1 * x) - acc;
        }
    }
    return F > 1e-29 ? F : 0;
}

/* dmat_cdf_array's loop (cdfdif_wrapper.pyx:35-53) after its argument checks;
 * returns 0, or -1 for parameters outside the support (the wrapper raises). */
int oracle_dmat_cdf_array(const double *x, int64_t n, double v, double sv, double a, double z,
                          double sz, double t, double st, double p_outlier, double w_outlier,
                          double *out)
{
    if ((sv < 0) || (a <= 0) || (z < 0) || (z > 1) || (sz < 0) || (sz > 1) || (z + sz / 2. > 1) ||
        (z - sz / 2. < 0) || (t - st / 2. < 0) || (t < 0) || (st < 0) ||
        !((p_outlier >= 0) && (p_outlier <= 1)))
        return -1;
    const double epsi = 1e-10;
    const double par[7] = {a / 10., t, sv / 10. + epsi, z * (a / 10.), sz * (a / 10.) + epsi,
                           st + epsi, v / 10.};
    for (int64_t i = 0; i < n; i++) {
        double pb;
        const int bnd = x[i] > 0;
        double y = oracle_cdfdif(fabs(x[i]), bnd, par, &pb);
        const double sg = x[i] > 0 ? 1.0 : (x[i] < 0 ? -1.0 : (x[i] == 0 ? 0.0 : x[i]));
        y = (1 - pb) + sg * y; /* np.sign: NaN stays NaN */
        out[i] = y * (1 - p_outlier) + (x[i] + (1. / (2 * w_outlier))) * w_outlier * p_outlier;
    }
    return 0;
}

/* the same loop over n_threads OpenMP threads (the multi-core CPU baseline;
 * not the reference's build) */
int oracle_dmat_cdf_array_omp(const double *x, int64_t n, double v, double sv, double a,
                              double z, double sz, double t, double st, double p_outlier,
                              double w_outlier, double *out, int n_threads)
{
    int rc = 0, used = 1;
#pragma omp parallel num_threads(n_threads > 0 ? n_threads : 1)
    {
#pragma omp single
        {
#ifdef _OPENMP
            used = omp_get_num_threads();
#endif
        }
        const int64_t nt = used;
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        const int64_t lo = n * tid / nt, hi = n * (tid + 1) / nt;
        if (oracle_dmat_cdf_array(x + lo, hi - lo, v, sv, a, z, sz, t, st, p_outlier, w_outlier,
                                  out + lo) != 0)
            rc = -1;
    }
    return rc < 0 ? -1 : used;
}
