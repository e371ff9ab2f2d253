// cdfdif_kernels.hip — gfx950 kernel of the DMAT / Tuerlinckx (2004) diffusion
// CDF with across-trial variability, the reference's `cdfdif_wrapper` module:
//
//   dmat_cdf_array   src/cdfdif_wrapper.pyx:16-53   (per-trial loop + outlier mix)
//   cdfdif           src/cdfdif.c:59-221            (6-point Gauss-Hermite over the
//                    drift x 6-point Gauss-Legendre over the start point, series in
//                    the boundary eigenfunctions, closed-form integral over Ter)
//
// Layout: everything that depends only on the call's parameters — the scaled
// quadrature nodes and weights, log(w_gh), and P(boundary) (cdfdif.c:84-113:
// 36 exp pairs) — is computed once per block by its first wave into LDS and
// read by every lane as broadcast loads. Two passes:
//   dmat_cdf_kernel  one trial per lane (wave64, 256-thread blocks); finishes
//                    trials below the Ter window and beyond it when the series
//                    converges within kLaneTerms terms, defers the rest;
//   cdf_wave_kernel  one wave per deferred trial: the terms of 64 consecutive
//                    v in parallel (sequential accumulation in v order), or
//                    the 36 + 6 window-branch series one per lane.
//
// Numerics: every basic operation follows the reference's expression order
// (-ffp-contract=off), and the transcendental calls are the reference's
// calls, so the result differs from the x86-64 build only through libm-vs-OCML
// ulps. That matters here: with sz = 0 or st = 0 the wrapper substitutes
// 1e-10 (cdfdif_wrapper.pyx:38-41) and cdfdif divides differences of nearly
// equal terms by sZ*st ~ 1e-20 (cdfdif.c:148), so the reference's own value
// carries that cancellation; tests/test_cdfdif.py states the tolerances.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wfpt_internal.h"

#pragma clang fp contract(off)

namespace wfpt {

namespace {

constexpr double kCPi = 3.1415926535897932384626433832795028841971693993751;  // cdfdif.c:27
constexpr double kDelta = 1e-29;   // series convergence (cdfdif.c:67)
constexpr double kEps = 1e-7;      // |xi node| ~ 0 test (cdfdif.c:68)
constexpr double kMinRT = 0.001;   // cdfdif.c:69
constexpr int kVMax = 5000;        // cdfdif.c:71
constexpr int kCdfBlock = 256;

// Gauss-Hermite (drift) and Gauss-Legendre (start point) 6-point rules, the
// published tables of Tuerlinckx (2004) as the reference lists them
// (cdfdif.c:78-81, including the last-digit asymmetries of the Legendre rows).
__constant__ double kGK[6] = {-2.3506049736744922818, -1.3358490740136970132,
                              -.43607741192761650950, .43607741192761650950,
                              1.3358490740136970132,  2.3506049736744922818};
__constant__ double kWGH[6] = {.45300099055088421593e-2, .15706732032114842368,
                               .72462959522439207571,    .72462959522439207571,
                               .15706732032114842368,    .45300099055088421593e-2};
__constant__ double kGZ[6] = {-.93246951420315193904, -.66120938646626381541,
                              -.23861918608319693247, .23861918608319712676,
                              .66120938646626459256,  .93246951420315160597};
__constant__ double kWG[6] = {.17132449237917049545, .36076157304813916138,
                              .46791393457269092604, .46791393457269092604,
                              .36076157304813843973, .17132449237917132812};

// Parameter-only state of one cdfdif call (cdfdif.c:61-113), in LDS.
struct CdfShared {
  double gk[6], w_gh[6], lw[6], gz[6], w_g[6];
  double term[36];  // prob terms, (i, m) row-major
  double prob;      // P(boundary) = sum_z (cdfdif.c:113)
};

// par: a, Ter, eta, z, sZ, st, nu (cdfdif_wrapper.pyx:36-42 already applied)
struct CdfPar {
  double a, Ter, eta, z, sZ, st, nu;
};

__device__ inline void cdf_setup(const CdfPar& P, CdfShared& S) {
  const int l = threadIdx.x;
  if (l < 6) {
    S.gk[l] = ((1.41421356237309505 * kGK[l]) * P.eta) + P.nu;  // cdfdif.c:86
    S.w_gh[l] = kWGH[l] / 1.772453850905515882;                 // cdfdif.c:88
    S.lw[l] = log(S.w_gh[l]);
    S.gz[l] = ((.5 * P.sZ) * kGZ[l]) + P.z;  // cdfdif.c:92
    S.w_g[l] = kWG[l];
  }
  __syncthreads();
  if (l < 36) {  // cdfdif.c:96-112, one (z node i, drift node m) term per lane
    const int i = l / 6, m = l % 6;
    const double g = S.gk[m];
    double r;
    if (fabs(g) > kEps)
      r = ((exp((-200 * S.gz[i]) * g) - 1) / (exp((-200 * P.a) * g) - 1)) * S.w_gh[m];
    else
      r = (S.gz[i] / P.a) * S.w_gh[m];
    S.term[l] = r;
  }
  __syncthreads();
  if (l == 0) {  // the reference's summation order
    double sum_z = 0;
    for (int i = 0; i < 6; ++i) {
      double sum_nu = 0;
      for (int m = 0; m < 6; ++m) sum_nu += S.term[i * 6 + m];
      sum_z += (sum_nu * S.w_g[i]) / 2;
    }
    S.prob = sum_z;
  }
  __syncthreads();
}

// Lane l's value broadcast to the wave through scalar registers (a constant l:
// two v_readlane_b32, no LDS round trip); WFPT_CDF_READLANE=0: __shfl.
#ifndef WFPT_CDF_READLANE
#define WFPT_CDF_READLANE 1
#endif
__device__ inline double bcast_lane(double v, int l) {
#if WFPT_CDF_READLANE
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
#else
  return __shfl(v, l, 64);
#endif
}

// Lane base + k's value within a group of G lanes. G = 4 with WFPT_CDF_DPP:
// a quad_perm DPP move per half (no LDS round trip), else __shfl.
#ifndef WFPT_CDF_DPP
#define WFPT_CDF_DPP 1
#endif
template <int K>
__device__ inline double quad_bcast(double v) {
  constexpr int ctrl = K | (K << 2) | (K << 4) | (K << 6);  // quad_perm [K, K, K, K]
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)b, ctrl, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), ctrl, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int G>
__device__ inline double group_bcast(double v, int base, int k) {
  if (WFPT_CDF_DPP && G == 4) {
    switch (k) {
      case 0: return quad_bcast<0>(v);
      case 1: return quad_bcast<1>(v);
      case 2: return quad_bcast<2>(v);
      default: return quad_bcast<3>(v);
    }
  }
  return __shfl(v, base + k, 64);
}

// Series convergence test shared by the three series (cdfdif.c:144-146, 177-179, 202-204).
__device__ inline bool converged(double h0, double h1, double h2) {
  return (fabs(h0 - h1) < kDelta) && (fabs(h1 - h2) < kDelta) && (h2 > 0);
}

// Per-trial quantities of cdfdif (cdfdif.c:61-69, 116-120) and its branch:
// 0 = t below the Ter window (F = 0, :213-216), 1 = beyond it (:121-149),
// 2 = inside it (:151-211).
struct CdfTrial {
  double t, Z_U, Z_L, lower_t, upper_t, p0, p1;
  int x, sg, sh, branch;
};

// Z_U / Z_L of boundary x (cdfdif.c:116-117): parameter-only, per boundary.
__device__ inline void z_bounds(int x, const CdfPar& P, double& Z_U, double& Z_L) {
  const double a = P.a, z = P.z, sZ = P.sZ;
  Z_U = (((1 - x) * z) + (x * (a - z))) + (sZ / 2);
  Z_L = (((1 - x) * z) + (x * (a - z))) - (sZ / 2);
}

__device__ inline CdfTrial cdf_prepare(double t, int x, const CdfPar& P, const CdfShared& S) {
  const double Ter = P.Ter, st = P.st;
  CdfTrial T;
  T.t = t;
  T.x = x;
  z_bounds(x, P, T.Z_U, T.Z_L);
  T.lower_t = Ter - (st / 2);
  T.sg = 2 * x - 1;  // (2*x-1)
  T.sh = 1 - 2 * x;  // (1-2*x)
  T.branch = 0;
  T.upper_t = T.p0 = T.p1 = 0.0;
  if (((t - Ter) + (st / 2)) > kMinRT) {
    T.upper_t = t < (Ter + (st / 2)) ? t : (Ter + (st / 2));
    T.p1 = (S.prob * (T.upper_t - T.lower_t)) / st;
    T.p0 = ((1 - S.prob) * (T.upper_t - T.lower_t)) / st;
    T.branch = (t > (Ter + (st / 2))) ? 1 : 2;
  }
  return T;
}

// Term (v, m) of the series beyond the window (cdfdif.c:130-143) in three
// factors. Beyond the window upper_t = Ter + st/2 for every trial, so only
// exp(dh * (t - upper_t) + lx) depends on the trial: denom, dh, lx and fact
// depend on (v, m) and the boundary x alone, and cdf_table_kernel evaluates
// them once per call with these same helpers (bit-identical terms).
__device__ inline double beyond_denom(int v, double g, double a2) {
  const double pv = ((kCPi * kCPi) * (double)(v * v)) / (100 * a2);
  return ((100 * g) * g) + pv;
}

// log(1 - exp(dh * (upper_t - lower_t))), dh = -denom/2 (cdfdif.c:141-142).
// Below -40 the exponential is < 2^-54, so 1 - e rounds to 1 and the log is 0
// exactly (in any libm): the same value without the two calls.
__device__ inline double beyond_lx(double dh, double width) {
  const double e = dh * width;
  return e < -40.0 ? 0.0 : log(1 - exp(e));
}

// fact of (v, m) on boundary x (cdfdif.c:133-140)
__device__ inline double beyond_fact(int v, int m, int x, double denom, const CdfPar& P,
                                     const CdfShared& S) {
  const double a = P.a;
  double Z_U, Z_L;
  z_bounds(x, P, Z_U, Z_L);
  const int sg = 2 * x - 1;
  const double l100 = log(100.);
  const double sifa = (kCPi * v) / a;
  const double sU = sin(sifa * Z_U), cU = cos(sifa * Z_U);
  const double sL = sin(sifa * Z_L), cL = cos(sifa * Z_L);
  const double g = S.gk[m];
  const double ld = 3 * log(denom);
  const double upp = exp(((((sg * Z_U) * g) * 100) - ld + S.lw[m]) - (2 * l100));
  const double low = exp(((((sg * Z_L) * g) * 100) - ld + S.lw[m]) - (2 * l100));
  return (upp * ((((sg * g) * sU) * 100) - (sifa * cU))) -
         (low * ((((sg * g) * sL) * 100) - (sifa * cL)));
}

// Term v of the series beyond the window, v * sum_nu, evaluated in full
// (cdf_wave_kernel's terms past the per-call table).
__device__ inline double beyond_term(int v, const CdfTrial& T, const CdfPar& P,
                                     const CdfShared& S) {
  const double a2 = P.a * P.a, t_up = T.t - T.upper_t, width = T.upper_t - T.lower_t;
  double sum_nu = 0;
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const double denom = beyond_denom(v, S.gk[m], a2);
    const double dh = -.5 * denom;
    const double fact = beyond_fact(v, m, T.x, denom, P, S);
    const double exdif = exp((dh * t_up) + beyond_lx(dh, width));
    sum_nu += fact * exdif;
  }
  return v * sum_nu;
}

__device__ inline double beyond_F(double h2, const CdfTrial& T, const CdfPar& P) {
  const double a2 = P.a * P.a;
  return ((T.p0 * (1 - T.x)) + (T.p1 * T.x)) - (((h2 * 4) * kCPi) / ((a2 * P.sZ) * P.st));  // :148
}

// Window branch, drift node m with |gk| > eps, start-point node i: the
// increment of sum_z (cdfdif.c:161-182). Term v of its series is
// (v sin(sifa zzz)) exp(-denom/2 (t - lower_t) - 2 log(denom)), where only
// t - lower_t depends on the trial: for v < kWinTerms the other factors come
// from the per-call table (window_terms, the same operations), past it they
// are computed here.
constexpr int kWinTerms = 512;
#ifndef WFPT_CDF_CHUNK
#define WFPT_CDF_CHUNK 8
#endif
constexpr int kWinChunk = WFPT_CDF_CHUNK;
static_assert(kWinTerms % kWinChunk == 0 && kVMax % kWinChunk == 0, "kWinChunk");
struct CdfWinTable {
  double vs[kWinTerms][2][6];  // v sin(sifa zzz(x, i))
  double dh[kWinTerms][6];     // -denom(v, m) / 2
  double l2[kWinTerms][6];     // 2 log(denom(v, m))
};

// The beyond-window factors for v < kBeyTerms in global memory, v fastest so
// the wave kernel's 64 lanes (64 consecutive v) read them coalesced: its
// series terms from one exp per drift node, the same operations as
// beyond_term (bit-identical terms).
constexpr int kBeyTerms = 512;
#ifndef WFPT_CDF_BEY
#define WFPT_CDF_BEY 1
#endif
struct CdfBeyTable {
  double dh[6][kBeyTerms];       // -denom(v, m) / 2
  double lx[6][kBeyTerms];       // log(1 - exp(dh * st_window))
  double fact[2][6][kBeyTerms];  // fact(v, m) per boundary x
};

// The first kWinStage rows of the window table, staged into LDS by the wave
// at its first window trial (one coalesced pass instead of a load round trip
// per chunk of terms).
constexpr int kWinStage = 64;
static_assert(kWinStage % kWinChunk == 0 && kWinStage <= kWinTerms, "kWinStage");
struct CdfWinStage {
  double vs[kWinStage][2][6];
  double dh[kWinStage][6];
  double l2[kWinStage][6];
};
__device__ inline void stage_window(const CdfWinTable* __restrict__ W, CdfWinStage& L, int lane) {
  const double* vs = &W->vs[0][0][0];
  const double* dh = &W->dh[0][0];
  const double* l2 = &W->l2[0][0];
  double* lvs = &L.vs[0][0][0];
  double* ldh = &L.dh[0][0];
  double* ll2 = &L.l2[0][0];
  // constant trip counts, so every load is issued before the first store
  static_assert(kWinStage * 6 % 64 == 0, "stage rows");
  double a[kWinStage * 12 / 64], b[kWinStage * 6 / 64], c[kWinStage * 6 / 64];
#pragma unroll
  for (int j = 0; j < kWinStage * 12 / 64; ++j) a[j] = vs[j * 64 + lane];
#pragma unroll
  for (int j = 0; j < kWinStage * 6 / 64; ++j) {
    b[j] = dh[j * 64 + lane];
    c[j] = l2[j * 64 + lane];
  }
#pragma unroll
  for (int j = 0; j < kWinStage * 12 / 64; ++j) lvs[j * 64 + lane] = a[j];
#pragma unroll
  for (int j = 0; j < kWinStage * 6 / 64; ++j) {
    ldh[j * 64 + lane] = b[j];
    ll2[j * 64 + lane] = c[j];
  }
}

__device__ inline double window_zzz(int x, int i, const CdfPar& P, const CdfShared& S) {
  const double gzi = S.gz[i];
  return ((P.a - gzi) * x) + (gzi * (1 - x));
}
__device__ inline double window_denom(int v, double g, double a2) {
  return ((g * g) * 100) + (((kCPi * v) * (kCPi * v)) / (a2 * 100));
}
__device__ inline double window_vs(int v, double zzz, double a) {
  const double sifa = (kCPi * v) / a;
  return v * sin(sifa * zzz);
}

__device__ inline double window_mi(int m, int i, const CdfTrial& T, const CdfPar& P,
                                   const CdfShared& S, const CdfWinTable* __restrict__ W,
                                   const CdfWinStage& WS) {
  const double a = P.a, a2 = a * a, st = P.st, t = T.t, lower_t = T.lower_t;
  const int x = T.x, sg = T.sg, sh = T.sh;
  const double g = S.gk[m];
  const double B = ((sh * g) * kCPi) * .01;
  const double sD = sinh(((sh * g) * a) / .01);
  const double zzz = window_zzz(x, i, P, S);
  const double ser = (((-((a * a2) / B)) * sinh(((zzz * sh) * g) / .01)) / (sD * sD)) +
                     ((((zzz * a2) / B) * cosh((((a - zzz) * sh) * g) / .01)) / sD);
  const double tl = t - lower_t;
  double h0 = 0, h1 = 0, h2 = 0;
  // kWinChunk terms at a time: their loads and exps are independent, then they
  // are added one by one with the test (terms past the stopping one are
  // computed and dropped: the same partial sums and stopping term)
  bool done = false;
  for (int v0 = 0; v0 < kVMax && !done; v0 += kWinChunk) {
    double term[kWinChunk];
    if (v0 < kWinStage) {
#pragma unroll
      for (int u = 0; u < kWinChunk; ++u) {
        const int v = v0 + u;
        term[u] = WS.vs[v][x][i] * exp((WS.dh[v][m] * tl) - WS.l2[v][m]);
      }
    } else if (v0 < kWinTerms) {
#pragma unroll
      for (int u = 0; u < kWinChunk; ++u) {
        const int v = v0 + u;
        term[u] = W->vs[v][x][i] * exp((W->dh[v][m] * tl) - W->l2[v][m]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kWinChunk; ++u) {
        const int v = v0 + u;
        const double denom = window_denom(v, g, a2);
        term[u] = window_vs(v, zzz, a) * exp(((-.5 * denom) * tl) - (2 * log(denom)));
      }
    }
#pragma unroll
    for (int u = 0; u < kWinChunk; ++u) {
      if (!done) {
        h0 = h1;
        h1 = h2;
        h2 = h1 + term[u];
        done = converged(h0, h1, h2);
      }
    }
  }
  return ((((.5 * S.w_g[i]) * (ser - (4 * h2))) * (kCPi / 100)) / (a2 * st)) *
         exp((((sg * zzz) * g) * 100));
}

// Window branch, drift node ~ 0: sum_z (cdfdif.c:187-206).
__device__ inline double window_m0(const CdfTrial& T, const CdfPar& P) {
  const double a = P.a, a2 = a * a, st = P.st, sZ = P.sZ, t = T.t, lower_t = T.lower_t;
  const double Z_U = T.Z_U, Z_L = T.Z_L;
  const double su = ((-(Z_U * Z_U)) / (12 * a2) + ((Z_U * Z_U) * Z_U) / ((12 * a) * a2)) -
                    ((((Z_U * Z_U) * Z_U) * Z_U) / ((48 * a2) * a2));
  const double sl = ((-(Z_L * Z_L)) / (12 * a2) + ((Z_L * Z_L) * Z_L) / ((12 * a) * a2)) -
                    ((((Z_L * Z_L) * Z_L) * Z_L) / ((48 * a2) * a2));
  double h0 = 0, h1 = 0, h2 = 0;
  bool done = false;  // v = 1 .. kVMax - 1 in chunks, as window_mi
  for (int v0 = 0; v0 < kVMax && !done; v0 += kWinChunk) {
    double term[kWinChunk];
#pragma unroll
    for (int u = 0; u < kWinChunk; ++u) {
      const int v = v0 + u;
      const double sifa = (kCPi * v) / a;
      const double denom = ((kCPi * v) * (kCPi * v)) / (a2 * 100);
      term[u] = ((1 / ((((((((kCPi * kCPi) * kCPi) * kCPi) * v) * v) * v) * v))) *
                 (cos(sifa * Z_L) - cos(sifa * Z_U))) *
                exp((-.5 * denom) * (t - lower_t));
    }
#pragma unroll
    for (int u = 0; u < kWinChunk; ++u) {
      if (!done && v0 + u >= 1) {
        h0 = h1;
        h1 = h2;
        h2 = h1 + term[u];
        done = converged(h0, h1, h2);
      }
    }
  }
  return (((400 * a2) * a) * ((sl - su) - h2)) / (st * sZ);
}

// cdfdif.c:218 (a NaN ends as 0 too), then the wrapper's fold and outlier mix
// (cdfdif_wrapper.pyx:48, 11-12, 51).
__device__ inline double cdf_output(double Fnew, double xi, double p_outlier, double w_outlier,
                                    const CdfShared& S) {
  double y = Fnew > kDelta ? Fnew : 0;
  const double sgn = xi > 0 ? 1.0 : (xi < 0 ? -1.0 : (xi == 0 ? 0.0 : xi));  // np.sign
  y = (1 - S.prob) + (sgn * y);
  return (y * (1 - p_outlier)) + (((xi + (1. / (2 * w_outlier))) * w_outlier) * p_outlier);
}

// Per-call tables of the series beyond the window for v < kLaneTerms, rows
// padded to kTabRow so the two boundary rows of fact fall in different LDS
// banks. Written by cdf_table_kernel, staged into LDS by dmat_cdf_kernel.
constexpr int kLaneTerms = 48;
constexpr int kTabRow = kLaneTerms + 4;
struct CdfTable {
  CdfShared S;
  double dh[6][kTabRow];       // -denom(v, m) / 2
  double lx[6][kTabRow];       // log(1 - exp(dh * st_window))
  double fact[2][6][kTabRow];  // fact(v, m) per boundary x
};

// One block per drift node m, one lane per v: the parameter-only state
// (cdf_setup) and the (v, m) factors of the beyond-window series.
constexpr int kWinVsBlocks = kWinTerms * 12 / 64, kWinDenBlocks = kWinTerms * 6 / 64;
constexpr int kBeyBlocks = kBeyTerms * 6 / 64;
constexpr int kCdfTableBlocks = 6 + kWinVsBlocks + kWinDenBlocks + kBeyBlocks;
__global__ __launch_bounds__(64) void cdf_table_kernel(CdfPar P, CdfTable* tab, CdfWinTable* W,
                                                       CdfBeyTable* B) {
  __shared__ CdfShared S;
  cdf_setup(P, S);
  if (blockIdx.x >= 6 + kWinVsBlocks + kWinDenBlocks) {  // the wave kernel's beyond table
    const int e = (blockIdx.x - (6 + kWinVsBlocks + kWinDenBlocks)) * 64 + threadIdx.x;
    const int m = e / kBeyTerms, v = e % kBeyTerms;
    const double a2 = P.a * P.a;
    const double width = (P.Ter + (P.st / 2)) - (P.Ter - (P.st / 2));  // upper_t - lower_t
    const double denom = beyond_denom(v, S.gk[m], a2);
    const double dh = -.5 * denom;
    B->dh[m][v] = dh;
    B->lx[m][v] = beyond_lx(dh, width);
    B->fact[0][m][v] = beyond_fact(v, m, 0, denom, P, S);
    B->fact[1][m][v] = beyond_fact(v, m, 1, denom, P, S);
    return;
  }
  if (blockIdx.x >= 6) {  // the window series' tables
    const double a2 = P.a * P.a;
    const int b = blockIdx.x - 6;
    if (b < kWinVsBlocks) {
      const int e = b * 64 + threadIdx.x, v = e / 12, x = (e % 12) / 6, i = e % 6;
      W->vs[v][x][i] = window_vs(v, window_zzz(x, i, P, S), P.a);
    } else {
      const int e = (b - kWinVsBlocks) * 64 + threadIdx.x, v = e / 6, m = e % 6;
      const double denom = window_denom(v, S.gk[m], a2);
      W->dh[v][m] = -.5 * denom;
      W->l2[v][m] = 2 * log(denom);
    }
    return;
  }
  const int m = blockIdx.x, v = threadIdx.x;
  if (m == 0) {
    const double* src = (const double*)&S;
    double* dst = (double*)&tab->S;
    for (int k = v; k < (int)(sizeof(CdfShared) / sizeof(double)); k += 64) dst[k] = src[k];
  }
  if (v < kLaneTerms) {
    const double a2 = P.a * P.a;
    const double width = (P.Ter + (P.st / 2)) - (P.Ter - (P.st / 2));  // upper_t - lower_t
    const double denom = beyond_denom(v, S.gk[m], a2);
    const double dh = -.5 * denom;
    tab->dh[m][v] = dh;
    tab->lx[m][v] = beyond_lx(dh, width);
    tab->fact[0][m][v] = beyond_fact(v, m, 0, denom, P, S);
    tab->fact[1][m][v] = beyond_fact(v, m, 1, denom, P, S);
  }
}

// Per-trial pass, G lanes per trial: trials below the window, and trials
// beyond it whose series converges within kLaneTerms terms, are finished
// here. Each step the G lanes of a trial evaluate G consecutive terms from the
// LDS tables (one exp per drift node), then every lane of the group adds them
// in v order with the reference's convergence test, so the partial sums —
// and the stopping term — are the reference's (cdfdif.c:128-147). The rest —
// window trials (36 series of up to 5000 terms each) and slowly converging
// series near the window edge — are appended to `defer` for cdf_wave_kernel.
template <int G>
__global__ __launch_bounds__(kCdfBlock) void dmat_cdf_kernel(const double* xs, int64_t n,
                                                             CdfPar P, const CdfTable* tab,
                                                             double p_outlier, double w_outlier,
                                                             double* out, int* defer,
                                                             int* n_defer) {
  static_assert(kLaneTerms % G == 0 && 64 % G == 0, "group size");
  __shared__ CdfTable L;
  {
    const double* src = (const double*)tab;
    double* dst = (double*)&L;
    for (int k = threadIdx.x; k < (int)(sizeof(CdfTable) / sizeof(double)); k += kCdfBlock)
      dst[k] = src[k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, j = lane % G, base = lane - j;
  const int64_t per_block = kCdfBlock / G;
  for (int64_t b = blockIdx.x; b * per_block < n; b += gridDim.x) {
    const int64_t i = b * per_block + threadIdx.x / G;
    const bool live = i < n;
    const double xi = live ? xs[i] : 0.0;
    const CdfTrial T = cdf_prepare(fabs(xi), xi > 0, P, L.S);  // boundary, cdfdif_wrapper.pyx:46
    const double t_up = T.t - T.upper_t;
    bool pend = live && T.branch == 1, conv = false;
    double h0 = 0, h1 = 0, h2 = 0;
    for (int v0 = 0; v0 < kLaneTerms && __ballot(pend); v0 += G) {
      const int v = v0 + j;
      double term = 0.0;
      if (pend) {
        double sum_nu = 0;
#pragma unroll
        for (int m = 0; m < 6; ++m)
          sum_nu += L.fact[T.x][m][v] * exp((L.dh[m][v] * t_up) + L.lx[m][v]);
        term = v * sum_nu;
      }
#pragma unroll
      for (int k = 0; k < G; ++k) {
        const double tk = G == 1 ? term : group_bcast<G>(term, base, k);
        if (pend) {
          h0 = h1;
          h1 = h2;
          h2 = h1 + tk;
          if (converged(h0, h1, h2)) {
            pend = false;
            conv = true;
          }
        }
      }
    }
    const bool deferred = live && (T.branch == 2 || (T.branch == 1 && !conv));
    if (live && !deferred && j == 0)
      out[i] = cdf_output(T.branch == 1 ? beyond_F(h2, T, P) : 0.0, xi, p_outlier, w_outlier, L.S);
    // wave-aggregated append (order irrelevant: outputs are per trial)
    const bool app = deferred && j == 0;
    const unsigned long long bal = __ballot(app);
    if (bal) {
      int at = 0;
      if (lane == 0) at = atomicAdd(n_defer, __popcll(bal));
      at = __shfl(at, 0, 64);
      if (app) defer[at + __popcll(bal & ((1ull << lane) - 1ull))] = (int)i;
    }
  }
}

// One wave per deferred trial. Beyond the window: the terms of 64
// consecutive v are computed one per lane, then accumulated in v order with
// the reference's convergence test (sequential sum, so the partial sums are
// the reference's). Inside the window: lane m*6+i runs the (m, i) series,
// lanes 36+m the drift-node-~0 series, and sum_z / sum_nu are combined in the
// reference's order.
__global__ __launch_bounds__(64) void cdf_wave_kernel(const double* xs, CdfPar P,
                                                     const CdfTable* tab,
                                                     const CdfWinTable* __restrict__ W,
                                                     const CdfBeyTable* __restrict__ B,
                                                     double p_outlier,
                                                     double w_outlier, double* out,
                                                     const int* defer, const int* n_defer) {
  const int nd = *n_defer;
  if ((int)blockIdx.x >= nd) return;
  __shared__ CdfShared S;
  __shared__ CdfWinStage WS;
  {
    const double* src = (const double*)&tab->S;
    double* dst = (double*)&S;
    for (int k = threadIdx.x; k < (int)(sizeof(CdfShared) / sizeof(double)); k += 64)
      dst[k] = src[k];
  }
  __syncthreads();
  const int lane = threadIdx.x;
  bool staged = false;
  for (int k = blockIdx.x; k < nd; k += gridDim.x) {
    const int idx = defer[k];
    const double xi = xs[idx];
    const CdfTrial T = cdf_prepare(fabs(xi), xi > 0, P, S);
    double F;
#ifdef WFPT_CDF_DEBUG
    const long long dbg_t0 = __builtin_amdgcn_s_memrealtime();
    long long dbg_t1 = dbg_t0;
    int dbg_rounds = 0;
#endif
    if (T.branch == 1) {
      // h1, h2: the last two partial sums (the reference's sequential
      // additions, cdfdif.c:128-147). Per round the 64 additions run without
      // a test between them (lane j keeps the sum after term j), then every
      // lane tests its own step at once and the first converged step ends the
      // series: the same sums and the same stopping term as one test per step.
      double h1 = 0, h2 = 0;
      bool conv = false;
      // the table's factors of the next round are loaded one round ahead, so
      // their latency overlaps this round's sequential additions
      double qf[6], qd[6], ql[6];
      const double* fx = &B->fact[T.x][0][0];
#pragma unroll
      for (int mm = 0; mm < 6; ++mm) {
        qf[mm] = fx[mm * kBeyTerms + lane];
        qd[mm] = B->dh[mm][lane];
        ql[mm] = B->lx[mm][lane];
      }
      for (int v0 = 0; v0 < kVMax && !conv; v0 += 64) {
        const int v = v0 + lane;
        double term = 0.0;
        if (WFPT_CDF_BEY && v0 < kBeyTerms) {  // wave-uniform: kBeyTerms is a multiple of 64
          double cf[6], cd[6], cx[6];
#pragma unroll
          for (int mm = 0; mm < 6; ++mm) {
            cf[mm] = qf[mm];
            cd[mm] = qd[mm];
            cx[mm] = ql[mm];
          }
          if (v0 + 64 < kBeyTerms) {
#pragma unroll
            for (int mm = 0; mm < 6; ++mm) {
              qf[mm] = fx[mm * kBeyTerms + v + 64];
              qd[mm] = B->dh[mm][v + 64];
              ql[mm] = B->lx[mm][v + 64];
            }
          }
          const double t_up = T.t - T.upper_t;
          double sum_nu = 0;
#pragma unroll
          for (int mm = 0; mm < 6; ++mm) sum_nu += cf[mm] * exp((cd[mm] * t_up) + cx[mm]);
          term = v * sum_nu;
        } else if (v < kVMax) {
          term = beyond_term(v, T, P, S);
        }
        const int m = (kVMax - v0 < 64) ? kVMax - v0 : 64;
        double h = h2, hk = 0.0;
#pragma unroll
        for (int j = 0; j < 64; ++j) {
          h = h + bcast_lane(term, j);
          hk = lane == j ? h : hk;
        }
        const double up1 = __shfl(hk, (lane + 63) & 63, 64), up2 = __shfl(hk, (lane + 62) & 63, 64);
        const double hm1 = lane >= 1 ? up1 : h2;
        const double hm2 = lane >= 2 ? up2 : (lane == 1 ? h2 : h1);
        const unsigned long long cb = __ballot(lane < m && converged(hm2, hm1, hk));
        const int last = cb ? __ffsll((long long)cb) - 1 : m - 1;
        conv = cb != 0ull;
        h1 = __shfl(hk, last > 0 ? last - 1 : 0, 64);
        if (last == 0) h1 = h2;
        h2 = __shfl(hk, last, 64);
#ifdef WFPT_CDF_DEBUG
        ++dbg_rounds;
#endif
      }
      F = beyond_F(h2, T, P);
    } else {
      if (!staged) {  // wave-uniform
        stage_window(W, WS, lane);
        __syncthreads();
        staged = true;
      }
      double val = 0.0;
      if (lane < 36) {
        const int m = lane / 6, i = lane % 6;
        if (fabs(S.gk[m]) > kEps) val = window_mi(m, i, T, P, S, W, WS);
      } else if (lane < 42) {
        if (!(fabs(S.gk[lane - 36]) > kEps)) val = window_m0(T, P);
      }
#ifdef WFPT_CDF_DEBUG
      dbg_t1 = __builtin_amdgcn_s_memrealtime();
#endif
      double sum_nu = 0;
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        double sum_z = 0;
        if (fabs(S.gk[m]) > kEps) {
#pragma unroll
          for (int i = 0; i < 6; ++i) sum_z += bcast_lane(val, m * 6 + i);
        } else {
          sum_z = bcast_lane(val, 36 + m);
        }
        sum_nu += sum_z * S.w_gh[m];
      }
      F = ((T.p0 * (1 - T.x)) + (T.p1 * T.x)) - sum_nu;  // cdfdif.c:210
    }
    if (lane == 0) out[idx] = cdf_output(F, xi, p_outlier, w_outlier, S);
#ifdef WFPT_CDF_DEBUG
    // diagnostic builds: -(rounds 1e12 + series ticks 1e6 + elapsed ticks) in
    // place of the value (100 MHz ticks from the trial's start)
    if (lane == 0)
      out[idx] = -((double)dbg_rounds * 1e12 + (double)(dbg_t1 - dbg_t0) * 1e6 +
                   (double)(__builtin_amdgcn_s_memrealtime() - dbg_t0));
#endif
  }
}

}  // namespace

// dmat_cdf_array on device x[n] (cdfdif_wrapper.pyx:16-53); *n_defer must be
// 0 (the caller clears it on the stream); tab holds kCdfTableDoubles doubles
// (the per-call tables).
// par holds the wrapper's transformed parameters (a/10, t, sv/10+1e-10,
// z*a/10, sz*a/10+1e-10, st+1e-10, v/10).
#ifndef WFPT_CDF_WAVES
#define WFPT_CDF_WAVES 4096
#endif
#ifndef WFPT_CDF_GROUP
#define WFPT_CDF_GROUP 4
#endif
// the buffer: CdfTable, then CdfWinTable at kCdfTableBeyond doubles
constexpr int kCdfTableBeyond = 1344;
static_assert(sizeof(CdfTable) <= kCdfTableBeyond * sizeof(double), "kCdfTableBeyond");
constexpr int kCdfTableWave = kCdfTableBeyond + 512 * 24;  // CdfBeyTable
static_assert(sizeof(CdfWinTable) == 512 * 24 * sizeof(double), "CdfWinTable");
static_assert(kCdfTableWave * sizeof(double) + sizeof(CdfBeyTable) <=
                  kCdfTableDoubles * sizeof(double), "kCdfTableDoubles");

void launch_dmat_cdf(const double* x, int64_t n, const double par[7], double p_outlier,
                     double w_outlier, double* out, double* tab, int* defer, int* n_defer,
                     hipStream_t s) {
  if (n <= 0) return;
  CdfPar P;
  P.a = par[0];
  P.Ter = par[1];
  P.eta = par[2];
  P.z = par[3];
  P.sZ = par[4];
  P.st = par[5];
  P.nu = par[6];
  CdfTable* T = reinterpret_cast<CdfTable*>(tab);
  CdfWinTable* W = reinterpret_cast<CdfWinTable*>(tab + kCdfTableBeyond);
  CdfBeyTable* B = reinterpret_cast<CdfBeyTable*>(tab + kCdfTableWave);
  hipLaunchKernelGGL(cdf_table_kernel, dim3(kCdfTableBlocks), dim3(64), 0, s, P, T, W, B);
  constexpr int G = WFPT_CDF_GROUP;
  const int64_t per_block = kCdfBlock / G;
  int64_t nb = (n + per_block - 1) / per_block;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(dmat_cdf_kernel<G>, dim3(nb), dim3(kCdfBlock), 0, s, x, n, P, T, p_outlier,
                     w_outlier, out, defer, n_defer);
  // one wave per deferred trial on a fixed grid (it reads the count itself)
  const int64_t gw = n < WFPT_CDF_WAVES ? n : WFPT_CDF_WAVES;
  hipLaunchKernelGGL(cdf_wave_kernel, dim3(gw), dim3(64), 0, s, x, P, T, W, B, p_outlier,
                     w_outlier, out, defer, n_defer);
}

}  // namespace wfpt
