// wfpt_device.hpp — device-side WFPT density for gfx950 (CDNA4), fp64.
//
// Restates the reference's numerics (src/pdf.pxi:28-146, src/integrate.pxi:12-206)
// for one-trial-per-lane execution:
//   * every *decision* (series branch, term count K, adaptive stop test, node
//     coordinates) is computed with the same IEEE operations in the same order
//     as the reference, so the quadrature tree is identical; a stop test
//     decided within kTieBand of its threshold, and a density that hinges on
//     subnormal rounding, send the trial to the exact path (wfpt_exact.hpp);
//   * work that depends only on the non-decision time node t (the series
//     branch and K, sqrt/log terms, sv normalisers) is hoisted out of the z
//     integral: one `TNode` per t node serves all z nodes;
//   * adaptive trees up to kTreeDepth levels per axis complete inside the
//     wave that owns the trial (engine_kernel, wfpt_kernels.hip: tree_node /
//     tree_value over the dyadic points); deeper trees continue on a
//     per-lane walk with an explicit stack (adaptive_walk).
// Compiled with -ffp-contract=off: no FMA contraction, like the x86-64 build
// of the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wfpt_amd.h"
#include "wfpt_crlibm.hpp"
#include "wfpt_exact.hpp"

#pragma clang fp contract(off)

namespace wfpt {

constexpr double kPi = 3.14159265358979323846;  // M_PI
constexpr double kPi2 = kPi * kPi;             // M_PI**2 (pdf.pxi:37, 62)

struct Params {
  double v, sv, a, z, sz, t, st, p_outlier;
};
struct Knobs {
  double err;
  int n_st, n_sz, use_adaptive;
  double simps_err, w_outlier;
};

enum Mode : int {
  kDirect = 0,   // sz = st = 0: one pdf_sv (pdf.pxi:129)
  kAdaptT = 1,   // st only, adaptive (pdf.pxi:132)
  kAdaptZ = 2,   // sz only, adaptive (pdf.pxi:139)
  kAdaptTZ = 3,  // sz and st, adaptive 2-D (pdf.pxi:144)
  kFixedT = 4,   // fixed Simpson variants (pdf.pxi:134, 141, 146)
  kFixedZ = 5,
  kFixedTZ = 6,
  kRuntime = 7,  // per-trial parameters: mode decided per lane
};

// Host+device: mode after full_pdf's st/sz < 1e-3 zeroing (pdf.pxi:122-146).
__host__ __device__ inline int select_mode(double sz, double st, int use_adaptive) {
  const bool zst = !(st >= 1e-3), zsz = !(sz >= 1e-3);
  if (zsz) {
    if (zst) return kDirect;
    return use_adaptive > 0 ? kAdaptT : kFixedT;
  }
  if (zst) return use_adaptive ? kAdaptZ : kFixedZ;
  return use_adaptive ? kAdaptTZ : kFixedTZ;
}

// ---------------------------------------------------------------------------
// Routing of trials whose value hinges on last-bit rounding (wfpt_exact.hpp).
//
// kExactBelow: a trial density below it (or zero, negative, NaN) is recomputed
// on the exact path: there intermediate values can be subnormal, where one
// rounding is up to 1e-5 relative, and a zero / negative / NaN outcome is a
// decision, not a rounding.
// kTieBand: an adaptive stop test |S2 - S| <= 15 err decided within this
// relative band of its threshold sends the trial to the exact path (the fast
// path's node values carry ~1e-14 relative error; the band is 1000x wider).
constexpr double kExactBelow = 1e-290;
constexpr double kTieBand = 1e-11;

// A settled density 0 < p <= kExactBelow (its tree decided with the
// reference's operations, no near-tie flagged) when the call's outlier mixture
// adds w_outlier p_outlier >= kMixAbsorb: any value within the fast path's
// error of p (< 1e-289) satisfies p' (1 - p_outlier) < w_outlier p_outlier
// 2^-54, so the reference's mixture p' (1 - p_outlier) + w_outlier p_outlier
// (wfpt.pyx:44, :70) rounds to w_outlier p_outlier exactly and the trial's
// output does not depend on p: it is settled as 0 (the same mixture bits)
// instead of being recomputed on the exact path. Without the mixture
// (full_pdf, p_outlier = 0) such a density still takes the exact path.
constexpr double kMixAbsorb = 1e-250;
#ifndef WFPT_TINY_MIX
#define WFPT_TINY_MIX 1
#endif
__host__ __device__ inline bool tiny_absorbed(double p, double p_outlier, double w_outlier) {
  return WFPT_TINY_MIX && p > 0.0 && p <= kExactBelow && w_outlier * p_outlier >= kMixAbsorb;
}

// UNROLL: the t-node loop fully unrolled (node positions, q hints and
// accumulators without per-node selects or loop-carried copies; 5x the code).
// The lean pass unrolls its boundary-uniform call site (WFPT_LEAN_UNROLL):
// 127 VGPRs = 4 waves/SIMD instead of 168 = 3, and C3's level 0 -13%.
#ifndef WFPT_LEAN_UNROLL
#define WFPT_LEAN_UNROLL 1
#endif
// WFPT_FAST_L0_UNROLL: the same for the per-node and per-trial-parameter
// level-0 passes (fast_level0: no scratch, node kernel -18%); the engine's
// level 0 keeps the loop (measured: the unrolled copy slows its stress set 4%)
#ifndef WFPT_FAST_L0_UNROLL
#define WFPT_FAST_L0_UNROLL 1
#endif
enum Flag : int {
  kFlagDepth = 1,     // refinement deeper than the stack (WFPT_MAX_DEPTH)
  kFlagBudget = 2,    // more than kEvalBudget pdf_sv evaluations in one trial
  kFlagExact = 4,     // recompute on the exact path
  kFlagFallback = 8,  // tree deeper than the breadth-first levels: per-lane walk
};
constexpr int kFlagErrors = kFlagDepth | kFlagBudget;


// ---------------------------------------------------------------------------
// Per-t-node quantities of ftt_01w / pdf_sv that do not depend on w (= z).
//
// Decisions (pos, small/large branch, K) are computed with the reference's
// exact operations. Values use cheaper equivalent forms whose rounding differs
// by a few ulp (trials whose value hinges on last-bit rounding are sent to the
// exact path, wfpt_exact.hpp):
//   * exp(-k^2 pi^2 tt/2) = q^(k^2), q = exp(-pi^2 tt/2), by two products per k;
//   * sin(k pi w) by the Chebyshev recurrence from one sincospi(w);
//   * exp(log p + c) = p * exp(c)  (overflow of exp(c) falls back to the
//     literal form; p < 0 keeps the reference's NaN from log);
//   * divisions by per-node constants become multiplications by reciprocals.
constexpr double kDblMin = 2.2250738585072014e-308;

// sin(pi w) and cos(pi w) for w in [0, 1] (the only range full_pdf produces:
// validity + flip keep every z node in [0, 1]). Exact reduction t = 2w,
// n = rint(t), f = t - n in [-1/2, 1/2], x = f pi/2 in [-pi/4, pi/4]; Taylor
// polynomials to x^17 / x^18 (truncation < 1e-19) by FMA Horner: <= 1.1 ulp
// relative (checked against 120-bit arithmetic). 30 fp64 ops instead of OCML's
// general-range sincospi (127). w == 1 is seeded with the reference's own
// sin(fl(pi)) = 1.2246e-16 so the z = 1 edge keeps its nonzero value.
// One Horner step of sincospi01: on the device a three-operand v_fma_f64 with
// the coefficient in SGPRs (see horner below: fma() costs a v_mov_b64 per
// step there), on the host fma() (the host builds the sine tables from the same
// correctly rounded operations, so both produce the same bits).
__host__ __device__ inline double horner_hd(double p, double r, double c) {
#if defined(__HIP_DEVICE_COMPILE__) && (!defined(WFPT_HORNER_ASM) || WFPT_HORNER_ASM)
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(p), "v"(r), "s"(c));
  return d;
#else
  return fma(p, r, c);
#endif
}

__host__ __device__ inline void sincospi01(double w, double& s, double& c) {
  const double t = 2.0 * w;
  const double n = rint(t);
  const double f = t - n;
  const double x = f * 1.5707963267948966;  // pi/2
  const double x2 = x * x;
  double ps = 0x1.952c77030ad4ap-49;
  ps = horner_hd(ps, x2, -0x1.ae7f3e733b81fp-41);
  ps = horner_hd(ps, x2, 0x1.6124613a86d09p-33);
  ps = horner_hd(ps, x2, -0x1.ae64567f544e4p-26);
  ps = horner_hd(ps, x2, 0x1.71de3a556c734p-19);
  ps = horner_hd(ps, x2, -0x1.a01a01a01a01ap-13);
  ps = horner_hd(ps, x2, 0x1.1111111111111p-7);
  ps = horner_hd(ps, x2, -0x1.5555555555555p-3);
  const double sx = fma(x * x2, ps, x);
  double pc = -0x1.6827863b97d97p-53;
  pc = horner_hd(pc, x2, 0x1.ae7f3e733b81fp-45);
  pc = horner_hd(pc, x2, -0x1.93974a8c07c9dp-37);
  pc = horner_hd(pc, x2, 0x1.1eed8eff8d898p-29);
  pc = horner_hd(pc, x2, -0x1.27e4fb7789f5cp-22);
  pc = horner_hd(pc, x2, 0x1.a01a01a01a01ap-16);
  pc = horner_hd(pc, x2, -0x1.6c16c16c16c17p-10);
  pc = horner_hd(pc, x2, 0x1.5555555555555p-5);
  const double cx = fma(x2 * x2, pc, fma(-0.5, x2, 1.0));
  const bool q1 = n == 1.0, q2 = n == 2.0;
  s = q1 ? cx : (q2 ? -sx : sx);
  c = q1 ? -sx : (q2 ? -cx : cx);
  if (w == 1.0) {
    s = 1.2246467991473532e-16;  // sin(M_PI) in double, as the reference computes
    c = -1.0;
  }
}

constexpr double kInvSqrt2Pi = 0.398942280401432677939946059934;  // 1 / sqrt(2 pi)

struct TNode {
  double xx;    // x - t_node: the `x` argument of pdf_sv
  double tt;    // xx / a^2 (pdf.pxi:98)
  double m;     // small-t: -1/(2 tt) exponent multiplier; large-t: q = exp(-pi^2 tt / 2)
  double q2;    // large-t: q^2
  double rn;    // small-t: 1 / sqrt(2 pi tt^3)  (pdf.pxi:57)
  double sc;    // 1/a^2, times 1/sqrt(sv^2 xx + 1) when sv > 0
  double cden;  // sv: 1 / (2 sv^2 xx + 2)
  double vvx;   // v^2 * xx
  int K;        // number of series terms (pdf.pxi:52, 60)
  int small;    // 1 => small-time series
  int pos;      // xx > 0 (else density 0, pdf.pxi:92)
  int amb;      // the decision sits within 1e-12 of a threshold: exact path
};

// Series branch and term count of one t node (pdf.pxi:36-60): small-time
// series iff ks < kl, K = ceil(min). kl and ks feed ONLY these two decisions.
struct Decision {
  int small, K, amb;
};

// fp32 estimate of the decision (~1e-7 relative). Returns false — the caller
// must then run the reference's fp64 operations — when any decision is within
// 1e-5 (relative) of flipping or an fp32 argument is out of range. args_out:
// the small-time log argument 2 sqrt(2 pi tt) err (for the monotonicity test
// of shared decisions).
// Hardware fp32 log / sqrt / reciprocal for the estimate (v_log_f32,
// v_sqrt_f32, v_rcp_f32: ~1 ulp on the normal range these arguments stay in,
// i.e. relative errors ~1e-7 in kl / ks, 100x inside the 1e-5 guard band).
__device__ inline float log32(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }
__device__ inline float sqrt32(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ inline float rcp32(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ inline bool decide32(double tt, double err, Decision& D, float& args_out) {
  args_out = 2.0f;
  if (!(tt > 1e-30 && tt < 1e30 && err > 1e-30 && err < 1e30)) return false;
  const float ttf = (float)tt, errf = (float)err;
  const float sqtf = sqrt32(ttf);
  const float ipsf = rcp32((float)kPi * sqtf);
  const float argl = ((float)kPi * ttf) * errf;
  const float args = (2.0f * sqrt32((2.0f * (float)kPi) * ttf)) * errf;
  args_out = args;
  const bool use_l = argl < 1.0f;
  const bool use_s = args < 1.0f;
  const float tol = 1e-5f;
  // |dL| <~ 1e-7 |L| from fp32 rounding + the hardware log; the relative error
  // it induces in kl/ks is <= |dL| / (2|L|) ~ 1e-7, 100x inside tol (and |L| >=
  // 0.1 is still required below, as for the correctly rounded logf).
  const bool rng = (use_l && !(argl > 1e-30f)) || (use_s && !(args > 1e-30f));
  if (rng) return false;
  const float Ll = use_l ? log32(argl) : -1.0f;
  const float Ls = use_s ? log32(args) : -1.0f;
  float klf = use_l ? sqrt32((-2.0f * Ll) * rcp32((float)kPi2 * ttf)) : ipsf;
  float ksf = use_s ? 2.0f + sqrt32((-2.0f * ttf) * Ls) : 2.0f;
  const float b2 = sqtf + 1.0f;
  const bool amb_t = fabsf(argl - 1.0f) <= tol || fabsf(args - 1.0f) <= tol;
  const bool amb_l = use_l && fabsf(klf - ipsf) <= tol * klf;
  const bool amb_s = use_s && fabsf(ksf - b2) <= tol * ksf;
  if (use_l) klf = (klf < ipsf) ? ipsf : klf;
  if (use_s) ksf = (ksf < b2) ? b2 : ksf;
  const float kk = (ksf < klf) ? ksf : klf;
  const bool amb_b = fabsf(ksf - klf) <= tol * klf;
  const bool amb_k = fabsf(kk - rintf(kk)) <= tol * kk;
  if (Ll > -0.1f || Ls > -0.1f || amb_t || amb_l || amb_s || amb_b || amb_k) return false;
  if (!(kk < 1e6f)) return false;  // huge / non-finite K: decide64's conversion
  D.small = ksf < klf;
  D.K = (int)ceilf(kk);
  D.amb = 0;
  return true;
}

// The reference's fp64 operations (pdf.pxi:36-60), reached when the fp32
// estimate is within 1e-5 of a threshold. OCML's log differs from glibc's by
// <= 1 ulp, so a decision within 1e-12 (relative) of a threshold is marked
// ambiguous and the trial goes to the exact path (glibc-equal log).
__device__ inline Decision decide64(double tt, double err) {
  double kl, ks;
  const double sqt = sqrt(tt);
  const double inv_pi_sqt = 1. / (kPi * sqt);
  const double arg_l = (kPi * tt) * err;
  const double arg_s = (2.0 * sqrt((2.0 * kPi) * tt)) * err;
  if (arg_l < 1.0) {
    kl = sqrt((-2.0 * log(arg_l)) / (kPi2 * tt));
    kl = (kl < inv_pi_sqt) ? inv_pi_sqt : kl;
  } else {
    kl = inv_pi_sqt;
  }
  if (arg_s < 1.0) {
    ks = 2.0 + sqrt((-2.0 * tt) * log(arg_s));
    const double b = sqt + 1.0;
    ks = (ks < b) ? b : ks;
  } else {
    ks = 2.0;
  }
  Decision D;
  D.small = ks < kl;
  const double kk = D.small ? ks : kl;
  D.K = wfpt_x::ref_int(ceil(kk));  // the reference's x86 conversion
  constexpr double tol = 1e-12;
  D.amb = fabs(arg_l - 1.0) <= tol || fabs(arg_s - 1.0) <= tol || fabs(ks - kl) <= tol * kl ||
          fabs(kk - rint(kk)) <= tol * kk;
  return D;
}

// qhint >= 0: exp(-pi^2 tt / 2) of this node computed by the caller (a
// recurrence over the t grid); < 0: computed here. has_known: `known` is the
// node's decision, established by the caller (shared over a trial's t grid).
// ia2: 1 / a^2 of the call, computed once by the caller. tt comes from a
// product: it feeds the fp32 decision estimate (1e-5 guard band) and values
// only; the fp64 decision, reached near a threshold, divides exactly as
// pdf.pxi:98.
__device__ inline TNode tnode_setup_r(double xx, double v, double sv, double a, double ia2,
                                      double err, double qhint = -1.0, bool has_known = false,
                                      Decision known = Decision{0, 0, 0}) {
  TNode T;
  T.xx = xx;
  T.pos = xx > 0;
  T.tt = 0.0;
  T.m = 0.0;
  T.q2 = 0.0;
  T.rn = 0.0;
  T.sc = 0.0;
  T.cden = 0.0;
  T.vvx = 0.0;
  T.K = 0;
  T.small = 0;
  T.amb = 0;
  if (!T.pos) return T;
  const double a2 = a * a;
  const double tt = xx * ia2;
  T.tt = tt;
  Decision D;
  float args;
  if (has_known) D = known;
  else if (!decide32(tt, err, D, args)) D = decide64(xx / a2, err);
  T.amb = D.amb;
  if (D.small) {
    T.small = 1;
    T.K = D.K;
    // values only: 1/sqrt(2 pi tt^3) and -1/(2 tt) from one rsqrt
    const double r = rsqrt(tt), r2 = r * r;
    T.rn = kInvSqrt2Pi * (r2 * r);
    T.m = -0.5 * r2;
  } else {
    T.small = 0;
    T.K = D.K;
    T.m = qhint >= 0.0 ? qhint : exp((-kPi2 * tt) / 2.0);
    T.q2 = T.m * T.m;
  }
  // values only: 1/(2u) and 1/(a^2 sqrt(u)), u = sv^2 xx + 1, from one rsqrt
  T.sc = ia2;
  if (sv != 0) {
    const double r = rsqrt(((sv * sv) * xx) + 1.0);
    T.cden = (0.5 * r) * r;
    T.sc = T.sc * r;
  }
  T.vvx = (v * v) * xx;
  return T;
}
__device__ inline TNode tnode_setup(double xx, double v, double sv, double a, double err,
                                    double qhint = -1.0, bool has_known = false,
                                    Decision known = Decision{0, 0, 0}) {
  return tnode_setup_r(xx, v, sv, a, 1.0 / (a * a), err, qhint, has_known, known);
}

// Series accumulation c + a b. Values only (never a decision input: the series
// choice, K and the Simpson stop tests use the reference's operations, and a
// stop test within kTieBand = 1e-11 of its threshold is re-decided on the exact
// path), so one fused rounding instead of two is within the few-ulp value
// error the recurrences already carry. WFPT_SERIES_FMA=0 restores mul + add.
#ifndef WFPT_SERIES_FMA
#define WFPT_SERIES_FMA 1
#endif
__host__ __device__ inline double madd(double a, double b, double c) {
#if WFPT_SERIES_FMA
  return fma(a, b, c);
#else
  return c + a * b;
#endif
}
// a b - c (the Chebyshev step 2cos(pi w) sin(k pi w) - sin((k-1) pi w))
__host__ __device__ inline double msub(double a, double b, double c) {
#if WFPT_SERIES_FMA
  return fma(a, b, -c);
#else
  return a * b - c;
#endif
}

// Exponentials of the single-node path (tnode_ftt / tnode_pdf_sv; defined
// after exp_val): values only, the fitted exp with its argument clamped to
// [-1100, 1100] (exp_val would make NaN of +-inf; the clamp keeps 0 / inf and
// NaN). WFPT_NODE_FAST_EXP=0: OCML's exp.
#ifndef WFPT_NODE_FAST_EXP
#define WFPT_NODE_FAST_EXP 1
#endif
__device__ inline double exp_node(double x);

// f(t|0,1,w) from a prepared t node (pdf.pxi:49-65).
__device__ inline double tnode_ftt(const TNode& T, double w) {
  double p = 0.0;
  const int K = T.K;
  if (T.small) {
    const int lower = (int)(-floor((K - 1) / 2.));
    const int upper = (int)ceil((K - 1) / 2.);
    for (int k = lower; k <= upper; ++k) {
      const double wk = w + (double)(2 * k);
      p = madd(wk, exp_node((wk * wk) * T.m), p);
    }
    p = p * T.rn;
  } else {
    double s1, c1;
    sincospi01(w, s1, c1);
    const double tc = c1 + c1;
    double sk = s1, skm1 = 0.0;          // sin(k pi w), sin((k-1) pi w)
    double e = T.m, r = T.m * T.q2;      // q^(k^2), q^(2k+1)
    if (K >= 1) p = e * s1;
    for (int k = 2; k <= K; ++k) {
      const double sn = msub(tc, sk, skm1);
      skm1 = sk;
      sk = sn;
      e = e * r;
      r = r * T.q2;
      p = madd((double)k * e, sk, p);
    }
    p = p * kPi;
  }
  return p;
}

// pdf_sv(xx, v, sv, a, w, err) (pdf.pxi:74-102) from a prepared t node.
__device__ inline double tnode_pdf_sv(const TNode& T, double w, double v, double sv, double a) {
  if (!T.pos) return 0.0;
  const double p = tnode_ftt(T, w);
  if (sv == 0) {
    const double ex = exp_node((((-v) * a) * w) - (T.vvx * 0.5));
    return (p * ex) * T.sc;
  }
  if (p < 0) return __builtin_nan("");  // log(p < 0) in the reference
  const double azsv = (a * w) * sv;
  const double c = (((azsv * azsv) - (((2.0 * a) * v) * w)) - T.vvx) * T.cden;
  const double ec = exp_node(c);
  const double r = (p * ec) * T.sc;
  if (__builtin_isinf(ec))  // exp(c) overflow: the literal form
    return (exp(log(p) + (((azsv * azsv) - (((2.0 * a) * v) * w)) - T.vvx) /
                             (((2.0 * (sv * sv)) * T.xx) + 2.0)) /
            sqrt(((sv * sv) * T.xx) + 1.0)) /
           (a * a);
  return r;
}

__device__ inline double pdf_sv(double xx, double v, double sv, double a, double w, double err,
                                int& flags) {
  const TNode T = tnode_setup(xx, v, sv, a, err);
  if (T.amb) flags |= kFlagExact;
  return tnode_pdf_sv(T, w, v, sv, a);
}


// ---------------------------------------------------------------------------
// The reference's stop test of adaptiveSimpsonsAux (integrate.pxi:105 / 170):
// true = refine. Marks kFlagExact when the test is decided inside kTieBand.
__host__ __device__ inline bool simpson_refine(double S, double S2, double err, int bottom,
                                               int& flags) {
  if (bottom <= 0) return false;
  const double d = fabs(S2 - S), thr = 15 * err;
  if (fabs(d - thr) <= kTieBand * ((fabs(S) + fabs(S2)) + thr)) flags |= kFlagExact;
  return !(d <= thr);
}

// ---------------------------------------------------------------------------
// Adaptive Simpson (integrate.pxi:72-141, 143-206) as an iterative walk.
struct Frame {
  double lb, ub, S, fb, fe, fm, err, left, hs;
};

// Tie resolution inside a per-lane walk. A stop test decided within kTieBand
// is re-decided from the interval's 5 points evaluated on the exact path
// (literal expressions, glibc-equal libm): the reference's own S and S2, so
// only that decision pays exact evaluations (deep trees run ~1e5 tests per
// trial, where whole-trial exact recomputation would dominate). NoResolve
// instead abandons the trial (kFlagExact: the caller recomputes it exactly).
struct NoResolve {
  static constexpr bool kResolves = false;
  __device__ bool operator()(double, double, double, bool, double, int) const { return false; }
};
template <class GX>
struct XResolve {
  static constexpr bool kResolves = true;
  GX gx;  // exact f(u), the reference's integrand value (divided by its width)
  // [lb, ub]: the interval; its S came from (hs / 6) (root prologue) or
  // (hs / 12) (a parent's Sleft / Sright, hs = the parent's width), each over
  // (f(lb) + 4 f(c)) + f(ub) (integrate.pxi:133-134, 105-107).
  __device__ bool operator()(double lb, double ub, double hs, bool root, double err,
                             int bottom) const {
    const double c = (ub + lb) / 2.;
    const double d = (lb + c) / 2., e = (c + ub) / 2.;
    const double fb = gx(lb), fd = gx(d), fm = gx(c), fe = gx(e), fu = gx(ub);
    const double S = root ? (hs / 6) * ((fb + (4 * fm)) + fu) : (hs / 12) * ((fb + (4 * fm)) + fu);
    const double h = ub - lb;
    const double S2 = ((h / 12) * ((fb + (4 * fd)) + fm)) + ((h / 12) * ((fm + (4 * fe)) + fu));
    return !(bottom <= 0 || fabs(S2 - S) <= 15 * err);
  }
};
template <class GX>
__device__ inline XResolve<GX> make_xresolve(GX gx) {
  return XResolve<GX>{gx};
}

// Depth <= N frames held in registers: every access is a compile-time index
// after unrolling, so the array is scalarised (no scratch).
template <int N>
struct RegStack {
  static constexpr int kCap = N;
  Frame f[N];
  __device__ inline Frame get(int i) const {
    Frame r = f[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
      if (i == k) r = f[k];
    return r;
  }
  __device__ inline double left(int i) const {
    double r = f[0].left;
#pragma unroll
    for (int k = 1; k < N; ++k)
      if (i == k) r = f[k].left;
    return r;
  }
  __device__ inline void set(int i, const Frame& x) {
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (i == k) f[k] = x;
  }
  __device__ inline void set_left(int i, double v) {
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (i == k) f[k].left = v;
  }
};

// Arbitrary depth (up to N): plain private array (scratch memory).
template <int N>
struct MemStack {
  static constexpr int kCap = N;
  Frame f[N];
  __device__ inline Frame get(int i) const { return f[i]; }
  __device__ inline double left(int i) const { return f[i].left; }
  __device__ inline void set(int i, const Frame& x) { f[i] = x; }
  __device__ inline void set_left(int i, double v) { f[i].left = v; }
};

constexpr long long kEvalBudget = 1ll << 24;

// Integrates g over [lb0, ub0] exactly like adaptiveSimpsons_1D/_2D followed by
// adaptiveSimpsonsAux(_2D): g(c) must already include the division by ZT (or
// st). Every lane walks its own tree; each loop trip evaluates g at the 3
// prologue nodes or the 2 new nodes of one interval from ONE call site. A
// near-tie stop test is re-decided by `resolve` (XResolve) or abandons the
// trial (NoResolve); depth past the stack or the evaluation budget abandon it
// too (flags set, NaN returned): no input keeps a wave busy without bound.
template <class Stack, class G, class R = NoResolve>
__device__ inline double adaptive_walk(G&& g, double lb0, double ub0, double err0, int depth,
                                       int& flags, const long long& ne, const R& resolve = R()) {
  Stack stk;
  double lb = lb0, ub = ub0, err = err0;
  double S = 0.0, fb = 0.0, fe = 0.0, fm = 0.0;
  double hs = 0.0;    // width the current S was computed with
  bool sroot = true;  // S from the prologue (hs / 6) rather than a parent (hs / 12)
  bool init = true;
  int bottom = depth, sp = 0;
  unsigned right_mask = 0u;  // bit i: frame i has finished its left child
  double result = 0.0;
  for (;;) {
    const double c = (ub + lb) / 2.;
    const double p0 = init ? lb : (lb + c) / 2.;
    const double p1 = init ? ub : (c + ub) / 2.;
    const int n = init ? 3 : 2;
    double y0 = 0.0, y1 = 0.0, y2 = 0.0;
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
      const double p = (i == 0) ? p0 : ((i == 1) ? p1 : c);
      const double y = g(p);
      if (i == 0) y0 = y;
      else if (i == 1) y1 = y;
      else y2 = y;
    }
    if (ne > kEvalBudget) flags |= kFlagBudget;
    if (flags & (kFlagErrors | kFlagExact)) {
      result = __builtin_nan("");
      break;
    }
    const double h = ub - lb;
    if (init) {  // adaptiveSimpsons_1D / _2D prologue
      fb = y0;
      fe = y1;
      fm = y2;
      S = (h / 6) * ((fb + (4 * fm)) + fe);
      hs = h;
      sroot = true;
      init = false;
      continue;
    }
    // adaptiveSimpsonsAux body (integrate.pxi:105-112 / 170-178)
    const double fd = y0, fee = y1;
    const double Sl = (h / 12) * ((fb + (4 * fd)) + fm);
    const double Sr = (h / 12) * ((fm + (4 * fee)) + fe);
    const double S2 = Sl + Sr;
    bool refine = simpson_refine(S, S2, err, bottom, flags);
    if (flags & kFlagExact) {
      if (!R::kResolves) {
        result = __builtin_nan("");
        break;
      }
      flags &= ~kFlagExact;
      refine = resolve(lb, ub, hs, sroot, err, bottom);
    }
    if (refine && sp >= Stack::kCap) {
      flags |= kFlagDepth;
      result = __builtin_nan("");
      break;
    }
    if (refine) {
      Frame fr;
      fr.lb = c;
      fr.ub = ub;
      fr.S = Sr;
      fr.fb = fm;
      fr.fe = fe;
      fr.fm = fee;
      fr.err = err / 2;
      fr.left = 0.0;
      fr.hs = h;
      stk.set(sp, fr);
      ++sp;
      ub = c;
      err = err / 2;
      S = Sl;
      hs = h;
      sroot = false;
      fe = fm;
      fm = fd;
      bottom -= 1;
      continue;
    }
    double val = S2 + (S2 - S) / 15;
    bool done = false;
    for (;;) {  // return up the tree: left + right in reference order
      if (sp == 0) {
        result = val;
        done = true;
        break;
      }
      const int top = sp - 1;
      if (!((right_mask >> top) & 1u)) {
        const Frame fr = stk.get(top);
        stk.set_left(top, val);
        right_mask |= (1u << top);
        lb = fr.lb;
        ub = fr.ub;
        S = fr.S;
        fb = fr.fb;
        fe = fr.fe;
        fm = fr.fm;
        err = fr.err;
        hs = fr.hs;
        sroot = false;
        bottom = depth - sp;
        break;
      }
      val = stk.left(top) + val;
      right_mask &= ~(1u << top);
      --sp;
    }
    if (done) break;
  }
  return result;
}

// Fixed composite Simpson, integrate.pxi:12-45. Returns the integral; the
// reference leaves `y` uninitialised when n == 0 (0 here).
__device__ inline double simpson_1d(double x, double v, double sv, double a, double z, double t,
                                    double err, double lb_z, double ub_z, int n_sz, double lb_t,
                                    double ub_t, int n_st, long long& ne, int& flags) {
  double ht, hz;
  const int n = (n_st < n_sz) ? n_sz : n_st;
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
  ++ne;
  double S = pdf_sv(x - lb_t, v, sv, a, lb_z, err, flags);
  double y = 0.0;
  for (int i = 1; i <= n; ++i) {
    const double z_tag = lb_z + hz * i;
    const double t_tag = lb_t + ht * i;
    ++ne;
    y = pdf_sv(x - t_tag, v, sv, a, z_tag, err, flags);
    if (i & 1) S += (4 * y);
    else S += (2 * y);
  }
  S = S - y;
  S = S / ((ub_t - lb_t) + (ub_z - lb_z));
  return ((ht + hz) * S) / 3;
}

__device__ inline double simpson_2d(double x, double v, double sv, double a, double z, double t,
                                    double err, double lb_z, double ub_z, int n_sz, double lb_t,
                                    double ub_t, int n_st, long long& ne, int& flags) {
  const double ht = (ub_t - lb_t) / n_st;
  double S = simpson_1d(x, v, sv, a, z, lb_t, err, lb_z, ub_z, n_sz, 0, 0, 0, ne, flags);
  double y = 0.0;
  for (int i_t = 1; i_t <= n_st; ++i_t) {
    const double t_tag = lb_t + ht * i_t;
    y = simpson_1d(x, v, sv, a, z, t_tag, err, lb_z, ub_z, n_sz, 0, 0, 0, ne, flags);
    if (i_t & 1) S += (4 * y);
    else S += (2 * y);
  }
  S = S - y;
  S = S / (ub_t - lb_t);
  return (ht * S) / 3;
}

// full_pdf's prologue (pdf.pxi:111-125): validity, boundary flip, |x|, the
// st / sz < 1e-3 zeroing. valid == 0: density 0 (pdf.pxi:111-113).
struct Trial {
  double x, v, z, sz, st;
  int valid;
};

__device__ inline Trial trial_setup(double x, const Params& P) {
  Trial T;
  double v = P.v, z = P.z, st = P.st, sz = P.sz;
  const double a = P.a, sv = P.sv, t = P.t;
  T.valid = !((z < 0) || (z > 1) || (a < 0) || (t < 0) || (st < 0) || (sv < 0) || (sz < 0) ||
              (sz > 1) || ((fabs(x) - (t - st / 2.)) < 0) || (z + sz / 2. > 1) ||
              (z - sz / 2. < 0) || (t - st / 2. < 0));
  if (x > 0) {
    v = -v;
    z = 1. - z;
  }
  T.x = fabs(x);
  if (st < 1e-3) st = 0;
  if (sz < 1e-3) sz = 0;
  T.v = v;
  T.z = z;
  T.st = st;
  T.sz = sz;
  return T;
}

// trial_setup for a trial whose boundary is known to the caller (flip ==
// (x > 0)): the same values, but v and z come from `flip` alone, so inside a
// pass over one boundary (flip wave-uniform) they are wave-uniform too.
__device__ inline Trial trial_setup_b(double x, const Params& P, bool flip) {
  Trial T;
  const double a = P.a, sv = P.sv, t = P.t, st0 = P.st, sz0 = P.sz;
  T.valid = !((P.z < 0) || (P.z > 1) || (a < 0) || (t < 0) || (st0 < 0) || (sv < 0) ||
              (sz0 < 0) || (sz0 > 1) || ((fabs(x) - (t - st0 / 2.)) < 0) ||
              (P.z + sz0 / 2. > 1) || (P.z - sz0 / 2. < 0) || (t - st0 / 2. < 0));
  T.v = flip ? -P.v : P.v;
  T.z = flip ? 1. - P.z : P.z;
  T.x = fabs(x);
  T.st = (st0 < 1e-3) ? 0.0 : st0;
  T.sz = (sz0 < 1e-3) ? 0.0 : sz0;
  return T;
}

// full_pdf (pdf.pxi:104-146) for one trial: the general per-lane walk (the
// fallback for trees deeper than the breadth-first levels, fixed Simpson,
// per-trial parameters). MODE is the integration family (kRuntime: per lane).
template <int MODE, class Stack>
__device__ inline double full_pdf(double x0, const Params& P, const Knobs& K, long long& ne,
                                  int& flags) {
  const Trial tr = trial_setup(x0, P);
  if (!tr.valid) return 0.0;
  const double a = P.a, sv = P.sv, t = P.t;
  const double x = tr.x, v = tr.v, z = tr.z, st = tr.st, sz = tr.sz;
  const int mode = (MODE == kRuntime) ? select_mode(sz, st, K.use_adaptive) : MODE;
  const double err = K.err;

  if (mode == kDirect) {
    ++ne;
    return pdf_sv(x - t, v, sv, a, z, err, flags);
  }
  if (mode == kAdaptZ) {
    // adaptiveSimpsons_1D over z at fixed t: one t node for every evaluation
    const double lb_z = z - sz / 2., ub_z = z + sz / 2.;
    const double iZT = 1.0 / (ub_z - lb_z);
    const TNode T = tnode_setup(x - t, v, sv, a, err);
    if (T.amb) flags |= kFlagExact;
    auto g = [&](double zc) -> double {
      ++ne;
      return tnode_pdf_sv(T, zc, v, sv, a) * iZT;
    };
    const double ZT = ub_z - lb_z;
    auto rz = make_xresolve([=](double zc) { return wfpt_x::pdf_sv(x - t, v, sv, a, zc, err) / ZT; });
    return adaptive_walk<Stack>(g, lb_z, ub_z, K.simps_err, K.n_sz, flags, ne, rz);
  }
  if (mode == kAdaptT) {
    const double lb_t = t - st / 2., ub_t = t + st / 2.;
    const double iZT = 1.0 / (ub_t - lb_t);
    auto g = [&](double tc) -> double {
      ++ne;
      return pdf_sv(x - tc, v, sv, a, z, err, flags) * iZT;
    };
    const double ZT = ub_t - lb_t;
    auto rt = make_xresolve([=](double tc) { return wfpt_x::pdf_sv(x - tc, v, sv, a, z, err) / ZT; });
    return adaptive_walk<Stack>(g, lb_t, ub_t, K.simps_err, K.n_st, flags, ne, rt);
  }
  if (mode == kAdaptTZ) {
    const double lb_z = z - sz / 2., ub_z = z + sz / 2.;
    const double lb_t = t - st / 2., ub_t = t + st / 2.;
    const double iZT = 1.0 / (ub_z - lb_z), istw = 1.0 / (ub_t - lb_t);
    const double ZT = ub_z - lb_z, stw = ub_t - lb_t;
    const double se = K.simps_err;
    const int nsz = K.n_sz;
    auto outer = [&](double tc) -> double {
      const TNode T = tnode_setup(x - tc, v, sv, a, err);
      if (T.amb) flags |= kFlagExact;
      auto inner = [&](double zc) -> double {
        ++ne;
        return tnode_pdf_sv(T, zc, v, sv, a) * iZT;
      };
      auto rz = make_xresolve([=](double zc) { return wfpt_x::pdf_sv(x - tc, v, sv, a, zc, err) / ZT; });
      return adaptive_walk<Stack>(inner, lb_z, ub_z, se, nsz, flags, ne, rz) * istw;
    };
    // exact outer values: the reference's z integral at tc (its own walk)
    auto rt = make_xresolve([=](double tc) {
      wfpt_x::Ctx C;
      auto inner_x = [&](double zc) { return wfpt_x::pdf_sv(x - tc, v, sv, a, zc, err) / ZT; };
      return wfpt_x::adaptive(inner_x, lb_z, ub_z, se, nsz, C) / stw;
    });
    return adaptive_walk<Stack>(outer, lb_t, ub_t, K.simps_err, K.n_st, flags, ne, rt);
  }
  if (mode == kFixedT)
    return simpson_1d(x, v, sv, a, z, t, err, z, z, 0, t - st / 2., t + st / 2., K.n_st, ne,
                      flags);
  if (mode == kFixedZ)
    return simpson_1d(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., K.n_sz, t, t, 0, ne,
                      flags);
  return simpson_2d(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., K.n_sz, t - st / 2.,
                    t + st / 2., K.n_st, ne, flags);
}

// The exact path for one trial (wfpt_exact.hpp), out of line: the kernels call
// it only for the rare trials routed there, and it must not add to their
// register allocation. Returns the density; flags gets kFlagDepth/Budget.
__device__ __noinline__ double exact_pdf(double x, Params P, Knobs K, long long* ne, int* flags) {
  wfpt_x::Ctx C;
  const double p = wfpt_x::full_pdf(x, P.v, P.sv, P.a, P.z, P.sz, P.t, P.st, K.err, K.n_st,
                                    K.n_sz, K.use_adaptive, K.simps_err, C);
  *ne += C.ne;
  *flags |= C.ovf;
  return p;
}

// The general per-lane walk, out of line (trees deeper than the breadth-first
// levels); a near-tie on it goes to the exact path.
template <int MODE>
__device__ __noinline__ double fallback_pdf(double x, Params P, Knobs K, long long* ne,
                                            int* flags) {
  long long n = 0;
  int f = 0;
  double p = full_pdf<MODE, MemStack<WFPT_MAX_DEPTH>>(x, P, K, n, f);
  if (f & kFlagExact) {
    n = 0;
    f = 0;
    p = exact_pdf(x, P, K, &n, &f);
  }
  *ne += n;
  *flags |= f;
  return p;
}

// Settles a trial density: a value that hinges on last-bit rounding (zero,
// negative, NaN, below kExactBelow, or kFlagExact raised on the way: a
// near-tie or an ambiguous series decision) is recomputed on the exact path,
// unless it is a structural zero (invalid parameters, or no evaluation point
// with x - t_node > 0: no arithmetic produced it).
__device__ inline double settle(double p, double x, const Params& P, const Knobs& K, bool structural,
                                long long& ne, int& flags) {
  if (!(flags & kFlagExact) && (p > kExactBelow || structural)) return p;
  flags &= ~kFlagExact;
  long long n = 0;
  const double q = exact_pdf(x, P, K, &n, &flags);
  ne = n;
  return q;
}

// ---------------------------------------------------------------------------
// Per-trial part of the root-level z grid. The 5 z nodes (lb, d, c, e, ub of
// integrate.pxi:114-141 / 143-178) are the same for every t node of a trial,
// so everything that depends on z alone is computed once per trial:
//   * sin/cos(pi g_0), sin/cos(pi g_4) and sin/cos(pi (g_4 - g_0) / 4), from
//     which each large-time t node rotates to g_1..g_3 (angle addition); g_4 is
//     evaluated directly so the w = 1 edge keeps the reference's sin(pi);
//   * the z-only part A_j of the drift-factor exponent (pdf.pxi:96-101):
//     c_j = (A_j - v^2 x) / (2 sv^2 x + 2)   (sv > 0),  c_j = A_j - v^2 x / 2  (sv = 0).
// g[] holds the reference's own node coordinates (every polynomial in w uses
// them); only transcendental factors use the rotations / recurrences.
struct ZGrid {
  double g[5];
  double s0, c0, s4, c4, sd, cd;
  double A[5];
  double h6, h12;  // (g4 - g0) / 6 and / 12: the Simpson weights of this grid's interval
};

__device__ inline ZGrid zgrid_setup(double lb, double ub, double v, double sv, double a) {
  ZGrid G;
  const double c = (ub + lb) / 2.;
  G.g[0] = lb;
  G.g[1] = (lb + c) / 2.;
  G.g[2] = c;
  G.g[3] = (c + ub) / 2.;
  G.g[4] = ub;
  sincospi01(G.g[0], G.s0, G.c0);
  sincospi01(G.g[4], G.s4, G.c4);
  sincospi01((G.g[4] - G.g[0]) * 0.25, G.sd, G.cd);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    if (sv == 0) {
      G.A[i] = ((-v) * a) * G.g[i];
    } else {
      const double azsv = (a * G.g[i]) * sv;
      G.A[i] = (azsv * azsv) - (((2.0 * a) * v) * G.g[i]);
    }
  }
  G.h6 = (G.g[4] - G.g[0]) / 6;
  G.h12 = (G.g[4] - G.g[0]) / 12;
  return G;
}

// exp(x) for the grid evaluation's finite arguments (series terms and drift
// factors, values only): x = k ln2 + r, |r| <= ln2/2, a degree-11 polynomial
// (Chebyshev-node fit: max relative error 1.2e-16 in double Horner steps),
// then ldexp, which also saturates to inf / 0 / subnormals for |x| > 709. No
// special-case selects (OCML's exp carries them for inf / NaN arguments,
// which the hot call sites never pass: their arguments are bounded by the
// -600 / 600 guards around them; the rare sites use exp_sat). WFPT_FAST_EXP=0
// restores OCML's exp.
#ifndef WFPT_FAST_EXP
#define WFPT_FAST_EXP 1
#endif
// One Horner step p r + c as a single three-operand v_fma_f64. Written with
// fma(), the compiler selects the two-address v_fmac_f64 and, because the
// coefficient c stays live for the next call site, copies it into the
// accumulator first (a v_mov_b64 per step: 9 extra VALU instructions per
// exponential). WFPT_HORNER_ASM=0 restores fma().
#ifndef WFPT_HORNER_ASM
#define WFPT_HORNER_ASM 1
#endif
__device__ inline double horner(double p, double r, double c) {
#if WFPT_HORNER_ASM
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(p), "v"(r), "s"(c));
  return d;
#else
  return fma(p, r, c);
#endif
}

// WFPT_EXP_ESTRIN: the degree-11 polynomial by Estrin's scheme (dependency
// depth 4 instead of Horner's 11, three more operations): the exponentials
// sit on the level-0 pass's longest dependency chains. Values only (the
// rounding differs from Horner's by an ulp; decisions keep their tie band).
#ifndef WFPT_EXP_ESTRIN
#define WFPT_EXP_ESTRIN 0
#endif
// WFPT_EXP_TABLE: exp_val as 2^(k/64) from a 64-entry table times a degree-5
// polynomial: x = (64 e + j) ln2/64 + r, |r| <= ln2/128, exp(x) = 2^e T[j]
// (1 + r + ... + r^5/120) (truncation < 4e-17 relative, ~1.5 ulp with the
// table's and Horner's roundings): 10 fp64 operations and a table load per
// exponential instead of 15 (and a 7-deep chain instead of 13). Values only,
// like exp_val.
#ifndef WFPT_EXP_TABLE
#define WFPT_EXP_TABLE 0
#endif
__device__ const double kExp2J64[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0};
// WFPT_EXP_TABLE=2: the table read from LDS (each kernel copies it at entry:
// exp_table_init), =1: from global memory
#if WFPT_EXP_TABLE == 2
__shared__ double sExp2J64[64];
#define WFPT_EXP_TAB sExp2J64
#else
#define WFPT_EXP_TAB kExp2J64
#endif
__device__ inline void exp_table_init() {
#if WFPT_EXP_TABLE == 2
  for (int k = threadIdx.x; k < 64; k += blockDim.x) sExp2J64[k] = kExp2J64[k];
  __syncthreads();
#endif
}
__device__ inline double exp_val_tab(double x) {
  const double kd = rint(x * 92.33248261689366);  // 64 / ln2
  double r = fma(-kd, 0x1.62e42fefa39efp-7, x);  // ln2 / 64, two parts
  r = fma(-kd, 0x1.abc9e3b39803fp-62, r);
  const int k = (int)kd;
  const double t = WFPT_EXP_TAB[k & 63];
  double p = horner(0x1.1111111111111p-7, r, 0x1.5555555555555p-5);
  p = horner(p, r, 0x1.5555555555555p-3);
  p = horner(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(t * p, k >> 6);
}
__device__ inline double exp_val(double x) {
#if WFPT_FAST_EXP && WFPT_EXP_TABLE
  return exp_val_tab(x);
#elif WFPT_FAST_EXP && WFPT_EXP_ESTRIN
  const double k = rint(x * 1.4426950408889634);
  double r = fma(-k, 6.9314718055994529e-01, x);
  r = fma(-k, 2.3190468138462996e-17, r);
  const double r2 = r * r;
  const double r4 = r2 * r2;
  const double r8 = r4 * r4;
  const double q0 = r + 1.0;
  const double q1 = fma(1.666666666666668e-01, r, 5.000000000000019e-01);
  const double q2 = fma(8.333333333319601e-03, r, 4.16666666664881e-02);
  const double q3 = fma(1.9841269890047113e-04, r, 1.3888888952314775e-03);
  const double q4 = fma(2.755724091857897e-06, r, 2.4801485482328494e-05);
  const double q5 = fma(2.5110037605963777e-08, r, 2.763263963904103e-07);
  const double s0 = fma(q1, r2, q0);
  const double s1 = fma(q3, r2, q2);
  const double s2 = fma(q5, r2, q4);
  const double p = fma(s2, r8, fma(s1, r4, s0));
  return ldexp(p, (int)k);
#elif WFPT_FAST_EXP
  const double k = rint(x * 1.4426950408889634);
  double r = fma(-k, 6.9314718055994529e-01, x);
  r = fma(-k, 2.3190468138462996e-17, r);
  double p = 2.5110037605963777e-08;
  p = horner(p, r, 2.763263963904103e-07);
  p = horner(p, r, 2.755724091857897e-06);
  p = horner(p, r, 2.4801485482328494e-05);
  p = horner(p, r, 1.9841269890047113e-04);
  p = horner(p, r, 1.3888888952314775e-03);
  p = horner(p, r, 8.333333333319601e-03);
  p = horner(p, r, 4.16666666664881e-02);
  p = horner(p, r, 1.666666666666668e-01);
  p = horner(p, r, 5.000000000000019e-01);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)k);
#else
  return exp(x);
#endif
}

// Large-time sines of a grid (pdf.pxi:61-62: sin(k pi w) at the grid's 5
// nodes), k = 1..kSinK, exactly as tnode_pdf_sv_grid5's recurrence produces
// them: sin / cos of nodes 1..3 rotated from node 0 (node 4 direct), then
// s_k = 2 cos(pi w) s_{k-1} - s_{k-2} in the same fused operations. Built on
// the host per call (RootGrids) so the lean pass reads them instead of
// recomputing them per lane; bit-identical to the per-lane recurrence.
constexpr int kSinK = 8;
// WFPT_SIN_PREFETCH=0: each row of the table is loaded where it is used
#ifndef WFPT_SIN_PREFETCH
#define WFPT_SIN_PREFETCH 0
#endif
__host__ __device__ inline void sin_rot(const ZGrid& G, double (&sj)[5], double (&cj)[5]) {
  sj[0] = G.s0;
  cj[0] = G.c0;
  sj[4] = G.s4;
  cj[4] = G.c4;
  for (int j = 1; j < 4; ++j) {
    sj[j] = fma(sj[j - 1], G.cd, cj[j - 1] * G.sd);
    cj[j] = fma(cj[j - 1], G.cd, -(sj[j - 1] * G.sd));
  }
}
// 2 cos(pi g_i) of node i (the recurrence's multiplier)
__host__ __device__ inline double sin_tc(const ZGrid& G, int i) {
  double sj[5], cj[5];
  sin_rot(G, sj, cj);
  const double c = i == 0 ? cj[0] : i == 1 ? cj[1] : i == 2 ? cj[2] : i == 3 ? cj[3] : cj[4];
  return c + c;
}
__host__ __device__ inline void sin_table(const ZGrid& G, double (&S)[kSinK + 1][5]) {
  double sj[5], cj[5];
  sin_rot(G, sj, cj);
  for (int i = 0; i < 5; ++i) {
    const double tc = cj[i] + cj[i];
    S[0][i] = 0.0;
    S[1][i] = sj[i];
    for (int k = 2; k <= kSinK; ++k) S[k][i] = msub(tc, S[k - 1][i], S[k - 2][i]);
  }
}

// Element i (a run-time index) of a 5-element register array, and its store:
// selects, so the array stays in registers inside a non-unrolled loop.
// Written out with constant subscripts (no loop): every access is a constant
// index from the start, so the array is split into registers, never
// promoted to memory.
__device__ inline double pick5(const double (&v)[5], int i) {
  const double a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3], a4 = v[4];
  return i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : i == 3 ? a3 : a4;
}
__device__ inline void put5(double (&v)[5], int i, double x) {
  v[0] = i == 0 ? x : v[0];
  v[1] = i == 1 ? x : v[1];
  v[2] = i == 2 ? x : v[2];
  v[3] = i == 3 ? x : v[3];
  v[4] = i == 4 ? x : v[4];
}

// The rare paths' exponentials, whose arguments can be infinite (|v| ~ 1e154
// makes v^2 x overflow; a subnormal tt makes the exponent multiplier
// overflow): libm's exp, which gives 0 for -inf like the reference
// (exp_val's range reduction would make NaN of it).
__device__ inline double exp_sat(double x) { return exp(x); }

// log of a trial's density term (wfpt.pyx:44, :70 — every per-trial log the
// kernels emit). Values only: the published fdlibm reduction x = 2^k (1 + f),
// sqrt(2)/2 <= 1 + f < sqrt(2), s = f / (2 + f) (hardware reciprocal + two
// Newton steps + one residual correction), log(1 + f) = f - (hfsq - s (hfsq +
// R(s^2))) with fdlibm's degree-7 R, plus k ln2 in two parts. <= 0.81 ulp
// (2e7 random arguments incl. subnormals against long double, unbiased), 38
// VALU operations against OCML's double-double log (~98). Zero, negative,
// infinite and NaN arguments take OCML's log. WFPT_FAST_LOG=0: OCML's log.
#ifndef WFPT_FAST_LOG
#define WFPT_FAST_LOG 1
#endif
__device__ inline double log_val(double x) {
#if WFPT_FAST_LOG
  if (!(x > 0.0 && x < __builtin_inf())) return log(x);
  int e;
  double m = frexp(x, &e);
  if (m < 0.70710678118654752440) {
    m = m + m;
    e -= 1;
  }
  const double f = m - 1.0;
  const double d = 2.0 + f;
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  double sq = f * r;
  sq = fma(r, fma(-d, sq, f), sq);
  const double z = sq * sq, w = z * z;
  const double t1 = w * horner(fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01), w,
                               3.999999999940941908e-01);
  const double t2 = z * horner(horner(fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                      w, 2.857142874366239149e-01),
                               w, 6.666666666666735130e-01);
  const double R = t2 + t1;
  const double hfsq = (0.5 * f) * f;
  const double k = (double)e;
  return k * 6.93147180369123816490e-01 -
         ((hfsq - fma(sq, hfsq + R, k * 1.90821492927058770002e-10)) - f);
#else
  return log(x);
#endif
}

__device__ inline double exp_node(double x) {
#if WFPT_FAST_EXP && WFPT_NODE_FAST_EXP
  x = x < -1100.0 ? -1100.0 : (x > 1100.0 ? 1100.0 : x);
  return exp_val(x);
#else
  return exp(x);
#endif
}

// Small-time series and drift factor of a grid in one 2-D recurrence
// (WFPT_SMALL_2D). Every term of pdf.pxi:55-57 times the drift factor of
// pdf.pxi:95-101 is exp(phi(j, k)) with
//   phi(j, k) = m (g_j + 2k)^2 + c_j,   j = 0..4 (z node), k = lower..upper,
// a quadratic in (j, k) on the equally spaced grid: its second differences
// are constants (8m in k, 2 m h^2 + d2 in j, 4 m h mixed), so the whole
// 5 x K table follows from six exponentials by products (the 1-D form below
// takes 2 per term k plus 3 for the drift). Values only, like the 1-D
// recurrences: ~K^2/2 + K + 4 chained roundings (< 40 ulp at K <= 8), far
// inside kTieBand. Returns false, and the caller evaluates the grid the 1-D
// way, when a term or an intermediate ratio could leave the normal range
// (every exponent is affine or quadratic over the table: its corners bound
// it) or a node's series is not positive (the fix-up path's semantics).
#ifndef WFPT_SMALL_2D
#define WFPT_SMALL_2D 1
#endif
__device__ inline bool small_grid2d(const TNode& T, const ZGrid& G, double sv, double (&out)[5]) {
  const int K = T.K;
  if (K > 8) return false;
  const int lower = (int)(-floor((K - 1) / 2.));
  const int upper = (int)ceil((K - 1) / 2.);
  const double m = T.m;
  // the drift exponent (A_i - vvx / 2 for sv = 0, (A_i - vvx) cden otherwise)
  // as one expression: the multiplier 1 is exact, so no per-node select
  const double dv = (sv == 0) ? T.vvx * 0.5 : T.vvx, dm = (sv == 0) ? 1.0 : T.cden;
  double c[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) c[i] = (G.A[i] - dv) * dm;
  const double lo2 = (double)(2 * lower);
  const double u0 = G.g[0] + lo2, u4 = G.g[4] + (double)(2 * upper);
  const double h = G.g[1] - G.g[0];
  const double d1 = c[1] - c[0];
  const double d2 = (c[2] - c[1]) - d1;
  const double a00 = m * (u0 * u0) + c[0];  // phi(0, lower)
  const double aR = m * (h * (2.0 * u0 + h)) + d1;  // phi(1, lower) - phi(0, lower)
  const double aQj = (2.0 * m) * (h * h) + d2;
  const double aP = (4.0 * m) * (u0 + 1.0);  // phi(0, lower + 1) - phi(0, lower)
  const double aQk = 8.0 * m;
  const double aQjk = (4.0 * m) * h;
  const double cmax = fmax(fmax(fmax(c[0], c[1]), fmax(c[2], c[3])), c[4]);
  const double cmin = fmin(fmin(fmin(c[0], c[1]), fmin(c[2], c[3])), c[4]);
  const double U = fmax(fabs(u0), fabs(u4));
  const double km1 = (double)(K - 1);
  // j-ratios at the table's corners (j = 0..3, k = lower..upper), k-ratios at
  // k = lower and upper - 1
  const double rmax = fmax(fmax(fabs(aR), fabs(aR + 3.0 * aQj)),
                           fmax(fabs(aR + km1 * aQjk), fabs((aR + 3.0 * aQj) + km1 * aQjk)));
  const double pmax = fmax(fabs(aP), fabs(aP + (km1 - 1.0) * aQk));
  const double qmax = fmax(fmax(fabs(aQj), fabs(aQk)), fabs(aQjk));
  constexpr double B = 640.0;
  const bool safe = (cmax < B) & (m * (U * U) + cmin > -B) & (fmax(fmax(rmax, pmax), qmax) < B);
  if (!safe) return false;
  double E0 = exp_val(a00), R0 = exp_val(aR), P = exp_val(aP);
  const double Qj = exp_val(aQj), Qk = exp_val(aQk), Qjk = exp_val(aQjk);
  double s[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) s[i] = 0.0;
  double k2 = lo2;
  for (int k = lower; k <= upper; ++k) {
    double E = E0, R = R0;
    s[0] = madd(G.g[0] + k2, E, s[0]);
#pragma unroll
    for (int i = 1; i < 5; ++i) {
      E = E * R;
      if (i < 4) R = R * Qj;
      s[i] = madd(G.g[i] + k2, E, s[i]);
    }
    E0 = E0 * P;
    P = P * Qk;
    R0 = R0 * Qjk;
    k2 = k2 + 2.0;
  }
  const double f = T.rn * T.sc;
  bool clean = true;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    out[i] = s[i] * f;
    clean = clean & (s[i] > 0) & !__builtin_isinf(out[i]);
  }
  return clean;
}

// pdf_sv at the 5 root-level z nodes of one t node (the values of
// tnode_pdf_sv at each node to a few ulp):
//   * small-t series: the exponents (g_j + 2k)^2 m are quadratic in j on the
//     equally spaced grid, so per term k two exponentials (j = 0 and the first
//     ratio) and one shared second-difference factor replace five; exponents
//     below -600 (subnormal territory) take the direct exps;
//   * large-t series: the Chebyshev recurrence in k from the rotated sin/cos;
//   * the drift factor exp(c_j): three exponentials and the second-difference
//     recurrence (direct exps when |c| > 600).
// stab (nullable): the grid's large-time sine table sin(k pi g_i), row k at
// stab + 5 k (k = 1..kSinK; SinTable); null: the Chebyshev recurrence in
// registers.
// Returns false when a node's drift factor overflowed with a positive series
// value (exp(c) = inf): then LITERAL fills that node with the reference's
// literal form (below); LITERAL = false (the level-0-only passes, whose
// register budget the rare form would take) leaves it inf. Either way the
// caller decides: a t node's root z grid (kAdaptTZ) hands such a node's z
// integral to a z walk, whose grids take the literal values.
template <bool LITERAL = true>
__device__ inline bool tnode_pdf_sv_grid5(const TNode& T, const ZGrid& G, double v, double sv,
                                          double a, double (&out)[5],
                                          const double* stab = nullptr) {
  double p[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) p[i] = 0.0;
  if (!T.pos) {
#pragma unroll
    for (int i = 0; i < 5; ++i) out[i] = 0.0;
    return true;
  }
  const int K = T.K;
#if defined(WFPT_KO_SMALL) || defined(WFPT_KO_LARGE)
  // timing experiments only (tools/ab_variants.py): wrong values
#ifdef WFPT_KO_SMALL
  if (T.small) {
#else
  if (!T.small) {
#endif
#pragma unroll
    for (int i = 0; i < 5; ++i) out[i] = T.sc * 0.25;
    return true;
  }
#endif
#if WFPT_SMALL_2D
  if (T.small && small_grid2d(T, G, sv, out)) return true;
#endif
  if (T.small) {
    const int lower = (int)(-floor((K - 1) / 2.));
    const int upper = (int)ceil((K - 1) / 2.);
    double qq = 0.0;
    bool have_q = false;
    for (int k = lower; k <= upper; ++k) {
      const double k2 = (double)(2 * k);
      // ek_j = (g_j + 2k)^2 m <= 0 is convex in j: the ends are the minima.
      // Operands are formed where they are used (the grid is wave-uniform in
      // the lean pass), not held as arrays across the branch.
      const double w0 = G.g[0] + k2, w4 = G.g[4] + k2;
      const double e0 = (w0 * w0) * T.m, e4 = (w4 * w4) * T.m;
      // with WFPT_SMALL_2D the 2-D table above takes every grid it can, so
      // this branch only sees the rare ones: node by node below
      if (!WFPT_SMALL_2D && e0 > -600.0 && e4 > -600.0) {
        const double w1 = G.g[1] + k2, w2 = G.g[2] + k2;
        const double e1 = (w1 * w1) * T.m, e2 = (w2 * w2) * T.m;
        const double d1 = e1 - e0;
        if (!have_q) {
          qq = exp_val((e2 - e1) - d1);
          have_q = true;
        }
        double E = exp_val(e0);
        double R = exp_val(d1);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          p[i] = madd(G.g[i] + k2, E, p[i]);
          E = E * R;
          R = R * qq;
        }
      } else {
        // rare (an end exponent in subnormal territory): one node per trip,
        // so the hot path's register allocation does not carry five
        // interleaved exponentials
#pragma unroll 1
        for (int i = 0; i < 5; ++i) {
          const double wi = pick5(G.g, i) + k2;
          put5(p, i, madd(wi, exp_sat((wi * wi) * T.m), pick5(p, i)));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) p[i] = p[i] * T.rn;
  } else if (stab) {
    // the sines of the (wave-uniform) grid from the call's table: the same
    // values the recurrence below produces (sin_table), read with scalar
    // loads instead of carried in 15 vector registers per lane
    double e = T.m, r = T.m * T.q2;
#if WFPT_SIN_PREFETCH
    if (K <= kSinK) {
      // each row's scalar loads are issued one row ahead of their use, so
      // the wait overlaps the previous row's products
      double row[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) row[i] = stab[5 + i];
      for (int k = 1; k <= K; ++k) {
        const int kq = k + 1 <= kSinK ? k + 1 : kSinK;
        double nxt[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) nxt[i] = stab[5 * kq + i];
        if (k == 1) {
#pragma unroll
          for (int i = 0; i < 5; ++i) p[i] = T.m * row[i];
        } else {
          e = e * r;
          r = r * T.q2;
          const double ke = (double)k * e;
#pragma unroll
          for (int i = 0; i < 5; ++i) p[i] = madd(ke, row[i], p[i]);
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) row[i] = nxt[i];
      }
    } else {
#else
    if (K >= 1) {
#pragma unroll
      for (int i = 0; i < 5; ++i) p[i] = T.m * stab[5 + i];
    }
    if (K <= kSinK) {
      for (int k = 2; k <= K; ++k) {
        e = e * r;
        r = r * T.q2;
        const double ke = (double)k * e;
#pragma unroll
        for (int i = 0; i < 5; ++i) p[i] = madd(ke, stab[5 * k + i], p[i]);
      }
    } else {
#endif
      // beyond the table (err far below 1e-10): the recurrence one node at
      // a time (few live registers)
#pragma unroll 1
      for (int i = 0; i < 5; ++i) {
        const double s1 = stab[5 + i];
        const double tci = sin_tc(G, i);
        double e1 = T.m, r1 = T.m * T.q2, sk = s1, skm1 = 0.0, pi = T.m * s1;
        for (int k = 2; k <= K; ++k) {
          e1 = e1 * r1;
          r1 = r1 * T.q2;
          const double sn = msub(tci, sk, skm1);
          skm1 = sk;
          sk = sn;
          pi = madd((double)k * e1, sk, pi);
        }
        put5(p, i, pi);
      }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) p[i] = p[i] * kPi;
  } else {
    double sj[5], cj[5];
    sj[0] = G.s0;
    cj[0] = G.c0;
    sj[4] = G.s4;
    cj[4] = G.c4;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      sj[j] = fma(sj[j - 1], G.cd, cj[j - 1] * G.sd);
      cj[j] = fma(cj[j - 1], G.cd, -(sj[j - 1] * G.sd));
    }
    double tc[5], sk[5], skm1[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      tc[i] = cj[i] + cj[i];
      sk[i] = sj[i];
      skm1[i] = 0.0;
      if (K >= 1) p[i] = T.m * sj[i];
    }
    // two terms per trip, the two sin registers swapping roles (no moves)
    double e = T.m, r = T.m * T.q2;
    int k = 2;
    for (; k + 1 <= K; k += 2) {
      e = e * r;
      r = r * T.q2;
      const double ke = (double)k * e;
      e = e * r;
      r = r * T.q2;
      const double ke1 = (double)(k + 1) * e;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        skm1[i] = msub(tc[i], sk[i], skm1[i]);  // sin(k pi w)
        p[i] = madd(ke, skm1[i], p[i]);
        sk[i] = msub(tc[i], skm1[i], sk[i]);    // sin((k+1) pi w)
        p[i] = madd(ke1, sk[i], p[i]);
      }
    }
    if (k <= K) {
      e = e * r;
      const double ke = (double)k * e;
#pragma unroll
      for (int i = 0; i < 5; ++i) p[i] = madd(ke, msub(tc[i], sk[i], skm1[i]), p[i]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) p[i] = p[i] * kPi;
  }
#ifdef WFPT_KO_LDRIFT
  if (!T.small) {  // timing experiment only: no drift factor
#pragma unroll
    for (int i = 0; i < 5; ++i) out[i] = p[i] * T.sc;
    return true;
  }
#endif
  // exponent of the drift factor at each node (quadratic in g), formed where
  // it is used: A_i - vvx / 2 for sv = 0, (A_i - vvx) cden otherwise, as one
  // expression (the multiplier 1 is exact: no per-node select)
  const double dv = (sv == 0) ? T.vvx * 0.5 : T.vvx, dm = (sv == 0) ? 1.0 : T.cden;
  auto cexp = [&](int i) -> double { return (G.A[i] - dv) * dm; };
  double ex[5];
  const double c0 = cexp(0), c2 = cexp(2), c4 = cexp(4);
  const bool moderate = fabs(c0) < 600.0 && fabs(c2) < 600.0 && fabs(c4) < 600.0;
  if (moderate) {
    // c_j = c0 + j d1 + j(j-1)/2 d2  ->  E_j = E_{j-1} * R * Q^(j-1)
    const double c1 = cexp(1);
    const double d1 = c1 - c0;
    const double d2 = (c2 - c1) - d1;
    ex[0] = exp_val(c0);
    double rr = exp_val(d1);
    const double qd = exp_val(d2);
#pragma unroll
    for (int j = 1; j < 5; ++j) {
      ex[j] = ex[j - 1] * rr;
      rr = rr * qd;
    }
  } else {  // rare: one node per trip (register allocation as above)
#pragma unroll 1
    for (int i = 0; i < 5; ++i) {
      const double Ai = pick5(G.A, i);
      put5(ex, i, exp_sat((Ai - dv) * dm));
    }
  }
  // the common case: every series value positive and every product finite;
  // the rare fix-ups below run only on lanes that need one (same values)
  bool clean = true;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    out[i] = (p[i] * ex[i]) * T.sc;
    clean = clean & (p[i] > 0) & !__builtin_isinf(out[i]);
  }
  if (__builtin_expect(clean, 1)) return true;
  if (!LITERAL) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      double r2 = out[i];
      if (sv != 0 && p[i] < 0) r2 = __builtin_nan("");
      if (p[i] == 0) r2 = 0.0 * T.sc;
      ok = ok & !(__builtin_isinf(r2) && p[i] > 0);
      out[i] = r2;
    }
    return ok;
  }
  bool ok = true;
#pragma unroll 1
  for (int i = 0; i < 5; ++i) {
    double r2 = pick5(out, i);
    const double pi = pick5(p, i);
    if (sv != 0 && pi < 0) r2 = __builtin_nan("");  // log(p < 0) in the reference
    // exp(log 0 + c) = 0 even if e^c = inf; 0 * sc keeps the reference's
    // 0 / (a*a) = NaN at a == 0
    if (pi == 0) r2 = 0.0 * T.sc;
    // exp(c) overflow with a finite true value (sv > 0): the reference's
    // literal form exp(log p + c) / sqrt(sv^2 x + 1) / a^2 (pdf.pxi:102), a
    // value like the others (the stop tests keep their tie band). sv = 0: the
    // reference's p exp(c) / a^2 (pdf.pxi:85) overflows to inf as well.
    const bool ovf = __builtin_isinf(r2) && pi > 0;
    ok = ok & !ovf;
    if (ovf && sv != 0) {
      const double w = pick5(G.g, i);
      const double azsv = (a * w) * sv;
      r2 = (exp(log(pi) + (((azsv * azsv) - (((2.0 * a) * v) * w)) - T.vvx) /
                              (((2.0 * (sv * sv)) * T.xx) + 2.0)) /
            sqrt(((sv * sv) * T.xx) + 1.0)) /
           (a * a);
    }
    put5(out, i, r2);
  }
  return ok;
}

// ---------------------------------------------------------------------------
// Adaptive trees (the reference's adaptiveSimpsonsAux recursion) over the
// dyadic points of the root interval.
//
// Node order used below: lb, d, c, e, ub of an interval (integrate.pxi:114-141
// prologue nodes lb, c, ub + the root aux nodes d, e). The level-0 engine
// (wfpt_kernels.hip: engine_kernel) completes trees of up to kTreeDepth
// refinement levels per axis in-wave (HDDM's n_st = n_sz = 2 default); deeper
// trees continue on the per-lane walk (kFlagFallback). A tree's values live at
// the kTreePoints dyadic points P_0..P_kTreeW of its root interval.
constexpr int kTreeDepth = 2;
constexpr int kTreeW = 4 << kTreeDepth;
constexpr int kTreePoints = kTreeW + 1;

enum Outcome : int { kFinal = 0, kTree = 1, kExact = 2 };

// The reference's Simpson estimates of one interval from its 5 values.
struct Simp {
  double S, Sl, Sr, S2;
};
__host__ __device__ inline Simp simp5(double h, double fb, double fd, double fm, double fe,
                                     double fu) {
  Simp s;
  s.S = (h / 6) * ((fb + (4 * fm)) + fu);
  s.Sl = (h / 12) * ((fb + (4 * fd)) + fm);
  s.Sr = (h / 12) * ((fm + (4 * fe)) + fu);
  s.S2 = s.Sl + s.Sr;
  return s;
}

// simp5 with the interval's weights h/6, h/12 precomputed (the same IEEE
// divisions of the same h: bit-identical).
__device__ inline Simp simp5p(double h6, double h12, double fb, double fd, double fm, double fe,
                              double fu) {
  Simp s;
  s.S = h6 * ((fb + (4 * fm)) + fu);
  s.Sl = h12 * ((fb + (4 * fd)) + fm);
  s.Sr = h12 * ((fm + (4 * fe)) + fu);
  s.S2 = s.Sl + s.Sr;
  return s;
}
// The leaf value S2 + (S2 - S) / 15 of an interval that stops refining
// (integrate.pxi:106,171), with 1/15 as a product: a value, never a decision
// input at its own level (the stop test reads S and S2), within an ulp of the
// quotient. Every site that must produce the same bits for a t node's root z
// integral (inner_root, the engine's task completion) uses this.
constexpr double kInv15 = 1.0 / 15.0;
__device__ inline double simp_value(const Simp& s) { return s.S2 + (s.S2 - s.S) * kInv15; }

// The z integral at one t node (adaptiveSimpsons_1D over z, integrate.pxi:
// 114-141), root level only: the root's 5 evaluations 5-wide on the grid and
// its stop test. repair = the test asks for refinement (the value is then the
// root estimate; the caller defers the trial).
__device__ inline double inner_root(const TNode& T, const ZGrid& G, double iZz, double v,
                                    double sv, double a, const Knobs& K, int& flags,
                                    long long& ne, bool& repair,
                                    const double* stab = nullptr) {
  double f[5];
  // an overflowed drift factor marks the z integral as refining: in every
  // call sequence the t node's value then comes from a z walk, whose grids
  // take the literal form (its values here are not used; their stop test
  // raises no flag)
  const bool ovf = !tnode_pdf_sv_grid5<false>(T, G, v, sv, a, f, stab);
#pragma unroll
  for (int i = 0; i < 5; ++i) f[i] = f[i] * iZz;
  ne += 5;
  const Simp s = simp5p(G.h6, G.h12, f[0], f[1], f[2], f[3], f[4]);
  int fl = 0;
  repair = simpson_refine(s.S, s.S2, K.simps_err, K.n_sz, fl) || ovf;
  flags |= ovf ? 0 : fl;
  return simp_value(s);
}

// Root interval of the adaptive tree: over t for kAdaptT / kAdaptTZ, over z
// for kAdaptZ.
template <int MODE>
__device__ inline void tree_root(const Trial& tr, const Params& P, double& lb, double& ub) {
  if (MODE == kAdaptZ) {
    lb = tr.z - tr.sz / 2.;
    ub = tr.z + tr.sz / 2.;
  } else {
    lb = P.t - tr.st / 2.;
    ub = P.t + tr.st / 2.;
  }
}

// Level-0 pass of one trial for an adaptive (or direct) MODE, one trial per
// lane (the direct family and the per-node path): the reference's prologue +
// root aux node of every adaptive Simpson it runs (1, 5, 5 or 25 pdf_sv
// evaluations).
//   kFinal: p is the trial density (0 for invalid parameters);
//   kTree:  the root stop test asks for refinement, or (kAdaptTZ) some t
//           node's z integral needs refinement (bit k of `pend`: tree point
//           k * kTreeW / 4); f[] = the root interval's values at lb, d, c, e, ub;
//   kExact: the value hinges on last-bit rounding (recomputed exactly).
template <int MODE, bool UNROLL = false, bool KEEP_F = true>
__device__ inline int eng_level0(double x0, const Params& P, const Knobs& K, const ZGrid& G,
                                 double& p, double (&f)[5], long long& ne, unsigned& pend);

// KEEP_F = false: f[] is not written (a caller that only needs p and the
// outcome: the per-node level 0, whose deferred chunks redo their level 0);
// the root Simpson sums are accumulated as the t nodes complete (the lean
// pass's form: the same values, fewer live registers)
template <int MODE, bool KEEP_F = true>
__device__ inline int fast_level0(double x0, const Params& P, const Knobs& K, double& p,
                                  double (&f)[5], long long& ne, int& flags, unsigned& pend) {
  const Trial tr = trial_setup(x0, P);
  p = 0.0;
  pend = 0u;
  if (!tr.valid) return kFinal;
  const double a = P.a, sv = P.sv, t = P.t, err = K.err;
  const double x = tr.x, v = tr.v, z = tr.z;
  if (MODE == kDirect) {
    ne += 1;
    p = pdf_sv(x - t, v, sv, a, z, err, flags);
    if (flags & kFlagExact) return kExact;
    if (p > kExactBelow || x - t <= 0) return kFinal;
    if (!tiny_absorbed(p, P.p_outlier, K.w_outlier)) return kExact;
    p = 0.0;
    return kFinal;
  }
  // adaptive families: the engine's level 0 (eng_level0, defined below) on
  // this trial's own root z grid
  ZGrid G{};
  if (MODE == kAdaptZ || MODE == kAdaptTZ)
    G = zgrid_setup(z - tr.sz / 2., z + tr.sz / 2., v, sv, a);
  (void)t;
  (void)x;
  return eng_level0<MODE, WFPT_FAST_L0_UNROLL != 0, KEEP_F>(x0, P, K, G, p, f, ne, pend);
}

// The engine's level 0 (kAdaptT / kAdaptTZ): the same operations as
// fast_level0, factored so that any single t node j of a trial's root
// interval can be evaluated on its own (a split chunk's level-0 task) with
// exactly the bits the per-lane loop produces. The z grid is the call's table
// (EngTables), shared by both.
struct L0Hints {
  // q of t node j is q0 R^j (formed per node: two registers instead of five
  // held across the node loop; the products are the ones a table would hold)
  double q0, R;
  double ia2;  // 1 / a^2
  Decision D0, D4;
  bool ok0, ok4, shared;
  __device__ double qh(int j) const {
    if (q0 < 0.0) return -1.0;
    const double R2 = R * R;
    const double Rj = j == 1 ? R : j == 2 ? R2 : j == 3 ? R2 * R : R2 * R2;
    return j == 0 ? q0 : q0 * Rj;
  }
};
__device__ inline L0Hints l0_hints(double x, double lb, double ub, double a, double err) {
  L0Hints H;
  H.q0 = -1.0;
  H.R = 0.0;
  H.D0 = Decision{0, 0, 0};
  H.D4 = Decision{0, 0, 0};
  H.ok0 = H.ok4 = H.shared = false;
  const double a2 = a * a;
  const double ia2 = 1.0 / a2;
  H.ia2 = ia2;
  // values only (the fp32 decision estimates below have a 1e-5 guard band)
  const double q0 = exp_node((-kPi2 * ((x - lb) * ia2)) * 0.5);
  const double R = exp_node((kPi2 * (ub - lb)) * (0.125 * ia2));
  if (q0 > 1e-280 && R < 1e10 && x - lb > 0) {
    H.q0 = q0;
    H.R = R;
  }
  if (x - ub > 0) {
    float args0, args4;
    H.ok0 = decide32((x - lb) * ia2, err, H.D0, args0);
    H.ok4 = decide32((x - ub) * ia2, err, H.D4, args4);
    H.shared = H.ok0 && H.ok4 && args0 < 0.5f && H.D0.small == H.D4.small && H.D0.K == H.D4.K;
  }
  return H;
}
// t node j (0..4: lb, d, c, e, ub) of the trial's root t interval: its value
// (kAdaptT: pdf_sv / st; kAdaptTZ: the z integral's root estimate / st),
// kFlagExact in flags for an ambiguous decision or a near-tie, pend = the z
// integral asks for refinement.
template <int MODE>
__device__ inline double l0_node(const Trial& tr, const Params& P, const Knobs& K, double lb,
                                 double ub, const L0Hints& H, int j, const ZGrid& G, int& flags,
                                 bool& pend, long long& ne, const double* stab = nullptr) {
  const double a = P.a, sv = P.sv, err = K.err;
  const double x = tr.x, v = tr.v, z = tr.z;
  const double iw = 1.0 / (ub - lb);
  const double c = (ub + lb) / 2.;
  const double d = (lb + c) / 2., e = (c + ub) / 2.;
  const double tc = j == 0 ? lb : j == 1 ? d : j == 2 ? c : j == 3 ? e : ub;
  const double qh = H.qh(j);
  const bool known = j == 0 ? H.ok0 : (j == 4 ? H.ok4 : H.shared);
  const TNode T = tnode_setup_r(x - tc, v, sv, a, H.ia2, err, qh, known, j == 4 ? H.D4 : H.D0);
  pend = false;
  if (T.amb) {
    flags |= kFlagExact;
    return 0.0;
  }
#ifdef WFPT_KO_NODE
  if (MODE == kAdaptTZ) {  // timing experiment only: no grid evaluation
    ne += 5;
    return T.sc * iw;
  }
#endif
  if (MODE == kAdaptTZ) {
    const double iZz = 1.0 / ((z + tr.sz / 2.) - (z - tr.sz / 2.));
    return inner_root(T, G, iZz, v, sv, a, K, flags, ne, pend, stab) * iw;
  }
  ne += 1;
  return tnode_pdf_sv(T, z, v, sv, a) * iw;
}

// The engine's level 0 of one trial (as fast_level0, on the table's z grid):
// kFinal (p), kTree (f[], pend) or kExact.
// KEEP_F = false (the lean pass, which never reads f[]): the root Simpson
// sums are accumulated as the t nodes complete, in the reference's
// expression order (three registers across the node loop instead of five).
// Overflowed drift factors (tnode_pdf_sv_grid5): kAdaptTZ's t-node root
// grids hand them to z walks in every pass (inner_root); kAdaptZ's root grid
// takes the literal form when LITERAL (the engine's own level 0, not
// unrolled), otherwise (the unrolled level-0-only passes: lean, small,
// per-node / per-trial fast) the trial returns kTree, i.e. it is handed to the
// engine — every call sequence gives it the same bits.
template <int MODE, bool KEEP_F = true, bool UNROLL = false, bool LITERAL = !UNROLL>
__device__ inline int eng_level0_t(const Trial& tr, const Params& P, const Knobs& K,
                                   const ZGrid& G, double& p, double (&f)[5], long long& ne,
                                   unsigned& pend, const double* stab = nullptr) {
  p = 0.0;
  pend = 0u;
  if (!tr.valid) return kFinal;
  double lb, ub;
  tree_root<MODE>(tr, P, lb, ub);
  // formed here: a one-bit mask across the node loop instead of a double
  const bool structural = (MODE == kAdaptZ) ? tr.x - P.t <= 0 : tr.x - lb <= 0;
  int flags = 0;
  if (MODE == kAdaptZ) {
    const double iw = 1.0 / (ub - lb);
    const TNode T = tnode_setup(tr.x - P.t, tr.v, P.sv, P.a, K.err);
    if (T.amb) return kExact;
    // (kAdaptZ: the root grid's values are the tree's; an overflow hands a
    // level-0-only pass's trial to the engine, which uses the literal values)
    if (!tnode_pdf_sv_grid5<LITERAL>(T, G, tr.v, P.sv, P.a, f, stab) && !LITERAL) return kTree;
#pragma unroll
    for (int i = 0; i < 5; ++i) f[i] = f[i] * iw;
    ne += 5;
  } else {
    const L0Hints H = l0_hints(tr.x, lb, ub, P.a, K.err);
    if (!KEEP_F) {
      // X, Y, Z after node j:  0: f0 | 1: f0, f0+4f1 | 2: f2, f0+4f2, Sl |
      // 3: f2+4f3, f0+4f2, Sl | 4: -> S = h6((f0+4f2)+f4), Sr = h12((f2+4f3)+f4)
      const double h = ub - lb;
      double X = 0.0, Y = 0.0, Z = 0.0, y4 = 0.0;
#define WFPT_L0_ACC_NODE(j)                                                      \
  {                                                                              \
    bool pj;                                                                     \
    const double y = l0_node<MODE>(tr, P, K, lb, ub, H, j, G, flags, pj, ne, stab);  \
    if (flags & kFlagExact) return kExact;                                       \
    if (pj) pend |= 1u << ((j) * (kTreeW / 4));                                  \
    const double x4 = X + (4 * y);                                               \
    if ((j) == 2) Z = (h / 12) * (Y + y);                                        \
    Y = ((j) == 1 || (j) == 2) ? x4 : Y;                                         \
    X = ((j) == 0 || (j) == 2) ? y : ((j) == 3 ? x4 : X);                        \
    y4 = y;                                                                      \
  }
      if constexpr (UNROLL) {
#pragma unroll
        for (int j = 0; j < 5; ++j) WFPT_L0_ACC_NODE(j)
      } else {
#pragma unroll 1
        for (int j = 0; j < 5; ++j) WFPT_L0_ACC_NODE(j)
      }
#undef WFPT_L0_ACC_NODE
      if (pend) return kTree;
      Simp s;
      s.S = (h / 6) * (Y + y4);
      s.Sl = Z;
      s.Sr = (h / 12) * (X + y4);
      s.S2 = s.Sl + s.Sr;
      const int bottom = K.n_st;
      const bool refine = simpson_refine(s.S, s.S2, K.simps_err, bottom, flags);
      if (flags & kFlagExact) return kExact;
      if (refine) return kTree;
      p = s.S2 + (s.S2 - s.S) / 15;
      if (p > kExactBelow || structural) return kFinal;
      if (!tiny_absorbed(p, P.p_outlier, K.w_outlier)) return kExact;
      p = 0.0;
      return kFinal;
    }
#define WFPT_L0_F_NODE(j)                                                        \
  {                                                                              \
    bool pj;                                                                     \
    const double y = l0_node<MODE>(tr, P, K, lb, ub, H, j, G, flags, pj, ne, stab);  \
    if (flags & kFlagExact) return kExact;                                       \
    if (pj) pend |= 1u << ((j) * (kTreeW / 4));                                  \
    if ((j) == 0) f[0] = y;                                                      \
    else if ((j) == 1) f[1] = y;                                                 \
    else if ((j) == 2) f[2] = y;                                                 \
    else if ((j) == 3) f[3] = y;                                                 \
    else f[4] = y;                                                               \
  }
    if constexpr (UNROLL) {
#pragma unroll
      for (int j = 0; j < 5; ++j) WFPT_L0_F_NODE(j)
    } else {
#pragma unroll 1
      for (int j = 0; j < 5; ++j) WFPT_L0_F_NODE(j)
    }
#undef WFPT_L0_F_NODE
  }
  if (pend) return kTree;
  const Simp s = simp5(ub - lb, f[0], f[1], f[2], f[3], f[4]);
  const int bottom = (MODE == kAdaptZ) ? K.n_sz : K.n_st;
  const bool refine = simpson_refine(s.S, s.S2, K.simps_err, bottom, flags);
  if (flags & kFlagExact) return kExact;
  if (refine) return kTree;
  p = s.S2 + (s.S2 - s.S) / 15;
  if (p > kExactBelow || structural) return kFinal;
  if (!tiny_absorbed(p, P.p_outlier, K.w_outlier)) return kExact;
  p = 0.0;
  return kFinal;
}
template <int MODE, bool UNROLL, bool KEEP_F>
__device__ inline int eng_level0(double x0, const Params& P, const Knobs& K, const ZGrid& G,
                                 double& p, double (&f)[5], long long& ne, unsigned& pend) {
  return eng_level0_t<MODE, KEEP_F, UNROLL>(trial_setup(x0, P), P, K, G, p, f, ne, pend);
}

// z grids of the engine, relative to the dyadic points P of [lb_z, ub_z]:
// kGridRoot {P0, P4, P8, P12, P16} (the root interval's lb, d, c, e, ub),
// kGridL1 {P2, P6, P10, P14, +1 unused} (the aux nodes of both halves),
// kGridL2L {P1, P3, P5, P7, P9}, kGridL2R {P7, P9, P11, P13, P15} (the aux
// nodes of the four quarters; P7 is taken from L2L, P9 from L2R). Five
// equally spaced points each, so tnode_pdf_sv_grid5 serves all four.
enum GridSel : int { kGridRoot = 0, kGridL1 = 1, kGridL2L = 2, kGridL2R = 3 };
// Dyadic point P_k (k = 0..kTreeW) of [lb, ub] as the reference's recursion
// computes it: every interval's midpoint is (ub + lb) / 2 of its own bounds
// and its aux nodes (lb + c) / 2, (c + ub) / 2 (integrate.pxi:94-104) are its
// children's midpoints, so P_k is the end of the chain of midpoints that
// bisects down to k (IEEE addition is commutative: operand order is moot).
__host__ __device__ inline double dyadic_point(double lb, double ub, int k) {
  if (k <= 0) return lb;
  if (k >= kTreeW) return ub;
  int lo = 0, hi = kTreeW;
  for (;;) {
    const int mid = (lo + hi) >> 1;
    const double c = (ub + lb) / 2.;
    if (k == mid) return c;
    if (k < mid) {
      hi = mid;
      ub = c;
    } else {
      lo = mid;
      lb = c;
    }
  }
}

__host__ __device__ inline ZGrid zgrid_of(double lb, double ub, int sel, double v, double sv,
                                          double a) {
  ZGrid G;
  const int k0 = sel == kGridRoot ? 0 : sel == kGridL1 ? 2 : sel == kGridL2L ? 1 : 7;
  const int dk = sel == kGridRoot ? 4 : sel == kGridL1 ? 4 : 2;
#pragma unroll
  for (int i = 0; i < 5; ++i) G.g[i] = dyadic_point(lb, ub, k0 + i * dk);
  // the unused fifth node of kGridL1 (P18, past ub <= 1 by sz / 8): any
  // finite coordinate of the same spacing
  if (sel == kGridL1) G.g[4] = G.g[3] + (G.g[3] - G.g[2]);
  sincospi01(G.g[0], G.s0, G.c0);
  sincospi01(G.g[4], G.s4, G.c4);
  sincospi01((G.g[4] - G.g[0]) * 0.25, G.sd, G.cd);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    if (sv == 0) {
      G.A[i] = ((-v) * a) * G.g[i];
    } else {
      const double azsv = (a * G.g[i]) * sv;
      G.A[i] = (azsv * azsv) - (((2.0 * a) * v) * G.g[i]);
    }
  }
  G.h6 = (G.g[4] - G.g[0]) / 6;
  G.h12 = (G.g[4] - G.g[0]) / 12;
  return G;
}


// The reference's recursion (adaptiveSimpsonsAux, integrate.pxi:94-112 /
// 159-178) over a tree of depth <= kTreeDepth whose values f[k] at the dyadic
// points P[k] of the root interval are in registers, in straight-line form:
// prologue S of the root, then per visited interval its S2 from its 5 values,
// the stop test (bottom = depth - level, eps halved per level) and either the
// leaf value S2 + (S2 - S) / 15 or left + right. lv: the deepest level whose
// values are known. Returns the integral when no visited interval asks for
// values below lv; otherwise need = the refining intervals of level lv
// (bit m: interval m of that level), and for lv == kTreeDepth those mean a
// deeper tree. flags gets kFlagExact for a stop test inside kTieBand; nref =
// visited refined intervals (2 new nodes x 2 evaluations each). used
// (optional): bit k set for every point f[k] the recursion read (the points
// the reference evaluates).
__host__ __device__ inline double tree17(const double (&f)[kTreePoints],
                                         const double (&P)[kTreePoints], double err, int depth,
                                         int lv, int& flags, unsigned& need, int& nref,
                                         unsigned* used = nullptr) {
  need = 0u;
  nref = 0;
  if (used) *used = 0x11111u;  // points 0, 4, 8, 12, 16
  const double h0 = P[kTreeW] - P[0];
  const double S0 = (h0 / 6) * ((f[0] + (4 * f[8])) + f[16]);
  const Simp r = simp5(h0, f[0], f[4], f[8], f[12], f[16]);
  if (!simpson_refine(S0, r.S2, err, depth, flags)) return r.S2 + (r.S2 - S0) / 15;
  nref = 1;
  if (lv == 0) {
    need = 1u;
    return 0.0;
  }
  double vh[2];
  if (used) *used |= 0x4444u;  // the halves' aux points 2, 6, 10, 14
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int lo = 8 * m;
    const double S = m ? r.Sr : r.Sl;
    const Simp s = simp5(P[lo + 8] - P[lo], f[lo], f[lo + 2], f[lo + 4], f[lo + 6], f[lo + 8]);
    if (!simpson_refine(S, s.S2, err / 2, depth - 1, flags)) {
      vh[m] = s.S2 + (s.S2 - S) / 15;
      continue;
    }
    ++nref;
    if (lv == 1) {
      need |= 1u << m;
      vh[m] = 0.0;
      continue;
    }
    if (used) *used |= 0xAAu << lo;  // the half's quarter aux points lo + 1, 3, 5, 7
    double vq[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int l2 = lo + 4 * q;
      const double Sq = q ? s.Sr : s.Sl;
      const Simp u = simp5(P[l2 + 4] - P[l2], f[l2], f[l2 + 1], f[l2 + 2], f[l2 + 3], f[l2 + 4]);
      if (simpson_refine(Sq, u.S2, (err / 2) / 2, depth - 2, flags)) need |= 1u << (2 * m + q);
      vq[q] = u.S2 + (u.S2 - Sq) / 15;
    }
    vh[m] = vq[0] + vq[1];
  }
  return need ? 0.0 : vh[0] + vh[1];
}

// Per-call tables of the engine (host-computed from the call's parameters,
// passed by value): the z grids of both boundaries (trial_setup's flip x > 0:
// v = -v, z = 1 - z), the dyadic points of the t tree and of both z trees.
struct EngTables {
  ZGrid G[2][4];
  double tP[kTreePoints];
  double zP[2][kTreePoints];
  double iz[2];  // 1 / (ub_z - lb_z) per boundary
};

__host__ __device__ inline void eng_tables(const Params& P, EngTables& T) {
  for (int k = 0; k < kTreePoints; ++k) T.tP[k] = dyadic_point(P.t - P.st / 2., P.t + P.st / 2., k);
  for (int flip = 0; flip < 2; ++flip) {
    const double zf = flip ? 1. - P.z : P.z, vf = flip ? -P.v : P.v;
    const double zl = zf - P.sz / 2., zu = zf + P.sz / 2.;
    for (int sel = 0; sel < 4; ++sel) T.G[flip][sel] = zgrid_of(zl, zu, sel, vf, P.sv, P.a);
    for (int k = 0; k < kTreePoints; ++k) T.zP[flip][k] = dyadic_point(zl, zu, k);
    T.iz[flip] = 1.0 / (zu - zl);
  }
}

// The root z grids of both boundaries alone (the lean level-0 pass): the
// same zgrid_of calls as eng_tables' G[flip][kGridRoot], so bit-identical.
struct RootGrids {
  ZGrid G[2];
  double S[2][kSinK + 1][5];  // their large-time sine tables (sin_table)
};
__host__ __device__ inline void root_grids(const Params& P, RootGrids& R) {
  for (int flip = 0; flip < 2; ++flip) {
    const double zf = flip ? 1. - P.z : P.z, vf = flip ? -P.v : P.v;
    R.G[flip] = zgrid_of(zf - P.sz / 2., zf + P.sz / 2., kGridRoot, vf, P.sv, P.a);
    sin_table(R.G[flip], R.S[flip]);
  }
}

// Per-call constants of the direct family (simple DDM: one pdf_sv per trial,
// pdf.pxi:74-102 at w = z) for both boundaries, computed once on the host with
// the device's operations (bit-identical): the flipped v and w (pdf.pxi:
// 116-118), sin(pi w) and 2 cos(pi w) of the large-time series (tnode_ftt),
// the drift exponent's trial-independent part (-v) a w, and 1 / a^2
// (tnode_setup). `ok`: trial_setup's validity tests that do not involve x.
struct DirectArgs {
  double v[2], w[2], s1[2], tc[2], dn[2];
  double ia2;
  int ok;
};
__host__ __device__ inline void direct_args(const Params& P, DirectArgs& D) {
  for (int b = 0; b < 2; ++b) {
    const double v = b ? -P.v : P.v, w = b ? 1. - P.z : P.z;
    D.v[b] = v;
    D.w[b] = w;
    double s1, c1;
    sincospi01(w, s1, c1);
    D.s1[b] = s1;
    D.tc[b] = c1 + c1;
    D.dn[b] = ((-v) * P.a) * w;
  }
  D.ia2 = 1.0 / (P.a * P.a);
  const double a = P.a, sv = P.sv, t = P.t, st0 = P.st, sz0 = P.sz;
  D.ok = !((P.z < 0) || (P.z > 1) || (a < 0) || (t < 0) || (st0 < 0) || (sv < 0) ||
           (sz0 < 0) || (sz0 > 1) || (P.z + sz0 / 2. > 1) || (P.z - sz0 / 2. < 0) ||
           (t - st0 / 2. < 0));
}

// tnode_ftt with the large-time sines given (DirectArgs): the same operations.
__device__ inline double tnode_ftt_sc(const TNode& T, double w, double s1, double tc) {
  double p = 0.0;
  const int K = T.K;
  if (T.small) {
    const int lower = (int)(-floor((K - 1) / 2.));
    const int upper = (int)ceil((K - 1) / 2.);
    for (int k = lower; k <= upper; ++k) {
      const double wk = w + (double)(2 * k);
      p = madd(wk, exp_node((wk * wk) * T.m), p);
    }
    p = p * T.rn;
  } else {
    double sk = s1, skm1 = 0.0;
    double e = T.m, r = T.m * T.q2;
    if (K >= 1) p = e * s1;
    for (int k = 2; k <= K; ++k) {
      const double sn = msub(tc, sk, skm1);
      skm1 = sk;
      sk = sn;
      e = e * r;
      r = r * T.q2;
      p = madd((double)k * e, sk, p);
    }
    p = p * kPi;
  }
  return p;
}

// fast_level0<kDirect> of a trial on boundary b with the call's DirectArgs:
// the same operations (trial_setup's validity, tnode_setup, tnode_pdf_sv, the
// settlement), with the trial-independent parts read from D.
__device__ inline int direct_level0(double x0, const Params& P, const Knobs& K,
                                    const DirectArgs& D, int b, double& p, long long& ne,
                                    int& flags) {
  p = 0.0;
  const double x = fabs(x0);
  if (!(D.ok && !((x - (P.t - P.st / 2.)) < 0))) return kFinal;
  const double a = P.a, sv = P.sv, t = P.t;
  const double v = D.v[b], w = D.w[b];
  ne += 1;
  const TNode T = tnode_setup_r(x - t, v, sv, a, D.ia2, K.err);
  if (T.amb) flags |= kFlagExact;
  if (T.pos) {
    const double f = tnode_ftt_sc(T, w, D.s1[b], D.tc[b]);
    if (sv == 0) {
      const double ex = exp_node(D.dn[b] - (T.vvx * 0.5));
      p = (f * ex) * T.sc;
    } else {
      p = tnode_pdf_sv(T, w, v, sv, a);  // (sv > 0: the general form)
    }
  }
  if (flags & kFlagExact) return kExact;
  if (p > kExactBelow || x - t <= 0) return kFinal;
  if (!tiny_absorbed(p, P.p_outlier, K.w_outlier)) return kExact;
  p = 0.0;
  return kFinal;
}

// P(hit upper boundary), pdf.pxi:67-72
__device__ inline double prob_ub(double v, double a, double z) {
  if (v == 0) return z;
  return (exp(((-2.0 * a) * z) * v) - 1.0) / (exp((-2.0 * a) * v) - 1.0);
}

}  // namespace wfpt
