// wfpt_exact.hpp — the exact path: full_pdf in the reference's literal
// expression order with correctly rounded transcendentals (wfpt_crlibm.hpp).
//
// Restates src/pdf.pxi:28-146 and src/integrate.pxi:12-206 operation for
// operation (no hoisting, no recurrences, no reciprocals): with glibc-equal
// exp/log/sin/pow(., 3) the result is the reference's double except where
// glibc itself misrounds (~0.1% of calls). It costs ~10x the fast path, and
// the kernels send a trial here only when its value hinges on last-bit
// rounding:
//   * its density is zero, negative, NaN or below kExactBelow (subnormal
//     roundings of intermediate values are ~1e-5 relative there);
//   * an adaptive stop test |S2 - S| <= 15 err sits inside kTieBand of its
//     threshold (the fast path's values carry ~1e-14 relative error);
//   * fixed Simpson (use_adaptive = 0) gives such a density.
// Host and device (WFPT_HD): tests/test_exact_path.py compiles it with gcc
// (tests/c/exact_host.cpp) and compares it with the reference fixtures and the
// oracle (bit for bit except where glibc misrounds).
#pragma once
#include "wfpt_crlibm.hpp"

#pragma clang fp contract(off)

namespace wfpt_x {

using namespace wfpt_cr;

constexpr double kPi = 3.14159265358979323846;
constexpr double kPi2 = kPi * kPi;
constexpr int kMaxDepth = 24;              // WFPT_MAX_DEPTH
constexpr long long kEvalBudget = 1ll << 24;  // WFPT_EVAL_BUDGET

// <int>(double) as the reference's x86-64 build converts (cvttsd2si): a value
// outside int's range, inf or NaN gives INT_MIN (the "integer indefinite"),
// where gfx950's conversion saturates. A non-finite term count (tt = 0 from
// an overflowing a, err = 0) thus runs no series term, as in the reference,
// instead of ~2^31 of them.
WFPT_HD int ref_int(double v) {
  return (v < 2147483648.0 && v > -2147483649.0) ? (int)v : (-2147483647 - 1);
}

// pdf.pxi:28-65
WFPT_HD double ftt_01w(double tt, double w, double err) {
  double kl, ks, p;
  if ((kPi * tt) * err < 1.0) {
    kl = sqrt((-2.0 * cr_log((kPi * tt) * err)) / (kPi2 * tt));
    const double b = 1. / (kPi * sqrt(tt));
    kl = (kl < b) ? b : kl;
  } else {
    kl = 1. / (kPi * sqrt(tt));
  }
  if ((2.0 * sqrt((2.0 * kPi) * tt)) * err < 1.0) {
    ks = 2.0 + sqrt((-2.0 * tt) * cr_log((2.0 * sqrt((2.0 * kPi) * tt)) * err));
    const double b = sqrt(tt) + 1.0;
    ks = (ks < b) ? b : ks;
  } else {
    ks = 2.0;
  }
  p = 0.0;
  if (ks < kl) {
    const int K = ref_int(ceil(ks));
    const int lower = ref_int(-floor((K - 1) / 2.));
    const int upper = ref_int(ceil((K - 1) / 2.));
    for (int k = lower; k <= upper; ++k) {
      const double wk = w + (double)(2 * k);
      p = p + wk * cr_exp(((-(wk * wk)) / 2.0) / tt);
    }
    p = p / sqrt((2.0 * kPi) * cr_cube(tt));
  } else {
    const int K = ref_int(ceil(kl));
    for (int k = 1; k <= K; ++k) {
      const double dk = (double)k;
      p = p + (dk * cr_exp((((-(dk * dk)) * kPi2) * tt) / 2.0)) * cr_sin((dk * kPi) * w);
    }
    p = p * kPi;
  }
  return p;
}

// pdf.pxi:74-85
WFPT_HD double pdf(double x, double v, double a, double w, double err) {
  if (x <= 0) return 0.0;
  const double tt = x / (a * a);
  const double p = ftt_01w(tt, w, err);
  return (p * cr_exp((((-v) * a) * w) - (((v * v) * x) / 2.))) / (a * a);
}

// pdf.pxi:87-102
WFPT_HD double pdf_sv(double x, double v, double sv, double a, double z, double err) {
  if (x <= 0) return 0.0;
  if (sv == 0) return pdf(x, v, a, z, err);
  const double tt = x / (a * a);
  const double p = ftt_01w(tt, z, err);
  const double azsv = (a * z) * sv;
  return (cr_exp(cr_log(p) + ((((azsv * azsv) - (((2.0 * a) * v) * z)) - ((v * v) * x)) /
                              (((2.0 * (sv * sv)) * x) + 2.0))) /
          sqrt(((sv * sv) * x) + 1.0)) /
         (a * a);
}

struct Ctx {
  long long ne = 0;  // pdf_sv evaluations
  int ovf = 0;       // 1: depth beyond kMaxDepth, 2: evaluation budget
};

struct Frame {
  double lb, ub, S, fb, fe, fm, err, left;
};

// adaptiveSimpsons_1D/_2D + Aux (integrate.pxi:72-206) over [lb0, ub0] as an
// explicit stack walk; g(u) already divides by ZT (or st). Children are
// visited left then right and combined as left + right, as the recursion does.
template <class G>
WFPT_HD double adaptive(G&& g, double lb0, double ub0, double err0, int depth, Ctx& C) {
  Frame stk[kMaxDepth];
  unsigned right = 0u;
  int sp = 0;
  double lb = lb0, ub = ub0, err = err0;
  const double h0 = ub - lb;
  const double c0 = (lb + ub) / 2.;
  double fb = g(lb), fe = g(ub), fm = g(c0);
  double S = (h0 / 6) * ((fb + (4 * fm)) + fe);
  int bottom = depth;
  for (;;) {
    if (C.ne > kEvalBudget) {
      C.ovf |= 2;
      return __builtin_nan("");
    }
    const double c = (ub + lb) / 2.;
    const double d = (lb + c) / 2., e = (c + ub) / 2.;
    const double h = ub - lb;
    const double fd = g(d), fee = g(e);
    const double Sl = (h / 12) * ((fb + (4 * fd)) + fm);
    const double Sr = (h / 12) * ((fm + (4 * fee)) + fe);
    const double S2 = Sl + Sr;
    if (!(bottom <= 0 || fabs(S2 - S) <= 15 * err)) {
      if (sp >= kMaxDepth) {
        C.ovf |= 1;
        return __builtin_nan("");
      }
      stk[sp] = Frame{c, ub, Sr, fm, fe, fee, err / 2, 0.0};
      ++sp;
      ub = c;
      err = err / 2;
      S = Sl;
      fe = fm;
      fm = fd;
      bottom -= 1;
      continue;
    }
    double val = S2 + (S2 - S) / 15;
    for (;;) {
      if (sp == 0) return val;
      const int top = sp - 1;
      if (!((right >> top) & 1u)) {
        const Frame fr = stk[top];
        stk[top].left = val;
        right |= 1u << top;
        lb = fr.lb;
        ub = fr.ub;
        S = fr.S;
        fb = fr.fb;
        fe = fr.fe;
        fm = fr.fm;
        err = fr.err;
        bottom = depth - sp;
        break;
      }
      val = stk[top].left + val;
      right &= ~(1u << top);
      --sp;
    }
  }
}

// integrate.pxi:12-45 (y = 0 where the reference leaves it uninitialised, n = 0)
WFPT_HD double simpson_1d(double x, double v, double sv, double a, double z, double t, double err,
                          double lb_z, double ub_z, int n_sz, double lb_t, double ub_t, int n_st,
                          Ctx& C) {
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
  ++C.ne;
  double S = pdf_sv(x - lb_t, v, sv, a, lb_z, err);
  double y = 0.0;
  for (int i = 1; i <= n; ++i) {
    const double z_tag = lb_z + hz * i;
    const double t_tag = lb_t + ht * i;
    ++C.ne;
    y = pdf_sv(x - t_tag, v, sv, a, z_tag, err);
    if (i & 1) S += (4 * y);
    else S += (2 * y);
  }
  S = S - y;
  S = S / ((ub_t - lb_t) + (ub_z - lb_z));
  return ((ht + hz) * S) / 3;
}

// integrate.pxi:47-70
WFPT_HD double simpson_2d(double x, double v, double sv, double a, double z, double err,
                          double lb_z, double ub_z, int n_sz, double lb_t, double ub_t, int n_st,
                          Ctx& C) {
  const double ht = (ub_t - lb_t) / n_st;
  double S = simpson_1d(x, v, sv, a, z, lb_t, err, lb_z, ub_z, n_sz, 0, 0, 0, C);
  double y = 0.0;
  for (int i_t = 1; i_t <= n_st; ++i_t) {
    const double t_tag = lb_t + ht * i_t;
    y = simpson_1d(x, v, sv, a, z, t_tag, err, lb_z, ub_z, n_sz, 0, 0, 0, C);
    if (i_t & 1) S += (4 * y);
    else S += (2 * y);
  }
  S = S - y;
  S = S / (ub_t - lb_t);
  return (ht * S) / 3;
}

// pdf.pxi:104-146
WFPT_HD double full_pdf(double x, double v, double sv, double a, double z, double sz, double t,
                        double st, double err, int n_st, int n_sz, int use_adaptive,
                        double simps_err, Ctx& C) {
  if ((z < 0) || (z > 1) || (a < 0) || (t < 0) || (st < 0) || (sv < 0) || (sz < 0) || (sz > 1) ||
      ((fabs(x) - (t - st / 2.)) < 0) || (z + sz / 2. > 1) || (z - sz / 2. < 0) ||
      (t - st / 2. < 0))
    return 0.0;
  if (x > 0) {
    v = -v;
    z = 1. - z;
  }
  x = fabs(x);
  if (st < 1e-3) st = 0;
  if (sz < 1e-3) sz = 0;
  if (sz == 0) {
    if (st == 0) {
      ++C.ne;
      return pdf_sv(x - t, v, sv, a, z, err);
    }
    if (use_adaptive > 0) {
      const double lb = t - st / 2., ub = t + st / 2., ZT = ub - lb;
      auto g = [&](double tc) -> double {
        ++C.ne;
        return pdf_sv(x - tc, v, sv, a, z, err) / ZT;
      };
      return adaptive(g, lb, ub, simps_err, n_st, C);
    }
    return simpson_1d(x, v, sv, a, z, t, err, z, z, 0, t - st / 2., t + st / 2., n_st, C);
  }
  if (st == 0) {
    if (use_adaptive) {
      const double lb = z - sz / 2., ub = z + sz / 2., ZT = ub - lb;
      auto g = [&](double zc) -> double {
        ++C.ne;
        return pdf_sv(x - t, v, sv, a, zc, err) / ZT;
      };
      return adaptive(g, lb, ub, simps_err, n_sz, C);
    }
    return simpson_1d(x, v, sv, a, z, t, err, z - sz / 2., z + sz / 2., n_sz, t, t, 0, C);
  }
  if (use_adaptive) {
    const double lb_z = z - sz / 2., ub_z = z + sz / 2., ZT = ub_z - lb_z;
    const double lb_t = t - st / 2., ub_t = t + st / 2., stw = ub_t - lb_t;
    auto outer = [&](double tc) -> double {
      auto inner = [&](double zc) -> double {
        ++C.ne;
        return pdf_sv(x - tc, v, sv, a, zc, err) / ZT;
      };
      return adaptive(inner, lb_z, ub_z, simps_err, n_sz, C) / stw;
    };
    return adaptive(outer, lb_t, ub_t, simps_err, n_st, C);
  }
  return simpson_2d(x, v, sv, a, z, err, z - sz / 2., z + sz / 2., n_sz, t - st / 2., t + st / 2.,
                    n_st, C);
}

}  // namespace wfpt_x
