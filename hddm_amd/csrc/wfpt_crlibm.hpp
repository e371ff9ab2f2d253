// wfpt_crlibm.hpp — correctly rounded exp / log / sin / cube for the exact path.
//
// The reference's CPU build evaluates exp, log, sin and pow(tt, 3.) with
// glibc's libm, whose results are correctly rounded in all but ~0.05% of
// calls (its FMA and non-FMA variants disagree that often). gfx950's OCML
// differs from glibc in 1-24% of calls (tools/libm_probe.hip, measured). The
// exact path (wfpt_exact.hpp) is used for the rare trials whose result hinges
// on last-bit rounding (subnormal / zero densities, near-ties of the adaptive
// stop test), so there every transcendental is evaluated in double-double
// (~2^-100 relative) and rounded once: the same double as glibc except where
// glibc itself misrounds. Double-double primitives use fma() for exact
// products; nothing here depends on FMA contraction of plain expressions.
//
// Host and device: tests/test_crlibm.py compiles this header with gcc and
// checks it against glibc and against exact rational arithmetic.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define WFPT_HD __host__ __device__ inline
#else
#define WFPT_HD static inline
#endif

#pragma clang fp contract(off)

namespace wfpt_cr {

struct dd {
  double hi, lo;
};

WFPT_HD dd two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return dd{s, (a - (s - bb)) + (b - bb)};
}
WFPT_HD dd fast_two_sum(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return dd{s, b - (s - a)};
}
WFPT_HD dd two_prod(double a, double b) {
  const double p = a * b;
  return dd{p, fma(a, b, -p)};
}
WFPT_HD dd dd_add(dd x, dd y) {
  dd s = two_sum(x.hi, y.hi);
  const dd t = two_sum(x.lo, y.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
WFPT_HD dd dd_add_d(dd x, double y) {
  dd s = two_sum(x.hi, y);
  s.lo += x.lo;
  return fast_two_sum(s.hi, s.lo);
}
WFPT_HD dd dd_mul(dd x, dd y) {
  dd p = two_prod(x.hi, y.hi);
  p.lo += x.hi * y.lo + x.lo * y.hi;
  return fast_two_sum(p.hi, p.lo);
}
WFPT_HD dd dd_mul_d(dd x, double y) {
  dd p = two_prod(x.hi, y);
  p.lo += x.lo * y;
  return fast_two_sum(p.hi, p.lo);
}

// Round (x.hi + x.lo) * 2^e to the nearest double once (normal, subnormal or
// overflow): the value is first brought into [1, 2) by an exact scaling.
WFPT_HD double dd_ldexp_round(dd x, int e) {
  if (x.hi == 0.0) return x.hi;
  int ex;
  (void)frexp(x.hi, &ex);  // x.hi in [2^(ex-1), 2^ex)
  const int te = ex - 1 + e;  // exponent of the result
  if (te >= -1022) {
    // normal range: x.hi is already the rounded dd value (|lo| <= ulp/2);
    // a tie (|lo| == ulp/2 exactly) is resolved by the sum
    const double r = x.hi + x.lo;
    return ldexp(r, e);
  }
  // subnormal: quantum 2^-1074. Scale so the quantum becomes 2^-52 relative
  // to 1: y = x * 2^(e + 1022) in (0, 1), then round 1 + y at 2^-52 once.
  const double sign = x.hi < 0 ? -1.0 : 1.0;
  const double yh = ldexp(fabs(x.hi), e + 1022);
  const double yl = ldexp(x.hi < 0 ? -x.lo : x.lo, e + 1022);
  const double s = 1.0 + yh;
  const double err = (1.0 - s) + yh;
  const double r = s + (err + yl);
  return sign * ldexp(r - 1.0, -1022);
}

constexpr double kLn2H = 0x1.62e42fefa39efp-1, kLn2M = 0x1.abc9e3b39803fp-56,
                 kLn2L = 0x1.7b57a079a1934p-111;
constexpr double kInvLn2 = 0x1.71547652b82fep+0;

// 1/n! as double-double, n = 0..16 (exact rationals rounded, tools: Python
// decimal at 80 digits)
WFPT_HD dd inv_fact(int n) {
  switch (n) {
    case 0: case 1: return dd{1.0, 0.0};
    case 2: return dd{0x1.0p-1, 0.0};
    case 3: return dd{0x1.5555555555555p-3, 0x1.5555555555555p-57};
    case 4: return dd{0x1.5555555555555p-5, 0x1.5555555555555p-59};
    case 5: return dd{0x1.1111111111111p-7, 0x1.1111111111111p-63};
    case 6: return dd{0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65};
    case 7: return dd{0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73};
    case 8: return dd{0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76};
    case 9: return dd{0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73};
    case 10: return dd{0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76};
    case 11: return dd{0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80};
    case 12: return dd{0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83};
    case 13: return dd{0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87};
    case 14: return dd{0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92};
    case 15: return dd{0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97};
    case 16: return dd{0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101};
    case 17: return dd{0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103};
    case 18: return dd{0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107};
    case 19: return dd{0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112};
    case 20: return dd{0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120};
    case 21: return dd{0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120};
    case 22: return dd{0x1.0ce396db7f853p-70, -0x1.aebcdbd20331cp-124};
    case 23: return dd{0x1.761b41316381ap-75, -0x1.3423c7d91404fp-130};
    case 24: return dd{0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135};
    case 25: return dd{0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139};
    case 26: return dd{0x1.88e85fc6a4e5ap-89, -0x1.71c37ebd16540p-143};
    case 27: return dd{0x1.d1ab1c2dccea3p-94, 0x1.054d0c78aea14p-149};
    case 28: return dd{0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153};
    default: return dd{0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157};  // 29
  }
}

// exp(x) = 2^k * exp(r) as an unrounded double-double times 2^k.
// |r| <= ln2/2; exp(r) = exp(r / 64)^64 with a degree-11 Taylor polynomial.
WFPT_HD dd exp_dd(double x, int* k_out) {
  const double kd = rint(x * kInvLn2);
  // r = x - k ln2, ln2 in three parts, every product exact in two_prod form
  dd r = dd_add(dd{x, 0.0}, [&] { const dd p = two_prod(kd, kLn2H); return dd{-p.hi, -p.lo}; }());
  r = dd_add(r, [&] { const dd p = two_prod(kd, kLn2M); return dd{-p.hi, -p.lo}; }());
  r = dd_add_d(r, -(kd * kLn2L));
  const dd rs{ldexp(r.hi, -6), ldexp(r.lo, -6)};
  dd p = inv_fact(11);
  for (int n = 10; n >= 0; --n) p = dd_add(dd_mul(p, rs), inv_fact(n));
  for (int i = 0; i < 6; ++i) p = dd_mul(p, p);
  *k_out = (int)kd;
  return p;
}

WFPT_HD double cr_exp(double x) {
  if (x != x) return x;
  if (x > 709.79) return INFINITY;
  if (x < -746.0) return 0.0;
  int k;
  const dd p = exp_dd(x, &k);
  return dd_ldexp_round(p, k);
}

// log(m), m in [sqrt(1/2), sqrt(2)), as a double-double.
WFPT_HD dd log_mant_dd(double m) {
  const double u = m - 1.0;  // exact (Sterbenz)
  if (fabs(u) < 0x1p-5) {
    // log(1 + u) = 2 atanh(s), s = u / (2 + u): s^2 < 2.5e-4, 11 odd terms
    const dd den = two_sum(2.0, u);
    // s = u / den in double-double: q0 = u / den.hi, correct with the residual
    const double q0 = u / den.hi;
    const dd qd = dd_mul_d(den, q0);
    const double rem = ((u - qd.hi) - qd.lo);
    const double q1 = rem / den.hi;
    const dd s = fast_two_sum(q0, q1);
    const dd s2 = dd_mul(s, s);
    dd acc{1.0 / 23.0, 0.0};
    for (int n = 21; n >= 1; n -= 2) {
      // 1/n as double-double
      const double h = 1.0 / n;
      const double l = fma(-h, (double)n, 1.0) / n;
      acc = dd_add(dd_mul(acc, s2), dd{h, l});
    }
    const dd r = dd_mul(acc, s);
    return dd{2.0 * r.hi, 2.0 * r.lo};
  }
  // Newton step on exp: y1 = y0 + (m e^-y0 - 1) - (m e^-y0 - 1)^2 / 2
  const double y0 = log(m);
  int k;
  dd e = exp_dd(-y0, &k);
  e = dd{ldexp(e.hi, k), ldexp(e.lo, k)};
  const dd me = dd_mul_d(e, m);
  const dd t = dd_add_d(me, -1.0);
  const dd t2 = dd_mul(t, t);
  dd y = dd_add(dd{y0, 0.0}, t);
  y = dd_add(y, dd{-0.5 * t2.hi, -0.5 * t2.lo});
  return y;
}

WFPT_HD double cr_log(double x) {
  if (x != x || x < 0) return __builtin_nan("");
  if (x == 0) return -INFINITY;
  if (x == INFINITY) return x;
  int e;
  double m = frexp(x, &e);  // [0.5, 1)
  if (m < 0.7071067811865476) {
    m *= 2.0;
    e -= 1;
  }
  const dd lm = log_mant_dd(m);
  const double ed = (double)e;
  // e ln2 in three parts: e * kLn2H is exact in two_prod form
  dd s = two_prod(ed, kLn2H);
  s = dd_add(s, two_prod(ed, kLn2M));
  s = dd_add_d(s, ed * kLn2L);
  const dd y = dd_add(s, lm);
  return y.hi + y.lo;
}

// pi/2 in four Cody-Waite parts (33, 33, 29 bits, then a full double)
constexpr double kPio2_1 = 0x1.921fb544p+0, kPio2_2 = 0x1.0b4611a6p-34,
                 kPio2_3 = 0x1.3198a2ep-69, kPio2_4 = 0x1.b839a252049c1p-104;
constexpr double kTwoOverPi = 0x1.45f306dc9c883p-1;

// sin / cos of a double-double |r| <= pi/4 + tiny: Taylor to degree 29 / 28
WFPT_HD dd sin_dd(dd r) {
  const dd r2 = dd_mul(r, r);
  dd p = inv_fact(29);
  for (int n = 27; n >= 1; n -= 2) {
    p = dd_mul(p, r2);
    const dd c = inv_fact(n);
    p = ((n >> 1) & 1) ? dd_add(p, dd{-c.hi, -c.lo}) : dd_add(p, c);  // (-1)^((n-1)/2) / n!
  }
  return dd_mul(p, r);
}
WFPT_HD dd cos_dd(dd r) {
  const dd r2 = dd_mul(r, r);
  dd p = inv_fact(28);
  for (int n = 26; n >= 0; n -= 2) {
    p = dd_mul(p, r2);
    const dd c = inv_fact(n);
    p = ((n >> 1) & 1) ? dd_add(p, dd{-c.hi, -c.lo}) : dd_add(p, c);
  }
  return p;
}

// sin(x) for |x| < 2^20 (the exact path's arguments are k pi w, k <= a few
// hundred); larger arguments fall back to the platform sin.
WFPT_HD double cr_sin(double x) {
  if (x != x) return x;
  if (fabs(x) >= 0x1p20) return sin(x);
  if (x == 0) return x;
  const double nd = rint(x * kTwoOverPi);
  // r = x - n pi/2: x - n P1 is exact (n < 2^21, P1 has 33 bits, Sterbenz)
  const double r1 = x - nd * kPio2_1;
  dd r = two_sum(r1, -(nd * kPio2_2));  // n * P2 exact (21 + 33 bits)
  r = dd_add_d(r, -(nd * kPio2_3));     // exact product
  r = dd_add(r, dd{-(nd * kPio2_4), -fma(nd, kPio2_4, -(nd * kPio2_4))});
  const long long n = (long long)nd;
  const int q = (int)(n & 3);
  dd v;
  if (q == 0) v = sin_dd(r);
  else if (q == 1) v = cos_dd(r);
  else if (q == 2) { v = sin_dd(r); v = dd{-v.hi, -v.lo}; }
  else { v = cos_dd(r); v = dd{-v.hi, -v.lo}; }
  return v.hi + v.lo;
}

// x^3 correctly rounded (the reference's pow(tt, 3.)); exact double-double
// product, scaled so that no partial product leaves the normal range.
WFPT_HD double cr_cube(double x) {
  if (x != x || x == 0 || isinf(x)) return x * x * x;
  int e;
  const double m = frexp(x, &e);  // |m| in [0.5, 1): m^3 exact in dd+ (<= 159 bits)
  const dd m2 = two_prod(m, m);
  dd m3 = two_prod(m2.hi, m);
  const dd t = two_prod(m2.lo, m);
  m3 = dd_add(m3, t);
  return dd_ldexp_round(m3, 3 * e);
}

}  // namespace wfpt_cr
