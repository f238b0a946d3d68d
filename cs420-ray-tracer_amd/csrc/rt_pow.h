// rt_pow.h -- pow(x, y) for the specular term when the shininess is not a
// whole number (the reference: pow(r_dot_v, mat.shininess), include/scene.h:113,
// glibc; the shininess is any double the parser accepts, scene_loader.h:66-70).
//
// glibc's pow is correctly rounded except in a small fraction of cases (its
// documented bound is 0.52 ulp); ocml's fp64 pow is not (14 % of the
// renderer's operands differ from glibc by an ulp, tests/test_gpu_powcheck.py).
// dd_pow computes x^y = exp(y ln x) in double-double to ~2^-85 relative and
// rounds once, so it is the correctly rounded x^y except within ~2^-30 ulp of a
// rounding boundary: it differs from glibc only where glibc is not correctly
// rounded (tests/test_pow.py measures both against a 256-bit reference).
//
//   ln x = e ln2 + logc[i] + log1p(r): x = 2^e m, i = the top 7 bits of m's
//          mantissa, r = fma(m, invc[i], -1) exact (invc[i] a multiple of
//          1/256, |r| < 2^-7); log1p(r) = r - r^2/2 + r^3/3 - r^4/4 (double-
//          double) + r^5 (1/5 - r/6 + ... + r^8/13) (double).
//   z    = y ln x (double-double); |z| > 700 is refused (the caller falls back
//          to ocml's pow: such results are below 1e-304 or above 1e304).
//   x^y  = 2^(k/128) exp(r'): k = rint(z 128/ln2), r' = z - k ln2/128 (ln2/128
//          in three parts, the first exact times k), |r'| <= 2^-8.5;
//          exp(r') - 1 = r' + r'^2/2 + r'^3/6 (double-double) + r'^4/24 +
//          r'^5 (1/5! + ... + r'^4/9!) (double); 2^(j/128) from the table;
//          T + T (exp(r') - 1) summed exactly up to a round-to-odd remainder,
//          then rounded once.
// Constants: rt_pow_tables.h, generated in 60-digit decimal arithmetic by
// scripts/gen_pow_tables.py.  Only IEEE +, -, *, fma and rint are used, so
// the host build (tests/native/pow_host.cpp, g++ -ffp-contract=off) returns
// the same bits as the device.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define RTP_FN __device__ __forceinline__
#define RTP_TAB static __device__ const
#else
#define RTP_FN static inline
#define RTP_TAB static const
#endif
#define RTP_CONST static constexpr

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace rtk {

#include "rt_pow_tables.h"

struct DDv {
  double h, l;
};
RTP_FN DDv dd_two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return DDv{s, (a - (s - bb)) + (b - bb)};
}
RTP_FN DDv dd_fast2(double a, double b) {  // |a| >= |b| or a == 0
  const double s = a + b;
  return DDv{s, b - (s - a)};
}
RTP_FN DDv dd_add(DDv a, DDv b) {  // accurate under cancellation
  DDv s = dd_two_sum(a.h, b.h);
  const DDv t = dd_two_sum(a.l, b.l);
  s.l += t.h;
  s = dd_fast2(s.h, s.l);
  s.l += t.l;
  return dd_fast2(s.h, s.l);
}
RTP_FN DDv dd_mul(DDv a, DDv b) {
  const double p = a.h * b.h;
  double e = __builtin_fma(a.h, b.h, -p);
  e += a.h * b.l + a.l * b.h;
  return dd_fast2(p, e);
}

// x > 0 finite, y finite, 0 < |y| <= 2^16: the operands dd_pow takes.
RTP_FN bool dd_pow_ok(double x, double y) {
  return x > 0.0 && x <= 0x1.fffffffffffffp1023 && y != 0.0 && y >= -65536.0 && y <= 65536.0;
}

// x^y for dd_pow_ok operands, in `out`; false when |y ln x| > 700.
RTP_FN bool dd_pow(double x, double y, double &out) {
  uint64_t ix = __builtin_bit_cast(uint64_t, x);
  int e = (int)(ix >> 52) - 1023;
  if ((ix >> 52) == 0) {  // subnormal x: scale by 2^54 (exact)
    ix = __builtin_bit_cast(uint64_t, x * 0x1p54);
    e = (int)(ix >> 52) - 1023 - 54;
  }
  const int i = (int)((ix >> 45) & 127);
  const double m = __builtin_bit_cast(double, (ix & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  const double r = __builtin_fma(m, kPowInvc[i], -1.0);  // exact: |r| < 2^-7 (generator)
  const double ef = (double)(e + (i >> 6));               // i >= 64: m/2, exponent + 1
  // log1p(r)
  const double r2h = r * r, r2l = __builtin_fma(r, r, -r2h);
  const DDv r3 = dd_mul(DDv{r2h, r2l}, DDv{r, 0.0});
  const double r4h = r2h * r2h;
  const DDv r4 = dd_fast2(r4h, __builtin_fma(r2h, r2h, -r4h) + 2.0 * r2h * r2l);
  double t = kPowLogTail[8];
  for (int k = 7; k >= 0; --k) t = t * r + kPowLogTail[k];
  DDv acc = dd_add(DDv{-0.25 * r4.h, -0.25 * r4.l}, DDv{(r4h * r) * t, 0.0});
  acc = dd_add(acc, dd_mul(r3, DDv{kPowThirdHi, kPowThirdLo}));
  acc = dd_add(acc, DDv{-0.5 * r2h, -0.5 * r2l});
  acc = dd_add(acc, DDv{r, 0.0});
  // ln x = e ln2 + logc + log1p(r)
  const double p = ef * kPowLn2Hi;
  const DDv l2 = dd_fast2(p, __builtin_fma(ef, kPowLn2Hi, -p) + ef * kPowLn2Lo);
  const DDv lnx = dd_add(dd_add(l2, DDv{kPowLogc[i][0], kPowLogc[i][1]}), acc);
  // z = y ln x
  const DDv z = dd_mul(lnx, DDv{y, 0.0});
  if (!(z.h >= -700.0 && z.h <= 700.0)) return false;
  // exp(z) = 2^(k/128) exp(r')
  const double kd = __builtin_rint(z.h * kPowInvLn2N);
  const int k = (int)kd;
  const DDv t1 = dd_two_sum(z.h, -(kd * kPowLn2N1));  // kd * L1 exact (|k| < 2^18, L1 has 35 bits)
  const double p2 = kd * kPowLn2N2, p2e = __builtin_fma(kd, kPowLn2N2, -p2);
  const DDv s = dd_two_sum(t1.h, -p2);
  const DDv rr = dd_two_sum(s.h, (((t1.l + z.l) - p2e) - kd * kPowLn2N3) + s.l);
  const double rh = rr.h;
  const double q2h = rh * rh;
  const DDv q2 = dd_fast2(q2h, __builtin_fma(rh, rh, -q2h) + 2.0 * rh * rr.l);
  const DDv q3 = dd_mul(q2, rr);
  double w = kPowExpTail[5];
  for (int j = 4; j >= 1; --j) w = w * rh + kPowExpTail[j];
  const double q4 = q2.h * q2.h;
  DDv em = dd_add(dd_mul(q3, DDv{kPowSixthHi, kPowSixthLo}), DDv{q4 * kPowExpTail[0] + (q4 * rh) * w, 0.0});
  em = dd_add(em, DDv{0.5 * q2.h, 0.5 * q2.l});
  em = dd_add(em, rr);  // exp(r') - 1
  // 2^(j/128) exp(r') = T + T em, T = Th + Tl: the leading sum exactly, the
  // rest rounded to odd so the last rounding is the correct one even where the
  // result lies next to a midpoint (x within a few ulps of 1: (1 - 2^-53)^1.5
  // = 1 - 1.5 2^-53 + 0.375 2^-106 must not round like the midpoint)
  const int j = k & 127, sc = k >> 7;  // k = 128 sc + j (arithmetic shift: floor)
  const double Th = kPowExp2[j][0], Tl = kPowExp2[j][1];
  const DDv Tem = dd_mul(DDv{Th, Tl}, em);
  const DDv s0 = dd_two_sum(Th, Tem.h);  // exact
  const DDv u = dd_two_sum(Tl, Tem.l), v = dd_two_sum(s0.l, u.h);
  const DDv wv = dd_two_sum(v.h, v.l + u.l);
  double wo = wv.h;
  if (wv.l != 0.0) {  // round to odd: an inexact even w moves to its odd neighbour towards the exact sum
    const uint64_t b = __builtin_bit_cast(uint64_t, wv.h);
    if (!(b & 1)) wo = __builtin_bit_cast(double, ((wv.l > 0.0) == (wv.h > 0.0)) ? b + 1 : b - 1);
  }
  out = (s0.h + wo) * __builtin_bit_cast(double, (uint64_t)(sc + 1023) << 52);  // |sc| <= 1010: exact
  return true;
}

}  // namespace rtk
