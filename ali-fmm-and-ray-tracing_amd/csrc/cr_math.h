// cr_math.h — correctly rounded atan, sin, cos, tan in double precision, for host and device.
//
// The reference's operators call glibc's atan / sin / cos / tan (numba lowers math.* to libm);
// glibc's results are the correctly rounded ones on essentially every argument, ocml's differ in
// the last bit on about 1 % of them, and one such bit, once a node is accepted, propagates through
// every later update of the heap walk.  These evaluate each function in double-double arithmetic
// (error below 2^-85 relative) and round once, so the device reproduces glibc's bits wherever
// glibc is correctly rounded (checked against the host libm: tests/test_crmath.py).
//
//   atan: x -> u in [0, 1] (1/x as a double-double when |x| > 1), u = k/128 + ..., atan u =
//         atan(k/128) + atan(t), t = (u - k/128) / (1 + u k/128), |t| <= 2^-8, odd series in t.
//   sin/cos: x = j pi/128 + r (pi/128 in three parts, |r| <= pi/256), sin(j pi/128 + r) from the
//         quarter-period table and the series of sin r, cos r - 1.
// Valid for |x| < 2^14 (sin/cos/tan: the operators' angles are below 2 pi); beyond that, the
// libm function is used (never the case on the solver's paths).
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define CR_HD __host__ __device__ inline
// the double-double paths (~1 argument in 2^9); inlined: an out-of-line call costs the callers
// spills across it (measured slower in the band and init kernels)
#define CR_COLD __host__ __device__ inline
#else
#define CR_HD inline
#define CR_COLD inline
#endif
#define CR_TABLE static constexpr
#define CR_CONST static constexpr
#include "cr_tables.h"

namespace crm {

struct dd {
  double h, l;
};

CR_HD dd two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
CR_HD dd fast_two_sum(double a, double b) {  // |a| >= |b| (or a == 0)
  const double s = a + b;
  return {s, b - (s - a)};
}
CR_HD dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
CR_HD dd add(dd a, dd b) {
  dd s = two_sum(a.h, b.h);
  return fast_two_sum(s.h, s.l + (a.l + b.l));
}
CR_HD dd mul(dd a, dd b) {
  dd p = two_prod(a.h, b.h);
  return fast_two_sum(p.h, p.l + (a.h * b.l + a.l * b.h));
}
CR_HD dd div(dd a, dd b) {
  const double q = a.h / b.h;
  const double r = (fma(-q, b.h, a.h) + a.l) - q * b.l;
  return fast_two_sum(q, r / b.h);
}
// a / n for a small integer n (exact remainder through fma)
CR_HD dd div_n(dd a, double n) {
  const double h = a.h / n;
  return fast_two_sum(h, (fma(-h, n, a.h) + a.l) / n);
}
// Table reads.  A translation unit that defines CR_LDS_TABLES keeps the tables in LDS on the
// device (a table entry is then an LDS read instead of a dependent global load, which the
// latency-bound solver kernels would wait on): each of its kernels calls crm::lds_init() with
// all threads and synchronises before the first use.
constexpr int kTabWords = 2 * (129 + 65);
#if defined(__HIP_DEVICE_COMPILE__) && defined(CR_LDS_TABLES)
__shared__ double crm_lds_tab[kTabWords];
__device__ inline void lds_init() {
  for (int k = threadIdx.x; k < kTabWords; k += blockDim.x)
    crm_lds_tab[k] = k < 258 ? (&kAtanTab[0][0])[k] : (&kSinTab[0][0])[k - 258];
}
CR_HD dd tab_atan(int i) { return {crm_lds_tab[2 * i], crm_lds_tab[2 * i + 1]}; }
CR_HD dd tab_sin(int i) { return {crm_lds_tab[258 + 2 * i], crm_lds_tab[259 + 2 * i]}; }
#else
CR_HD void lds_init() {}
CR_HD dd tab_atan(int i) { return {kAtanTab[i][0], kAtanTab[i][1]}; }
CR_HD dd tab_sin(int i) { return {kSinTab[i][0], kSinTab[i][1]}; }
#endif

// atan(t) for a double-double |t| <= 2^-8 + 2^-20: t + t P(t^2), P = -q/3 + q^2 (1/5 - q/7 + ...)
CR_HD dd atan_small(dd t) {
  dd q = two_prod(t.h, t.h);
  q.l += 2.0 * t.h * t.l;
  const double x = q.h;
  const double R = ((((-1.0 / 15 * x + 1.0 / 13) * x - 1.0 / 11) * x + 1.0 / 9) * x - 1.0 / 7) * x + 1.0 / 5;
  const dd q3 = div_n(q, 3.0);
  const dd P = add({-q3.h, -q3.l}, {x * x * R, 0.0});
  return add(t, mul(t, P));
}

CR_COLD double atan_accurate(double x) {
  const double a = fabs(x);
  const bool inv = a > 1.0;
  dd u{a, 0.0};
  if (inv) {
    const double h = 1.0 / a;
    u = {h, fma(-h, a, 1.0) / a};
  }
  const int k = (int)(u.h * 128.0 + 0.5);
  const double c = k * (1.0 / 128);
  const dd n = two_sum(u.h - c, u.l);  // u.h - c exact (Sterbenz: c/2 <= u.h <= 2c for k >= 1)
  dd p = two_prod(u.h, c);
  p.l += u.l * c;
  dd d = two_sum(1.0, p.h);
  d = fast_two_sum(d.h, d.l + p.l);
  dd r = add(tab_atan(k), atan_small(div(n, d)));
  if (inv) r = add({kPio2H, kPio2L}, {-r.h, -r.l});
  return copysign(r.h + r.l, x);
}

// sin and cos of x as double-doubles (|x| < 2^14)
CR_COLD void sincos_dd(double x, dd& s, dd& c) {
  const double jd = nearbyint(x * k128OverPi);
  const int j = (int)jd;
  // r = x - j pi/128: j kP1 exact (33-bit kP1, |j| < 2^20), x - j kP1 exact (Sterbenz)
  const double r1 = x - jd * kP1;
  const dd p2 = two_prod(jd, kP2);
  dd r = two_sum(r1, -p2.h);
  r = fast_two_sum(r.h, (r.l - p2.l) - jd * kP3);
  // sin r = r + r S, cos r = 1 + C; q = r^2
  dd q = two_prod(r.h, r.h);
  q.l += 2.0 * r.h * r.l;
  const double y = q.h;
  const dd q2 = mul(q, q);
  const dd q6 = div_n(q, 6.0), q2_120 = div_n(q2, 120.0), q2_24 = div_n(q2, 24.0);
  const double ys = q2.h * y * ((-1.0 / 39916800 * y + 1.0 / 362880) * y - 1.0 / 5040);
  const double yc = q2.h * y * (((1.0 / 479001600 * y - 1.0 / 3628800) * y + 1.0 / 40320) * y - 1.0 / 720);
  const dd S = add(add({-q6.h, -q6.l}, q2_120), {ys, 0.0});  // sin r = r (1 + S)
  const dd C = add(add({-0.5 * q.h, -0.5 * q.l}, q2_24), {yc, 0.0});  // cos r = 1 + C
  // sin / cos of (j mod 256) pi/128 = qd pi/2 + a from the quarter-period table
  const int m = j & 255, qd = m >> 6, i = m & 63;
  const dd sa = tab_sin(i), ca = tab_sin(64 - i);
  const dd nsa{-sa.h, -sa.l}, nca{-ca.h, -ca.l};
  const dd sj = qd == 0 ? sa : qd == 1 ? ca : qd == 2 ? nsa : nca;
  const dd cj = qd == 0 ? ca : qd == 1 ? nsa : qd == 2 ? nca : sa;
  const dd sr = add(r, mul(r, S));  // sin r
  // sin x = sj + sj C + cj sin r ;  cos x = cj + cj C - sj sin r
  const dd ssr = mul(sj, sr);
  s = add(sj, add(mul(sj, C), mul(cj, sr)));
  c = add(cj, add(mul(cj, C), {-ssr.h, -ssr.l}));
}

// Fast paths: the same reductions with the series tails in double (error below 2^-63 of the
// result), then a rounding test: when the approximation's error interval straddles a rounding
// boundary (about 1 argument in 2^9), the double-double evaluation above decides.
CR_HD bool rounds_same(double h, double l, double e) { return h + (l + e) == h + (l - e); }

CR_HD double atan(double x) {
  const double a = fabs(x);
  if (!(a <= 0x1p60)) return a != a ? x + x : copysign(kPio2H, x);  // NaN; pi/2 - 1/a rounds to pi/2
  if (a < 0x1p-27) return x;  // |atan x - x| < |x|^3 / 3: below half an ulp
  const bool inv = a > 1.0;
  double uh = a, ul = 0.0;
  if (inv) {
    uh = 1.0 / a;
    ul = fma(-uh, a, 1.0) * uh;
  }
  const int k = (int)(uh * 128.0 + 0.5);
  const double c = k * (1.0 / 128);
  const double nh = uh - c;  // exact (Sterbenz)
  const double ph = uh * c, pl = fma(uh, c, -ph) + ul * c;
  const double dh = 1.0 + ph, dl = ((1.0 - dh) + ph) + pl;  // 1 >= |ph|
  const double th = nh / dh;
  const double tl = ((fma(-th, dh, nh) + ul) - th * dl) / dh;
  const double q = th * th;
  const double tP = th * q * ((((1.0 / 13 * q - 1.0 / 11) * q + 1.0 / 9) * q - 1.0 / 7) * q * q + (1.0 / 5 * q - 1.0 / 3));
  // atan u = A_k + t + t P
  const dd A = tab_atan(k);
  dd r = two_sum(A.h, th);
  r.l += (A.l + tl) + tP;
  if (inv) {
    dd v = two_sum(kPio2H, -r.h);
    v.l += kPio2L - r.l;
    r = v;
  }
  const double h = r.h + r.l, l = r.l - (h - r.h);
  if (rounds_same(h, l, fabs(h) * 0x1p-63)) return copysign(h, x);
  return copysign(atan_accurate(a), x);
}

// sin x ~ s + ls and cos x ~ c + lc (|x| < 2^14), each within 2^-62 of the result relative to it
// (the bound the rounding tests below rely on)
CR_HD void sincos_fast(double x, double& s, double& ls, double& c, double& lc) {
  const double jd = nearbyint(x * k128OverPi);
  const int j = (int)jd;
  const double r1 = x - jd * kP1;
  const double p2h = jd * kP2, p2l = fma(jd, kP2, -p2h);
  const double rh0 = r1 - p2h;
  const double rl0 = ((r1 - rh0) - p2h) - p2l - jd * kP3;  // r1 - rh0 - p2h exact (|r1| >= |p2h|)
  const double rh = rh0 + rl0, rl = rl0 - (rh - rh0);
  const double q = rh * rh;
  const double S = q * ((((-1.0 / 39916800 * q + 1.0 / 362880) * q - 1.0 / 5040) * q + 1.0 / 120) * q - 1.0 / 6);
  const double C = q * ((((1.0 / 3628800 * -q + 1.0 / 40320) * q - 1.0 / 720) * q + 1.0 / 24) * q - 0.5);
  const int m = j & 255, qd = m >> 6, i = m & 63;
  const dd sa = tab_sin(i), ca = tab_sin(64 - i);
  const dd nsa{-sa.h, -sa.l}, nca{-ca.h, -ca.l};
  const dd sj = qd == 0 ? sa : qd == 1 ? ca : qd == 2 ? nsa : nca;
  const dd cj = qd == 0 ? ca : qd == 1 ? nsa : qd == 2 ? nca : sa;
  // sin r = r + r S with r = rh + rl: rh + (rl + rh S)
  const double sr_l = rl + rh * S;
  // sin x = sj + cj rh + [sj C + cj (rl + rh S) + cj_l rh + sj_l]
  const dd ps = two_prod(cj.h, rh);
  const dd s0 = two_sum(sj.h, ps.h);
  const double sl = s0.l + (ps.l + sj.l + sj.h * C + cj.h * sr_l + cj.l * rh);
  // cos x = cj - sj rh + [cj C - sj (rl + rh S) - sj_l rh + cj_l]
  const dd pc = two_prod(-sj.h, rh);
  const dd c0 = two_sum(cj.h, pc.h);
  const double cl = c0.l + (pc.l + cj.l + cj.h * C - sj.h * sr_l - sj.l * rh);
  s = s0.h + sl;
  c = c0.h + cl;
  ls = sl - (s - s0.h);
  lc = cl - (c - c0.h);
}

CR_HD void sincos(double x, double* sp, double* cp) {
  if (!(fabs(x) < 0x1p14)) {
    *sp = ::sin(x);
    *cp = ::cos(x);
    return;
  }
  double s, ls, c, lc;
  sincos_fast(x, s, ls, c, lc);
  if (rounds_same(s, ls, fabs(s) * 0x1p-62) && rounds_same(c, lc, fabs(c) * 0x1p-62)) {
    *sp = fabs(x) < 0x1p-26 ? x : s;
    *cp = c;
    return;
  }
  dd sd, cd;
  sincos_dd(x, sd, cd);
  *sp = fabs(x) < 0x1p-26 ? x : sd.h + sd.l;
  *cp = cd.h + cd.l;
}

CR_HD double sin(double x) {
  double s, c;
  sincos(x, &s, &c);
  return s;
}
CR_HD double cos(double x) {
  double s, c;
  sincos(x, &s, &c);
  return c;
}
// tan = sin / cos from the fast path's pairs (relative error below 2^-61 + the quotient's
// 2^-104), rounding test at 2^-59; the double-double evaluation decides the rest
CR_HD double tan(double x) {
  if (!(fabs(x) < 0x1p14)) return ::tan(x);
  if (fabs(x) < 0x1p-27) return x;
  double sh, sl, ch, cl;
  sincos_fast(x, sh, sl, ch, cl);
  const double q = sh / ch;
  const double r = ((fma(-q, ch, sh) + sl) - q * cl) / ch;
  const double h = q + r, l = r - (h - q);
  if (rounds_same(h, l, fabs(h) * 0x1p-59)) return h;
  dd s, c;
  sincos_dd(x, s, c);
  const dd t = div(s, c);
  return t.h + t.l;
}

}  // namespace crm
