// dd_dev.h — double-double arithmetic (error-free transforms on FMA) and the kernel fields'
// transcendentals to ~1e-30 relative, for the kernel-parameter contraction of large factors
// (pgrad.hip, DD): sum_c S_c f_c(theta) cancels ~1e8-fold at C5, so the fp64 rounding of the
// derivative fields f_c themselves -- not the solves -- sets its accuracy (DESIGN.md §3,
// tools/c5_kp_split.py).  Host and device (tools/probes/dd_check.hip checks exp / sincos against
// quad precision on the host).
#pragma once
#include <hip/hip_runtime.h>

// Error-free transforms need every product and sum rounded where it is written: HIP device code
// defaults to -ffp-contract=fast, which fuses a product into a LATER addition (e.g. two_prod's
// a*b into quick's a + b) and silently breaks them (measured: 1e-10 relative on the GPU, exact
// on the host).  Every function here switches contraction off for its own body.
#define DD_EXACT _Pragma("clang fp contract(off)")

namespace gpk {
namespace dd {

struct D {
  double h, l;  // value h + l, |l| <= ulp(h) / 2
};

__host__ __device__ inline D two_sum(double a, double b) {
  DD_EXACT
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline D quick(double a, double b) {
  DD_EXACT  // |a| >= |b|
  const double s = a + b;
  return {s, b - (s - a)};
}
__host__ __device__ inline D two_prod(double a, double b) {
  DD_EXACT
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
__host__ __device__ inline D of(double a) {
  DD_EXACT return {a, 0.0}; }
__host__ __device__ inline D neg(D a) {
  DD_EXACT return {-a.h, -a.l}; }
__host__ __device__ inline D add(D a, D b) {
  DD_EXACT  // IEEE-style (accurate) addition
  D s = two_sum(a.h, b.h);
  const D t = two_sum(a.l, b.l);
  s.l += t.h;
  s = quick(s.h, s.l);
  s.l += t.l;
  return quick(s.h, s.l);
}
__host__ __device__ inline D sub(D a, D b) {
  DD_EXACT return add(a, neg(b)); }
__host__ __device__ inline D add_d(D a, double b) {
  DD_EXACT
  D s = two_sum(a.h, b);
  s.l += a.l;
  return quick(s.h, s.l);
}
__host__ __device__ inline D mul(D a, D b) {
  DD_EXACT
  D p = two_prod(a.h, b.h);
  p.l = fma(a.h, b.l, fma(a.l, b.h, p.l));
  return quick(p.h, p.l);
}
__host__ __device__ inline D mul_d(D a, double b) {
  DD_EXACT
  D p = two_prod(a.h, b);
  p.l = fma(a.l, b, p.l);
  return quick(p.h, p.l);
}
__host__ __device__ inline D div_d(D a, double b) {
  DD_EXACT
  const double q1 = a.h / b;
  const D p = two_prod(q1, b);
  const double r = ((a.h - p.h) - p.l) + a.l;
  return quick(q1, r / b);
}
__host__ __device__ inline D scale2(D a, int k) {
  DD_EXACT return {ldexp(a.h, k), ldexp(a.l, k)}; }  // exact

// e^x, x <= ~700 (e^x = 0 below -708): x = k ln2 + t, e^t = (1 + p(t / 512))^512 kept as
// expm1 through the nine squarings (q <- 2q + q^2), Taylor to t^9 / 9! (|t / 512| <= 6.8e-4)
__host__ __device__ inline D exp(D x) {
  DD_EXACT
  if (x.h < -708.0) return {0.0, 0.0};
  const double LN2_1 = 6.9314718055994529e-01, LN2_2 = 2.3190468138462996e-17, LN2_3 = 5.707708438416212e-34;
  const double k = rint(x.h / LN2_1);
  D t = sub(x, two_prod(k, LN2_1));
  t = sub(t, two_prod(k, LN2_2));
  t = add_d(t, -k * LN2_3);
  t = scale2(t, -9);
  // q = e^t - 1 = t + t^2/2 + ... + t^9/9!  (Horner: t (1 + t (1/2 + t (1/6 + ...))))
  D q = of(1.0 / 362880.0);
  q = add_d(mul(q, t), 1.0 / 40320.0);
  q = add_d(mul(q, t), 1.0 / 5040.0);
  q = add_d(mul(q, t), 1.0 / 720.0);
  q = add_d(mul(q, t), 1.0 / 120.0);
  q = add_d(mul(q, t), 1.0 / 24.0);
  q = add(mul(q, t), D{1.6666666666666666e-01, 9.2518585385429707e-18});  // 1/6
  q = add_d(mul(q, t), 0.5);
  q = add_d(mul(q, t), 1.0);
  q = mul(q, t);
  for (int i = 0; i < 9; ++i) q = add(scale2(q, 1), mul(q, q));  // (1 + q)^2 - 1
  return scale2(add_d(q, 1.0), (int)k);
}

// sin and cos of x (|x| up to ~1e5): x = k pi/2 + t (pi/2 in three parts), u = t / 16, Taylor to
// u^13 / u^12, four double-angle steps, quadrant by k mod 4
__host__ __device__ inline void sincos(D x, D& S, D& C) {
  DD_EXACT
  const double P1 = 1.5707963267948966e+00, P2 = 6.123233995736766e-17, P3 = -1.4973849048591698e-33;
  const double k = rint(x.h / P1);
  D t = sub(x, two_prod(k, P1));
  t = sub(t, two_prod(k, P2));
  t = add_d(t, -k * P3);
  const D u = scale2(t, -4);
  const D u2 = mul(u, u);
  D s = of(1.0 / 6227020800.0);  // 1/13!
  s = add_d(mul(s, u2), -1.0 / 39916800.0);
  s = add_d(mul(s, u2), 1.0 / 362880.0);
  s = add_d(mul(s, u2), -1.0 / 5040.0);
  s = add(mul(s, u2), D{8.3333333333333332e-03, 1.1564823173178714e-19});  // 1/120
  s = add(mul(s, u2), D{-1.6666666666666666e-01, -9.2518585385429707e-18});  // -1/6
  s = add_d(mul(s, u2), 1.0);
  s = mul(s, u);
  D c = of(1.0 / 479001600.0);  // 1/12!
  c = add_d(mul(c, u2), -1.0 / 3628800.0);
  c = add_d(mul(c, u2), 1.0 / 40320.0);
  c = add(mul(c, u2), D{-1.3888888888888889e-03, 5.3005439543735771e-20});  // -1/720
  c = add(mul(c, u2), D{4.1666666666666664e-02, 2.3129646346357427e-18});  // 1/24
  c = add_d(mul(c, u2), -0.5);
  c = add_d(mul(c, u2), 1.0);
  for (int i = 0; i < 4; ++i) {
    const D s2 = scale2(mul(s, c), 1);
    c = mul(sub(c, s), add(c, s));
    s = s2;
  }
  const long q = ((long)k) & 3;
  if (q == 0) { S = s; C = c; }
  else if (q == 1) { S = c; C = neg(s); }
  else if (q == 2) { S = neg(s); C = neg(c); }
  else { S = neg(c); C = s; }
}

}  // namespace dd
}  // namespace gpk
