// Host check of csrc/dd_dev.h's exp and sincos against quad precision (libquadmath): worst
// relative error over arguments spanning the kernel fields' ranges (tools/probes, not the product).
#include <quadmath.h>
#include <cstdio>
#include <cstdlib>
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/fields_dd.h"

using gpk::dd::D;
static __float128 q(D a) { return (__float128)a.h + (__float128)a.l; }
static D from(__float128 x) { double h = (double)x; double l = (double)(x - (__float128)h); return {h, l}; }

int main() {
  srand(7);
  double we = 0, ws = 0, wc = 0;
  for (int i = 0; i < 200000; ++i) {
    const double u = rand() / (double)RAND_MAX;
    // exp: -r, r in [0, 60] (Matern's sqrt5 a d; SE's a d^2)
    const __float128 r = (__float128)(60.0 * u) + (__float128)(u * 1e-17);
    const D e = gpk::dd::exp(from(-r));
    const __float128 ex = expq(-r);
    const double re = (double)fabsq((q(e) - ex) / ex);
    if (re > we) we = re;
    // sincos: phase in [0, 1200]
    const __float128 x = (__float128)(1200.0 * u) + (__float128)(u * 3e-14);
    D S, C;
    gpk::dd::sincos(from(x), S, C);
    const __float128 sx = sinq(x), cx = cosq(x);
    const double rs = (double)fabsq(q(S) - sx), rc = (double)fabsq(q(C) - cx);  // absolute (|sin| <= 1)
    if (rs > ws) ws = rs;
    if (rc > wc) wc = rc;
  }
  // the six derivative fields (Matern52_Cos, DERIV 1 and 2) against the same formulas in quad
  // precision (oracle/gp_oracle.py _radial / _cosine with the fp64 constants)
  double wf = 0;
  for (int i = 0; i < 20000; ++i) {
    const double d = rand() / (double)RAND_MAX, a = 1.0 + 40.0 * rand() / (double)RAND_MAX;
    const double f = 40.0 * rand() / (double)RAND_MAX, om = gpk::TWO_PI * f;
    const double oml = fma(gpk::TWO_PI, f, -om);
    for (int deriv = 1; deriv <= 2; ++deriv) {
      D F[6];
      if (deriv == 1) gpk::fields_dd<true, true, 1>(d, a, om, oml, F[0], F[1], F[2], F[3], F[4], F[5]);
      else gpk::fields_dd<true, true, 2>(d, a, om, oml, F[0], F[1], F[2], F[3], F[4], F[5]);
      const __float128 Q5 = (__float128)gpk::SQRT5, TP = (__float128)gpk::TWO_PI, A = a, Dd = d;
      const __float128 r = Q5 * A * Dd, E = expq(-r);
      const __float128 m0 = (1 + r + r * r / 3) * E, m1 = -(Q5 * A / 3) * r * (1 + r) * E;
      const __float128 m2 = (5 * A * A / 3) * (r * r - r - 1) * E, m0l = -(r * r / 3) * (1 + r) * E;
      const __float128 m1l = -(Q5 * A / 3) * r * (2 + 2 * r - r * r) * E;
      const __float128 m2l = (5 * A * A / 3) * (-r * r * r + 5 * r * r - 2 * r - 2) * E;
      const __float128 w = TP * (__float128)f, C = cosq(w * Dd), S = sinq(w * Dd);
      const __float128 c0 = C, c1 = -w * S, c2 = -w * w * C, c0f = -TP * Dd * S;
      const __float128 c1f = -TP * S - TP * w * Dd * C, c2f = -2 * TP * w * C + TP * w * w * Dd * S;
      __float128 R[6] = {m0 * c0, m0l * c0, m0 * c0f, 0, 0, 0};
      if (deriv == 2) {
        R[3] = m2 * c0 + 2 * m1 * c1 + m0 * c2; R[4] = m2l * c0 + 2 * m1l * c1 + m0l * c2; R[5] = m2 * c0f + 2 * m1 * c1f + m0 * c2f;
      } else {
        R[3] = m1 * c0 + m0 * c1; R[4] = m1l * c0 + m0l * c1; R[5] = m1 * c0f + m0 * c1f;
      }
      // error relative to the field's scale at this point (|m| |c| products: no cancellation scale)
      const __float128 sc = (fabsq(m0) + fabsq(m1) + fabsq(m2) + fabsq(m0l) + fabsq(m1l) + fabsq(m2l)) * (1 + fabsq(w) * fabsq(w)) * (1 + TP * (1 + Dd) * (1 + fabsq(w)));
      for (int x = 0; x < 6; ++x) {
        if (sc == 0) continue;
        const double e = (double)(fabsq(q(F[x]) - R[x]) / sc);
        if (e > wf) wf = e;
      }
    }
  }
  std::printf("fields_dd: worst error / field scale %.3e\n", wf);
  std::printf("dd exp: worst relative error %.3e over r in [0, 60]\n", we);
  std::printf("dd sincos: worst absolute error sin %.3e cos %.3e over x in [0, 1200]\n", ws, wc);
  return (we < 1e-27 && ws < 1e-27 && wc < 1e-27 && wf < 1e-26) ? 0 : 1;
}
