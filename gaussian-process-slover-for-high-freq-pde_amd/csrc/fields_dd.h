// fields_dd.h — the kernel-parameter contraction's derivative fields in double-double (pgrad.hip
// DD; host-checked against quad precision by tools/probes/dd_check.hip).
#pragma once
#include "gpk_internal.h"
#include "dd_dev.h"

namespace gpk {

// The six derivative fields of one mixture component at distance d in double-double (DD): the
// same formulas as the fp64 loop of pgrad_kernel (oracle/gp_oracle.py param_grad_contract,
// code/kernel_matrix.py:114-193), on the exact arguments sqrt5 a d / a d^2 and (om + oml) d.
template <bool MATERN, bool COS, int DERIV>
__host__ __device__ inline void fields_dd(double d, double a, double om, double oml, dd::D& fw, dd::D& fl,
                                          dd::D& ff, dd::D& dw, dd::D& dl, dd::D& df) {
  DD_EXACT
  using namespace dd;
  D m0, m1, m2, m0l, m1l, m2l;
  if (MATERN) {
    const D p = two_prod(SQRT5, a);            // sqrt5 a
    const D r = mul_d(p, d), r2 = mul(r, r);
    const D E = dd::exp(neg(r));
    const D ka = div_d(p, 3.0);                // sqrt5 a / 3
    const D k2 = div_d(mul_d(two_prod(a, a), 5.0), 3.0);  // 5 a^2 / 3
    const D r2t = div_d(r2, 3.0), opr = add_d(r, 1.0), kar = mul(ka, r);
    m0 = mul(add(opr, r2t), E);
    m1 = neg(mul(mul(kar, opr), E));
    m2 = mul(mul(k2, add_d(sub(r2, r), -1.0)), E);
    m0l = neg(mul(mul(r2t, opr), E));
    m1l = neg(mul(mul(kar, sub(add_d(scale2(r, 1), 2.0), r2)), E));
    m2l = mul(mul(k2, add_d(sub(add(neg(mul(r2, r)), mul_d(r2, 5.0)), scale2(r, 1)), -2.0)), E);
  } else {
    const D d2 = two_prod(d, d), t = mul_d(d2, a), g = dd::exp(neg(t));
    const D ad = two_prod(a, d), a2 = two_prod(a, a), a2d2 = mul(a2, d2);
    m0 = g;
    m1 = neg(mul(scale2(ad, 1), g));
    m2 = mul(add_d(scale2(a2d2, 2), -2.0 * a), g);
    m0l = neg(mul(t, g));
    m1l = mul(add(neg(scale2(ad, 1)), scale2(mul_d(a2d2, d), 1)), g);
    m2l = mul(add(add_d(mul_d(a2d2, 10.0), -2.0 * a), neg(scale2(mul(mul_d(a2, a), mul(d2, d2)), 2))), g);
  }
  if (COS) {
    const D w = {om, oml};                     // 2 pi f, exactly
    D S, C;
    dd::sincos(mul_d(w, d), S, C);
    const D wS = mul(w, S), wC = mul(w, C), w2 = mul(w, w);
    const D c0 = C, c1 = neg(wS), c2 = neg(mul(w2, C));
    const D c0f = neg(mul_d(mul_d(S, d), TWO_PI));
    const D c1f = sub(neg(mul_d(S, TWO_PI)), mul_d(mul_d(wC, d), TWO_PI));
    const D c2f = add(neg(mul_d(wC, 2.0 * TWO_PI)), mul_d(mul_d(mul(w2, S), d), TWO_PI));
    fw = mul(m0, c0);
    fl = mul(m0l, c0);
    ff = mul(m0, c0f);
    if (DERIV == 2) {
      dw = add(add(mul(m2, c0), scale2(mul(m1, c1), 1)), mul(m0, c2));
      dl = add(add(mul(m2l, c0), scale2(mul(m1l, c1), 1)), mul(m0l, c2));
      df = add(add(mul(m2, c0f), scale2(mul(m1, c1f), 1)), mul(m0, c2f));
    } else {
      dw = add(mul(m1, c0), mul(m0, c1));
      dl = add(mul(m1l, c0), mul(m0l, c1));
      df = add(mul(m1, c0f), mul(m0, c1f));
    }
  } else {
    fw = m0;
    fl = m0l;
    ff = of(0.0);
    dw = DERIV == 2 ? m2 : m1;
    dl = DERIV == 2 ? m2l : m1l;
    df = of(0.0);
  }
}

}  // namespace gpk
