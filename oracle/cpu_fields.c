/* CPU oracle helper (TEST INFRASTRUCTURE / CPU BASELINE ONLY — never shipped, never on the
 * product path).  Plain-C OpenMP restatement of the O(N^2 Q) elementwise half of the
 * reference's hot path:
 *
 *   - kappa / D_x1_kappa / DD_x1_kappa blocks   code/kernel_matrix.py:21-30, :49-57, :114-193
 *   - the parameter-gradient contraction that jax.grad pushes through vmap(kappa) and
 *     vmap(grad(grad(kappa)))                   code/model_GP_solver_2d.py:107-117,179
 *
 * Closed forms: SURVEY.md Appendix B (same formulas as oracle/gp_oracle.py, which is the
 * pure-NumPy statement this file is tested against in tests/test_oracle.py).  Dense linear
 * algebra of the CPU baseline stays in NumPy/SciPy (OpenBLAS LU), as in gp_oracle.py.
 *
 * kind: 0 SE_Cos_1d, 1 Matern52_Cos_1d, 2 SE_1d, 3 Matern52_1d.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SQRT5 2.23606797749978969641
#define TWO_PI 6.28318530717958647692

typedef struct {
  double m0, m1, m2, m0l, m1l, m2l;
} radial_t;
typedef struct {
  double c0, c1, c2, c0f, c1f, c2f;
} cosine_t;

static inline void radial(int kind, double d, double a, int want_l, radial_t* o) {
  if (kind == 1 || kind == 3) { /* Matern52: r = sqrt5 a d (code/kernel_matrix.py:147-151) */
    double r = SQRT5 * a * d, E = exp(-r);
    double ka = SQRT5 * a / 3.0, k2 = 5.0 * a * a / 3.0;
    o->m0 = (1.0 + r + r * r / 3.0) * E;
    o->m1 = -ka * r * (1.0 + r) * E;
    o->m2 = k2 * (r * r - r - 1.0) * E;
    if (want_l) {
      o->m0l = -(r * r / 3.0) * (1.0 + r) * E;
      o->m1l = -ka * r * (2.0 + 2.0 * r - r * r) * E;
      o->m2l = k2 * (-r * r * r + 5.0 * r * r - 2.0 * r - 2.0) * E;
    }
  } else { /* SE: exp(-d^2 e^{log-ls}) (code/kernel_matrix.py:125) */
    double d2 = d * d, g = exp(-a * d2);
    o->m0 = g;
    o->m1 = -2.0 * a * d * g;
    o->m2 = (4.0 * a * a * d2 - 2.0 * a) * g;
    if (want_l) {
      o->m0l = -a * d2 * g;
      o->m1l = (-2.0 * a * d + 2.0 * a * a * d2 * d) * g;
      o->m2l = (10.0 * a * a * d2 - 2.0 * a - 4.0 * a * a * a * d2 * d2) * g;
    }
  }
}

static inline void cosine(int kind, double d, double f, int want_f, cosine_t* o) {
  if (kind == 0 || kind == 1) { /* cos(2 pi f d) (code/kernel_matrix.py:127,153) */
    double w = TWO_PI * f, C = cos(w * d), S = sin(w * d);
    o->c0 = C;
    o->c1 = -w * S;
    o->c2 = -w * w * C;
    if (want_f) {
      o->c0f = -TWO_PI * d * S;
      o->c1f = -TWO_PI * S - TWO_PI * w * d * C;
      o->c2f = -2.0 * TWO_PI * w * C + TWO_PI * w * w * d * S;
    }
  } else {
    o->c0 = 1.0;
    o->c1 = o->c2 = o->c0f = o->c1f = o->c2f = 0.0;
  }
}

/* K[n1*n2] (kappa, + jitter on i==j when add_jitter) and, if D != NULL, the deriv-order
 * derivative block (1: D_x1_kappa, 2: DD_x1_kappa).  Row-major, x1 indexes rows. */
void oracle_kd(int kind, int deriv, const double* x1, int n1, const double* x2, int n2,
               const double* logw, const double* logls, const double* freq, int Q,
               double jitter, int add_jitter, double* K, double* D) {
  double* w = (double*)malloc(sizeof(double) * Q * 2);
  double* a = w + Q;
  for (int q = 0; q < Q; ++q) {
    w[q] = exp(logw[q]);
    a[q] = exp(logls[q]);
  }
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n1; ++i) {
    for (int j = 0; j < n2; ++j) {
      double diff = x1[i] - x2[j];
      double d = fabs(diff), s = diff >= 0.0 ? 1.0 : -1.0; /* JAX abs' (0) = +1 */
      double k = 0.0, dv = 0.0;
      for (int q = 0; q < Q; ++q) {
        radial_t m;
        cosine_t c;
        radial(kind, d, a[q], 0, &m);
        cosine(kind, d, freq[q], 0, &c);
        k += w[q] * (m.m0 * c.c0);
        if (deriv == 1)
          dv += w[q] * (m.m1 * c.c0 + m.m0 * c.c1);
        else if (deriv == 2)
          dv += w[q] * (m.m2 * c.c0 + 2.0 * m.m1 * c.c1 + m.m0 * c.c2);
      }
      if (add_jitter && i == j) k += jitter;
      K[(size_t)i * n2 + j] = k;
      if (D) D[(size_t)i * n2 + j] = deriv == 1 ? dv * s : dv;
    }
  }
  free(w);
}

/* out[0:Q] = dL/dfreq, out[Q:2Q] = dL/dlog-ls, out[2Q:3Q] = dL/dlog-w of
 *   sum_ij GK[i,j] K_ij(theta) + GD[i,j] D_ij(theta)   over an n x n block of x. */
void oracle_param_grad(int kind, int deriv, const double* x, int n, const double* logw,
                       const double* logls, const double* freq, int Q, const double* GK,
                       const double* GD, double* out) {
  double* w = (double*)malloc(sizeof(double) * Q * 2);
  double* a = w + Q;
  for (int q = 0; q < Q; ++q) {
    w[q] = exp(logw[q]);
    a[q] = exp(logls[q]);
  }
  memset(out, 0, sizeof(double) * 3 * Q);
#pragma omp parallel
  {
    double* acc = (double*)calloc(3 * Q, sizeof(double));
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) {
      for (int j = 0; j < n; ++j) {
        double diff = x[i] - x[j];
        double d = fabs(diff), s = diff >= 0.0 ? 1.0 : -1.0;
        double gk = GK[(size_t)i * n + j], gd = GD ? GD[(size_t)i * n + j] : 0.0;
        for (int q = 0; q < Q; ++q) {
          radial_t m;
          cosine_t c;
          radial(kind, d, a[q], 1, &m);
          cosine(kind, d, freq[q], 1, &c);
          double fw = gk * (m.m0 * c.c0), fl = gk * (m.m0l * c.c0), ff = gk * (m.m0 * c.c0f);
          if (deriv == 2) {
            fw += gd * (m.m2 * c.c0 + 2.0 * m.m1 * c.c1 + m.m0 * c.c2);
            fl += gd * (m.m2l * c.c0 + 2.0 * m.m1l * c.c1 + m.m0l * c.c2);
            ff += gd * (m.m2 * c.c0f + 2.0 * m.m1 * c.c1f + m.m0 * c.c2f);
          } else if (deriv == 1) {
            double gs = gd * s;
            fw += gs * (m.m1 * c.c0 + m.m0 * c.c1);
            fl += gs * (m.m1l * c.c0 + m.m0l * c.c1);
            ff += gs * (m.m1 * c.c0f + m.m0 * c.c1f);
          }
          acc[q] += ff;
          acc[Q + q] += fl;
          acc[2 * Q + q] += fw;
        }
      }
    }
#pragma omp critical
    for (int t = 0; t < 3 * Q; ++t) out[t] += acc[t];
    free(acc);
  }
  for (int q = 0; q < Q; ++q) {
    out[q] *= w[q];
    out[Q + q] *= w[q];
    out[2 * Q + q] *= w[q];
    if (!(kind == 0 || kind == 1)) out[q] = 0.0;
  }
  free(w);
}
