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
 * Performance structure (so the CPU baseline is a credible stand-in for JAX/XLA-CPU): rows
 * are split over OpenMP threads; the inner loop runs over the columns j of a row with
 * `omp simd`, so exp/sin/cos vectorise through glibc's libmvec (built with -ffast-math);
 * square symmetric blocks evaluate only j <= i and mirror, exactly like the GPU path.
 *
 * kind: 0 SE_Cos_1d, 1 Matern52_Cos_1d, 2 SE_1d, 3 Matern52_1d.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SQRT5 2.23606797749978969641
#define TWO_PI 6.28318530717958647692

static inline int is_matern(int k) { return k == 1 || k == 3; }
static inline int has_cos(int k) { return k == 0 || k == 1; }

/* One row i of K (and D) over columns j in [0, jend): accumulate component q into kr/dr. */
static inline __attribute__((always_inline)) void row_kd_t(const int mat, const int deriv, double xi,
                                                            const double* x2, int jend, double w,
                                                            double a, double om, double* kr,
                                                            double* dr) {
#pragma omp simd
  for (int j = 0; j < jend; ++j) {
    const double diff = xi - x2[j];
    const double d = fabs(diff);
    double m0, m1, m2;
    if (mat) {
      const double r = SQRT5 * a * d, E = exp(-r);
      m0 = (1.0 + r + r * r * (1.0 / 3.0)) * E;
      m1 = -(SQRT5 / 3.0) * a * r * (1.0 + r) * E;
      m2 = (5.0 / 3.0) * a * a * (r * r - r - 1.0) * E;
    } else {
      const double g = exp(-a * d * d);
      m0 = g;
      m1 = -2.0 * a * d * g;
      m2 = (4.0 * a * a * d * d - 2.0 * a) * g;
    }
    /* non-cosine kinds pass om = 0: cos = 1, sin = 0 exactly */
    const double C = cos(om * d), S = sin(om * d);
    const double c0 = C, c1 = -om * S, c2 = -om * om * C;
    kr[j] += w * (m0 * c0);
    if (deriv == 2) dr[j] += w * (m2 * c0 + 2.0 * m1 * c1 + m0 * c2);
    if (deriv == 1) dr[j] += w * ((m1 * c0 + m0 * c1) * (diff >= 0.0 ? 1.0 : -1.0));
  }
}

static void row_kd(int kind, int deriv, double xi, const double* x2, int jend, double w,
                   double a, double f, double* kr, double* dr) {
  const double om = has_cos(kind) ? TWO_PI * f : 0.0;
  /* every (radial, deriv) combination gets its own branch-free simd loop */
  if (is_matern(kind)) {
    if (deriv == 2) row_kd_t(1, 2, xi, x2, jend, w, a, om, kr, dr);
    else if (deriv == 1) row_kd_t(1, 1, xi, x2, jend, w, a, om, kr, dr);
    else row_kd_t(1, 0, xi, x2, jend, w, a, om, kr, dr);
  } else {
    if (deriv == 2) row_kd_t(0, 2, xi, x2, jend, w, a, om, kr, dr);
    else if (deriv == 1) row_kd_t(0, 1, xi, x2, jend, w, a, om, kr, dr);
    else row_kd_t(0, 0, xi, x2, jend, w, a, om, kr, dr);
  }
}

/* K[n1*n2] (kappa, + jitter on i==j when add_jitter) and, if D != NULL, the deriv-order
 * derivative block (1: D_x1_kappa, 2: DD_x1_kappa).  Row-major, x1 indexes rows.
 * symmetric != 0 asserts x1 == x2 (square block): only j <= i is evaluated, then mirrored. */
void oracle_kd2(int kind, int deriv, const double* x1, int n1, const double* x2, int n2,
                const double* logw, const double* logls, const double* freq, int Q,
                double jitter, int add_jitter, int symmetric, double* K, double* D) {
  double* w = (double*)malloc(sizeof(double) * Q * 2);
  double* a = w + Q;
  for (int q = 0; q < Q; ++q) {
    w[q] = exp(logw[q]);
    a[q] = exp(logls[q]);
  }
#pragma omp parallel for schedule(dynamic, 8)
  for (int i = 0; i < n1; ++i) {
    const int jend = symmetric ? i + 1 : n2;
    double* kr = K + (size_t)i * n2;
    double* dr = D ? D + (size_t)i * n2 : NULL;
    double tmp[1];
    memset(kr, 0, sizeof(double) * jend);
    if (dr) memset(dr, 0, sizeof(double) * jend);
    for (int q = 0; q < Q; ++q)
      row_kd(kind, D ? deriv : 0, x1[i], x2, jend, w[q], a[q], freq[q], kr, dr ? dr : tmp);
    if (add_jitter && i < n2) kr[i] += jitter;
  }
  if (symmetric) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n1; ++i)
      for (int j = i + 1; j < n2; ++j) {
        K[(size_t)i * n2 + j] = K[(size_t)j * n2 + i];
        if (D) D[(size_t)i * n2 + j] = (deriv == 1) ? -D[(size_t)j * n2 + i] : D[(size_t)j * n2 + i];
      }
  }
  free(w);
}

/* legacy entry (full evaluation), kept for the tests */
void oracle_kd(int kind, int deriv, const double* x1, int n1, const double* x2, int n2,
               const double* logw, const double* logls, const double* freq, int Q,
               double jitter, int add_jitter, double* K, double* D) {
  oracle_kd2(kind, deriv, x1, n1, x2, n2, logw, logls, freq, Q, jitter, add_jitter, 0, K, D);
}

static inline __attribute__((always_inline)) void pg_row_t(const int mat, const int deriv, int jend,
                                                            const double* dd, const double* wk,
                                                            const double* wd, double aq, double om,
                                                            double* osf, double* osl, double* osw) {
  double sf = 0.0, sl = 0.0, sw = 0.0;
#pragma omp simd reduction(+ : sf, sl, sw)
  for (int j = 0; j < jend; ++j) {
    const double d = dd[j];
    double m0, m1, m2, m0l, m1l, m2l;
    if (mat) {
      const double r = SQRT5 * aq * d, E = exp(-r), r2 = r * r;
      const double ka = (SQRT5 / 3.0) * aq, k2 = (5.0 / 3.0) * aq * aq;
      m0 = (1.0 + r + r2 * (1.0 / 3.0)) * E;
      m1 = -ka * r * (1.0 + r) * E;
      m2 = k2 * (r2 - r - 1.0) * E;
      m0l = -(r2 * (1.0 / 3.0)) * (1.0 + r) * E;
      m1l = -ka * r * (2.0 + 2.0 * r - r2) * E;
      m2l = k2 * (-r2 * r + 5.0 * r2 - 2.0 * r - 2.0) * E;
    } else {
      const double d2 = d * d, g = exp(-aq * d2);
      m0 = g;
      m1 = -2.0 * aq * d * g;
      m2 = (4.0 * aq * aq * d2 - 2.0 * aq) * g;
      m0l = -aq * d2 * g;
      m1l = (-2.0 * aq * d + 2.0 * aq * aq * d2 * d) * g;
      m2l = (10.0 * aq * aq * d2 - 2.0 * aq - 4.0 * aq * aq * aq * d2 * d2) * g;
    }
    /* non-cosine kinds pass om = 0: cos = 1, sin = 0; their freq gradient is zeroed later */
    const double C = cos(om * d), S = sin(om * d);
    const double c0 = C, c1 = -om * S, c2 = -om * om * C;
    const double c0f = -TWO_PI * d * S;
    const double c1f = -TWO_PI * S - TWO_PI * om * d * C;
    const double c2f = -2.0 * TWO_PI * om * C + TWO_PI * om * om * d * S;
    const double fw = m0 * c0, fl = m0l * c0, ff = m0 * c0f;
    double dw, dl, df;
    if (deriv == 2) {
      dw = m2 * c0 + 2.0 * m1 * c1 + m0 * c2;
      dl = m2l * c0 + 2.0 * m1l * c1 + m0l * c2;
      df = m2 * c0f + 2.0 * m1 * c1f + m0 * c2f;
    } else if (deriv == 1) {
      dw = m1 * c0 + m0 * c1;
      dl = m1l * c0 + m0l * c1;
      df = m1 * c0f + m0 * c1f;
    } else {
      dw = dl = df = 0.0;
    }
    sw += wk[j] * fw + wd[j] * dw;
    sl += wk[j] * fl + wd[j] * dl;
    sf += wk[j] * ff + wd[j] * df;
  }
  *osf = sf;
  *osl = sl;
  *osw = sw;
}

/* out[0:Q] = dL/dfreq, out[Q:2Q] = dL/dlog-ls, out[2Q:3Q] = dL/dlog-w of
 *   sum_ij GK[i,j] K_ij(theta) + GD[i,j] D_ij(theta)   over an n x n block of x.
 * Pairs j < i carry the mirror's weight (K, DD symmetric; D_x1 sign folded into the weight). */
void oracle_param_grad(int kind, int deriv, const double* x, int n, const double* logw,
                       const double* logls, const double* freq, int Q, const double* GK,
                       const double* GD, double* out) {
  const int mat = is_matern(kind), cs = has_cos(kind);
  if (!GD) deriv = 0;
  double* w = (double*)malloc(sizeof(double) * Q * 2);
  double* a = w + Q;
  for (int q = 0; q < Q; ++q) {
    w[q] = exp(logw[q]);
    a[q] = exp(logls[q]);
  }
  memset(out, 0, sizeof(double) * 3 * Q);
  /* per-row partials, summed in row order afterwards: the result does not depend on the thread
   * count or the dynamic schedule (the GPU comparisons need a reproducible oracle) */
  double* rowp = (double*)calloc((size_t)n * 3 * Q, sizeof(double));
#pragma omp parallel
  {
    double* wk = (double*)malloc(sizeof(double) * n);
    double* wd = (double*)malloc(sizeof(double) * n);
    double* dd = (double*)malloc(sizeof(double) * n);
#pragma omp for schedule(dynamic, 8)
    for (int i = 0; i < n; ++i) {
      double* acc = rowp + (size_t)i * 3 * Q;
      /* weights of the unordered pairs (i, j), j <= i */
      for (int j = 0; j <= i; ++j) {
        const double diff = x[i] - x[j];
        const double sij = diff >= 0.0 ? 1.0 : -1.0, sji = -diff >= 0.0 ? 1.0 : -1.0;
        double gkij = GK[(size_t)i * n + j], gkji = GK[(size_t)j * n + i];
        double gdij = GD ? GD[(size_t)i * n + j] : 0.0, gdji = GD ? GD[(size_t)j * n + i] : 0.0;
        if (deriv == 1) {
          gdij *= sij;
          gdji *= sji;
        }
        dd[j] = fabs(diff);
        wk[j] = (j == i) ? gkij : gkij + gkji;
        wd[j] = (j == i) ? gdij : gdij + gdji;
      }
      for (int q = 0; q < Q; ++q) {
        const double aq = a[q], om = cs ? TWO_PI * freq[q] : 0.0;
        double sf = 0.0, sl = 0.0, sw = 0.0;
        if (mat) {
          if (deriv == 2) pg_row_t(1, 2, i + 1, dd, wk, wd, aq, om, &sf, &sl, &sw);
          else if (deriv == 1) pg_row_t(1, 1, i + 1, dd, wk, wd, aq, om, &sf, &sl, &sw);
          else pg_row_t(1, 0, i + 1, dd, wk, wd, aq, om, &sf, &sl, &sw);
        } else {
          if (deriv == 2) pg_row_t(0, 2, i + 1, dd, wk, wd, aq, om, &sf, &sl, &sw);
          else if (deriv == 1) pg_row_t(0, 1, i + 1, dd, wk, wd, aq, om, &sf, &sl, &sw);
          else pg_row_t(0, 0, i + 1, dd, wk, wd, aq, om, &sf, &sl, &sw);
        }
        acc[q] = sf;
        acc[Q + q] = sl;
        acc[2 * Q + q] = sw;
      }
    }
    free(wk);
    free(wd);
    free(dd);
  }
  for (int i = 0; i < n; ++i)
    for (int t = 0; t < 3 * Q; ++t) out[t] += rowp[(size_t)i * 3 * Q + t];
  free(rowp);
  for (int q = 0; q < Q; ++q) {
    out[q] *= w[q];
    out[Q + q] *= w[q];
    out[2 * Q + q] *= w[q];
    if (!cs) out[q] = 0.0;
  }
  free(w);
}
