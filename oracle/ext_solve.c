/* Extended-precision (x87 80-bit long double) LU factorisation and solves -- TEST INFRASTRUCTURE.
 *
 * The oracle's "exact arithmetic" yardstick (gp_oracle.set_extended): jnp.linalg.solve /
 * slogdet (LAPACK getrf + getrs, partial pivoting; reference call sites
 * code/model_GP_solver_2d.py:104-105,157-162, code/model_GP_solver_1d.py:92,135-137) restated in
 * long double (eps 5.4e-20), so that the fp64 solves of the oracle and of the device can both be
 * measured against a value whose own rounding error is ~2000x smaller.  Same algorithm as the
 * NumPy long-double loops in gp_oracle.py (_ext_lu_py / _ext_solve_py), blocked (NB rows /
 * columns) and OpenMP over rows so that the 4096-point factors of config C5 take seconds.
 *
 * Layout: row-major; LU holds L (unit lower, below the diagonal) and U; perm[i] is the original
 * row now at position i.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NB 64
#define JB 512 /* rhs columns per inner block: one 8-KB row chunk stays in L1 */

static void swap_rows(long double* A, int n, int a, int b) {
  long double* ra = A + (size_t)a * n;
  long double* rb = A + (size_t)b * n;
  for (int j = 0; j < n; ++j) { const long double t = ra[j]; ra[j] = rb[j]; rb[j] = t; }
}

/* in place, partial pivoting (right-looking, NB-column panels); 0, or k+1 on a zero pivot */
int ld_lu(int n, long double* A, int* perm) {
  for (int i = 0; i < n; ++i) perm[i] = i;
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int k1 = k0 + NB < n ? k0 + NB : n;
    /* panel: columns [k0, k1) of rows [k0, n), unblocked with row swaps across the full width */
    for (int k = k0; k < k1; ++k) {
      int p = k;
      long double best = fabsl(A[(size_t)k * n + k]);
      for (int i = k + 1; i < n; ++i) {
        const long double v = fabsl(A[(size_t)i * n + k]);
        if (v > best) { best = v; p = i; }
      }
      if (best == 0.0L) return k + 1;
      if (p != k) {
        swap_rows(A, n, k, p);
        const int t = perm[k]; perm[k] = perm[p]; perm[p] = t;
      }
      const long double* rk = A + (size_t)k * n;
      const long double piv = rk[k];
#pragma omp parallel for schedule(static)
      for (int i = k + 1; i < n; ++i) {
        long double* ri = A + (size_t)i * n;
        const long double l = ri[k] / piv;
        ri[k] = l;
        for (int j = k + 1; j < k1; ++j) ri[j] -= l * rk[j];
      }
    }
    if (k1 == n) break;
    /* U12 = L11^{-1} A12 (rows [k0, k1), columns [k1, n)) */
    for (int k = k0; k < k1; ++k) {
      const long double* rk = A + (size_t)k * n;
      for (int i = k + 1; i < k1; ++i) {
        long double* ri = A + (size_t)i * n;
        const long double l = ri[k];
        for (int j = k1; j < n; ++j) ri[j] -= l * rk[j];
      }
    }
    /* A22 -= L21 U12: each row of A22 stays in cache while the NB rows of U12 stream by */
#pragma omp parallel for schedule(static)
    for (int i = k1; i < n; ++i) {
      long double* ri = A + (size_t)i * n;
      int k = k0;
      for (; k + 4 <= k1; k += 4) {
        const long double c0 = ri[k], c1 = ri[k + 1], c2 = ri[k + 2], c3 = ri[k + 3];
        const long double* r0 = A + (size_t)k * n;
        const long double* r1 = r0 + n;
        const long double* r2 = r1 + n;
        const long double* r3 = r2 + n;
        for (int j = k1; j < n; ++j) ri[j] = ri[j] - c0 * r0[j] - c1 * r1[j] - c2 * r2[j] - c3 * r3[j];
      }
      for (; k < k1; ++k) {
        const long double l = ri[k];
        const long double* rk = A + (size_t)k * n;
        for (int j = k1; j < n; ++j) ri[j] -= l * rk[j];
      }
    }
  }
  return 0;
}

/* X = A^{-1} B for nrhs columns: B [n][nrhs] fp64 row-major -> X [n][nrhs] fp64, rounded once
 * from the long double result.  Blocked by NB rows: the diagonal block is solved, then every
 * later (earlier) row is updated by the block's NB rows (cache-resident) in parallel. */
void ld_lu_solve(int n, const long double* LU, const int* perm, int nrhs, const double* B, double* X) {
  long double* W = (long double*)malloc((size_t)n * nrhs * sizeof(long double));
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    const double* b = B + (size_t)perm[i] * nrhs;
    long double* w = W + (size_t)i * nrhs;
    for (int j = 0; j < nrhs; ++j) w[j] = (long double)b[j];
  }
  /* L (unit lower) */
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int k1 = k0 + NB < n ? k0 + NB : n;
    for (int k = k0; k < k1; ++k)
      for (int i = k + 1; i < k1; ++i) {
        const long double l = LU[(size_t)i * n + k];
        long double* wi = W + (size_t)i * nrhs;
        const long double* wk = W + (size_t)k * nrhs;
        for (int j = 0; j < nrhs; ++j) wi[j] -= l * wk[j];
      }
#pragma omp parallel for schedule(static)
    for (int i = k1; i < n; ++i) {
      long double* wi = W + (size_t)i * nrhs;
      for (int j0 = 0; j0 < nrhs; j0 += JB) {
        const int j1 = j0 + JB < nrhs ? j0 + JB : nrhs;
        int k = k0;
        for (; k + 4 <= k1; k += 4) {  /* 4 rows per pass: one 80-bit store per 4 products */
          const long double* c = LU + (size_t)i * n + k;
          const long double c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
          const long double* w0 = W + (size_t)k * nrhs;
          const long double* w1 = w0 + nrhs;
          const long double* w2 = w1 + nrhs;
          const long double* w3 = w2 + nrhs;
          for (int j = j0; j < j1; ++j) wi[j] = wi[j] - c0 * w0[j] - c1 * w1[j] - c2 * w2[j] - c3 * w3[j];
        }
        for (; k < k1; ++k) {
          const long double l = LU[(size_t)i * n + k];
          const long double* wk = W + (size_t)k * nrhs;
          for (int j = j0; j < j1; ++j) wi[j] -= l * wk[j];
        }
      }
    }
  }
  /* U (upper), bottom block first */
  for (int k1 = n; k1 > 0; k1 -= NB) {
    const int k0 = k1 - NB > 0 ? k1 - NB : 0;
    for (int k = k1 - 1; k >= k0; --k) {
      long double* wk = W + (size_t)k * nrhs;
      const long double d = LU[(size_t)k * n + k];
      for (int j = 0; j < nrhs; ++j) wk[j] /= d;
      for (int i = k0; i < k; ++i) {
        const long double u = LU[(size_t)i * n + k];
        long double* wi = W + (size_t)i * nrhs;
        for (int j = 0; j < nrhs; ++j) wi[j] -= u * wk[j];
      }
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < k0; ++i) {
      long double* wi = W + (size_t)i * nrhs;
      for (int j0 = 0; j0 < nrhs; j0 += JB) {
        const int j1 = j0 + JB < nrhs ? j0 + JB : nrhs;
        int k = k0;
        for (; k + 4 <= k1; k += 4) {  /* 4 rows per pass: one 80-bit store per 4 products */
          const long double* c = LU + (size_t)i * n + k;
          const long double c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
          const long double* w0 = W + (size_t)k * nrhs;
          const long double* w1 = w0 + nrhs;
          const long double* w2 = w1 + nrhs;
          const long double* w3 = w2 + nrhs;
          for (int j = j0; j < j1; ++j) wi[j] = wi[j] - c0 * w0[j] - c1 * w1[j] - c2 * w2[j] - c3 * w3[j];
        }
        for (; k < k1; ++k) {
          const long double u = LU[(size_t)i * n + k];
          const long double* wk = W + (size_t)k * nrhs;
          for (int j = j0; j < j1; ++j) wi[j] -= u * wk[j];
        }
      }
    }
  }
#pragma omp parallel for schedule(static)
  for (size_t e = 0; e < (size_t)n * nrhs; ++e) X[e] = (double)W[e];
  free(W);
}

/* sum log|U_kk| in long double, returned rounded to double */
double ld_lu_logabsdet(int n, const long double* LU) {
  long double s = 0.0L;
  for (int k = 0; k < n; ++k) s += logl(fabsl(LU[(size_t)k * n + k]));
  return (double)s;
}

void ld_from_double(size_t n, const double* a, long double* out) {
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) out[i] = (long double)a[i];
}
