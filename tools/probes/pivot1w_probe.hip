// Probe: single-wave register-resident 32x32 Cholesky + L^{-1} (candidate pivot factorisation)
// vs libgpk's 4-wave LDS version (spd_pivot.h).  One workgroup; timing by wall clock over
// repeated factorisations inside one launch; correctness vs the LDS version.
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/spd_pivot.h"
#include <cstdio>
#include <vector>
#include <cmath>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

using namespace gpk;

// Wave 0 only (lanes 0..63): lane l owns column c = l & 31, rows 16h..16h+15 (h = l >> 5) of A
// and M = L^{-1}, in registers.  Step k: the owners of row k publish A[k][:] and M[k][:] to LDS
// (they updated them last step); every lane reads p = A[k][k], A[k][c], M[k][c] and the row-k
// values A[k][i] of its 16 rows (= column k by symmetry), then updates in registers.
// No barriers: one wave, LDS ops are in order.  M rows are scaled lazily (as spd_pivot.h).
__device__ __forceinline__ double pivot_1wave(const double* Ain, double* Mout, double* rowA,
                                              double* rowM, double* pv, int lane, int* status) {
  const int c = lane & 31, h = lane >> 5;
  double a[16], m[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    a[r] = Ain[(16 * h + r) * SP + c];
    m[r] = (16 * h + r == c) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int hk = k >> 4, rk = k & 15;
    if (h == hk) {                 // owners of row k publish it
      rowA[(k & 1) * 32 + c] = a[rk];
      rowM[(k & 1) * 32 + c] = m[rk];
    }
    __builtin_amdgcn_wave_barrier();
    const double* ra = rowA + (k & 1) * 32;
    const double p = ra[k];
    const double akc = ra[c];
    const double mkc0 = rowM[(k & 1) * 32 + c];
    double aki[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) aki[r] = ra[16 * h + r];
    const double rs = rsqrt_f64(p);
    if (lane == 0) pv[k] = p;
    const double lck = akc * rs, mkc = mkc0 * rs;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 16 * h + r;
      const double lik = aki[r] * rs;
      if (i > k) {
        if (c > k) a[r] = fma(-lik, lck, a[r]);
        m[r] = fma(-lik, mkc, m[r]);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = 16 * h + r;
    Mout[i * SP + c] = m[r] * rsqrt_f64(pv[i]);
  }
  const double pk = pv[lane & 31];
  if (lane < 32 && !(pk > 0.0)) atomicOr(status, 1);
  double ls = (lane < 32) ? log(pk) : 0.0;
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  return ls;
}


// Blocked (b = 4) right-looking variant, 4 waves, thread t: column c = t&31, rows i0 + 8r.
// Per 4-column block B: every thread factors the 4x4 diagonal block D = L_D L_D^T redundantly in
// registers (W = L_D^{-1}), forms its panel rows l_iB = A_iB W^T, updates its trailing elements
// and its L^{-1} rows (X_B = W M_B; M_i -= l_iB X_B).  One barrier per block (8 per pivot).
// A and M are register-resident; LDS only carries the values other threads need.
__device__ __forceinline__ double pivot_blocked4(double* A, double* M, double* pv, int t, int* status) {
  const int c = t & 31, i0 = t >> 5;
  double a[4], m[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = A[(i0 + 8 * r) * SP + c];
    m[r] = (i0 + 8 * r == c) ? 1.0 : 0.0;
    M[(i0 + 8 * r) * SP + c] = m[r];
  }
  __syncthreads();
  double ls = 0.0;
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    const int b0 = 4 * kb;
    // reads: D (lower), row i panel A[i][B] for own rows, A[c][B], M[B][c]
    double D[4][4], aiB[4][4], acB[4], mB[4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int y = 0; y < 4; ++y) aiB[r][y] = A[(i0 + 8 * r) * SP + b0 + y];
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      acB[y] = A[c * SP + b0 + y];
      mB[y] = M[(b0 + y) * SP + c];
    }
    // 4x4 Cholesky (redundant per thread): L (lower), rinv[x] = 1/L_xx
    double L[4][4], rinv[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      double s = D[x][x];
#pragma unroll
      for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
      if (t == 0) pv[b0 + x] = s;
      rinv[x] = rsqrt_f64(s);
      L[x][x] = s * rinv[x];
#pragma unroll
      for (int y = x + 1; y < 4; ++y) {
        double q = D[y][x];
#pragma unroll
        for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
        L[y][x] = q * rinv[x];
      }
    }
    // W = L^{-1} (lower): W_xx = rinv_x, W_yx = -rinv_y sum_{z=x}^{y-1} L_yz W_zx
    double W[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      W[x][x] = rinv[x];
#pragma unroll
      for (int y = x + 1; y < 4; ++y) {
        double q = 0.0;
#pragma unroll
        for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
        W[y][x] = -q * rinv[y];
      }
    }
    // l_cB = A_cB W^T ; X_B = W m_B (column c of the new L^{-1} rows B)
    double lc[4], X[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      double q = 0.0, u = 0.0;
#pragma unroll
      for (int z = 0; z <= x; ++z) {
        q = fma(acB[z], W[x][z], q);
        u = fma(W[x][z], mB[z], u);
      }
      lc[x] = q;
      X[x] = u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 8 * r;
      if (i >= b0 && i < b0 + 4) {
        m[r] = X[i - b0];        // final row of L^{-1} (not re-published: nobody reads it again)
      } else if (i >= b0 + 4) {
        double li[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          double q = 0.0;
#pragma unroll
          for (int z = 0; z <= x; ++z) q = fma(aiB[r][z], W[x][z], q);
          li[x] = q;
        }
        double na = a[r], nm = m[r];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          if (c >= b0 + 4) na = fma(-li[x], lc[x], na);
          nm = fma(-li[x], X[x], nm);
        }
        a[r] = na;
        m[r] = nm;
      }
    }
    __syncthreads();  // everyone has read block kb's inputs
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 8 * r;
      if (i >= b0 + 4) {
        A[i * SP + c] = a[r];
        M[i * SP + c] = m[r];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(i0 + 8 * r) * SP + c] = m[r];
  if (t < 64) {
    const double pk = pv[t & 31];
    if (t < 32 && !(pk > 0.0)) atomicOr(status, 1);
    ls = (t < 32) ? log(pk) : 0.0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  }
  __syncthreads();
  return ls;
}

// Blocked (b = 4) right-looking variant, 4 waves, thread t: column c = t&31, rows i0 + 8r.
// Per 4-column block B: every thread factors the 4x4 diagonal block D = L_D L_D^T redundantly in
// registers (W = L_D^{-1}), forms its panel rows l_iB = A_iB W^T, updates its trailing elements
// and its L^{-1} rows (X_B = W M_B; M_i -= l_iB X_B).  One barrier per block (8 per pivot).
// A and M are register-resident; LDS only carries the values other threads need.
template <int BS, bool ONEBAR>
__device__ __forceinline__ double pivot_blockedT(double* A, double* M, double* pv, int t, int* status) {
  const int c = t & 31, i0 = t >> 5;
  double a[4], m[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = A[(i0 + 8 * r) * SP + c];
    m[r] = (i0 + 8 * r == c) ? 1.0 : 0.0;
    M[(i0 + 8 * r) * SP + c] = m[r];
  }
  __syncthreads();
  double ls = 0.0;
#pragma unroll
  for (int kb = 0; kb < 32 / BS; ++kb) {
    const int b0 = BS * kb;
    // reads: D (lower), row i panel A[i][B] for own rows, A[c][B], M[B][c]
    double D[BS][BS], aiB[4][BS], acB[BS], mB[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int y = 0; y < BS; ++y) aiB[r][y] = A[(i0 + 8 * r) * SP + b0 + y];
#pragma unroll
    for (int y = 0; y < BS; ++y) {
      acB[y] = A[c * SP + b0 + y];
      mB[y] = M[(b0 + y) * SP + c];
    }
    // 4x4 Cholesky (redundant per thread): L (lower), rinv[x] = 1/L_xx
    double L[BS][BS], rinv[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      double s = D[x][x];
#pragma unroll
      for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
      if (t == 0) pv[b0 + x] = s;
      rinv[x] = rsqrt_f64(s);
      L[x][x] = s * rinv[x];
#pragma unroll
      for (int y = x + 1; y < BS; ++y) {
        double q = D[y][x];
#pragma unroll
        for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
        L[y][x] = q * rinv[x];
      }
    }
    // W = L^{-1} (lower): W_xx = rinv_x, W_yx = -rinv_y sum_{z=x}^{y-1} L_yz W_zx
    double W[BS][BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      W[x][x] = rinv[x];
#pragma unroll
      for (int y = x + 1; y < BS; ++y) {
        double q = 0.0;
#pragma unroll
        for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
        W[y][x] = -q * rinv[y];
      }
    }
    // l_cB = A_cB W^T ; X_B = W m_B (column c of the new L^{-1} rows B)
    double lc[BS], X[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      double q = 0.0, u = 0.0;
#pragma unroll
      for (int z = 0; z <= x; ++z) {
        q = fma(acB[z], W[x][z], q);
        u = fma(W[x][z], mB[z], u);
      }
      lc[x] = q;
      X[x] = u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 8 * r;
      if (i >= b0 && i < b0 + BS) {
        m[r] = X[i - b0];        // final row of L^{-1} (not re-published: nobody reads it again)
      } else if (i >= b0 + BS) {
        double li[BS];
#pragma unroll
        for (int x = 0; x < BS; ++x) {
          double q = 0.0;
#pragma unroll
          for (int z = 0; z <= x; ++z) q = fma(aiB[r][z], W[x][z], q);
          li[x] = q;
        }
        double na = a[r], nm = m[r];
#pragma unroll
        for (int x = 0; x < BS; ++x) {
          if (c >= b0 + BS) na = fma(-li[x], lc[x], na);
          nm = fma(-li[x], X[x], nm);
        }
        a[r] = na;
        m[r] = nm;
      }
    }
    if (!ONEBAR) __syncthreads();  // (not needed: the writes below never change a value read above)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 8 * r;
      if (i >= b0 + BS) {
        A[i * SP + c] = a[r];
        M[i * SP + c] = m[r];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(i0 + 8 * r) * SP + c] = m[r];
  if (t < 64) {
    const double pk = pv[t & 31];
    if (t < 32 && !(pk > 0.0)) atomicOr(status, 1);
    ls = (t < 32) ? log(pk) : 0.0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  }
  __syncthreads();
  return ls;
}

template <int BS, bool ONEBAR>
__device__ __forceinline__ double pivot_blockedBF(double* A, double* M, double* pv, int t, int* status) {
  const int c = t & 31, i0 = t >> 5;
  double a[4], m[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = A[(i0 + 8 * r) * SP + c];
    m[r] = (i0 + 8 * r == c) ? 1.0 : 0.0;
    M[(i0 + 8 * r) * SP + c] = m[r];
  }
  __syncthreads();
  double ls = 0.0;
#pragma unroll
  for (int kb = 0; kb < 32 / BS; ++kb) {
    const int b0 = BS * kb;
    // reads: D (lower), row i panel A[i][B] for own rows, A[c][B], M[B][c]
    double D[BS][BS], aiB[4][BS], acB[BS], mB[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int y = 0; y < BS; ++y) aiB[r][y] = A[(i0 + 8 * r) * SP + b0 + y];
#pragma unroll
    for (int y = 0; y < BS; ++y) {
      acB[y] = A[c * SP + b0 + y];
      mB[y] = M[(b0 + y) * SP + c];
    }
    // 4x4 Cholesky (redundant per thread): L (lower), rinv[x] = 1/L_xx
    double L[BS][BS], rinv[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      double s = D[x][x];
#pragma unroll
      for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
      if (t == 0) pv[b0 + x] = s;
      rinv[x] = rsqrt_f64(s);
      L[x][x] = s * rinv[x];
#pragma unroll
      for (int y = x + 1; y < BS; ++y) {
        double q = D[y][x];
#pragma unroll
        for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
        L[y][x] = q * rinv[x];
      }
    }
    // W = L^{-1} (lower): W_xx = rinv_x, W_yx = -rinv_y sum_{z=x}^{y-1} L_yz W_zx
    double W[BS][BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      W[x][x] = rinv[x];
#pragma unroll
      for (int y = x + 1; y < BS; ++y) {
        double q = 0.0;
#pragma unroll
        for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
        W[y][x] = -q * rinv[y];
      }
    }
    // l_cB = A_cB W^T ; X_B = W m_B (column c of the new L^{-1} rows B)
    double lc[BS], X[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      double q = 0.0, u = 0.0;
#pragma unroll
      for (int z = 0; z <= x; ++z) {
        q = fma(acB[z], W[x][z], q);
        u = fma(W[x][z], mB[z], u);
      }
      lc[x] = q;
      X[x] = u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // branch-free: every thread does the work, selects the result
      const int i = i0 + 8 * r;
      double li[BS];
#pragma unroll
      for (int x = 0; x < BS; ++x) {
        double q = 0.0;
#pragma unroll
        for (int z = 0; z <= x; ++z) q = fma(aiB[r][z], W[x][z], q);
        li[x] = q;
      }
      double na = a[r], nm = m[r], xb = 0.0;
#pragma unroll
      for (int x = 0; x < BS; ++x) {
        na = fma(-li[x], lc[x], na);
        nm = fma(-li[x], X[x], nm);
        xb = (i == b0 + x) ? X[x] : xb;
      }
      const bool below = i >= b0 + BS, inB = (i >= b0) && !below;
      a[r] = (below && c >= b0 + BS) ? na : a[r];
      m[r] = below ? nm : (inB ? xb : m[r]);
    }
    if (!ONEBAR) __syncthreads();  // (not needed: the writes below never change a value read above)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 8 * r;
      if (i >= b0 + BS) {
        A[i * SP + c] = a[r];
        M[i * SP + c] = m[r];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(i0 + 8 * r) * SP + c] = m[r];
  if (t < 64) {
    const double pk = pv[t & 31];
    if (t < 32 && !(pk > 0.0)) atomicOr(status, 1);
    ls = (t < 32) ? log(pk) : 0.0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  }
  __syncthreads();
  return ls;
}

__global__ __launch_bounds__(256) void bench(const double* Kin, double* Mout, double* out, int reps,
                                             int variant, int* status, long long* cycles) {
  __shared__ double A[32 * SP], M[32 * SP], pv[32], rowA[64], rowM[64];
  const int t = threadIdx.x;
  double ls = 0.0;
  long long t0 = wall_clock64();
  long long c0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = t; e < 1024; e += 256) A[(e >> 5) * SP + (e & 31)] = Kin[e];
    __syncthreads();
    if (variant == 0) {
      ls = pivot_chol_inv_block(A, M, pv, t, status);
    } else if (variant == 2) {
      ls = pivot_blocked4(A, M, pv, t, status);
    } else if (variant == 3) {
      ls = pivot_blockedT<4, true>(A, M, pv, t, status);
    } else if (variant == 4) {
      ls = pivot_blockedT<8, true>(A, M, pv, t, status);
    } else if (variant == 5) {
      ls = pivot_blockedT<2, true>(A, M, pv, t, status);
    } else if (variant == 6) {
      ls = pivot_blockedBF<4, true>(A, M, pv, t, status);
    } else if (variant == 7) {
      ls = pivot_blockedBF<8, true>(A, M, pv, t, status);
    } else {
      if (t < 64) ls = pivot_1wave(A, M, rowA, rowM, pv, t, status);
      __syncthreads();
    }
  }
  long long t1 = wall_clock64();
  long long c1 = __builtin_amdgcn_s_memtime();
  for (int e = t; e < 1024; e += 256) Mout[e] = M[(e >> 5) * SP + (e & 31)];
  if (t == 0) { out[0] = ls; cycles[0] = t1 - t0; cycles[1] = c1 - c0; }
}

int main() {
  // SPD test block: Matern-like kernel matrix + jitter
  std::vector<double> K(1024);
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double d = fabs(i - j) * 0.07;
      K[i * 32 + j] = (1 + sqrt(5.0) * d + 5.0 / 3.0 * d * d) * exp(-sqrt(5.0) * d) * cos(3.0 * d) + (i == j ? 1e-3 : 0.0);
    }
  double *dK, *dM, *dout;
  int* st;
  long long* cyc;
  CHK(hipMalloc(&dK, 8192)); CHK(hipMalloc(&dM, 8192)); CHK(hipMalloc(&dout, 64));
  CHK(hipMalloc(&st, 4)); CHK(hipMalloc(&cyc, 16));
  CHK(hipMemcpy(dK, K.data(), 8192, hipMemcpyHostToDevice));
  CHK(hipMemset(st, 0, 4));
  int rate = 0;
  CHK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));
  std::vector<double> M0(1024), M1(1024), M2(1024), Mv(1024);
  double ls[8];
  for (int v = 0; v < 8; ++v) {
    const int reps = 200;
    hipLaunchKernelGGL(bench, dim3(1), dim3(256), 0, 0, dK, dM, dout, reps, v, st, cyc);
    CHK(hipDeviceSynchronize());
    long long c, cc[2];
    CHK(hipMemcpy(cc, cyc, 16, hipMemcpyDeviceToHost));
    c = cc[0];
    printf("   shader cycles per factorisation %.0f -> clock %.2f GHz\n", (double)cc[1] / reps,
           (double)cc[1] / ((double)c / (rate * 1e3)) / 1e9);
    CHK(hipMemcpy(v == 0 ? M0.data() : v == 1 ? M1.data() : v == 2 ? M2.data() : Mv.data(), dM, 8192, hipMemcpyDeviceToHost));
    if (v >= 3) {
      double md = 0, mx = 0;
      for (int i = 0; i < 1024; ++i) { md = fmax(md, fabs(M0[i] - Mv[i])); mx = fmax(mx, fabs(M0[i])); }
      printf("   variant %d: max |M0 - Mv| / max|M0| = %.3e\n", v, md / mx);
    }
    CHK(hipMemcpy(&ls[v], dout, 8, hipMemcpyDeviceToHost));
    printf("variant %d (%s): %.3f us per factorisation (wall clock %d kHz)\n", v,
           v == 0 ? "4-wave LDS" : v == 1 ? "1-wave registers" : v == 2 ? "blocked b=4" : v == 3 ? "blocked b=4 1bar" : v == 4 ? "blocked b=8 1bar" : v == 5 ? "blocked b=2 1bar" : v == 6 ? "branch-free b=4" : "branch-free b=8", (double)c / reps / (rate * 1e-3), rate);
  }
  double md = 0, mx = 0;
  for (int i = 0; i < 1024; ++i) { md = fmax(md, fabs(M0[i] - M1[i])); mx = fmax(mx, fabs(M0[i])); }
  int hs;
  CHK(hipMemcpy(&hs, st, 4, hipMemcpyDeviceToHost));
  printf("max |M0 - M1| / max|M0| = %.3e, logdet %.15e vs %.15e, status %d\n", md / mx, ls[0], ls[1], hs);
  md = 0;
  for (int i = 0; i < 1024; ++i) md = fmax(md, fabs(M0[i] - M2[i]));
  printf("max |M0 - M2| / max|M0| = %.3e, logdet %.15e\n", md / mx, ls[2]);
  // M2 * L = I check via K: M K M^T = I
  double e = 0;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    double s = 0; for (int p = 0; p < 32; ++p) for (int q = 0; q < 32; ++q) s += M2[i*32+p] * K[p*32+q] * M2[j*32+q];
    e = fmax(e, fabs(s - (i == j)));
  }
  printf("|M2 K M2^T - I|max = %.3e\n", e);
  return 0;
}
