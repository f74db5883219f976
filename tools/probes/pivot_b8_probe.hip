// Probe: the 32x32 SPD pivot factorisation (Cholesky + L^{-1} + log det) with 8-column blocks
// (4 block steps, rank-8 updates as two rank-4 MFMAs) vs spd_pivot.h's 4-column blocks (8 steps).
// One 256-thread workgroup; wall clock over repeated factorisations inside one launch.
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/spd_pivot.h"
#include <cstdio>
#include <vector>
#include <cmath>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

using namespace gpk;
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NEWTON>
__device__ __forceinline__ double rsq(double p) {
  double y = __builtin_amdgcn_rsq(p);
#pragma unroll
  for (int i = 0; i < NEWTON; ++i) {
    const double e = fma(-p * y, y, 1.0);
    y = fma(0.5 * y, e, y);
  }
  return y;
}

// 8-column blocks: 4 block steps (one barrier each); the rank-8 trailing updates as two rank-4
// MFMAs per accumulator; every lane factors the 8x8 diagonal block itself
__device__ double pivot_b8(double* A, double* M, double* pv, int t, int* status) {
  const int lane = t & 63, wv = t >> 6, wr = wv >> 1, wc = wv & 1;
  const int li = lane & 15, lk = lane >> 4;
  const int ri = 16 * wr + li, cj = 16 * wc + li;
  d4 accA, accM;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * wr + lk + 4 * r;
    accA[r] = A[row * SP + cj];
    accM[r] = (row == cj) ? 1.0 : 0.0;
    M[row * SP + cj] = accM[r];
  }
  const double s0 = lk == 0 ? 1.0 : 0.0, s1 = lk == 1 ? 1.0 : 0.0, s2 = lk == 2 ? 1.0 : 0.0,
               s3 = lk == 3 ? 1.0 : 0.0;
  __syncthreads();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const int b0 = 8 * kb;
    double D[8][8], ar[8], ac[8], mb[8];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
      for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
    for (int z = 0; z < 8; ++z) {
      ar[z] = A[ri * SP + b0 + z];
      ac[z] = A[cj * SP + b0 + z];
      mb[z] = M[(b0 + z) * SP + cj];
    }
    double L[8][8], rinv[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      double s = D[x][x];
#pragma unroll
      for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
      if (t == 0) pv[b0 + x] = s;
      rinv[x] = rsqrt_f64(s);
#pragma unroll
      for (int y = x + 1; y < 8; ++y) {
        double q = D[y][x];
#pragma unroll
        for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
        L[y][x] = q * rinv[x];
      }
    }
    double W[8][8];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      W[x][x] = rinv[x];
#pragma unroll
      for (int y = x + 1; y < 8; ++y) {
        double q = 0.0;
#pragma unroll
        for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
        W[y][x] = -q * rinv[y];
      }
#pragma unroll
      for (int y = 0; y < x; ++y) W[y][x] = 0.0;
    }
    double xv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double lr = 0.0, lc = 0.0, x = 0.0;
#pragma unroll
      for (int z = 0; z < 8; ++z) {
        const int o = 4 * h;
        const double w = fma(W[o][z], s0, fma(W[o + 1][z], s1, fma(W[o + 2][z], s2, W[o + 3][z] * s3)));
        lr = fma(ar[z], w, lr);
        lc = fma(ac[z], w, lc);
        x = fma(w, mb[z], x);
      }
      xv[h] = x;
      const double opa = (ri >= b0 + 8) ? -lr : 0.0;
      const double opb = (cj >= b0 + 8) ? lc : 0.0;
      accA = __builtin_amdgcn_mfma_f64_16x16x4f64(opa, opb, accA, 0, 0, 0);
      accM = __builtin_amdgcn_mfma_f64_16x16x4f64(opa, x, accM, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * wr + lk + 4 * r;
      if (16 * wr + 4 * r == b0) accM[r] = xv[0];
      if (16 * wr + 4 * r == b0 + 4) accM[r] = xv[1];
      if (kb < 3 && row >= b0 + 8) {
        if (cj >= b0 + 8) A[row * SP + cj] = accA[r];
        M[row * SP + cj] = accM[r];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(16 * wr + lk + 4 * r) * SP + cj] = accM[r];
  double ls = 0.0;
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
  __shared__ double A[32 * SP], M[2 * 32 * SP], Ab[32 * SP], pv[32];
  const int t = threadIdx.x;
  double ls = 0.0;
  long long t0 = wall_clock64();
  long long c0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = t; e < 1024; e += 256) A[(e >> 5) * SP + (e & 31)] = Kin[e];
    __syncthreads();
    if (variant == 0)
      ls = pivot_chol_inv_block(A, M, pv, t, status);
    else
      ls = pivot_b8(A, M, pv, t, status);
  }
  long long t1 = wall_clock64();
  long long c1 = __builtin_amdgcn_s_memtime();
  for (int e = t; e < 1024; e += 256) Mout[e] = M[(e >> 5) * SP + (e & 31)];
  if (t == 0) { out[0] = ls; cycles[0] = t1 - t0; cycles[1] = c1 - c0; }
}

int main() {
  const char* names[] = {"b=4, 8 block steps (spd_pivot.h)", "b=8, 4 block steps"};
  for (int mat = 0; mat < 2; ++mat) {
    std::vector<double> K(1024);
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        double d = fabs((double)(i - j)) * (mat == 0 ? 0.07 : 0.02);
        K[i * 32 + j] = (1 + sqrt(5.0) * d + 5.0 / 3.0 * d * d) * exp(-sqrt(5.0) * d) * cos(3.0 * d) +
                        (i == j ? (mat == 0 ? 1e-3 : 1e-6) : 0.0);
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
    std::vector<double> M0(1024), Mv(1024);
    double ls0 = 0;
    printf("matrix %d (%s)\n", mat, mat == 0 ? "moderate" : "ill-conditioned");
    for (int v = 0; v < 2; ++v) {
      const int reps = 200;
      hipLaunchKernelGGL(bench, dim3(1), dim3(256), 0, 0, dK, dM, dout, reps, v, st, cyc);
      CHK(hipDeviceSynchronize());
      long long cc[2];
      CHK(hipMemcpy(cc, cyc, 16, hipMemcpyDeviceToHost));
      CHK(hipMemcpy(v == 0 ? M0.data() : Mv.data(), dM, 8192, hipMemcpyDeviceToHost));
      double ls;
      CHK(hipMemcpy(&ls, dout, 8, hipMemcpyDeviceToHost));
      if (v == 0) ls0 = ls;
      const std::vector<double>& Mx = v == 0 ? M0 : Mv;
      double md = 0, mx = 0, e = 0;
      for (int i = 0; i < 1024; ++i) { md = fmax(md, fabs(M0[i] - Mx[i])); mx = fmax(mx, fabs(M0[i])); }
      for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
        double s = 0; for (int p = 0; p < 32; ++p) for (int q = 0; q < 32; ++q) s += Mx[i*32+p] * K[p*32+q] * Mx[j*32+q];
        e = fmax(e, fabs(s - (i == j)));
      }
      printf("  variant %d (%s): %.3f us (%.0f cycles) | max|M-M0|/max|M0| %.2e | |MKM^T-I| %.2e | logdet %.15e (d %.1e)\n",
             v, names[v], (double)cc[0] / reps / (rate * 1e-3), (double)cc[1] / reps, md / mx, e, ls, ls - ls0);
    }
    int hs;
    CHK(hipMemcpy(&hs, st, 4, hipMemcpyDeviceToHost));
    printf("  status %d\n", hs);
  }
  return 0;
}
