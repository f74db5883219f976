// Probe: where the 32x32 pivot factorisation's time goes (spd_pivot.h pivot_chol_inv_block, the
// pivot chain's serial step).  A copy of the block-step loop with parts switched off by a
// template mask (timing only -- the results of the partial variants are meaningless):
//   1 = the 4x4 diagonal Cholesky + rsqrt + W (replaced by constants)
//   2 = the two MFMA rank-4 updates
//   4 = the per-step barrier
//   8 = the per-step LDS reads (D, A's column block, M's rows)
//  16 = the per-step LDS writes of the updated entries
//  32 = (not a removal) the writes of the lower triangles only -- spd_pivot.h's form
// One 256-thread workgroup, repeated factorisations; wall clock per factorisation.
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/spd_pivot.h"
#include <cstdio>
#include <vector>
#include <cmath>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

using namespace gpk;

template <int OFF>
__device__ __forceinline__ double piv(double* A, double* M, double* pv, int t) {
  typedef double dv4 __attribute__((ext_vector_type(4)));
  const int lane = t & 63, wv = t >> 6, wr = wv >> 1, wc = wv & 1;
  const int li = lane & 15, lk = lane >> 4;
  const int ri = 16 * wr + li, cj = 16 * wc + li;
  dv4 accA, accM;
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
  for (int kb = 0; kb < 8; ++kb) {
    const int b0 = 4 * kb;
    double D[4][4], ar[4], ac[4], mb[4];
    if (OFF & 8) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
#pragma unroll
        for (int y = 0; y < 4; ++y) D[x][y] = (x == y) ? 2.0 + accA[0] * 1e-30 : 0.1;
        ar[x] = 0.01 * x + accA[1] * 1e-30; ac[x] = 0.02 * x; mb[x] = 0.03 * x + accM[0] * 1e-30;
      }
    } else {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        ar[z] = A[ri * SP + b0 + z];
        ac[z] = A[cj * SP + b0 + z];
        mb[z] = M[(b0 + z) * SP + cj];
      }
    }
    double W[4][4];
    if (OFF & 1) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) W[y][x] = (x == y) ? D[x][x] : (y > x ? D[y][x] : 0.0);
    } else {
      double L[4][4], rinv[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        double s = D[x][x];
#pragma unroll
        for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
        if (t == 0) pv[b0 + x] = s;
        rinv[x] = rsqrt_f64(s);
#pragma unroll
        for (int y = x + 1; y < 4; ++y) {
          double q = D[y][x];
#pragma unroll
          for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
          L[y][x] = q * rinv[x];
        }
      }
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
#pragma unroll
        for (int y = 0; y < x; ++y) W[y][x] = 0.0;
      }
    }
    double lr = 0.0, lc = 0.0, xv = 0.0;
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const double w = fma(W[0][z], s0, fma(W[1][z], s1, fma(W[2][z], s2, W[3][z] * s3)));
      lr = fma(ar[z], w, lr);
      lc = fma(ac[z], w, lc);
      xv = fma(w, mb[z], xv);
    }
    const double opa = (ri >= b0 + 4) ? -lr : 0.0;
    const double opb = (cj >= b0 + 4) ? lc : 0.0;
    if (OFF & 2) {
      accA[0] += opa * opb;
      accM[0] += opa * xv;
    } else {
      accA = __builtin_amdgcn_mfma_f64_16x16x4f64(opa, opb, accA, 0, 0, 0);
      accM = __builtin_amdgcn_mfma_f64_16x16x4f64(opa, xv, accM, 0, 0, 0);
    }
    if (!(OFF & 16)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * wr + lk + 4 * r;
        if (16 * wr + 4 * r == b0) accM[r] = xv;
        if (kb < 7 && row >= b0 + 4 && ((OFF & 32) == 0 || row >= cj)) {
          if (cj >= b0 + 4) A[row * SP + cj] = accA[r];
          M[row * SP + cj] = accM[r];
        }
      }
    }
    if (!(OFF & 4)) __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(16 * wr + lk + 4 * r) * SP + cj] = accM[r];
  __syncthreads();
  return accA[0] + accA[3];
}

template <int OFF>
__global__ __launch_bounds__(256) void bench(const double* Kin, double* out, int reps, long long* cyc) {
  __shared__ double A[32 * SP], M[32 * SP], pv[32];
  const int t = threadIdx.x;
  double ls = 0.0;
  const long long t0 = wall_clock64();
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = t; e < 1024; e += 256) A[(e >> 5) * SP + (e & 31)] = Kin[e];
    __syncthreads();
    ls += piv<OFF>(A, M, pv, t);
  }
  const long long t1 = wall_clock64();
  if (t == 0) { out[0] = ls; cyc[0] = t1 - t0; }
}

template <int OFF>
int run(const char* name, const double* dK, double* dout, long long* cyc, int rate) {
  const int reps = 400;
  hipLaunchKernelGGL(bench<OFF>, dim3(1), dim3(256), 0, 0, dK, dout, reps, cyc);
  CHK(hipDeviceSynchronize());
  hipLaunchKernelGGL(bench<OFF>, dim3(1), dim3(256), 0, 0, dK, dout, reps, cyc);
  CHK(hipDeviceSynchronize());
  long long c;
  CHK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
  printf("  off %2d %-44s %.3f us per factorisation\n", OFF, name, (double)c / reps / (rate * 1e-3));
  return 0;
}

int main() {
  std::vector<double> K(1024);
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double d = fabs((double)(i - j)) * 0.07;
      K[i * 32 + j] = (1 + sqrt(5.0) * d + 5.0 / 3.0 * d * d) * exp(-sqrt(5.0) * d) * cos(3.0 * d) + (i == j ? 1e-3 : 0.0);
    }
  double *dK, *dout;
  long long* cyc;
  CHK(hipMalloc(&dK, 8192)); CHK(hipMalloc(&dout, 64)); CHK(hipMalloc(&cyc, 16));
  CHK(hipMemcpy(dK, K.data(), 8192, hipMemcpyHostToDevice));
  int rate = 0;
  CHK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));
  printf("pivot parts (32x32, 8 block steps), wall clock %d kHz\n", rate);
  run<0>("full", dK, dout, cyc, rate);
  run<1>("- 4x4 Cholesky / rsqrt / W", dK, dout, cyc, rate);
  run<2>("- MFMA updates", dK, dout, cyc, rate);
  run<4>("- barriers", dK, dout, cyc, rate);
  run<8>("- LDS reads", dK, dout, cyc, rate);
  run<16>("- LDS writes", dK, dout, cyc, rate);
  run<1 | 2>("- Cholesky - MFMA", dK, dout, cyc, rate);
  run<1 | 8>("- Cholesky - LDS reads", dK, dout, cyc, rate);
  run<4 | 8 | 16>("- barriers - LDS", dK, dout, cyc, rate);
  run<1 | 2 | 4 | 8 | 16>("everything off (loop skeleton)", dK, dout, cyc, rate);
  run<32>("lower-triangle writes only", dK, dout, cyc, rate);
  run<0>("full (again)", dK, dout, cyc, rate);
  run<32>("lower-triangle writes only (again)", dK, dout, cyc, rate);
  return 0;
}
