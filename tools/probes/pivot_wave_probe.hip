#include <hip/hip_runtime.h>
constexpr int SP = 33;
__device__ __forceinline__ double rsqrt_f64(double p) {
  double y = __builtin_amdgcn_rsq(p);
  double e = fma(-p * y, y, 1.0);
  y = fma(0.5 * y, e, y);
  e = fma(-p * y, y, 1.0);
  return fma(0.5 * y, e, y);
}
__device__ __forceinline__ double rdlane(double v, int src) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), src);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), src);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// one wave; lane: column c = lane&31, half h = lane>>5; register slot m holds row h + 2*((m + t) mod 16)
// at pair t (arrays rotate by one slot per pair so the current row pair always sits in slot 0).
__device__ __forceinline__ double pivot_wave(const double* A, double* piv, double* bc, double* pvv, int lane) {
  const int c = lane & 31, h = lane >> 5;
  double a[16], g[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) { a[m] = A[(h + 2 * m) * SP + c]; g[m] = (h + 2 * m == c) ? 1.0 : 0.0; }
  for (int t = 0; t < 16; ++t) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int k = 2 * t + kh;
      const double p = rdlane(a[0], k + 32 * kh);          // A[k][k]: lane (c=k, h=kh), slot 0
      const double rs = rsqrt_f64(p);
      if (lane == 0) pvv[k] = p;
      const double sw = __shfl_xor(a[0], 32, 64);
      const double akc = (h == kh) ? a[0] : sw;             // A[k][c]
      const double lck = akc * rs;
      const double gsw = __shfl_xor(g[0], 32, 64);
      const double mkc = ((h == kh) ? g[0] : gsw) * rs;     // L^{-1}[k][c] (row k not yet scaled)
      if (h == kh) bc[c] = lck;                             // row k of L (scaled), by column
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int i = h + 2 * m + 2 * t;                    // row held in slot m (valid if m < 16 - t)
        const double lik = bc[i & 31];
        const bool upd = (m < 16 - t) && (i > k);
        a[m] = (upd && c > k) ? fma(-lik, lck, a[m]) : a[m];
        g[m] = upd ? fma(-lik, mkc, g[m]) : g[m];
      }
      __builtin_amdgcn_wave_barrier();
    }
    // rotate: slot 0 (rows 2t, 2t+1 done) goes to the back
    const double a0 = a[0], g0 = g[0];
#pragma unroll
    for (int m = 0; m < 15; ++m) { a[m] = a[m + 1]; g[m] = g[m + 1]; }
    a[15] = a0; g[15] = g0;
  }
  // after 16 rotations slot m holds row h + 2m again; scale rows by rs_k
#pragma unroll
  for (int m = 0; m < 16; ++m) piv[(h + 2 * m) * 32 + c] = g[m] * rsqrt_f64(pvv[h + 2 * m]);
  double ls = (lane < 32) ? log(pvv[lane]) : 0.0;
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  return ls;
}
__global__ __launch_bounds__(64) void kpv(const double* X, double* piv, double* out, int iters) {
  __shared__ double A[32 * SP], bc[32], pvv[32];
  for (int e = threadIdx.x; e < 1024; e += 64) A[(e >> 5) * SP + (e & 31)] = X[e];
  __syncthreads();
  double ls = 0;
  for (int it = 0; it < iters; ++it) ls += pivot_wave(A, piv, bc, pvv, threadIdx.x);
  if (threadIdx.x == 0) out[0] = ls;
}
int main() {
  double hX[1024];
  srand(1);
  // SPD: B B^T + 32 I
  double B[1024]; for (int i = 0; i < 1024; ++i) B[i] = (rand() / (double)RAND_MAX) - 0.5;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { double s = (i == j) ? 1.0 : 0.0; for (int k = 0; k < 32; ++k) s += B[i*32+k]*B[j*32+k]; hX[i*32+j] = s; }
  double *dX, *dP, *dO; hipMalloc(&dX, 8192); hipMalloc(&dP, 8192); hipMalloc(&dO, 8);
  hipMemcpy(dX, hX, 8192, hipMemcpyHostToDevice);
  kpv<<<1, 64>>>(dX, dP, dO, 1);
  double hP[1024], ls; hipMemcpy(hP, dP, 8192, hipMemcpyDeviceToHost); hipMemcpy(&ls, dO, 8, hipMemcpyDeviceToHost);
  // check: Li * X * Li^T = I
  double err = 0;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { double s = 0; for (int a = 0; a < 32; ++a) for (int b = 0; b < 32; ++b) s += hP[i*32+a]*hX[a*32+b]*hP[j*32+b]; err = fmax(err, fabs(s - (i==j))); }
  // upper triangle zero?
  double up = 0; for (int i = 0; i < 32; ++i) for (int j = i+1; j < 32; ++j) up = fmax(up, fabs(hP[i*32+j]));
  printf("max |Li X Li^T - I| = %.3e  upper=%.1e  logdet=%.12f\n", err, up, ls);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0); kpv<<<1, 64>>>(dX, dP, dO, 100); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); printf("pivot_wave: %.3f us per factorization\n", ms * 10.0);
  }
  return 0;
}
