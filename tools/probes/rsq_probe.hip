// rsq_probe.hip -- accuracy of v_rsq_f64 and of v_rsq_f64 + one / two Newton steps against
// 1/sqrt in long double on the host, and of one third-order (Householder) step
// y (1 + e/2 + 3e^2/8), e = 1 - p y^2 (decides the pivot's rsqrt_f64 in spd_pivot.h).
//   hipcc --offload-arch=gfx950 -O3 rsq_probe.hip -o rsq_probe && ./rsq_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void rsq(const double* x, double* r0, double* r1, double* r2, double* r3, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double p = x[i];
  double y = __builtin_amdgcn_rsq(p);
  r0[i] = y;
  {
    const double e3 = fma(-p * y, y, 1.0);
    r3[i] = fma(y * e3, fma(0.375, e3, 0.5), y);
  }
  double e = fma(-p * y, y, 1.0);
  y = fma(0.5 * y, e, y);
  r1[i] = y;
  e = fma(-p * y, y, 1.0);
  r2[i] = fma(0.5 * y, e, y);
}

int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), r0(n), r1(n), r2(n), r3(n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-30.0, 30.0);
  for (auto& v : x) v = std::exp(u(g));
  double *dx, *d0, *d1, *d2, *d3;
  hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8); hipMalloc(&d3, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  rsq<<<n / 256, 256>>>(dx, d0, d1, d2, d3, n);
  hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r3.data(), d3, n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, m2 = 0, m3 = 0;
  long d12 = 0;
  for (int i = 0; i < n; ++i) {
    const long double t = 1.0L / sqrtl((long double)x[i]);
    m0 = std::fmax(m0, (double)fabsl((r0[i] - t) / t));
    m1 = std::fmax(m1, (double)fabsl((r1[i] - t) / t));
    m2 = std::fmax(m2, (double)fabsl((r2[i] - t) / t));
    m3 = std::fmax(m3, (double)fabsl((r3[i] - t) / t));
    d12 += r1[i] != r2[i];
  }
  printf("max rel err: rsq %.3e (2^%.1f)  +1 Newton %.3e  +2 Newton %.3e  (eps %.3e); 1 vs 2 steps differ in %ld of %d\n",
         m0, std::log2(m0), m1, m2, 2.220446e-16, d12, n);
  printf("third-order step: max rel err %.3e\n", m3);
  return 0;
}
