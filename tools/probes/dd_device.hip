// Device vs host evaluation of csrc/fields_dd.h (probe): the same inputs through fields_dd on the
// GPU and on the host; prints the largest difference per field (should be 0: same IEEE operations).
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/fields_dd.h"

using gpk::dd::D;
struct In { double d, a, om, oml; };

template <int DERIV>
__global__ void k(const In* in, D* out, int n) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  D* o = out + 6 * i;
  gpk::fields_dd<true, true, DERIV>(in[i].d, in[i].a, in[i].om, in[i].oml, o[0], o[1], o[2], o[3], o[4], o[5]);
}

int main() {
  const int n = 4096;
  std::vector<In> in(n);
  srand(3);
  for (int i = 0; i < n; ++i) {
    const double f = 40.0 * rand() / RAND_MAX;
    in[i].d = 6.0 * rand() / RAND_MAX;
    in[i].a = 0.5 + 10.0 * rand() / RAND_MAX;
    in[i].om = gpk::TWO_PI * f;
    in[i].oml = fma(gpk::TWO_PI, f, -in[i].om);
  }
  In* din; D* dout;
  hipMalloc(&din, n * sizeof(In));
  hipMalloc(&dout, 6 * n * sizeof(D));
  hipMemcpy(din, in.data(), n * sizeof(In), hipMemcpyHostToDevice);
  for (int deriv = 1; deriv <= 2; ++deriv) {
    if (deriv == 1) hipLaunchKernelGGL(k<1>, dim3(n / 64), dim3(64), 0, 0, din, dout, n);
    else hipLaunchKernelGGL(k<2>, dim3(n / 64), dim3(64), 0, 0, din, dout, n);
    std::vector<D> dev(6 * n);
    hipMemcpy(dev.data(), dout, 6 * n * sizeof(D), hipMemcpyDeviceToHost);
    double worst[6] = {0}, worst_h[6] = {0};
    for (int i = 0; i < n; ++i) {
      D h[6];
      if (deriv == 1) gpk::fields_dd<true, true, 1>(in[i].d, in[i].a, in[i].om, in[i].oml, h[0], h[1], h[2], h[3], h[4], h[5]);
      else gpk::fields_dd<true, true, 2>(in[i].d, in[i].a, in[i].om, in[i].oml, h[0], h[1], h[2], h[3], h[4], h[5]);
      for (int x = 0; x < 6; ++x) {
        const D g = dev[6 * i + x];
        const double s = fabs(h[x].h) + 1e-300;
        const double e = fabs((g.h - h[x].h) + (g.l - h[x].l)) / s;
        if (e > worst[x]) worst[x] = e;
        const double eh = fabs(g.h - h[x].h) / s;
        if (eh > worst_h[x]) worst_h[x] = eh;
      }
    }
    std::printf("deriv %d: device vs host fields_dd, worst relative difference (h+l / h only):", deriv);
    for (int x = 0; x < 6; ++x) std::printf(" %.2e/%.2e", worst[x], worst_h[x]);
    std::printf("\n");
  }
  return 0;
}
