// Workgroup dispatch timing of a chain_kernel-shaped grid (probe; tools/probes, not the product).
// Kernel `hold` has chain_kernel's footprint (256 threads, __launch_bounds__(256, 2), ~50 KB of
// LDS, the VGPR budget pinned to 256 by the attribute below): every workgroup records its start on
// the 100 MHz device clock and its hardware placement (XCC, SE, CU), then stays resident for
// `hold_us` so that the grid fills the device as the chain does.  A one-workgroup kernel ahead of
// it records its own end, which prices the boundary.  Prints per linear workgroup id: start (us,
// relative to the earliest start), xcc/se/cu; and the boundary.
// usage: dispatch_probe [nwg=580] [lds_kb=50] [hold_us=60]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

__global__ void first(unsigned long long* endt) {
  if (threadIdx.x == 0) endt[0] = __builtin_amdgcn_s_memrealtime();
}

template <int LDSD>
__global__ __launch_bounds__(256, 2) void hold(unsigned long long* st, unsigned* where, int hold_ticks, double* sink) {
  __shared__ double lds[LDSD];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int wg = blockIdx.x + blockIdx.y * gridDim.x;
  if (threadIdx.x == 0) {
    st[wg] = t0;
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); // HW_REG_XCC_ID
    where[wg] = (xcc & 0xf) << 16 | ((hw >> 13) & 0x7) << 8 | ((hw >> 8) & 0xf);
  }
  // some VGPR pressure and LDS traffic so the allocation is what the attribute asks for
  double acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = threadIdx.x * 1.0 + i;
  lds[threadIdx.x % LDSD] = acc[threadIdx.x & 31];
  __syncthreads();
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < hold_ticks) {
    __builtin_amdgcn_s_sleep(10);
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = fma(acc[i], 1.0000001, lds[(threadIdx.x + i) % LDSD]);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 32; ++i) s += acc[i];
  if (s == 12345.678) sink[0] = s;
}

int main(int argc, char** argv) {
  const int nwg = argc > 1 ? std::atoi(argv[1]) : 580;
  const int lds_kb = argc > 2 ? std::atoi(argv[2]) : 50;
  const int hold_us = argc > 3 ? std::atoi(argv[3]) : 60;
  unsigned long long *st, *endt;
  unsigned* where;
  double* sink;
  CHK(hipMalloc(&st, nwg * 8));
  CHK(hipMalloc(&where, nwg * 4));
  CHK(hipMalloc(&endt, 8));
  CHK(hipMalloc(&sink, 8));
  auto run = [&](int rows) {
    dim3 g(nwg / rows, rows);
    hipLaunchKernelGGL(first, dim3(1), dim3(64), 0, 0, endt);
    if (lds_kb >= 40) hipLaunchKernelGGL((hold<6300>), g, dim3(256), 0, 0, st, where, hold_us * 100, sink);
    else hipLaunchKernelGGL((hold<1024>), g, dim3(256), 0, 0, st, where, hold_us * 100, sink);
    CHK(hipDeviceSynchronize());
  };
  for (int rep = 0; rep < 3; ++rep) run(nwg % 3 == 0 ? 3 : 1);  // warm up
  std::vector<unsigned long long> hs(nwg), he(1);
  std::vector<unsigned> hw(nwg);
  for (int rep = 0; rep < 2; ++rep) {
    run(nwg % 3 == 0 ? 3 : 1);
    CHK(hipMemcpy(hs.data(), st, nwg * 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(hw.data(), where, nwg * 4, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(he.data(), endt, 8, hipMemcpyDeviceToHost));
    const unsigned long long t0 = *std::min_element(hs.begin(), hs.end());
    std::printf("rep %d: nwg %d lds %d KB: boundary (first kernel end -> earliest start) %.2f us\n", rep, nwg,
                lds_kb, (double)(t0 - he[0]) / 100.0);
    for (int i = 0; i < nwg; ++i)
      if (i < 8 || i % 16 == 0 || (i >= 185 && i <= 200) || i >= nwg - 4)
        std::printf("  wg %4d start %6.2f us  xcc %u se %u cu %2u\n", i, (double)(hs[i] - t0) / 100.0,
                    hw[i] >> 16, (hw[i] >> 8) & 0xff, hw[i] & 0xff);
    // how many CUs hold 2+ workgroups
    std::vector<int> cnt(1 << 20, 0);
    int shared = 0;
    for (int i = 0; i < nwg; ++i) if (++cnt[hw[i]] == 2) ++shared;
    std::printf("  CUs with 2+ workgroups: %d; latest start %.2f us\n", shared,
                (double)(*std::max_element(hs.begin(), hs.end()) - t0) / 100.0);
  }
  return 0;
}
