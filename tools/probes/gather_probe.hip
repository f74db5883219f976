// Probe: HBM rate of the K-assembly gather (assemble.hip gather_kernel / gather_wide_kernel) at
// C5 size -- K, Kc and D of two 4096^2 factors written from class values, the int32 class id of
// every element read (940 MB per launch) -- against a pure streaming write of the same bytes.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 gather_probe.hip -o gather_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

struct Ax { const int* cid; const double* kv; const double* dv; double* K; double* Kc; double* D; int p; };
struct B2 { Ax a[2]; };

// V0: one 32x32 tile per workgroup, 4 rows per thread (gather_kernel)
__global__ __launch_bounds__(256) void v0(B2 b) {
  const Ax& A = b.a[blockIdx.x];
  const int T = A.p / 32, tile = blockIdx.y, I = tile / T, J = tile % T, t = threadIdx.x;
  const int j = J * 32 + (t & 31);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = I * 32 + (t >> 5) + 8 * r;
    const size_t o = (size_t)i * A.p + j;
    const int u = A.cid[o];
    double k = u >= 0 ? A.kv[u] : 0.0, d = u >= 0 ? A.dv[u] : 0.0;
    if (i == j) k += 1e-6;
    A.K[o] = k; A.Kc[o] = k; A.D[o] = d;
  }
}

// V1: 8 rows x 512 columns per workgroup, lane = 2 adjacent columns (gather_wide_kernel); NT: nontemporal stores
template <bool NT>
__global__ __launch_bounds__(256) void v1(B2 b) {
  const Ax& A = b.a[blockIdx.z];
  const int p = A.p, r0 = blockIdx.y * 8, c0 = blockIdx.x * 512, t = threadIdx.x, lane = t & 63, w = t >> 6;
  int2 id[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      id[h][q] = *reinterpret_cast<const int2*>(A.cid + (size_t)(r0 + w + 4 * h) * p + c0 + 128 * q + 2 * lane);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = r0 + w + 4 * h, j = c0 + 128 * q + 2 * lane;
      const int u0 = id[h][q].x, u1 = id[h][q].y;
      double k0 = u0 >= 0 ? A.kv[u0] : 0.0, k1 = u1 >= 0 ? A.kv[u1] : 0.0;
      const double d0 = u0 >= 0 ? A.dv[u0] : 0.0, d1 = u1 >= 0 ? A.dv[u1] : 0.0;
      if (i == j) k0 += 1e-6;
      if (i == j + 1) k1 += 1e-6;
      const size_t o = (size_t)i * p + j;
      if (NT) {
        __builtin_nontemporal_store(k0, A.K + o); __builtin_nontemporal_store(k1, A.K + o + 1);
        __builtin_nontemporal_store(k0, A.Kc + o); __builtin_nontemporal_store(k1, A.Kc + o + 1);
        __builtin_nontemporal_store(d0, A.D + o); __builtin_nontemporal_store(d1, A.D + o + 1);
      } else {
        *reinterpret_cast<double2*>(A.K + o) = make_double2(k0, k1);
        *reinterpret_cast<double2*>(A.Kc + o) = make_double2(k0, k1);
        *reinterpret_cast<double2*>(A.D + o) = make_double2(d0, d1);
      }
    }
}

// V2: one row segment of 1024 columns per wave, 4 columns per lane (int4 ids, two double2 per array)
__global__ __launch_bounds__(256) void v2(B2 b) {
  const Ax& A = b.a[blockIdx.z];
  const int p = A.p, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = blockIdx.y * 4 + w, c0 = blockIdx.x * 1024;
  int4 id[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) id[q] = *reinterpret_cast<const int4*>(A.cid + (size_t)i * p + c0 + 256 * q + 4 * lane);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = c0 + 256 * q + 4 * lane;
    const int u[4] = {id[q].x, id[q].y, id[q].z, id[q].w};
    double k[4], d[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      k[e] = u[e] >= 0 ? A.kv[u[e]] : 0.0;
      d[e] = u[e] >= 0 ? A.dv[u[e]] : 0.0;
      if (i == j + e) k[e] += 1e-6;
    }
    const size_t o = (size_t)i * p + j;
    *reinterpret_cast<double2*>(A.K + o) = make_double2(k[0], k[1]);
    *reinterpret_cast<double2*>(A.K + o + 2) = make_double2(k[2], k[3]);
    *reinterpret_cast<double2*>(A.Kc + o) = make_double2(k[0], k[1]);
    *reinterpret_cast<double2*>(A.Kc + o + 2) = make_double2(k[2], k[3]);
    *reinterpret_cast<double2*>(A.D + o) = make_double2(d[0], d[1]);
    *reinterpret_cast<double2*>(A.D + o + 2) = make_double2(d[2], d[3]);
  }
}

// V3: the same bytes as a pure stream (ids read, constants written): the launch's floor
__global__ __launch_bounds__(256) void v3(B2 b) {
  const Ax& A = b.a[blockIdx.z];
  const int p = A.p, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = blockIdx.y * 4 + w, c0 = blockIdx.x * 1024;
  int4 id[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) id[q] = *reinterpret_cast<const int4*>(A.cid + (size_t)i * p + c0 + 256 * q + 4 * lane);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const size_t o = (size_t)i * p + c0 + 256 * q + 4 * lane;
    const double v = (double)(id[q].x + id[q].w);
    *reinterpret_cast<double2*>(A.K + o) = make_double2(v, v);
    *reinterpret_cast<double2*>(A.K + o + 2) = make_double2(v, v);
    *reinterpret_cast<double2*>(A.Kc + o) = make_double2(v, v);
    *reinterpret_cast<double2*>(A.Kc + o + 2) = make_double2(v, v);
    *reinterpret_cast<double2*>(A.D + o) = make_double2(v, v);
    *reinterpret_cast<double2*>(A.D + o + 2) = make_double2(v, v);
  }
}

int main() {
  const int p = 4096, ncls = 20480;
  const size_t nn = (size_t)p * p;
  B2 b;
  std::vector<int> cid(nn);
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < p; ++j) cid[(size_t)i * p + j] = (std::abs(i - j) * 5 + ((i * 7 + j) & 3)) % ncls;
  std::vector<double> kv(ncls);
  for (int u = 0; u < ncls; ++u) kv[u] = 1.0 / (1 + u);
  for (int a = 0; a < 2; ++a) {
    int* dc; double *dk, *dd, *K, *Kc, *D;
    CHK(hipMalloc(&dc, nn * 4)); CHK(hipMalloc(&dk, ncls * 8)); CHK(hipMalloc(&dd, ncls * 8));
    CHK(hipMalloc(&K, nn * 8)); CHK(hipMalloc(&Kc, nn * 8)); CHK(hipMalloc(&D, nn * 8));
    CHK(hipMemcpy(dc, cid.data(), nn * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dk, kv.data(), ncls * 8, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dd, kv.data(), ncls * 8, hipMemcpyHostToDevice));
    b.a[a] = Ax{dc, dk, dd, K, Kc, D, p};
  }
  const double bytes = 2.0 * nn * (4 + 24);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) -> int {
    for (int w = 0; w < 3; ++w) launch();
    CHK(hipEventRecord(e0));
    const int it = 20;
    for (int k = 0; k < it; ++k) launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / it;
    printf("  %-48s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
    return 0;
  };
  printf("gather at C5 size: %.1f MB per launch\n", bytes / 1e6);
  timeit("V0 32x32 tile per WG (gather_kernel)", [&] { hipLaunchKernelGGL(v0, dim3(2, (p / 32) * (p / 32)), dim3(256), 0, 0, b); });
  timeit("V1 8x512 per WG, 2 cols/lane (gather_wide)", [&] { hipLaunchKernelGGL(v1<false>, dim3(p / 512, p / 8, 2), dim3(256), 0, 0, b); });
  timeit("V1 + nontemporal stores", [&] { hipLaunchKernelGGL(v1<true>, dim3(p / 512, p / 8, 2), dim3(256), 0, 0, b); });
  timeit("V2 4 rows x 1024 per WG, 4 cols/lane", [&] { hipLaunchKernelGGL(v2, dim3(p / 1024, p / 4, 2), dim3(256), 0, 0, b); });
  timeit("V3 floor: ids read, constants written", [&] { hipLaunchKernelGGL(v3, dim3(p / 1024, p / 4, 2), dim3(256), 0, 0, b); });
  timeit("V0 again", [&] { hipLaunchKernelGGL(v0, dim3(2, (p / 32) * (p / 32)), dim3(256), 0, 0, b); });
  return 0;
}
