// Probe: the software-pipelined 128x128 fp64 tile (csrc/gemm_tile_dev.h) against libgpk's
// gemm_huge_kernel on square n^3 products, all four transpose signatures; variants of issue
// priority and of the sched_group_barrier interleave.  Correctness against a naive fp64 kernel
// (max abs error / max abs value); TF/s with HIP events over 5 launches after a warm-up.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
//   -I include tools/probes/gemm_tile_probe.hip -o /tmp/gemm_tile_probe
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/gemm.hip"
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/gemm_tile_dev.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

using namespace gpk;

template <int TA, int TB, int PRIO, bool SCHED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void tile_kernel(const double* A, int lda, const double* B, int ldb, double* C, int ldc, int M, int N, int K,
                 int per_xcd) {
  using namespace tile;
  constexpr int GM = 4;
  const int tm = (M + TM - 1) / TM, tn = (N + TM - 1) / TM;
  const int o = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (o >= tm * tn) return;
  const int gsz = GM * tn, grp = o / gsz, first = grp * GM;
  const int gm = min(GM, tm - first), in = o - grp * gsz;
  const int ti = first + in % gm, tj = in / gm;
  const int i0 = ti * TM, j0 = tj * TM;
  __shared__ double lds[LDS_DOUBLES];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};
  product<TA, TB, false, PRIO, SCHED>(A, lda, B, ldb, K, M, N, i0, j0, 1.0, lds, t, wr, wc, lane, acc);
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i0 + 64 * wr + 16 * x + (lane >> 4) + 4 * r;
        const int col = j0 + 64 * wc + 16 * y + (lane & 15);
        if (row < M && col < N) C[(size_t)row * ldc + col] = acc[x][y][r];
      }
}

__global__ void ref_gemm(const double* A, int ta, const double* B, int tb, double* C, int n, int ld) {
  const int i = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int k = 0; k < n; ++k) {
    const double a = ta ? A[(size_t)k * ld + i] : A[(size_t)i * ld + k];
    const double b = tb ? B[(size_t)j * ld + k] : B[(size_t)k * ld + j];
    s = fma(a, b, s);
  }
  C[(size_t)i * ld + j] = s;
}

typedef void (*TileFn)(const double*, int, const double*, int, double*, int, int, int, int, int);
template <int PRIO, bool SCHED>
static TileFn tile_fn(int ta, int tb) {
  if (!ta && !tb) return tile_kernel<0, 0, PRIO, SCHED>;
  if (!ta && tb) return tile_kernel<0, 1, PRIO, SCHED>;
  if (ta && !tb) return tile_kernel<1, 0, PRIO, SCHED>;
  return tile_kernel<1, 1, PRIO, SCHED>;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int ld = n;
  const size_t nn = (size_t)n * ld;
  std::vector<double> h(nn);
  double *A, *B, *C, *R;
  CHK(hipMalloc(&A, nn * 8)); CHK(hipMalloc(&B, nn * 8)); CHK(hipMalloc(&C, nn * 8)); CHK(hipMalloc(&R, nn * 8));
  for (size_t i = 0; i < nn; ++i) h[i] = std::sin(0.37 * i) * 0.5;
  CHK(hipMemcpy(A, h.data(), nn * 8, hipMemcpyHostToDevice));
  for (size_t i = 0; i < nn; ++i) h[i] = std::cos(0.11 * i + 1.0) * 0.5;
  CHK(hipMemcpy(B, h.data(), nn * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const double flops = 2.0 * n * (double)n * n;
  const int tiles = ((n + 127) / 128) * ((n + 127) / 128), per = (tiles + 7) / 8;
  std::vector<double> hr(nn), hc(nn);
  auto err = [&]() {
    double md = 0, mx = 0;
    for (size_t i = 0; i < nn; ++i) { md = fmax(md, fabs(hc[i] - hr[i])); mx = fmax(mx, fabs(hr[i])); }
    return md / mx;
  };
  for (int ta = 0; ta < 2; ++ta)
    for (int tb = 0; tb < 2; ++tb) {
      hipLaunchKernelGGL(ref_gemm, dim3((n + 255) / 256, n), dim3(256), 0, 0, A, ta, B, tb, R, n, ld);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(hr.data(), R, nn * 8, hipMemcpyDeviceToHost));
      struct V { const char* name; TileFn fn; } vs[] = {
          {"tile regs sched ", tile_fn<0, true>(ta, tb)},
          {"tile regs nosch ", tile_fn<0, false>(ta, tb)},
      };
      for (const V& v : vs) {
        CHK(hipMemset(C, 0, nn * 8));
        hipLaunchKernelGGL(v.fn, dim3(8 * per), dim3(256), 0, 0, A, ld, B, ld, C, ld, n, n, n, per);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(hc.data(), C, nn * 8, hipMemcpyDeviceToHost));
        const double e = err();
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CHK(hipEventRecord(e0));
          for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(v.fn, dim3(8 * per), dim3(256), 0, 0, A, ld, B, ld, C, ld, n, n, n, per);
          CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
          float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
          best = fminf(best, ms / 5);
        }
        printf("n=%d ta=%d tb=%d %s: %.3f ms  %.1f TF/s  relerr %.2e\n", n, ta, tb, v.name, best, flops / best / 1e9, e);
      }
      {
        GemmDesc d{};
        d.A = A; d.lda = ld; d.ta = ta; d.B = B; d.ldb = ld; d.tb = tb; d.alpha = 1.0; d.C = C; d.ldc = ld;
        d.M = n; d.N = n; d.K = n; d.epi = EPI_STORE;
        CHK(launch_gemm_auto(&d, 1, nullptr, 0, GEMM_HUGE));
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(hc.data(), C, nn * 8, hipMemcpyDeviceToHost));
        const double e = err();
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CHK(hipEventRecord(e0));
          for (int it = 0; it < 5; ++it) CHK(launch_gemm_auto(&d, 1, nullptr, 0, GEMM_HUGE));
          CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
          float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
          best = fminf(best, ms / 5);
        }
        printf("n=%d ta=%d tb=%d libgpk huge     : %.3f ms  %.1f TF/s  relerr %.2e\n", n, ta, tb, best, flops / best / 1e9, e);
      }
      fflush(stdout);
    }
  return 0;
}
