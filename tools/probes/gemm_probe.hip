// Probe: per-launch cost of 256^3 fp64 GEMM variants in a graph of dependent launches.
//   v0: libgpk gemm_small_kernel (16x16 tile / WG, K split over 4 waves, global->VGPR)
//   v1: LDS-staged 16x16 tile / WG: 16-B coalesced loads of the A row-panel and B col-panel
//   v2: copy-only kernel (loads the same panels, no MFMA) -> memory-latency floor
//   v3: empty kernel (launch floor)
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/gemm.hip"
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

using namespace gpk;

// v1: C[16x16 tile] = A[i0:i0+16, :] * B[:, j0:j0+16], N = K = 256, row-major, ld = 256
template <int KD>
__global__ __launch_bounds__(256) void gemm_lds16(const double* __restrict__ A, const double* __restrict__ B,
                                                  double* __restrict__ C, int n) {
  const int tn = n >> 4;
  const int i0 = (blockIdx.x / tn) * 16, j0 = (blockIdx.x % tn) * 16;
  __shared__ double sA[16][KD + 2];   // row panel, +2 pad
  __shared__ double sB[KD][16 + 2];   // column panel
  __shared__ double part[4][256];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // A panel: 16 x KD doubles = 16*KD/2 double2 ; 256 threads
  for (int e = t; e < 16 * KD / 2; e += 256) {
    const int r = e / (KD / 2), c2 = e % (KD / 2);
    const double2 v = *reinterpret_cast<const double2*>(A + (size_t)(i0 + r) * n + 2 * c2);
    sA[r][2 * c2] = v.x; sA[r][2 * c2 + 1] = v.y;
  }
  for (int e = t; e < KD * 8; e += 256) {
    const int r = e >> 3, c2 = e & 7;
    const double2 v = *reinterpret_cast<const double2*>(B + (size_t)r * n + j0 + 2 * c2);
    sB[r][2 * c2] = v.x; sB[r][2 * c2 + 1] = v.y;
  }
  __syncthreads();
  const int li = lane & 15, lk = lane >> 4;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  const int kb = wv * (KD / 4);
#pragma unroll
  for (int s = 0; s < KD / 16; ++s) {
    const int k = kb + 4 * s + lk;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sA[li][k], sB[k][li], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) part[wv][lane * 4 + r] = acc[r];
  __syncthreads();
  if (wv) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = lane * 4 + r;
    C[(size_t)(i0 + (lane >> 4) + 4 * r) * n + j0 + (lane & 15)] =
        (part[0][q] + part[1][q]) + (part[2][q] + part[3][q]);
  }
}

template <int KD>
__global__ __launch_bounds__(256) void copy_panels(const double* __restrict__ A, const double* __restrict__ B,
                                                   double* __restrict__ C, int n) {
  const int tn = n >> 4;
  const int i0 = (blockIdx.x / tn) * 16, j0 = (blockIdx.x % tn) * 16;
  const int t = threadIdx.x;
  double s = 0.0;
  for (int e = t; e < 16 * KD / 2; e += 256) {
    const int r = e / (KD / 2), c2 = e % (KD / 2);
    const double2 v = *reinterpret_cast<const double2*>(A + (size_t)(i0 + r) * n + 2 * c2);
    s += v.x + v.y;
  }
  for (int e = t; e < KD * 8; e += 256) {
    const int r = e >> 3, c2 = e & 7;
    const double2 v = *reinterpret_cast<const double2*>(B + (size_t)r * n + j0 + 2 * c2);
    s += v.x + v.y;
  }
  C[(size_t)(i0 + (t >> 4)) * n + j0 + (t & 15)] = s;
}

__global__ void empty_k(double* C) {
  if (threadIdx.x == 1000) C[0] = 1.0;
}

int main() {
  const int n = 256, NL = 100;
  std::vector<double> h((size_t)n * n);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0 / (1.0 + (i % 97));
  double *A, *B, *C0, *C1;
  CHK(hipMalloc(&A, 8 * h.size())); CHK(hipMalloc(&B, 8 * h.size()));
  CHK(hipMalloc(&C0, 8 * h.size())); CHK(hipMalloc(&C1, 8 * h.size()));
  CHK(hipMemcpy(A, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
  CHK(hipMemcpy(B, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
  CHK(hipMemcpy(C0, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
  StepScalars* sc;
  CHK(hipMalloc(&sc, sizeof(StepScalars)));
  CHK(hipMemset(sc, 0, sizeof(StepScalars)));
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const char* names[] = {"v0 gemm_small (libgpk)", "v1 lds16 panels", "v2 copy panels only", "v3 empty"};
  for (int v = 0; v < 4; ++v) {
    hipGraph_t g; hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int l = 0; l < NL; ++l) {
      double* src = (l & 1) ? C1 : C0;   // dependent chain: C_{l+1} = A * C_l
      double* dst = (l & 1) ? C0 : C1;
      if (v == 0) {
        GemmDesc d{};
        d.A = A; d.lda = n; d.B = src; d.ldb = n; d.C = dst; d.ldc = n; d.M = n; d.N = n; d.K = n;
        d.alpha = 1.0; d.epi = EPI_STORE;
        CHK(launch_gemm_batch(&d, 1, (n / 16) * (n / 16), sc, s, 1));
      } else if (v == 1) {
        hipLaunchKernelGGL(gemm_lds16<256>, dim3((n / 16) * (n / 16)), dim3(256), 0, s, A, src, dst, n);
      } else if (v == 2) {
        hipLaunchKernelGGL(copy_panels<256>, dim3((n / 16) * (n / 16)), dim3(256), 0, s, A, src, dst, n);
      } else {
        hipLaunchKernelGGL(empty_k, dim3((n / 16) * (n / 16)), dim3(256), 0, s, dst);
      }
    }
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    CHK(hipEventRecord(e0, s));
    for (int r = 0; r < 5; ++r) CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-26s %.3f us per launch\n", names[v], ms * 1000.0 / (5 * NL));
  }
  // correctness of v1 vs v0 on one product
  {
    GemmDesc d{};
    d.A = A; d.lda = n; d.B = B; d.ldb = n; d.C = C0; d.ldc = n; d.M = n; d.N = n; d.K = n;
    d.alpha = 1.0; d.epi = EPI_STORE;
    CHK(launch_gemm_batch(&d, 1, (n / 16) * (n / 16), sc, s, 1));
    hipLaunchKernelGGL(gemm_lds16<256>, dim3((n / 16) * (n / 16)), dim3(256), 0, s, A, B, C1, n);
    std::vector<double> r0(h.size()), r1(h.size());
    CHK(hipMemcpy(r0.data(), C0, 8 * h.size(), hipMemcpyDeviceToHost));
    CHK(hipMemcpy(r1.data(), C1, 8 * h.size(), hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < h.size(); ++i) md = fmax(md, fabs(r0[i] - r1[i]));
    printf("max |v0 - v1| = %.3e (ref %.3e)\n", md, r0[12345]);
  }
  return 0;
}
