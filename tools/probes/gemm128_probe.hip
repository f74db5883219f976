// Probe: 128x128-tile fp64 MFMA GEMM (v_mfma_f64_16x16x4, 4 waves x 64x64) vs libgpk's 64x64
// gemm_big_kernel on the C5 shapes (4096^3, all four transpose combinations).
// Correctness against a naive fp64 kernel; TF/s with HIP events.
#include "../../gaussian-process-slover-for-high-freq-pde_amd/csrc/gemm.hip"
#include <cstdio>
#include <vector>
#include <cmath>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

using namespace gpk;

namespace h128 {
constexpr int TM = 128, KS = 16, S = 144;  // LDS row stride: k and k+1 rows 32 banks apart

template <int TA, int TB>
struct Regs { double2 a[4], b[4]; };

// global -> registers for K-step k0: op(A) tile [TM x KS], op(B) tile [KS x TM].  Every load
// instruction reads whole contiguous segments: a 128-double source row is one wave x 16 B, a
// 16-double source row is 8 lanes x 16 B.
template <int TA, int TB>
__device__ __forceinline__ void fetch(Regs<TA, TB>& R, const double* A, int lda, const double* B, int ldb,
                                      int M, int N, int i0, int j0, int k0, int t) {
  const double2 z = {0.0, 0.0};
  if (!TA) {  // A[i][k] (k contiguous, 16 per tile row): row (t>>3) + 32j, k pair 2(t&7)
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (t >> 3) + 32 * j;
      R.a[j] = (i0 + r < M) ? *reinterpret_cast<const double2*>(A + (size_t)(i0 + r) * lda + k0 + kc) : z;
    }
  } else {    // A[k][i] (i contiguous, 128 per tile row): k row (t>>6) + 4j, i pair 2(t&63)
    const int ic = 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kr = (t >> 6) + 4 * j;
      R.a[j] = (i0 + ic < M) ? *reinterpret_cast<const double2*>(A + (size_t)(k0 + kr) * lda + i0 + ic) : z;
    }
  }
  if (!TB) {  // B[k][j] (j contiguous)
    const int jc = 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kr = (t >> 6) + 4 * j;
      R.b[j] = (j0 + jc < N) ? *reinterpret_cast<const double2*>(B + (size_t)(k0 + kr) * ldb + j0 + jc) : z;
    }
  } else {    // B[j][k] (k contiguous)
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (t >> 3) + 32 * j;
      R.b[j] = (j0 + r < N) ? *reinterpret_cast<const double2*>(B + (size_t)(j0 + r) * ldb + k0 + kc) : z;
    }
  }
}

// registers -> LDS, both as [k][m] / [k][n]
template <int TA, int TB>
__device__ __forceinline__ void store(const Regs<TA, TB>& R, double* sA, double* sB, int t) {
  if (!TA) {
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (t >> 3) + 32 * j;
      sA[kc * S + r] = R.a[j].x;
      sA[(kc + 1) * S + r] = R.a[j].y;
    }
  } else {
    const int ic = 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<double2*>(sA + ((t >> 6) + 4 * j) * S + ic) = R.a[j];
  }
  if (!TB) {
    const int jc = 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<double2*>(sB + ((t >> 6) + 4 * j) * S + jc) = R.b[j];
  } else {
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (t >> 3) + 32 * j;
      sB[kc * S + r] = R.b[j].x;
      sB[(kc + 1) * S + r] = R.b[j].y;
    }
  }
}

__device__ __forceinline__ void mma(const double* sA, const double* sB, int wr, int wc, int lane,
                                    d4 (&acc)[4][4]) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < KS / 4; ++kk) {
    const int k = 4 * kk + lk;
    double a[4], b[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      a[x] = sA[k * S + 64 * wr + 16 * x + li];
      b[x] = sB[k * S + 64 * wc + 16 * x + li];
    }
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
        acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[y], acc[x][y], 0, 0, 0);
  }
}

template <int TA, int TB>
__global__ __launch_bounds__(256) void gemm128(const double* A, int lda, const double* B, int ldb,
                                               double* C, int ldc, int M, int N, int K, int per_xcd,
                                               int group_m) {
  const int tm = (M + TM - 1) / TM, tn = (N + TM - 1) / TM;
  const int o = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);  // XCD-major dealing
  if (o >= tm * tn) return;
  // grouped order: group_m tile rows advance together (A/B panel reuse in the XCD's L2)
  const int gsz = group_m * tn;
  const int grp = o / gsz, first = grp * group_m;
  const int gm = min(group_m, tm - first);
  const int in = o - grp * gsz;
  const int ti = first + in % gm, tj = in / gm;
  const int i0 = ti * TM, j0 = tj * TM;
  __shared__ double sA[2][KS * S], sB[2][KS * S];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};
  Regs<TA, TB> R;
  const int nk = K / KS;
  fetch<TA, TB>(R, A, lda, B, ldb, M, N, i0, j0, 0, t);
  store<TA, TB>(R, sA[0], sB[0], t);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) fetch<TA, TB>(R, A, lda, B, ldb, M, N, i0, j0, (kt + 1) * KS, t);
    mma(sA[cur], sB[cur], wr, wc, lane, acc);
    if (kt + 1 < nk) store<TA, TB>(R, sA[cur ^ 1], sB[cur ^ 1], t);
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i0 + 64 * wr + 16 * x + (lane >> 4) + 4 * r, col = j0 + 64 * wc + 16 * y + (lane & 15);
        if (row < M && col < N) C[(size_t)row * ldc + col] = acc[x][y][r];
      }
}
}  // namespace h128

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

static int g_ld = 0;
template <int TA, int TB>
static hipError_t run128(const double* A, const double* B, double* C, int n, int gm) {
  const int tiles = ((n + 127) / 128) * ((n + 127) / 128);
  const int per = (tiles + 7) / 8;
  const int ld = g_ld;
  hipLaunchKernelGGL((h128::gemm128<TA, TB>), dim3(8 * per), dim3(256), 0, 0, A, ld, B, ld, C, ld, n, n, n, per, gm);
  return hipGetLastError();
}

static hipError_t run128v(int ta, int tb, const double* A, const double* B, double* C, int n, int gm) {
  if (!ta && !tb) return run128<0, 0>(A, B, C, n, gm);
  if (!ta && tb) return run128<0, 1>(A, B, C, n, gm);
  if (ta && !tb) return run128<1, 0>(A, B, C, n, gm);
  return run128<1, 1>(A, B, C, n, gm);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int pad = argc > 2 ? atoi(argv[2]) : 0;
  g_ld = n + pad;
  const size_t nn = (size_t)n * g_ld;
  std::vector<double> h(nn);
  double *A, *B, *C, *R;
  CHK(hipMalloc(&A, nn * 8)); CHK(hipMalloc(&B, nn * 8)); CHK(hipMalloc(&C, nn * 8)); CHK(hipMalloc(&R, nn * 8));
  for (size_t i = 0; i < nn; ++i) h[i] = std::sin(0.37 * i) * 0.5;
  CHK(hipMemcpy(A, h.data(), nn * 8, hipMemcpyHostToDevice));
  for (size_t i = 0; i < nn; ++i) h[i] = std::cos(0.11 * i + 1.0) * 0.5;
  CHK(hipMemcpy(B, h.data(), nn * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const double flops = 2.0 * n * (double)n * n;
  for (int ta = 0; ta < 2; ++ta)
    for (int tb = 0; tb < 2; ++tb) {
      hipLaunchKernelGGL(ref_gemm, dim3((n + 255) / 256, n), dim3(256), 0, 0, A, ta, B, tb, R, n, g_ld);
      CHK(hipDeviceSynchronize());
      std::vector<double> hr(nn), hc(nn);
      CHK(hipMemcpy(hr.data(), R, nn * 8, hipMemcpyDeviceToHost));
      for (int gm : {4}) {
        CHK(run128v(ta, tb, A, B, C, n, gm));
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(hc.data(), C, nn * 8, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (size_t i = 0; i < nn; ++i) {
          if ((int)(i % g_ld) >= n) continue;
          md = fmax(md, fabs(hc[i] - hr[i])); mx = fmax(mx, fabs(hr[i]));
        }
        CHK(hipEventRecord(e0));
        for (int it = 0; it < 5; ++it) CHK(run128v(ta, tb, A, B, C, n, gm));
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("ld=%d gemm128 ta=%d tb=%d group_m=%d: %.3f ms  %.1f TF/s  maxerr %.2e\n", g_ld, ta, tb, gm, ms / 5, flops / (ms / 5) / 1e9, md / mx);
      }
      // libgpk big (64x64) and huge (128x128) kernels on the same shape
      for (int variant : {GEMM_BIG, GEMM_HUGE}) {
        GemmDesc d{};
        d.A = A; d.lda = g_ld; d.ta = ta; d.B = B; d.ldb = g_ld; d.tb = tb; d.alpha = 1.0; d.C = C; d.ldc = g_ld;
        d.M = n; d.N = n; d.K = n; d.epi = EPI_STORE;
        CHK(launch_gemm_auto(&d, 1, nullptr, 0, variant));
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(hc.data(), C, nn * 8, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (size_t i = 0; i < nn; ++i) {
          if ((int)(i % g_ld) >= n) continue;
          md = fmax(md, fabs(hc[i] - hr[i])); mx = fmax(mx, fabs(hr[i]));
        }
        CHK(hipEventRecord(e0));
        for (int it = 0; it < 5; ++it) CHK(launch_gemm_auto(&d, 1, nullptr, 0, variant));
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("libgpk %s ta=%d tb=%d: %.3f ms  %.1f TF/s  maxerr %.2e\n", variant == GEMM_BIG ? "big " : "huge",
               ta, tb, ms / 5, flops / (ms / 5) / 1e9, md / mx);
      }
    }
  return 0;
}
