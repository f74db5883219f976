// gemm_huge_dev.h — the 128x128-tile fp64 MFMA product loop (gfx950), shared by the large GEMM
// (gemm.hip gemm_huge_kernel) and the large-factor SPD inverse's update (spdinv_big.hip).
// A 128x128 output tile per 256-thread workgroup, each wave a 64x64 quadrant = 4x4
// v_mfma_f64_16x16x4 blocks (every LDS fragment feeds 4 MFMAs, 16 independent accumulation
// chains per wave); 16-deep K-steps through double-buffered LDS ([k][m] / [k][n], rows S = 140
// doubles apart), the next step prefetched global -> registers with 16-B loads that read whole
// contiguous segments.  LDS: 2 x 2 x KS x S doubles (70 KB).
// Row stride: a k-contiguous operand (A[i][k], B[j][k]) is transposed into LDS by 8-B stores,
// 8 k rows x 8 m columns per wave instruction; with S = 144 (a multiple of 16 doubles) the 8 k
// rows hit the same banks (8-way), with S = 140 (or 148, 156: S = 4 or 12 mod 16) they spread.
// C5 gemm_B stage 60.0 -> 63.6 TF/s, C5 step 43.0 -> 41.2 ms (same box; 152: 60.0, 164: 52.2
// -- one workgroup per CU).
#pragma once
#include "gpk_internal.h"

namespace gpk {

typedef double d4 __attribute__((ext_vector_type(4)));

namespace huge {
constexpr int TM = 128, KS = 16, S = 140, GROUP_M = 4;

struct Regs { double2 a[4], b[4]; };

// Branch-free: rows / columns past M, N (edge tiles of a 32-padded matrix) load a clamped,
// in-bounds address instead.  Those values only reach output rows / columns >= M, N, which are
// never stored, so no zeroing is needed -- and an unconditional load keeps the K-loop free of
// divergent control flow (a guarded load becomes an exec-mask branch, and the compiler then
// shuttles the 128 accumulators between VGPRs and AGPRs every K-step).
__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }

template <int ta, int tb>
__device__ __forceinline__ void fetch(Regs& R, const double* A, int lda, const double* B, int ldb,
                                      int M, int N, int i0, int j0, int k0, int t) {
  if (!ta) {  // A[i][k], k contiguous (16 per tile row): row (t>>3) + 32j, k pair 2(t&7)
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = i0 + (t >> 3) + 32 * j;
      R.a[j] = ld2(A + (size_t)min(r, M - 1) * lda + k0 + kc);
    }
  } else {    // A[k][i], i contiguous (128 per tile row): k row (t>>6) + 4j, i pair 2(t&63)
    const int ic = i0 + 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kr = (t >> 6) + 4 * j;
      R.a[j] = ld2(A + (size_t)(k0 + kr) * lda + min(ic, M - 2));
    }
  }
  if (!tb) {  // B[k][j], j contiguous
    const int jc = j0 + 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kr = (t >> 6) + 4 * j;
      R.b[j] = ld2(B + (size_t)(k0 + kr) * ldb + min(jc, N - 2));
    }
  } else {    // B[j][k], k contiguous
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = j0 + (t >> 3) + 32 * j;
      R.b[j] = ld2(B + (size_t)min(r, N - 1) * ldb + k0 + kc);
    }
  }
}

// registers -> LDS ([k][m] and [k][n]); A scaled by sa (the dual product's alpha2 / alpha)
template <int ta, int tb>
__device__ __forceinline__ void store(const Regs& R, double* sA, double* sB, double sa, int t) {
  if (!ta) {
    const int kc = 2 * (t & 7);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (t >> 3) + 32 * j;
      sA[kc * S + r] = sa * R.a[j].x;
      sA[(kc + 1) * S + r] = sa * R.a[j].y;
    }
  } else {
    const int ic = 2 * (t & 63);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double2 v = {sa * R.a[j].x, sa * R.a[j].y};
      *reinterpret_cast<double2*>(sA + ((t >> 6) + 4 * j) * S + ic) = v;
    }
  }
  if (!tb) {
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

// acc += sa * op(A) op(B) over K (multiple of 16... of 32 by the padding contract)
template <int ta, int tb>
__device__ __forceinline__ void product_t(const double* A, int lda, const double* B, int ldb,
                                          int K, int M, int N, int i0, int j0, double sa, double* sA0,
                                          double* sB0, int t, int wr, int wc, int lane, d4 (&acc)[4][4]) {
  constexpr int SZ = KS * S;
  Regs R;
  const int nk = K / KS;
  fetch<ta, tb>(R, A, lda, B, ldb, M, N, i0, j0, 0, t);
  store<ta, tb>(R, sA0, sB0, sa, t);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) fetch<ta, tb>(R, A, lda, B, ldb, M, N, i0, j0, (kt + 1) * KS, t);
    mma(sA0 + cur * SZ, sB0 + cur * SZ, wr, wc, lane, acc);
    if (kt + 1 < nk) store<ta, tb>(R, sA0 + (cur ^ 1) * SZ, sB0 + (cur ^ 1) * SZ, sa, t);
    __syncthreads();
  }
}

}  // namespace huge

}  // namespace gpk
