// gemm.hip — batched fp64 MFMA GEMM / GEMV with fused epilogues (gfx950).
//
// Every dense product of the log-joint step (code/model_GP_solver_2d.py:104-119 solves and
// matmuls, and the products of their reverse pass) becomes one
// descriptor of a batched launch: C = alpha*op(A)op(B) [+ alpha2*op(A2)op(B2)] + epilogue.
// The dual-product form fuses R = D1 A + Bt D2^T - F into one tile loop; epilogues also
// produce the reductions the loss needs (||R||^2, <U,S>) as deterministic per-tile partials.
//
// Tile: 32x32 per 256-thread workgroup; wave w owns the 16x16 quadrant (w>>1, w&1);
// K-steps of 32 staged through LDS; v_mfma_f64_16x16x4_f64 with the measured gfx950 map
// (A[i=l&15][k=l>>4], B[k=l>>4][j=l&15], C/D row=(l>>4)+4r, col=l&15).
#include "gpk_internal.h"

namespace gpk {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int GSA = 34;  // A-role LDS stride (doubles)
constexpr int GSB = 48;  // B-role LDS stride

__device__ __forceinline__ void stage_tiles(double* sA, double* sB, const double* A, int lda,
                                            int ta, const double* B, int ldb, int tb, int i0,
                                            int j0, int k0, int t) {
  const int c = t & 31, r0 = t >> 5;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int r = r0 + 8 * m;
    if (!ta)
      sA[r * GSA + c] = A[(size_t)(i0 + r) * lda + k0 + c];   // op(A)[i0+r][k0+c]
    else
      sA[c * GSA + r] = A[(size_t)(k0 + r) * lda + i0 + c];   // op(A)[i0+c][k0+r] = A[k0+r][i0+c]
    if (!tb)
      sB[r * GSB + c] = B[(size_t)(k0 + r) * ldb + j0 + c];   // op(B)[k0+r][j0+c]
    else
      sB[c * GSB + r] = B[(size_t)(j0 + r) * ldb + k0 + c];   // op(B)[k0+c][j0+r] = B[j0+r][k0+c]
  }
}

__device__ __forceinline__ d4 mma32(const double* sA, const double* sB, int wr, int wc, int lane,
                                    d4 acc) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const double a = sA[(16 * wr + li) * GSA + 4 * kk + lk];
    const double b = sB[(4 * kk + lk) * GSB + 16 * wc + li];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ double block_sum_256(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int t = threadIdx.x;
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  double s = 0.0;
  if (t == 0) s = (red[0] + red[1]) + (red[2] + red[3]);
  return s;
}

__global__ __launch_bounds__(256) void gemm_kernel(const GemmDesc* __restrict__ descs,
                                                   const StepScalars* __restrict__ sc) {
  const GemmDesc& d = descs[blockIdx.y];
  const int tn = d.N >> 5;
  const int tiles = (d.M >> 5) * tn;
  if ((int)blockIdx.x >= tiles) return;
  const int ti = blockIdx.x / tn, tj = blockIdx.x % tn;
  const int i0 = ti * 32, j0 = tj * 32;

  __shared__ double sA[32 * GSA];
  __shared__ double sB[32 * GSB];
  __shared__ double sred[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;

  d4 acc1 = {0.0, 0.0, 0.0, 0.0}, acc2 = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < d.K; k0 += 32) {
    stage_tiles(sA, sB, d.A, d.lda, d.ta, d.B, d.ldb, d.tb, i0, j0, k0, t);
    __syncthreads();
    acc1 = mma32(sA, sB, wr, wc, lane, acc1);
    __syncthreads();
  }
  for (int k0 = 0; k0 < d.K2; k0 += 32) {
    stage_tiles(sA, sB, d.A2, d.lda2, d.ta2, d.B2, d.ldb2, d.tb2, i0, j0, k0, t);
    __syncthreads();
    acc2 = mma32(sA, sB, wr, wc, lane, acc2);
    __syncthreads();
  }

  double alpha = d.alpha;
  if (d.vscale) alpha *= sc->v;
  double part = 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = i0 + 16 * wr + (lane >> 4) + 4 * r, col = j0 + 16 * wc + (lane & 15);
    double c = alpha * acc1[r];
    if (d.K2) c += d.alpha2 * acc2[r];
    switch (d.epi) {
      case EPI_STORE:
        if (d.beta != 0.0) c += d.beta * d.C0[(size_t)row * d.ldc0 + col];
        break;
      case EPI_RESID: {
        const size_t fo = (size_t)row * d.ldf + col;
        c -= d.F[fo];
        if (d.ac) {
          const double u = d.U[fo];
          c += u * (u * u - 1.0);
        }
        part += c * c;
        break;
      }
      case EPI_QUAD:
        part += c * d.U[(size_t)row * d.ldf + col];
        break;
      case EPI_HALFS:
        c += 0.5 * d.C0[(size_t)row * d.ldc0 + col];
        break;
    }
    d.C[(size_t)row * d.ldc + col] = c;
  }
  if (d.red) {
    double s = block_sum_256(part, sred);
    if (t == 0) d.red[blockIdx.x] = s;
  }
}

hipError_t launch_gemm_batch(const GemmDesc* descs_dev, int ndesc, int max_tiles,
                             const StepScalars* sc, hipStream_t s) {
  hipLaunchKernelGGL(gemm_kernel, dim3(max_tiles, ndesc), dim3(256), 0, s, descs_dev, sc);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// GEMV (1D solver, code/model_GP_solver_1d.py:92,97): one wave per row, 4 rows per block.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gemv_kernel(GemvDesc d) {
  __shared__ double sred[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int row = blockIdx.x * 4 + wv;
  double acc = 0.0;
  if (row < d.rows) {
    const double* a = d.A + (size_t)row * d.lda;
    for (int c = lane; c < d.p; c += 64) acc += a[c] * d.x[c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  double part = 0.0;
  if (lane == 0 && row < d.rows) {
    double y = d.alpha * acc;
    if (d.epi == EPI_RESID) {
      y -= d.F[row];
      if (d.ac) {
        const double u = d.U[row];
        y += u * (u * u - 1.0);
      }
      part = y * y;
    } else if (d.epi == EPI_QUAD) {
      part = y * d.U[row];
    }
    d.y[row] = y;
  }
  if (d.red) {
    if (lane == 0) sred[wv] = part;
    __syncthreads();
    if (t == 0) d.red[blockIdx.x] = (sred[0] + sred[1]) + (sred[2] + sred[3]);
  }
}

int gemv_blocks(int rows) { return (rows + 3) / 4; }

hipError_t launch_gemv(const GemvDesc& d, hipStream_t s) {
  hipLaunchKernelGGL(gemv_kernel, dim3(gemv_blocks(d.rows)), dim3(256), 0, s, d);
  return hipGetLastError();
}

}  // namespace gpk
