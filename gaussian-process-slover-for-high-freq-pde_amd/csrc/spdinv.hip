// spdinv.hip — SPD inverse + log-determinant of the covariance factors (gfx950, fp64 MFMA).
//
// Replaces jnp.linalg.solve (LU getrf/getrs) and jnp.linalg.slogdet (a second LU) of
//   code/model_GP_solver_1d.py:92,135-137 and code/model_GP_solver_2d.py:104-105,157-162.
// The step needs K^{-1} explicitly anyway (the log-det gradient is K^{-1}), so every solve
// becomes an MFMA GEMM against K^{-1} and the log-det falls out of the Cholesky pivots.
//
// Algorithm: blocked Cholesky-Gauss-Jordan sweep, 32x32 pivot blocks.  For pivot block P
// (the current Schur complement S = X_PP = L L^T, Cholesky-factored in LDS by one workgroup):
//     V   = L^{-1} X_P.                  (panel "TRSM" by MFMA against L^{-1})
//     X_RR -= V_R^T V_R                  (symmetric rank-32 update, like SYRK)
//     X_PR  = L^{-T} V_R,  X_RP = X_PR^T,  X_PP = -L^{-T} L^{-1}
// After every block is swept X = -K^{-1}; the last sweep flips the sign.  Using L^{-1}
// (not X_PP^{-1}) for the update keeps the accuracy of a Cholesky-based inverse: a plain
// block Gauss-Jordan with explicit X_PP^{-1} lost ~4 digits at cond(K) = 1e7.
// log det K = sum_k 2 sum_i log L_ii over pivot blocks.  A non-positive pivot raises
// GPK_ENOTPD through *status.
//
// One launch per pivot block (ping-pong X -> Y, no intra-launch hazards); a 256-thread
// workgroup owns one 32x32 output tile (4 waves x 16x16 v_mfma_f64_16x16x4 quadrants) and
// recomputes the two 32x32 panel pieces it needs; the workgroup that produces the NEXT
// pivot tile factors it in its tail, so the next launch finds L^{-1} ready: N/32 launches,
// batched over both Kronecker factors.
#include "gpk_internal.h"
#include "spd_pivot.h"

namespace gpk {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int SA = 34;  // LDS row stride for A-role tiles (conflict-free ds_read_b64 A[i][k])
constexpr int SB = 48;  // LDS row stride for B-role tiles (conflict-free B[k][j])
struct SpdBatch {
  double* X[2];   // buffer holding the assembled K (even sweeps read it)
  double* Y[2];   // pong buffer (odd sweeps read it)
  int p[2];
  int T[2];       // p / 32
  double* piv[2]; // [T][32*32] L^{-1} of each pivot block
  double* ldet[2];
  double* pst[2];  // refinement gate [2]: K_00, bits of max diag K^{-1} (gate_open)
  int n[2];        // true size: padded rows (identity) are left out of pst
  int* status[2];
};

__global__ __launch_bounds__(256) void pivot_init_kernel(SpdBatch b) {
  const int m = blockIdx.x;
  __shared__ double A[32 * SP], M[32 * SP], pv[32];
  const int t = threadIdx.x;
  const double* X = b.X[m];
  const int p = b.p[m];
  for (int e = t; e < 1024; e += 256) A[(e >> 5) * SP + (e & 31)] = X[(size_t)(e >> 5) * p + (e & 31)];
  __syncthreads();
  const double ls = pivot_chol_inv_block(A, M, pv, t, b.status[m]);
  double* piv = b.piv[m];
  for (int e = t; e < 1024; e += 256) piv[e] = M[(e >> 5) * SP + (e & 31)];
  if (t == 0) {
    b.ldet[m][0] = ls;
    b.pst[m][0] = X[0];  // K_00 = max diag K (stationary kernel + jitter)
    b.pst[m][1] = 0.0;   // max diag K^{-1}: atomicMax'd by the last sweep
  }
}

// acc += A(32x32, element (i,k) at a[i*sai + k*sak]) * B(32x32, (k,j) at bm[k*sbk + j*sbj]),
// this wave's 16x16 quadrant (wr, wc).  Strides let one LDS image serve transposed reads.
__device__ __forceinline__ d4 mma_t(const double* a, int sai, int sak, const double* bm, int sbk,
                                    int sbj, int wr, int wc, int lane, d4 acc) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = 4 * kk + lk;
    const double av = a[(16 * wr + li) * sai + k * sak];
    const double bv = bm[k * sbk + (16 * wc + li) * sbj];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ void store_quad(double* s, int ld, int wr, int wc, int lane, d4 v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) s[(16 * wr + (lane >> 4) + 4 * r) * ld + 16 * wc + (lane & 15)] = v[r];
}

__global__ __launch_bounds__(256) void sweep_kernel(SpdBatch b, int k) {
  const int m = blockIdx.y;
  const int p = b.p[m];
  const int T = b.T[m];
  if (k >= T) return;  // this factor is already inverted
  const int last = (k == T - 1);
  const int tile = blockIdx.x;
  if (tile >= T * T) return;
  const int I = tile / T, J = tile % T;
  const double* X = (k & 1) ? b.Y[m] : b.X[m];
  double* Y = (k & 1) ? b.X[m] : b.Y[m];
  const double* Li = b.piv[m] + (size_t)k * 1024;  // L^{-1} of pivot block k

  __shared__ double sL[32 * SA];                 // L^{-1}
  __shared__ double sXI[32 * SB], sXJ[32 * SB];  // X_PI, X_PJ, then V_I, V_J
  __shared__ double sP[32 * SP], sM[32 * SP], pv[32];  // next-pivot scratch
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int tx = t & 31, ty = t >> 5;
  const int P = k;

  // prefetch this wave's quadrant of X_IJ (consumed only in the epilogue)
  double xij[4] = {0.0, 0.0, 0.0, 0.0};
  if (I != P && J != P) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      xij[r] = X[(size_t)(I * 32 + 16 * wr + (lane >> 4) + 4 * r) * p + J * 32 + 16 * wc + (lane & 15)];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = ty + 8 * r;
    sL[row * SA + tx] = Li[row * 32 + tx];
    if (I != P) sXI[row * SB + tx] = X[(size_t)(P * 32 + row) * p + I * 32 + tx];
    if (J != P && J != I) sXJ[row * SB + tx] = X[(size_t)(P * 32 + row) * p + J * 32 + tx];
  }
  __syncthreads();
  const double* sVJ = (J == I) ? sXI : sXJ;
  // V_I = L^{-1} X_PI, V_J = L^{-1} X_PJ (in place, after everyone has read the inputs)
  d4 vi = {0.0, 0.0, 0.0, 0.0}, vj = {0.0, 0.0, 0.0, 0.0};
  if (I != P) vi = mma_t(sL, SA, 1, sXI, SB, 1, wr, wc, lane, vi);
  if (J != P && J != I) vj = mma_t(sL, SA, 1, sXJ, SB, 1, wr, wc, lane, vj);
  __syncthreads();
  if (I != P) store_quad(sXI, SB, wr, wc, lane, vi);
  if (J != P && J != I) store_quad(sXJ, SB, wr, wc, lane, vj);
  __syncthreads();

  d4 acc = {0.0, 0.0, 0.0, 0.0};
  if (I == P && J == P) {
    acc = mma_t(sL, 1, SA, sL, SA, 1, wr, wc, lane, acc);   // L^{-T} L^{-1}
  } else if (I == P) {
    acc = mma_t(sL, 1, SA, sVJ, SB, 1, wr, wc, lane, acc);  // L^{-T} V_J
  } else if (J == P) {
    acc = mma_t(sXI, 1, SB, sL, SA, 1, wr, wc, lane, acc);  // V_I^T L^{-1}
  } else {
    acc = mma_t(sXI, 1, SB, sVJ, SB, 1, wr, wc, lane, acc); // V_I^T V_J
  }

  const double fin = last ? -1.0 : 1.0;
  const bool nextpiv = (!last) && I == k + 1 && J == k + 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * wr + (lane >> 4) + 4 * r, col = 16 * wc + (lane & 15);
    const size_t o = (size_t)(I * 32 + row) * p + J * 32 + col;
    double y;
    if (I == P && J == P)
      y = -acc[r];
    else if (I == P || J == P)
      y = acc[r];
    else
      y = xij[r] - acc[r];
    Y[o] = y * fin;
    if (nextpiv) sP[row * SP + col] = y;
    if (last && I == J && row == col) pv[row] = (I * 32 + row < b.n[m]) ? y * fin : 0.0;
  }
  if (last && I == J) {  // block-uniform: refinement gate, max_i (K^{-1})_ii of this block
    __syncthreads();
    if (t == 0) {
      double mx = 0.0;
      for (int j = 0; j < 32; ++j) mx = fmax(mx, pv[j]);
      // positive doubles order like their bit patterns
      atomicMax(reinterpret_cast<unsigned long long*>(b.pst[m] + 1),
                (unsigned long long)__double_as_longlong(mx));
    }
    return;
  }
  if (!nextpiv) return;  // block-uniform
  __syncthreads();
  const double ls = pivot_chol_inv_block(sP, sM, pv, t, b.status[m]);
  double* piv = b.piv[m] + (size_t)(k + 1) * 1024;
  for (int e = t; e < 1024; e += 256) piv[e] = sM[(e >> 5) * SP + (e & 31)];
  if (t == 0) b.ldet[m][k + 1] = ls;
}

// One launch of the inverse: stage -1 = pivot_init, stage k >= 0 = sweep k (bench/profiling).
hipError_t launch_spd_stage(SpdArgs* a, int nmat, int stage, hipStream_t s) {
  SpdBatch b{};
  int Tmax = 0;
  for (int m = 0; m < nmat; ++m) {
    b.X[m] = a[m].X; b.Y[m] = a[m].Y; b.p[m] = a[m].p; b.T[m] = a[m].p / 32;
    b.piv[m] = a[m].piv; b.ldet[m] = a[m].ldet; b.status[m] = a[m].status;
    b.pst[m] = a[m].pst; b.n[m] = a[m].n;
    if (b.T[m] > Tmax) Tmax = b.T[m];
  }
  if (stage < 0)
    hipLaunchKernelGGL(pivot_init_kernel, dim3(nmat), dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL(sweep_kernel, dim3(Tmax * Tmax, nmat), dim3(256), 0, s, b, stage);
  return hipGetLastError();
}

hipError_t launch_spd_inverse(SpdArgs* a, int nmat, double** final_out, hipStream_t s,
                              bool pivot0_done) {
  SpdBatch b{};
  int Tmax = 0;
  for (int m = 0; m < nmat; ++m) {
    b.X[m] = a[m].X;
    b.Y[m] = a[m].Y;
    b.p[m] = a[m].p;
    b.T[m] = a[m].p / 32;
    b.piv[m] = a[m].piv;
    b.ldet[m] = a[m].ldet;
    b.pst[m] = a[m].pst;
    b.n[m] = a[m].n;
    b.status[m] = a[m].status;
    if (b.T[m] > Tmax) Tmax = b.T[m];
    // sweep k reads (k even ? X : Y) and writes the other; T sweeps end in:
    final_out[m] = (b.T[m] & 1) ? a[m].Y : a[m].X;
  }
  if (!pivot0_done) hipLaunchKernelGGL(pivot_init_kernel, dim3(nmat), dim3(256), 0, s, b);
  for (int k = 0; k < Tmax; ++k)
    hipLaunchKernelGGL(sweep_kernel, dim3(Tmax * Tmax, nmat), dim3(256), 0, s, b, k);
  return hipGetLastError();
}

}  // namespace gpk
