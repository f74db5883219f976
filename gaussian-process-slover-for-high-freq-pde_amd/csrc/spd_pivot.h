// spd_pivot.h — factorisation of one 32x32 SPD pivot block in LDS (shared by the SPD sweep
// and the assembly kernel, which factors pivot block 0 while the matrix is being assembled).
#pragma once
#include "gpk_internal.h"

namespace gpk {

constexpr int SP = 33;  // pivot scratch stride
typedef __attribute__((address_space(3))) double* lds_ptr;

__device__ __forceinline__ double rsqrt_f64(double p) {
  double y = __builtin_amdgcn_rsq(p);          // ~2^-29 relative
  double e = fma(-p * y, y, 1.0);              // 1 - p y^2
  y = fma(0.5 * y, e, y);
  e = fma(-p * y, y, 1.0);
  return fma(0.5 * y, e, y);
}

// One workgroup (256 threads): Cholesky of the 32x32 SPD block A = L L^T (LDS, stride SP,
// full symmetric storage; clobbered) and M = L^{-1} (LDS out, stride SP); returns log det A in
// thread 0 (and every thread < 64).
//
// Blocked right-looking, 4-column blocks B (8 block steps, one barrier each).  Thread t owns
// column c = t&31, rows i = (t>>5) + 8r (r = 0..3) of A and of M, in registers.  Per block,
// every thread factors the 4x4 diagonal block D = L_D L_D^T itself (W = L_D^{-1}; redundant
// but communication-free), then
//   l_iB = A_iB W^T,  l_cB = A_cB W^T                     (panel rows it needs)
//   A_ic -= l_iB . l_cB          (i, c below B)           (trailing update, its elements)
//   X_B = W M_B,c ;  M_ic -= l_iB . X_B  (i below B),  M_Bc = X_B  (final rows of L^{-1})
// and publishes its updated elements through LDS.  Writes never change a value read in the
// same block step (rows/columns of B and of earlier blocks are final), so one barrier per block
// suffices.  The 4x4 square roots use v_rsq_f64 + two Newton steps (no fp64 sqrt/div
// sequences).  Measured 7.0 us vs 12.5 us for the unblocked one-column-per-barrier form
// (tools/probes/pivot1w_probe.hip); results agree to 3e-13 relative (M K M^T = I to 3e-13).
// LP: the LDS pointer type -- plain double* when inlined into a kernel (address space inferred),
// lds_ptr (address_space(3)) when called through a non-inlined function, so that the callee
// still issues ds_read / ds_write instead of flat memory instructions.
template <int BS = 4, typename LP = double*>
__device__ __forceinline__ double pivot_chol_inv_block(LP A, LP M, LP pv, int t, int* status) {
  const int c = t & 31, i0 = t >> 5;
  double a[4], m[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = A[(i0 + 8 * r) * SP + c];
    m[r] = (i0 + 8 * r == c) ? 1.0 : 0.0;
    M[(i0 + 8 * r) * SP + c] = m[r];
  }
  __syncthreads();
#pragma unroll
  for (int kb = 0; kb < 32 / BS; ++kb) {
    const int b0 = BS * kb;
    double D[BS][BS], aiB[4][BS], acB[BS], mB[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int y = 0; y < BS; ++y) aiB[r][y] = A[(i0 + 8 * r) * SP + b0 + y];
#pragma unroll
    for (int y = 0; y < BS; ++y) {
      acB[y] = A[c * SP + b0 + y];
      mB[y] = M[(b0 + y) * SP + c];
    }
    // D = L_D L_D^T, rinv[x] = 1 / (L_D)_xx
    double L[BS][BS], rinv[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      double s = D[x][x];
#pragma unroll
      for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
      if (t == 0) pv[b0 + x] = s;
      rinv[x] = rsqrt_f64(s);
#pragma unroll
      for (int y = x + 1; y < BS; ++y) {
        double q = D[y][x];
#pragma unroll
        for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
        L[y][x] = q * rinv[x];
      }
    }
    // W = L_D^{-1}: W_xx = rinv_x, W_yx = -rinv_y sum_{z=x}^{y-1} L_yz W_zx
    double W[BS][BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      W[x][x] = rinv[x];
#pragma unroll
      for (int y = x + 1; y < BS; ++y) {
        double q = 0.0;
#pragma unroll
        for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
        W[y][x] = -q * rinv[y];
      }
    }
    double lc[BS], X[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      double q = 0.0, u = 0.0;
#pragma unroll
      for (int z = 0; z <= x; ++z) {
        q = fma(acB[z], W[x][z], q);
        u = fma(W[x][z], mB[z], u);
      }
      lc[x] = q;
      X[x] = u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // branch-free: compute, then select
      const int i = i0 + 8 * r;
      double li[BS];
#pragma unroll
      for (int x = 0; x < BS; ++x) {
        double q = 0.0;
#pragma unroll
        for (int z = 0; z <= x; ++z) q = fma(aiB[r][z], W[x][z], q);
        li[x] = q;
      }
      double na = a[r], nm = m[r], xb = 0.0;
#pragma unroll
      for (int x = 0; x < BS; ++x) {
        na = fma(-li[x], lc[x], na);
        nm = fma(-li[x], X[x], nm);
        xb = (i == b0 + x) ? X[x] : xb;
      }
      const bool below = i >= b0 + BS, inB = (i >= b0) && !below;
      a[r] = (below && c >= b0 + BS) ? na : a[r];
      m[r] = below ? nm : (inB ? xb : m[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 8 * r;
      if (i >= b0 + BS) {
        A[i * SP + c] = a[r];
        M[i * SP + c] = m[r];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(i0 + 8 * r) * SP + c] = m[r];
  double ls = 0.0;
  if (t < 64) {
    const double pk = pv[t & 31];
    if (t < 32 && !(pk > 0.0)) atomicOr(status, 1);
    ls = (t < 32) ? log(pk) : 0.0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  }
  __syncthreads();
  return ls;
}

}  // namespace gpk
