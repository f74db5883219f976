// spd_pivot.h — factorisation of one 32x32 SPD pivot block in LDS (shared by the SPD sweep
// and the assembly kernel, which factors pivot block 0 while the matrix is being assembled).
#pragma once
#include "gpk_internal.h"

namespace gpk {

constexpr int SP = 33;  // pivot scratch stride
typedef __attribute__((address_space(3))) double* lds_ptr;

// Every inter-workgroup wait of the persistent / flag-ordered kernels is bounded: 2^22 polls
// (seconds, far beyond any hand-off of a running step) and the wait gives up, setting status
// bit 2 -- the step then reports GPK_ENOTPD ("hand-off timed out") instead of hanging the device
// (a producer that is not resident, e.g. another process holding the CUs).  The host resets the
// hand-off slots after such a launch (gpk_api.cpp reset_handoffs).
// The poll budget, per translation unit that waits (spdinv, spdinv_big, assemble): SPIN_CAP
// unless gpk_set_wait_limit lowered it (tests force a timeout with 1: every wait whose first
// poll fails gives up).  A scalar constant-cache load per poll.
static __constant__ unsigned g_wait_limit = SPIN_CAP;
#define GPK_WAIT_LIMIT_SETTER(fn) \
  hipError_t fn(unsigned polls) { return hipMemcpyToSymbol(HIP_SYMBOL(g_wait_limit), &polls, sizeof polls); }

// Called on every poll of a wait that has not succeeded yet.  A wait gives up (status bit 2)
// when its budget is spent, or -- read every 64th poll, so a hand-off that arrives within 63
// polls (every one of a healthy step's critical hand-offs) costs no status load -- when another
// wait of the same handle already gave up (bit 2 set): its producer may be gone, and the rest of
// the grid and the later steps of a captured batch must drain within 64 polls per wait instead
// of each spending the whole budget.
__device__ __forceinline__ bool spin_give_up(unsigned spins, int* status) {
  bool give_up = spins + 1 >= g_wait_limit;
  if (!give_up && (spins & 63u) == 63u)
    give_up = (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2) != 0;
  if (give_up) atomicOr(status, 2);
  return give_up;
}

template <int SLEEP = 1>
__device__ __forceinline__ bool spin_until_ge(const unsigned int* c, unsigned int target, int* status) {
  for (unsigned spins = 0;
       __hip_atomic_load(const_cast<unsigned int*>(c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;
       ++spins) {
    if (spin_give_up(spins, status)) return false;
    __builtin_amdgcn_s_sleep(SLEEP);
  }
  return true;
}

// v_rsq_f64 is 2^-24.2 relative (tools/probes/rsq_probe.hip): one Newton step leaves 4e-15,
// two 1.4e-16.  One third-order step y (1 + e/2 + 3e^2/8), e = 1 - p y^2 (truncation ~e^3/3 =
// 2^-70) reaches the same accuracy in 4 dependent operations after the rsq instead of 6: the
// square roots are the serial part of the 32-column pivot chain.
__device__ __forceinline__ double rsqrt_f64(double p) {
  const double y = __builtin_amdgcn_rsq(p);
  const double e = fma(-p * y, y, 1.0);
  return fma(y * e, fma(0.375, e, 0.5), y);
}

// One workgroup (256 threads): Cholesky of the 32x32 SPD block A = L L^T (LDS, stride SP,
// full symmetric storage; clobbered) and M = L^{-1} (LDS out, stride SP); returns log det A in
// thread 0 (and every thread < 64).
//
// Blocked right-looking, 4-column blocks B (8 block steps, one barrier each), with the rank-4
// trailing updates of A and of M on v_mfma_f64_16x16x4 (k = 4 = the block width).  Wave
// (wr, wc) keeps the 16x16 quadrant (rows 16wr.., cols 16wc..) of A and of M in two MFMA
// accumulators for the whole factorisation (lane: rows 16wr + lk + 4r, column 16wc + li).  Per
// block every lane factors the 4x4 diagonal block D = L_D L_D^T itself (W = L_D^{-1}; redundant
// but communication-free), then forms the three operand values it owns:
//   A operand  -l_iB[lk] = -(A_iB W^T)[lk]       (i = 16wr + li, zero unless i is below B)
//   B operand   l_cB[lk] =  (A_cB W^T)[lk]       (c = 16wc + li, zero unless c is below B)
//   B operand   X[lk][c] =  (W M_B)[lk][c]
// and one MFMA each gives A_ic -= l_iB . l_cB and M_ic -= l_iB . X_B (rows below B); the rows of
// B become M_B = X.  Only entries that change are published to LDS, and the entries read in a
// block step (A's column block B and diagonal block, M's rows B) never change in it, so one
// barrier per block suffices and M needs no second buffer.  The 4x4 square roots use
// v_rsq_f64 + one third-order correction (rsqrt_f64 above).  Results are bitwise those of the VALU form it replaced (MFMA
// f64 accumulates the 4 products in the same order); 5.2 us vs 6.6 us per factorisation
// (tools/probes/pivot_mfma_probe.hip).
// LP: the LDS pointer type -- plain double* when inlined into a kernel (address space inferred),
// lds_ptr (address_space(3)) when called through a non-inlined function, so that the callee
// still issues ds_read / ds_write instead of flat memory instructions.
// Hook (optional): hook.early() runs in every thread before the barrier that ends block step 2,
// hook.pre() before the one that ends step 5 and hook.post() right after it -- a window to poll
// (without waiting) for the NEXT pivot's inputs and start their loads while this factorisation
// still has 2 block steps to go (chain_kernel's pivot chain).  The flag load needs the 3 steps
// in between to land (a read at step 4 checked at step 6 stalled every pivot by ~1 us), and a
// check at step 4 came too early for most inputs (C4: steps 2/5 beat 1/4 by ~1%).
struct NoPivotHook {
  __device__ constexpr bool waves() const { return false; }  // (pivot_chol_inv_1w: waves 1-3 skip it)
  __device__ void early() {}
  __device__ void pre() {}
  __device__ void post() {}
};
// UNROLL: the 8 block steps unrolled (the chain's pivot: constant LDS offsets) or kept as a loop
// (1: a quarter of the registers, for kernels that must stay at two waves per SIMD)
template <int BS = 4, typename LP = double*, typename Hook = NoPivotHook, int UNROLL = 8>
__device__ __forceinline__ double pivot_chol_inv_block(LP A, LP M, LP pv, int t, int* status,
                                                       Hook hook = Hook()) {
  static_assert(BS == 4, "the MFMA update is rank 4");
  typedef double dv4 __attribute__((ext_vector_type(4)));
  const int lane = t & 63, wv = t >> 6, wr = wv >> 1, wc = wv & 1;
  const int li = lane & 15, lk = lane >> 4;
  const int ri = 16 * wr + li, cj = 16 * wc + li;
  dv4 accA, accM;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * wr + lk + 4 * r;
    accA[r] = A[row * SP + cj];
    accM[r] = (row == cj) ? 1.0 : 0.0;
    M[row * SP + cj] = accM[r];
  }
  // (0/1 weights select row lk of W: a select chain on lk becomes a scratch-indexed array)
  const double s0 = lk == 0 ? 1.0 : 0.0, s1 = lk == 1 ? 1.0 : 0.0, s2 = lk == 2 ? 1.0 : 0.0,
               s3 = lk == 3 ? 1.0 : 0.0;
  __syncthreads();
#pragma unroll UNROLL
  for (int kb = 0; kb < 8; ++kb) {
    const int b0 = 4 * kb;
    double D[4][4], ar[4], ac[4], mb[4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      ar[z] = A[ri * SP + b0 + z];
      ac[z] = A[cj * SP + b0 + z];
      mb[z] = M[(b0 + z) * SP + cj];
    }
    // D = L_D L_D^T, rinv[x] = 1 / (L_D)_xx
    double L[4][4], rinv[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      double s = D[x][x];
#pragma unroll
      for (int z = 0; z < x; ++z) s = fma(-L[x][z], L[x][z], s);
      if (t == 0) pv[b0 + x] = s;
      rinv[x] = rsqrt_f64(s);
#pragma unroll
      for (int y = x + 1; y < 4; ++y) {
        double q = D[y][x];
#pragma unroll
        for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
        L[y][x] = q * rinv[x];
      }
    }
    // W = L_D^{-1}: W_xx = rinv_x, W_yx = -rinv_y sum_{z=x}^{y-1} L_yz W_zx, zero above
    double W[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      W[x][x] = rinv[x];
#pragma unroll
      for (int y = x + 1; y < 4; ++y) {
        double q = 0.0;
#pragma unroll
        for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
        W[y][x] = -q * rinv[y];
      }
#pragma unroll
      for (int y = 0; y < x; ++y) W[y][x] = 0.0;
    }
    double lr = 0.0, lc = 0.0, xv = 0.0;
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const double w = fma(W[0][z], s0, fma(W[1][z], s1, fma(W[2][z], s2, W[3][z] * s3)));
      lr = fma(ar[z], w, lr);
      lc = fma(ac[z], w, lc);
      xv = fma(w, mb[z], xv);
    }
    const double opa = (ri >= b0 + 4) ? -lr : 0.0;
    const double opb = (cj >= b0 + 4) ? lc : 0.0;
    accA = __builtin_amdgcn_mfma_f64_16x16x4f64(opa, opb, accA, 0, 0, 0);
    accM = __builtin_amdgcn_mfma_f64_16x16x4f64(opa, xv, accM, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * wr + lk + 4 * r;
      if (16 * wr + 4 * r == b0) accM[r] = xv;  // rows of B: M_B = X (final; written at the end)
      if (kb < 7 && row >= b0 + 4) {
        if (cj >= b0 + 4) A[row * SP + cj] = accA[r];
        M[row * SP + cj] = accM[r];
      }
    }
    if (kb == 2) hook.early();
    if (kb == 5) hook.pre();
    __syncthreads();
    if (kb == 5) hook.post();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(16 * wr + lk + 4 * r) * SP + cj] = accM[r];
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


// The same factorisation by ONE wave (wave 0; waves 1-3 only run the hook), bitwise equal to
// pivot_chol_inv_block (same operations per element, tools/probes/pivot_variants_probe.hip):
// wave 0 keeps the lower 16x16 tiles (0,0), (1,0), (1,1) of A and of M in six MFMA accumulators
// (register r of lane (li, lk) = element (16 I + lk + 4 r, 16 J + li)), so a block step needs no
// workgroup barrier (LDS operations of one wave are in order), and it publishes to LDS only what
// the NEXT block step reads -- A's next column block (rows at and below it) and M's next block
// rows -- instead of every updated entry.  4.3 us against 5.0 us per factorisation.
// The upper tile of A in LDS is left stale (read only for rows above the block, whose operand is
// masked to zero); the upper tile of M is zero.  M's LDS copy is complete on return.
// Hook: wave 0 runs early() after block step 2 and pre() / post() after block step 5, then meets
// waves 1-3 at ONE workgroup barrier (they wait there instead of polling LDS, which competed
// with wave 0's LDS traffic) and they run the three hook calls themselves, so per-thread
// prefetches (chain_master's PivotPrefetch) are issued at the same point of the factorisation as
// with the four-wave form.  hook.waves() == false (NoPivotHook): waves 1-3 go straight to the
// closing barrier.  (sflag: unused, kept for the call signature.)
template <typename LP = double*, typename Hook = NoPivotHook>
__device__ __forceinline__ double pivot_chol_inv_1w(LP A, LP M, LP pv, int t, int* status,
                                                    volatile int* sflag = nullptr, Hook hook = Hook()) {
  typedef double dv4 __attribute__((ext_vector_type(4)));
  double ls = 0.0;
  if (t < 64) {
    const int lane = t, li = lane & 15, lk = lane >> 4;
    dv4 a00, a10, a11, m00, m10, m11;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = lk + 4 * r;
      a00[r] = A[row * SP + li];
      a10[r] = A[(16 + row) * SP + li];
      a11[r] = A[(16 + row) * SP + 16 + li];
      m00[r] = (row == li) ? 1.0 : 0.0;
      m10[r] = 0.0;
      m11[r] = m00[r];
      M[row * SP + li] = m00[r];
      M[row * SP + 16 + li] = 0.0;
      M[(16 + row) * SP + li] = 0.0;
      M[(16 + row) * SP + 16 + li] = m11[r];
    }
    const double s0 = lk == 0 ? 1.0 : 0.0, s1 = lk == 1 ? 1.0 : 0.0, s2 = lk == 2 ? 1.0 : 0.0,
                 s3 = lk == 3 ? 1.0 : 0.0;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const int b0 = 4 * kb, b1 = b0 + 4, J0 = kb >> 2;
      double D[4][4], ar0[4], ar1[4], mb0[4], mb1[4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y <= x; ++y) D[x][y] = A[(b0 + x) * SP + b0 + y];
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        ar0[z] = J0 == 0 ? A[li * SP + b0 + z] : 0.0;
        ar1[z] = A[(16 + li) * SP + b0 + z];
        mb0[z] = M[(b0 + z) * SP + li];
        mb1[z] = J0 == 1 ? M[(b0 + z) * SP + 16 + li] : 0.0;
      }
      // D = L_D L_D^T, W = L_D^{-1}: pivot_chol_inv_block's arithmetic
      double L[4][4], rinv[4], W[4][4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        double sx = D[x][x];
#pragma unroll
        for (int z = 0; z < x; ++z) sx = fma(-L[x][z], L[x][z], sx);
        if (lane == 0) pv[b0 + x] = sx;
        rinv[x] = rsqrt_f64(sx);
#pragma unroll
        for (int y = x + 1; y < 4; ++y) {
          double q = D[y][x];
#pragma unroll
          for (int z = 0; z < x; ++z) q = fma(-L[y][z], L[x][z], q);
          L[y][x] = q * rinv[x];
        }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        W[x][x] = rinv[x];
#pragma unroll
        for (int y = x + 1; y < 4; ++y) {
          double q = 0.0;
#pragma unroll
          for (int z = x; z < y; ++z) q = fma(L[y][z], W[z][x], q);
          W[y][x] = -q * rinv[y];
        }
#pragma unroll
        for (int y = 0; y < x; ++y) W[y][x] = 0.0;
      }
      double l0 = 0.0, l1 = 0.0, x0 = 0.0, x1 = 0.0;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const double w = fma(W[0][z], s0, fma(W[1][z], s1, fma(W[2][z], s2, W[3][z] * s3)));
        l0 = fma(ar0[z], w, l0);
        l1 = fma(ar1[z], w, l1);
        x0 = fma(w, mb0[z], x0);
        x1 = fma(w, mb1[z], x1);
      }
      const double oa0 = (li >= b1) ? -l0 : 0.0, oa1 = (16 + li >= b1) ? -l1 : 0.0;
      const double ob0 = (li >= b1) ? l0 : 0.0, ob1 = (16 + li >= b1) ? l1 : 0.0;
      if (J0 == 0) {
        a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(oa0, ob0, a00, 0, 0, 0);
        a10 = __builtin_amdgcn_mfma_f64_16x16x4f64(oa1, ob0, a10, 0, 0, 0);
        m00 = __builtin_amdgcn_mfma_f64_16x16x4f64(oa0, x0, m00, 0, 0, 0);
      }
      a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(oa1, ob1, a11, 0, 0, 0);
      m10 = __builtin_amdgcn_mfma_f64_16x16x4f64(oa1, x0, m10, 0, 0, 0);
      m11 = __builtin_amdgcn_mfma_f64_16x16x4f64(oa1, x1, m11, 0, 0, 0);
      const int rb = kb & 3;  // the block's rows: register rb of tile row J0 (final: M_B = X)
      if (J0 == 0) {
        m00[rb] = x0;
      } else {
        m10[rb] = x0;
        m11[rb] = x1;
      }
      if (kb < 7) {  // publish what block step kb + 1 reads
        const int J1 = b1 >> 4, c1 = b1 & 15, r1 = (b1 & 15) >> 2;
        const bool mine = li >= c1 && li < c1 + 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = lk + 4 * r;
          if (J1 == 0) {
            if (mine && row >= b1) A[row * SP + li] = a00[r];
            if (mine) A[(16 + row) * SP + li] = a10[r];
          } else {
            if (mine && 16 + row >= b1) A[(16 + row) * SP + 16 + li] = a11[r];
          }
        }
        if (J1 == 0) {
          M[(lk + 4 * r1) * SP + li] = m00[r1];
        } else {
          M[(16 + lk + 4 * r1) * SP + li] = m10[r1];
          M[(16 + lk + 4 * r1) * SP + 16 + li] = m11[r1];
        }
      }
      if (kb == 2) hook.early();
      if (kb == 5) {
        hook.pre();
        hook.post();
        if (hook.waves()) __syncthreads();  // releases waves 1-3 (waiting there, not polling)
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = lk + 4 * r;
      M[row * SP + li] = m00[r];
      M[(16 + row) * SP + li] = m10[r];
      M[(16 + row) * SP + 16 + li] = m11[r];
    }
    const double pk = pv[lane & 31];
    if (lane < 32 && !(pk > 0.0)) atomicOr(status, 1);
    ls = (lane < 32) ? log(pk) : 0.0;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
  } else if (hook.waves()) {
    __syncthreads();  // wave 0 has passed block step 5
    hook.early();
    hook.pre();
    hook.post();
  }
  __syncthreads();
  return ls;
}

}  // namespace gpk
