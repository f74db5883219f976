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
#include <algorithm>

#include "gpk_internal.h"
#include "spd_pivot.h"
#include "gpk_trace.h"
#include "prep_dev.h"

namespace gpk {

GPK_WAIT_LIMIT_SETTER(wait_limit_spdinv)  // gpk_set_wait_limit

GPK_TRACE_TU(spdinv)

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
  const double ls = pivot_chol_inv_1w(A, M, pv, t, b.status[m]);
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
  // grid (nmat, tiles): the factors are interleaved in dispatch order, and tile numbering starts
  // at the tile that factors the next pivot (the critical path of the launch): it is dispatched
  // first instead of after up to 2 T^2 other workgroups
  const int m = blockIdx.x;
  const int p = b.p[m];
  const int T = b.T[m];
  if (k >= T) return;  // this factor is already inverted
  const int last = (k == T - 1);
  if ((int)blockIdx.y >= T * T) return;
  const int tile = (int)(blockIdx.y + (last ? 0 : (k + 1) * (T + 1))) % (T * T);
  const int I = tile / T, J = tile % T;
  // probes: the block that factors the next pivot (tile (0,0) of factor 0 in the last sweep)
  const bool trb = threadIdx.x == 0 && m == 0 && k < 16 && blockIdx.y == 0;
  if (trb) TR_LO(SLOT_SWEEP + k);
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
    if (trb) TR_HI(SLOT_SWEEP + k);
    return;
  }
  if (!nextpiv) {  // block-uniform
    if (trb) TR_HI(SLOT_SWEEP + k);
    return;
  }
  __syncthreads();
  if (trb) TR_LO(SLOT_SWEEP_PIVOT + k);
  const double ls = pivot_chol_inv_1w(sP, sM, pv, t, b.status[m]);
  double* piv = b.piv[m] + (size_t)(k + 1) * 1024;
  for (int e = t; e < 1024; e += 256) piv[e] = sM[(e >> 5) * SP + (e & 31)];
  if (t == 0) b.ldet[m][k + 1] = ls;
  if (trb) TR_HI(SLOT_SWEEP_PIVOT + k);
  if (trb) TR_HI(SLOT_SWEEP + k);
}

// ---- persistent dataflow form ("chain"): every sweep in ONE launch ------------------------
// The sweep above pays a launch boundary per pivot block: the pivot workgroup's pre-pivot work
// (~4 us of loads + two MFMA passes) plus the inter-kernel gap (~1.7 us) on top of the 5.4-us
// factorisation, 8 times at 256^2 (tools/timeline.py).  Here one workgroup per tile owns its
// tile for the whole inverse (in MFMA accumulators) and sweeps are ordered by flags:
//   * tile (I, J) is read by other workgroups only as the panel of sweep I; its owner publishes
//     it once, after sweep I-1, into the panel buffer PB (write-once, no ping-pong hazard);
//   * L^{-1} of pivot k is published once into piv[k] by the owner of (k, k);
//   * hand-offs follow MI355X_MICROARCH.md's sc1 row: payload stored sc1 by every wave, each
//     wave's vmcnt(0), a barrier, one lane's sc1 flag store; the consumer polls the flag with an
//     sc1 load, a barrier, then sc1 loads of the payload.
// The per-sweep critical path is the pivot owner's hop (poll + loads + two MFMA passes) plus its
// factorisation.  All workgroups wait on one another, so the grid must be co-resident: used
// only when the grid fits the device's co-resident capacity (spd_chain_capacity: occupancy per CU
// x CUs; two per CU on a full MI355X) and at most CHAIN_MAX_BLOCKS.  The arithmetic is the
// sweep kernel's operation for operation: the results are bitwise equal.
struct ChainFactor {
  double* X;            // in: assembled K (read mode); out: K^{-1}
  double* PB;           // panel buffer [p*p]: tile (I, J) as it is after sweep I-1
  double* piv;          // [T][32*32] L^{-1} of each pivot block
  double* ldet;         // [T]
  double* pst;          // refinement gate [2]
  int* status;
  unsigned int* flags;  // [T*TC] panel ready, [T] pivot ready, [T] (unused), [1] done counter
                        // (zero; re-armed by the last workgroup)
  double* gran;              // the pivot chain's input slots [T][2][1024] (chain_master)
  double* PB2;               // chain_multi: panel slots [2][p*p] by launch parity (self-validating)
  unsigned int* epoch;       // chain_multi: launch counter (its parity selects the PB2 half)
  int piv_off;               // offset of the pivot-ready flags (T * TC)
  int p, n, T;
  // gather mode: K from the distance classes (+ jitter), kept copy Kc and D written on the way
  const int* cid; const double* kval; const double* dval; const double* x; double jitter;
  double* Kc; double* D;
  // augmented right-hand sides: tile columns T.. of the sweep operator's upper-right block end
  // as K^{-1} [B_u | D^T]  (gpk_internal.h ChainArgs)
  int tu, td;
  const double* Bu; int ldbu, bu_t;
  double* Ou; int ldou, ou_t;
  double* Od; int ldod;
  double* PBa; int ldpba;
};
struct ChainBatch {
  ChainFactor f[2];
  int nmat;
  PrepArgs prep;  // published by workgroup (0, nmat) when the grid has that extra row
  int q;
  int mpos;       // chain_multi_kernel: linear index of the pivot chain's workgroup
};

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// bounded (spd_pivot.h spin_until_ge): a flag that never rises sets status bit 2
__device__ __forceinline__ void wait_flag(unsigned int* f, int* status) {
  (void)spin_until_ge<1>(f, 1u, status);
}
// every wave drained its sc1 stores -> barrier -> one lane raises the flag
__device__ __forceinline__ void signal_flag(unsigned int* f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The pivot chain's inputs travel as self-validating words (MI355X_MICROARCH.md hand-off row
// handoff-1to1; cdna_hip_programming.md Guideline 16 R2 with the data as its own flag): every
// fp64 element is ONE 8-byte sc1 store into a slot that holds a sentinel (a signalling-NaN bit
// pattern, which no floating-point operation produces: results are quieted) until it is
// written.  The producer neither drains its stores nor raises a flag; the pivot chain, the
// slot's only reader, loads the words, re-loads any that still hold the sentinel, and after
// consuming a slot writes the sentinel back (ready for the next launch; the buffer is
// initialised to the sentinel at create, gpk_api.cpp).  Slot k (hop k, the inputs of pivot
// k+1): [0] panel tile (k, k+1), [1] diagonal tile (k+1, k+1), both after sweep k-1; element
// e = 32 row + col of the tile.
__device__ __forceinline__ double* gran_at(const ChainFactor& F, int slot, int which, int e) {
  return F.gran + (size_t)(2 * slot + which) * 1024 + e;
}
__device__ __forceinline__ bool gran_ok(double v) {
  return __double_as_longlong(v) != (long long)CHAIN_SENTINEL;
}

// The pivot chain of one factor (chain_kernel, chain_multi_kernel): one workgroup factors every
// pivot block in order.  acc: this wave's quadrant of tile (0, 0) of K.  LDS: sXJ [32][SB],
// sP / sM [32][SP], pv [32].
template <bool ONEWAVE>
__device__ __forceinline__ void chain_master(const ChainFactor& F, int T, d4 acc, double* sXJ,
                                             double* sP, double* sM, double* pv, bool trm,
                                             bool early_flag, double* lw = nullptr) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int tx = t & 31, ty = t >> 5;
  unsigned int* piv_rdy = F.flags + F.piv_off;
  __shared__ int s_pflag;  // pivot_chol_inv_1w's "wave 0 passed block step 5" flag
    // (issue priority over the tile workgroup that may share its CU: this one is the chain)
  __builtin_amdgcn_s_setprio(3);
  // The pivot chain, kept in one workgroup: after factoring pivot k it holds L_k^{-1} in LDS,
  // so pivot k+1's Schur complement X_{k+1,k+1} - V^T V (V = L_k^{-1} X_{k,k+1}) needs no hop
  // for L_k^{-1}; its two inputs (the panel tile (k, k+1) and the diagonal tile (k+1, k+1)
  // after sweep k-1) are handed over (self-validating words, above) by their owners while this
  // workgroup is still factoring pivot k.  Same operations as the owner's update of that tile:
  // bitwise equal.  Their loads are issued inside that factorisation (PivotPrefetch, after block
  // step 5) and checked after it; words that were not yet written are re-loaded.
  // element of this thread: panel tile (LDS-staging layout: row ty + 8r, column tx) and the
  // diagonal tile (MFMA quadrant layout)
  auto ex = [&](int r) { return (ty + 8 * r) * 32 + tx; };
  auto ed = [&](int r) { return (16 * wr + (lane >> 4) + 4 * r) * 32 + 16 * wc + (lane & 15); };
  double gx[4], gd[4];
  auto issue = [&](int k) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gx[r] = ld_sc1(gran_at(F, k, 0, ex(r)));
      gd[r] = ld_sc1(gran_at(F, k, 1, ed(r)));
    }
  };
  struct PivotPrefetch {
    __device__ constexpr bool waves() const { return true; }  // every thread issues its own words
    decltype(issue)* f;
    int k, T;
    __device__ void early() {}
    __device__ void pre() {}
    __device__ void post() {
      if (k + 1 < T) (*f)(k);
    }
  };
  // L^{-1}_kp is stored right after its factorisation, but its flag is raised inside the next
  // hop (after the first product, when the stores have drained): the chain does not stall on
  // the write-back of every pivot (the last one is signalled at once)
  auto factor = [&](int kp) {
    if (trm && kp > 0 && kp < 17) TR_HI(SLOT_SWEEP + kp - 1);  // (inputs in: the hop ends)
    store_quad(sP, SP, wr, wc, lane, acc);
    __syncthreads();
    if (trm && kp > 0 && kp < 17) TR_LO(SLOT_SWEEP_PIVOT + kp - 1);
    if (trm && kp == 0) TR_LO(SLOT_PIVOT0);
    PivotPrefetch hook{&issue, kp, T};
    // ONEWAVE (chain_kernel): the one-wave factorisation (spd_pivot.h pivot_chol_inv_1w, 4.3 vs
    // 5.0 us), waves 1-3 issuing their prefetch words when wave 0 passes block step 5;
    // chain_multi_kernel keeps the four-wave form (its tile path is at the register limit: the
    // one-wave form's accumulators would spill there)
    double ls;
    if (ONEWAVE)
      ls = pivot_chol_inv_1w<double*, PivotPrefetch>(sP, sM, pv, t, F.status, &s_pflag, hook);
    else
      ls = pivot_chol_inv_block<4, double*, PivotPrefetch>(sP, sM, pv, t, F.status, hook);
    // lw (chain_multi): L^{-1}_kp as self-validating words in this launch's slots, no flag
    double* ldst = (lw ? lw : F.piv) + (size_t)kp * 1024;
    for (int e = t; e < 1024; e += 256) st_sc1(ldst + e, sM[(e >> 5) * SP + (e & 31)]);
    if (t == 0) F.ldet[kp] = ls;
    if (kp + 1 == T && !lw) signal_flag(piv_rdy + kp);
    if (trm && kp > 0 && kp < 17) TR_HI(SLOT_SWEEP_PIVOT + kp - 1);
    if (trm && kp == 0) TR_HI(SLOT_PIVOT0);
  };
  // refinement gate: K_00 = max diag K (stationary kernel + jitter), and max diag K^{-1}
  // zeroed here -- before piv_rdy[0] is raised (the vmcnt(0) ahead of that flag drains these
  // stores), so it precedes every diagonal tile's atomicMax, which waits on all piv_rdy[k]
  if (t == 0) {
    st_sc1(F.pst, acc[0]);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(F.pst + 1), 0ull, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t == 0) s_pflag = 0;  // (the barrier inside factor(0) orders it before the pivot)
  // lw: no pivot flags -- the zeroing above completes before any L^{-1} word is stored (every
  // diagonal tile's atomicMax comes after it has read L^{-1}_0's words)
  if (lw) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  factor(0);  // acc = tile (0, 0) of K, gathered above
  for (int k = 0; k + 1 < T; ++k) {
    // L_k's flag: raised inside the hop (below); with early_flag (chain_multi, whose inputs are
    // usually late) at once -- its stores drain while the inputs are awaited, and the tile
    // workgroups' sweep k (which produces pivot k+2's inputs) does not wait for this hop
    if (early_flag) {
      if (lw) __syncthreads();
      else signal_flag(piv_rdy + k);
    }
    bool ok = true;
#pragma unroll
    for (int r = 0; r < 4; ++r) ok = ok && gran_ok(gx[r]) && gran_ok(gd[r]);
    if (trm && !ok) { TR_LO(SLOT_PREFETCH_MISS); TR_HI(SLOT_PREFETCH_MISS); }  // (thread 0's words)
    // (per lane) words not yet written when they were loaded: load them again.  Bounded: a
    // hand-off that never arrives flags the status word (the step reports an error) instead of
    // hanging the device.
    for (unsigned spins = 0; !ok; ++spins) {
      if (spin_give_up(spins, F.status)) break;
      __builtin_amdgcn_s_sleep(1);
      issue(k);
      ok = true;
#pragma unroll
      for (int r = 0; r < 4; ++r) ok = ok && gran_ok(gx[r]) && gran_ok(gd[r]);
    }
    if (trm && k < 16) TR_LO(SLOT_SWEEP + k);
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // prefetched during pivot k's factorisation
      sXJ[(ty + 8 * r) * SB + tx] = gx[r];
      acc[r] = gd[r];
      // consumed: the sentinel back into the slot for the next launch
      st_sc1(gran_at(F, k, 0, ex(r)), __longlong_as_double((long long)CHAIN_SENTINEL));
      st_sc1(gran_at(F, k, 1, ed(r)), __longlong_as_double((long long)CHAIN_SENTINEL));
    }
    __syncthreads();
    d4 vj = {0.0, 0.0, 0.0, 0.0};
    vj = mma_t(sM, SP, 1, sXJ, SB, 1, wr, wc, lane, vj);  // V = L_k^{-1} X_{k,k+1}
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // L^{-1}_k's stores (long drained)
    __syncthreads();
    if (t == 0 && !early_flag && !lw) __hip_atomic_store(piv_rdy + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    store_quad(sXJ, SB, wr, wc, lane, vj);
    __syncthreads();
    d4 prod = {0.0, 0.0, 0.0, 0.0};
    prod = mma_t(sXJ, 1, SB, sXJ, SB, 1, wr, wc, lane, prod);  // V^T V
    acc = acc - prod;
    factor(k + 1);
  }
}

template <int DERIV, bool GATHER>
__global__ __launch_bounds__(256, 2) void chain_kernel(ChainBatch b) {
  const int m = blockIdx.y;
  if (m == b.nmat) {  // the step constants (+ a folded batch begin), off the critical path
    if (blockIdx.x == 0) publish_prep(b.prep, b.q);
    copy_snapshot(b.prep, blockIdx.x, gridDim.x);
    return;
  }
  const ChainFactor& F = b.f[m];
  const int T = F.T, p = F.p;
  const int TC = T + F.tu + F.td;  // tile columns: K, then the augmented B_u, D^T columns
  if ((int)blockIdx.x > T * TC) return;
  // the pivot chain's own workgroup (below) is tile index T*TC; it and the tiles feeding it are
  // dispatched in the grid's middle, alone on their CUs (gpk_internal.h chain_role)
  const int tile = chain_role(m, (int)blockIdx.x, T, TC);
  const bool master = tile == T * TC;
  const int I = master ? 0 : tile / TC, J = master ? 0 : tile % TC;
  const bool aug = J >= T;
  const int ja = J - T;  // augmented tile column
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int tx = t & 31, ty = t >> 5;
  unsigned int* panel_rdy = F.flags;
  unsigned int* piv_rdy = F.flags + T * TC;
  unsigned int* done = F.flags + T * TC + 2 * T;
  // panel tile (row k) of column J: K part in PB, augmented part in PBa
  auto panel_ptr = [&](int k, int row, int col) -> double* {
    return J < T ? F.PB + (size_t)(k * 32 + row) * p + J * 32 + col
                 : F.PBa + (size_t)(k * 32 + row) * F.ldpba + ja * 32 + col;
  };
  __shared__ double sL[32 * SA];
  __shared__ double sXI[32 * SB], sXJ[32 * SB];
  __shared__ double sP[32 * SP], sM[32 * SP], pv[32];
  __shared__ unsigned int s_last;
  // L_k^{-1} as self-validating words (chain_multi_kernel's form) in this launch's half of the
  // L^{-1} slots (PB2, launch parity; the other half is reset by the tile workgroups): the tile
  // workgroups see L_k^{-1} as soon as its stores land instead of after the pivot chain's flag,
  // which it raises only inside the next hop
  const unsigned ep = F.PB2 ? __hip_atomic_load(F.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  double* PLc = F.PB2 ? F.PB2 + (size_t)(ep & 1u) * chain_half(p, false) : nullptr;

  // own tile, this wave's quadrant: rows 16 wr + (lane >> 4) + 4 r, column 16 wc + (lane & 15)
  d4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = I * 32 + 16 * wr + (lane >> 4) + 4 * r, j = J * 32 + 16 * wc + (lane & 15);
    const size_t o = (size_t)i * p + j;
    if (aug) {  // B_u[i][j'] or D^T[i][j'] = D[j'][i] (j' = column inside the part)
      const int jl = ja * 32 + 16 * wc + (lane & 15);
      if (ja < F.tu) {
        acc[r] = F.bu_t ? F.Bu[(size_t)(jl) * F.ldbu + i] : F.Bu[(size_t)i * F.ldbu + jl];
      } else {
        const int jd = jl - 32 * F.tu;
        const size_t od = (size_t)jd * p + i;
        if (GATHER) {
          const int u = F.cid[od];
          double dv = u >= 0 ? F.dval[u] : 0.0;
          if (DERIV == 1 && u >= 0 && !(F.x[jd] - F.x[i] >= 0.0)) dv = -dv;
          acc[r] = dv;
        } else {
          acc[r] = F.D[od];
        }
      }
      continue;
    }
    if (GATHER) {
      const int u = F.cid[o];
      double kv, dv;
      if (u >= 0) {
        kv = F.kval[u];
        if (i == j) kv += F.jitter;
        dv = F.dval[u];
        if (DERIV == 1 && !(F.x[i] - F.x[j] >= 0.0)) dv = -dv;  // JAX abs'(0) = +1
      } else {
        kv = (i == j) ? 1.0 : 0.0;
        dv = 0.0;
      }
      if (!master) {
        if (F.Kc) F.Kc[o] = kv;
        if (DERIV && F.D) F.D[o] = dv;
      }
      acc[r] = kv;
    } else {
      acc[r] = F.X[o];
    }
  }
  auto publish_tile = [&](void) {  // panel tile (I, J) <- acc, then its flag
#pragma unroll
    for (int r = 0; r < 4; ++r) st_sc1(panel_ptr(I, 16 * wr + (lane >> 4) + 4 * r, 16 * wc + (lane & 15)), acc[r]);
    signal_flag(panel_rdy + I * TC + J);
  };
  // the pivot chain's inputs of hop kk (after sweep kk-1): panel tile (kk, kk+1) and diagonal
  // tile (kk+1, kk+1) as granules (chain_master), before any other store of the tile
  auto chain_inputs = [&](int kk) {
    const int which = (I == kk && J == kk + 1) ? 0 : (I == J && I == kk + 1) ? 1 : -1;
    if (which < 0 || kk + 1 >= T) return;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      st_sc1(gran_at(F, kk, which, (16 * wr + (lane >> 4) + 4 * r) * 32 + 16 * wc + (lane & 15)), acc[r]);
  };
  const bool trm = t == 0 && m == 0;  // probes (gpk_trace.h): factor 0's pivot owners
  if (master) {
    chain_master<true>(F, T, acc, sXJ, sP, sM, pv, trm, false, PLc);
  } else {
    if (trm && tile == 0) TR_LO(SLOT_GATHER);
    chain_inputs(0);                       // tiles (0, 1) and (1, 1) as they are before sweep 0
    if (I == 0 && J != 0) publish_tile();  // row 0 is the panel of sweep 0
    if (PLc) {  // this tile's share of the other half's L^{-1} slots (last launch's) -> sentinel
      double* PLo = F.PB2 + (size_t)((ep & 1u) ^ 1u) * chain_half(p, false);
      const int share = (T * 1024 + T * TC - 1) / (T * TC);
      const int e1 = min(T * 1024, (tile + 1) * share);
      for (int e = tile * share + t; e < e1; e += 256) PLo[e] = __longlong_as_double((long long)CHAIN_SENTINEL);
    }
  }

  for (int k = 0; k < T && !master; ++k) {
    const bool needI = I != k, needJ = J != k && J != I;
    // issue priority over the CU's other workgroup when this tile feeds sweep k+1's panel or
    // the pivot chain
    if (I == k + 1 || (I == k + 2 && J == k + 2)) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(0);
    // the panel tiles are usually published long before the pivot: fetch them first, then
    // wait for L^{-1}_k
    if (t == 0) {
      if (needI) wait_flag(panel_rdy + k * TC + I, F.status);
      if (needJ) wait_flag(panel_rdy + k * TC + J, F.status);
    }
    __syncthreads();
    double xi[4], xj[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = ty + 8 * r;
      xi[r] = needI ? ld_sc1(F.PB + (size_t)(k * 32 + row) * p + I * 32 + tx) : 0.0;
      xj[r] = needJ ? ld_sc1(panel_ptr(k, row, tx)) : 0.0;
    }
    const bool trl = t == 0 && m == 0 && k == T - 1 && I == T - 1 && J == T - 1;
    double lv[4];
    if (PLc) {
      // one thread polls one word of L_k^{-1} (the polling traffic of a flag), then every thread
      // loads its words and re-loads those still holding the sentinel (bounded)
      const double* Lw = PLc + (size_t)k * 1024;
      if (t == 0) {
        for (unsigned spins = 0; !gran_ok(ld_sc1(Lw + 1023)); ++spins) {
          if (spin_give_up(spins, F.status)) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (trl) TR_HI(SLOT_LAST_FLAG);
#pragma unroll
      for (int r = 0; r < 4; ++r) lv[r] = ld_sc1(Lw + (ty + 8 * r) * 32 + tx);
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int r = 0; r < 4; ++r) ok = ok && gran_ok(lv[r]);
        if (ok) break;
        if (spin_give_up(spins, F.status)) break;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!gran_ok(lv[r])) lv[r] = ld_sc1(Lw + (ty + 8 * r) * 32 + tx);
      }
    } else {
      if (t == 0) wait_flag(piv_rdy + k, F.status);
      __syncthreads();
      if (trl) TR_HI(SLOT_LAST_FLAG);
      const double* Li = F.piv + (size_t)k * 1024;
#pragma unroll
      for (int r = 0; r < 4; ++r) lv[r] = ld_sc1(Li + (ty + 8 * r) * 32 + tx);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = ty + 8 * r;
      sL[row * SA + tx] = lv[r];
      if (needI) sXI[row * SB + tx] = xi[r];
      if (needJ) sXJ[row * SB + tx] = xj[r];
    }
    __syncthreads();
    if (trl) TR_HI(SLOT_LAST_LDS);
    const double* sVJ = (J == I) ? sXI : sXJ;
    d4 vi = {0.0, 0.0, 0.0, 0.0}, vj = {0.0, 0.0, 0.0, 0.0};
    if (needI) vi = mma_t(sL, SA, 1, sXI, SB, 1, wr, wc, lane, vi);
    if (needJ) vj = mma_t(sL, SA, 1, sXJ, SB, 1, wr, wc, lane, vj);
    __syncthreads();
    if (needI) store_quad(sXI, SB, wr, wc, lane, vi);
    if (needJ) store_quad(sXJ, SB, wr, wc, lane, vj);
    __syncthreads();
    d4 prod = {0.0, 0.0, 0.0, 0.0};
    if (I == k && J == k) {
      prod = mma_t(sL, 1, SA, sL, SA, 1, wr, wc, lane, prod);   // L^{-T} L^{-1}
      acc = -prod;
    } else if (I == k) {
      acc = mma_t(sL, 1, SA, sVJ, SB, 1, wr, wc, lane, prod);  // L^{-T} V_J
    } else if (J == k) {
      acc = mma_t(sXI, 1, SB, sL, SA, 1, wr, wc, lane, prod);  // V_I^T L^{-1}
    } else {
      prod = mma_t(sXI, 1, SB, sVJ, SB, 1, wr, wc, lane, prod); // V_I^T V_J
      acc = acc - prod;
    }
    // panel of sweep k + 1 (the diagonal tile's panel slot is the pivot chain's: nobody reads
    // a (k, k) panel tile)
    chain_inputs(k + 1);  // tiles (k+1, k+2), (k+2, k+2) after sweep k: pivot k+2's inputs
    if (k + 1 < T && I == k + 1 && J != I) publish_tile();
    if (trl) TR_HI(SLOT_LAST_MMA);
    __syncthreads();  // LDS is refilled next sweep
  }
  if (aug && !master) {  // upper-right block: +K^{-1} B (B_u part possibly stored transposed)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = I * 32 + 16 * wr + (lane >> 4) + 4 * r, jl = ja * 32 + 16 * wc + (lane & 15);
      if (ja < F.tu) {
        if (F.ou_t) F.Ou[(size_t)jl * F.ldou + i] = acc[r];
        else F.Ou[(size_t)i * F.ldou + jl] = acc[r];
      } else {
        F.Od[(size_t)i * F.ldod + jl - 32 * F.tu] = acc[r];
      }
    }
  }
  // K^{-1} = -X after the last sweep
#pragma unroll
  for (int r = 0; r < 4 && !aug && !master; ++r) {
    const int row = 16 * wr + (lane >> 4) + 4 * r, col = 16 * wc + (lane & 15);
    const double y = -acc[r];
    F.X[(size_t)(I * 32 + row) * p + J * 32 + col] = y;
    if (I == J && row == col) pv[row] = (I * 32 + row < F.n) ? y : 0.0;
  }
  __syncthreads();
  if (I == J && t == 0 && !master) {  // refinement gate: max_i (K^{-1})_ii of this block
    double mx = 0.0;
    for (int j = 0; j < 32; ++j) mx = fmax(mx, pv[j]);
    atomicMax(reinterpret_cast<unsigned long long*>(F.pst + 1), (unsigned long long)__double_as_longlong(mx));
  }
  if (trm && tile == 0) TR_HI(SLOT_GATHER);
  // the last workgroup of this factor re-arms the flags for the next launch
  if (t == 0 && master && m == 1) TR_HI(SLOT_CHAIN_M1);
  if (t == 0 && master && m == 1) TR_LO(SLOT_CHAIN_M1);
  if (t == 0) s_last = atomicAdd(done, 1u) == (unsigned)(T * TC);  // T*TC tiles + the chain
  __syncthreads();
  if (t == 0 && m == 0 && I == T - 1 && J == T - 1 && !master) TR_HI(SLOT_LAST_OUT);
  if (t == 0 && m == 0 && I == T - 1 && J == TC - 1 && !master) TR_HI(SLOT_LAST_AUG);
  if (s_last && t == 0) TR_HI(SLOT_CHAIN_END);
  if (s_last) {
    for (int e = t; e < T * TC + 2 * T; e += 256)
      __hip_atomic_store(F.flags + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (PLc && t == 0) __hip_atomic_store(F.epoch, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- multi-tile chain: large factors (1D, p up to 2048) -------------------------------------
// chain_kernel owns one 32x32 tile per workgroup (T^2 workgroups: p <= ~700).  Here a workgroup
// owns a LOWER macro tile -- rows {2R, 2R+1} x one pair of 32-column tiles {2C, 2C+1}, C < R --
// and up to one tile of its macro row's diagonal 2x2 block (multi_role: the three lower tiles
// go to three different workgroups of the row from R = 3 on, so no workgroup updates more than
// five tiles per sweep) -- so p = 2048 needs 1 + 32*31/2 = 497 workgroups + the pivot chain
// (two per CU).  The pivot chain is chain_kernel's (chain_master); per sweep k a
// tile workgroup:
//   * waits for the panel tiles of its row / column pairs and L_k^{-1}, loads them (sc1);
//   * forms V = L_k^{-1} X_{k,.} for its (up to) four tile rows / columns (MFMA, LDS);
//   * updates its (up to) five tiles (seven in macro row 1) with chain_kernel's operations -- first the tiles that
//     feed the next sweep's panel or the pivot chain, published together (one drain + barrier),
//     then the rest.
// Storage is the lower triangle: panel slot (k, J) of PB holds X_{k,J} after sweep k-1; for J > k
// it is the transpose of lower tile (J, k), published transposed by its owner.  The same
// operation sequence per tile as chain_kernel (bitwise equal results); K^{-1} is written to both
// triangles at the end.  V tiles are XOR-swizzled in LDS (element (k, j) at 32k + (j ^ 16(k&1)):
// conflict-free fragment reads without padding), so the workgroup needs 42 KB.
__device__ __forceinline__ int vsw(int k, int j) { return 32 * k + (j ^ ((k & 1) << 4)); }

// acc += A B over one 32-deep product, this wave's quadrant; fa(i, k), fb(k, j) give the operands
template <class FA, class FB>
__device__ __forceinline__ d4 mma_f(FA fa, FB fb, int wr, int wc, int lane, d4 acc) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = 4 * kk + lk;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa(16 * wr + li, k), fb(k, 16 * wc + li), acc, 0, 0, 0);
  }
  return acc;
}

// slot s of a macro-tile workgroup: s < 4 the column pair c0 (rows 2R + (s >> 1), column
// 2 c0 + (s & 1)), s = 4..6 the diagonal block (2R,2R), (2R+1,2R), (2R+1,2R+1)
__host__ __device__ inline void multi_slot(int s, int R, int c0, int& I, int& J) {
  if (s < 4) {
    I = 2 * R + (s >> 1);
    J = 2 * c0 + (s & 1);
  } else {
    I = 2 * R + (s == 4 ? 0 : 1);
    J = 2 * R + (s == 6 ? 1 : 0);
  }
}

// macro-tile workgroup g (0-based) -> macro row R, its column pair c0 (-1: none) and the tiles of
// the diagonal 2x2 block it holds (dmask bit s - 4 for slot s).  Row 0: the diagonal block only;
// row R >= 1: R workgroups c0 = 0 .. R-1.  The pivot chain's inputs after sweep k are tiles
// (k+2, k+1) and (k+2, k+2), and every workgroup updates all of its tiles in every sweep, so the
// workgroup holding an input tile must not be slowed by extra tiles: (2R+1, 2R+1) goes to c0 =
// R-1, (2R, 2R) to R-2 and (2R+1, 2R) to R-3 (rows 1, 2: to c0 = 0 where those do not exist).
// Round 2's form gave the whole block to c0 = R-1: seven tiles, four of them in the critical
// pass of sweep 2R-1, which set the C2 sweep cycle.
__host__ __device__ inline void multi_role(int g, int& R, int& c0, int& dmask) {
  if (g == 0) {
    R = 0; c0 = -1; dmask = 7;
    return;
  }
  int r = 1, first = 1;  // first workgroup of macro row r: 1 + r(r-1)/2
  while (first + r <= g) { first += r; ++r; }
  R = r;
  c0 = g - first;
  const int o4 = r >= 2 ? r - 2 : 0, o5 = r >= 3 ? r - 3 : 0, o6 = r - 1;
  dmask = (c0 == o4 ? 1 : 0) | (c0 == o5 ? 2 : 0) | (c0 == o6 ? 4 : 0);
}

__host__ __device__ inline int multi_workgroups(int T) {  // per factor, + the pivot chain
  const int MT = (T + 1) / 2;
  return 1 + MT * (MT - 1) / 2 + 1;
}

template <int DERIV, bool GATHER>
__global__ __launch_bounds__(256, 2) void chain_multi_kernel(ChainBatch b) {
  const int m = blockIdx.y;
  if (m == b.nmat) {  // the step constants (+ a folded batch begin), off the critical path
    if (blockIdx.x == 0) publish_prep(b.prep, b.q);
    copy_snapshot(b.prep, blockIdx.x, gridDim.x);
    return;
  }
  const ChainFactor& F = b.f[m];
  const int T = F.T, p = F.p;
  const int nwg = multi_workgroups(T);
  if ((int)blockIdx.x >= nwg) return;
  // the pivot chain's workgroup sits at linear index mpos (host: a CU the dispatcher's second
  // pass over the CUs does not double up), the tile workgroups around it
  const int mpos = b.mpos < nwg ? b.mpos : 0;
  const bool master = (int)blockIdx.x == mpos;
  if (master && threadIdx.x == 0 && m == 0) TR_WHO(SLOT_MCP_MPOS, blockIdx.x);
  int R = 0, c0 = -1, dmask = 0;
  if (!master) multi_role((int)blockIdx.x - ((int)blockIdx.x > mpos ? 1 : 0), R, c0, dmask);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int tx = t & 31, ty = t >> 5;
  unsigned int* done = F.flags + T * T + 2 * T;
  // panel hand-off: self-validating words (chain_master's inputs, above) in the PB2 half of this
  // launch's parity; the other half (last launch's) is reset to the sentinel meanwhile, a chunk
  // per tile workgroup and sweep, off the critical path.  No flags, no drains.
  // L_k^{-1} travels the same way (PLc, after the panel slots in each half; no pivot flags): it
  // is normally written before the panel row it goes with, so it arrives with the panel's loads
  const unsigned ep = __hip_atomic_load(F.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const size_t hs = multi_half(p);
  double* PBc = F.PB2 + (size_t)(ep & 1u) * hs;
  double* PBo = F.PB2 + (size_t)((ep & 1u) ^ 1u) * hs;
  double* PLc = PBc + (size_t)p * p;
  // LDS: L_k^{-1} [32][SA] + four swizzled V tiles; the pivot chain's sXJ / sP / sM alias them
  __shared__ double pool[32 * SA + 4 * 1024];
  __shared__ double pv[32];
  __shared__ unsigned int s_last;
  __shared__ double sQ[4 * 16 * 17];  // per-wave transposition blocks (publish_stores)
  double* sL = pool;
  double* sV = pool + 32 * SA;

  auto valid = [&](int s) {
    if (master) return false;
    if (s < 4 && c0 < 0) return false;
    if (s >= 4 && !((dmask >> (s - 4)) & 1)) return false;
    int I, J;
    multi_slot(s, R, c0, I, J);
    return I < T && J <= I;
  };
  // gathered / read K value (and Kc, D written) at (i, j)
  auto kval_at = [&](int i, int j, bool write) -> double {
    const size_t o = (size_t)i * p + j;
    if (GATHER) {
      const int u = F.cid[o];
      double kv, dv;
      if (u >= 0) {
        kv = F.kval[u];
        if (i == j) kv += F.jitter;
        dv = F.dval[u];
        if (DERIV == 1 && !(F.x[i] - F.x[j] >= 0.0)) dv = -dv;  // JAX abs'(0) = +1
      } else {
        kv = (i == j) ? 1.0 : 0.0;
        dv = 0.0;
      }
      if (write) {
        if (F.Kc) F.Kc[o] = kv;
        if (DERIV && F.D) F.D[o] = dv;
      }
      return kv;
    }
    return F.X[o];
  };
  d4 acc[7];
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    acc[s] = d4{0.0, 0.0, 0.0, 0.0};
    if (!valid(s)) continue;
    int I, J;
    multi_slot(s, R, c0, I, J);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = I * 32 + 16 * wr + (lane >> 4) + 4 * r, j = J * 32 + 16 * wc + (lane & 15);
      acc[s][r] = kval_at(i, j, true);
      if (GATHER && I != J && (F.Kc || (DERIV && F.D))) (void)kval_at(j, i, true);  // mirrored Kc / D
    }
  }
  const bool trm = t == 0 && m == 0;
  if (master) {
    d4 a0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      a0[r] = kval_at(16 * wr + (lane >> 4) + 4 * r, 16 * wc + (lane & 15), false);
    double* sXJ = pool;             // [32][SB]
    double* sP = pool + 32 * SB;    // [32][SP]
    double* sM = sP + 32 * SP;      // [32][SP]
    chain_master<false>(F, T, a0, sXJ, sP, sM, pv, trm, true, PLc);
  }

  // hand-offs after sweep kk - 1 (kk = k + 1; kk = 0: before sweep 0): panel row kk -- tile
  // (kk, J), J < kk as is, tile (I, kk), I > kk transposed (stores of every publishing tile of
  // the pass, one drain + barrier, flags) -- and, as granules first, the pivot chain's inputs of
  // hop kk: tile (kk+1, kk) (= panel tile (kk, kk+1) transposed) and the diagonal tile
  // (kk+1, kk+1)
  auto publishes = [&](int s, int kk) {
    int I, J;
    multi_slot(s, R, c0, I, J);
    return kk < T && ((I == kk && J < kk) || (J == kk && I > kk));
  };
  auto chain_in = [&](int s, int kk) {
    int I, J;
    multi_slot(s, R, c0, I, J);
    return kk + 1 < T && I == kk + 1 && (J == kk || J == I);
  };
  // a wave's 16x16 quadrant stored transposed -- element (row, col) of the tile to
  // dst[col * ld + row] -- through its own LDS block (no workgroup barrier): each store
  // instruction then writes 4 whole 128-B column segments instead of 16 lines x 32 B
  auto put_transposed = [&](double* dst, size_t ld, const d4& a) {
    double* q = sQ + wv * (16 * 17);
#pragma unroll
    for (int r = 0; r < 4; ++r) q[((lane >> 4) + 4 * r) * 17 + (lane & 15)] = a[r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = lane + 64 * r, c = e >> 4, rr = e & 15;  // quadrant column c, row rr
      st_sc1(dst + (size_t)(16 * wc + c) * ld + 16 * wr + rr, q[rr * 17 + c]);
    }
    __builtin_amdgcn_wave_barrier();
  };
  // stores of the publishing tiles (sc1, not waited for here): which = 0 the pivot chain's input
  // tiles (granules, and their panel slots when they publish), 1 the other publishing tiles
  auto publish_stores = [&](int kk, int which) {
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      if (which != 0 || !valid(s) || !chain_in(s, kk)) continue;
      int I, J;
      multi_slot(s, R, c0, I, J);
      if (I == J) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * wr + (lane >> 4) + 4 * r, col = 16 * wc + (lane & 15);
          st_sc1(gran_at(F, kk, 1, row * 32 + col), acc[s][r]);
        }
      } else {  // (kk+1, kk) -> element (col, row) of panel tile (kk, kk+1)
        put_transposed(gran_at(F, kk, 0, 0), 32, acc[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      if (!valid(s) || !publishes(s, kk) || chain_in(s, kk) != (which == 0)) continue;
      int I, J;
      multi_slot(s, R, c0, I, J);
      if (I == kk) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * wr + (lane >> 4) + 4 * r, col = 16 * wc + (lane & 15);
          st_sc1(PBc + (size_t)(kk * 32 + row) * p + J * 32 + col, acc[s][r]);
        }
      } else {  // (I, kk) -> slot (kk, I) transposed
        put_transposed(PBc + (size_t)(kk * 32) * p + I * 32, (size_t)p, acc[s]);
      }
    }
  };
  if (!master) {
    publish_stores(0, 0);
    publish_stores(0, 1);
  }
  // this workgroup's share of the other half's reset: [rs0, rs1), a chunk per sweep
  const size_t ntot = hs;
  const int gidx = (int)blockIdx.x - ((int)blockIdx.x > mpos ? 1 : 0);
  const size_t share = (ntot + (nwg - 2)) / (nwg - 1);
  const size_t rs0 = std::min(ntot, (size_t)gidx * share), rs1 = std::min(ntot, rs0 + share);
  const size_t rchunk = (share + T - 1) / T;

  __shared__ unsigned s_lword_;  // sweep k + 1 once thread 0 has seen a word of L_k^{-1}
  volatile unsigned* s_lword = &s_lword_;
  if (t == 0) *s_lword = 0u;
  __syncthreads();
  // V slots: 0, 1 = rows 2R, 2R+1; 2, 3 = the plain column pair's columns 2c0, 2c0+1
  auto vslot_of_col = [&](int s) { return s < 4 ? 2 + (s & 1) : (s == 6 ? 1 : 0); };
  for (int k = 0; k < T && !master; ++k) {
    // probes (gpk_trace.h SLOT_MC_*): the workgroup owning tile (k+2, k+2), factor 0
    const bool trc = t == 0 && m == 0 && k < 16 &&
                     ((k + 2 == 2 * R && (dmask & 1)) || (k + 2 == 2 * R + 1 && (dmask & 4)));
    // issue priority: the sweep's front half (loads, V, the pass-0 tiles that feed sweep k+1 and
    // the pivot chain) over the pass-1 products of the workgroup sharing this CU
    __builtin_amdgcn_s_setprio(2);
    bool need[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int idx = v < 2 ? 2 * R + v : 2 * c0 + (v - 2);
      need[v] = (v < 2 || c0 >= 0) && idx < T && idx != k;
    }
    // panel tiles of sweep k: load, re-load the words still holding the sentinel (bounded)
    double xv[4][4];
    auto load_panel = [&]() {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int idx = v < 2 ? 2 * R + v : 2 * c0 + (v - 2);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          xv[v][r] = need[v] ? ld_sc1(PBc + (size_t)(k * 32 + ty + 8 * r) * p + idx * 32 + tx) : 0.0;
      }
    };
    auto panel_ok = [&]() {
      bool ok = true;
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) ok = ok && gran_ok(xv[v][r]);
      return ok;
    };
    // re-load while waiting: only each tile's first word (r = 0) until those are in, then the
    // words still holding the sentinel -- a quarter of the polling traffic of ~500 waiting
    // workgroups, which otherwise delays the very stores they wait for
    auto reload_panel = [&]() {
      bool head = true;
#pragma unroll
      for (int v = 0; v < 4; ++v) head = head && gran_ok(xv[v][0]);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int idx = v < 2 ? 2 * R + v : 2 * c0 + (v - 2);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (need[v] && !gran_ok(xv[v][r]) && (r == 0 || head))
            xv[v][r] = ld_sc1(PBc + (size_t)(k * 32 + ty + 8 * r) * p + idx * 32 + tx);
      }
    };
    // L_k^{-1}'s words (row ty + 8r, column tx), loaded with the panel's; only the words still
    // holding the sentinel are loaded again
    const double* Li = PLc + (size_t)k * 1024;
    double lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lv[r] = __longlong_as_double((long long)CHAIN_SENTINEL);
    auto load_l = [&]() {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!gran_ok(lv[r])) lv[r] = ld_sc1(Li + (ty + 8 * r) * 32 + tx);
    };
    auto l_ok = [&]() {
      bool ok = true;
#pragma unroll
      for (int r = 0; r < 4; ++r) ok = ok && gran_ok(lv[r]);
      return ok;
    };
    // L_k^{-1}: while the panel is awaited, thread 0 polls ONE of its words (a flag's polling
    // traffic); once that word is in, every thread issues its own words with its next panel
    // re-load, so they arrive under the panel wait instead of one round trip after it.  Polling
    // all of L_k^{-1}'s words with the panel had ~500 workgroups re-loading the same 8 KB while
    // the pivot was being factored (measured: C2 0.638 -> 0.676 ms), and so did loading them
    // once with the panel's first attempt (0.614 -> 0.677 ms): no thread touches the slots
    // before that one word is in.
    load_panel();
    if (t == 0) lv[0] = ld_sc1(Li);  // (thread 0's first word is the one polled)
    bool lissued = false;
    for (unsigned spins = 0; !panel_ok(); ++spins) {
      if (spin_give_up(spins, F.status)) break;
      if (!lissued) {
        if (t == 0 && gran_ok(lv[0])) *s_lword = k + 1;
        if (*s_lword == (unsigned)(k + 1)) {
          load_l();
          lissued = true;
        }
      }
      __builtin_amdgcn_s_sleep(1);
      reload_panel();
      if (t == 0 && !lissued) lv[0] = ld_sc1(Li);
    }
    if (trc) TR_HI(SLOT_MC_PANEL + k);
    load_l();  // (the words not yet loaded, or still holding the sentinel)
    for (unsigned spins = 0; !l_ok(); ++spins) {
      if (spin_give_up(spins, F.status)) break;
      __builtin_amdgcn_s_sleep(1);
      load_l();
    }
    if (trc) TR_HI(SLOT_MC_PIV + k);
    // probes (trace build): every workgroup that publishes panel row k + 1 in this sweep's pass 0,
    // [first, last] of its inputs-in and of its publication (SLOT_MCP_IN / SLOT_MCP_OUT)
    [[maybe_unused]] bool pubk = false;
#ifdef GPK_TRACE
#pragma unroll
    for (int s = 0; s < 7; ++s) pubk = pubk || (valid(s) && publishes(s, k + 1));
    pubk = pubk && t == 0 && m == 0 && k < 16;
    if (pubk) { TR_LO(SLOT_MCP_IN + k); TR_HI(SLOT_MCP_IN + k); TR_WHO(SLOT_MCP_WHO_IN + k, blockIdx.x); }
#endif
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = ty + 8 * r;
      sL[row * SA + tx] = lv[r];
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (need[v]) sV[v * 1024 + vsw(row, tx)] = xv[v][r];
    }
    __syncthreads();
    if (trc) TR_HI(SLOT_MC_LDS + k);
    d4 vv[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      vv[v] = d4{0.0, 0.0, 0.0, 0.0};
      if (!need[v]) continue;
      const double* X = sV + v * 1024;
      vv[v] = mma_f([&](int i, int kq) { return sL[i * SA + kq]; }, [&](int kq, int j) { return X[vsw(kq, j)]; },
                    wr, wc, lane, vv[v]);  // V = L_k^{-1} X_{k,idx}
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      if (!need[v]) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sV[v * 1024 + vsw(16 * wr + (lane >> 4) + 4 * r, 16 * wc + (lane & 15))] = vv[v][r];
    }
    __syncthreads();
    if (trc) TR_HI(SLOT_MC_V + k);
    // the tiles that publish after this sweep (and the pivot chain's inputs) first, their
    // stores, then the rest.  (Forming V_I^T V_J as P_I^T (M_k P_J), M_k = L_k^{-T} L_k^{-1},
    // halves the V products but moved no sweep: the critical merged workgroups keep 4 products,
    // and the 5-step C2 trajectory drifted past the oracle budget -- measured, reverted.)
    // pass 0: the pivot chain's input tiles (its next hop waits on them), stored at once; pass 1:
    // the other tiles that publish panel row k + 1; pass 2: the rest.  (A loop: unrolled three
    // times it spilled 108 B per lane.)
#pragma unroll 1
    for (int pass = 0; pass < 3; ++pass) {
#pragma unroll
      for (int s = 0; s < 7; ++s) {
        if (!valid(s)) continue;
        const int ps = chain_in(s, k + 1) ? 0 : publishes(s, k + 1) ? 1 : 2;
        if (ps != pass) continue;
        int I, J;
        multi_slot(s, R, c0, I, J);
        const double* VI = sV + (s < 4 ? (s >> 1) : (s == 4 ? 0 : 1)) * 1024;
        const double* VJ = sV + vslot_of_col(s) * 1024;
        auto lt = [&](int i, int kq) { return sL[kq * SA + i]; };  // L^T (i, k) = L (k, i)
        auto lk = [&](int kq, int j) { return sL[kq * SA + j]; };
        auto vit = [&](int i, int kq) { return VI[vsw(kq, i)]; };  // V_I^T
        auto vj = [&](int kq, int j) { return VJ[vsw(kq, j)]; };
        d4 prod = {0.0, 0.0, 0.0, 0.0};
        if (I == k && J == k) {
          prod = mma_f(lt, lk, wr, wc, lane, prod);  // L^{-T} L^{-1}
          acc[s] = -prod;
        } else if (I == k) {
          acc[s] = mma_f(lt, vj, wr, wc, lane, prod);  // L^{-T} V_J
        } else if (J == k) {
          acc[s] = mma_f(vit, lk, wr, wc, lane, prod);  // V_I^T L^{-1}
        } else {
          prod = mma_f(vit, vj, wr, wc, lane, prod);  // V_I^T V_J
          acc[s] = acc[s] - prod;
        }
      }
      if (pass == 1 && trc) TR_HI(SLOT_MC_PROD + k);
      if (pass < 2 && k + 1 < T) publish_stores(k + 1, pass);
      if (pass == 1 && trc) TR_HI(SLOT_MC_PUB + k);
      if (pass == 1 && pubk) { TR_LO(SLOT_MCP_OUT + k); TR_HI(SLOT_MCP_OUT + k); TR_WHO(SLOT_MCP_WHO_OUT + k, blockIdx.x); }
      if (pass == 1) __builtin_amdgcn_s_setprio(0);
    }
    {  // reset chunk k of this workgroup's share of the other half
      const size_t b0 = rs0 + (size_t)k * rchunk, b1 = std::min(rs1, b0 + rchunk);
      for (size_t e = b0 + t; e < b1; e += 256)
        PBo[e] = __longlong_as_double((long long)CHAIN_SENTINEL);
    }
    __syncthreads();  // LDS is refilled next sweep
    if (trc) TR_HI(SLOT_MC_DONE + k);
  }
  // K^{-1} = -X, both triangles; refinement gate over the diagonal tiles
  double mx = 0.0;
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    if (!valid(s)) continue;
    int I, J;
    multi_slot(s, R, c0, I, J);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * wr + (lane >> 4) + 4 * r, col = 16 * wc + (lane & 15);
      const double y = -acc[s][r];
      F.X[(size_t)(I * 32 + row) * p + J * 32 + col] = y;
      if (I != J) F.X[(size_t)(J * 32 + col) * p + I * 32 + row] = y;
      else if (row == col && I * 32 + row < F.n) mx = fmax(mx, y);
    }
  }
  if (dmask & 5) {  // holds a diagonal tile
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if (lane == 0 && mx > 0.0)
      atomicMax(reinterpret_cast<unsigned long long*>(F.pst + 1), (unsigned long long)__double_as_longlong(mx));
  }
  // the last workgroup of this factor re-arms the flags for the next launch
  __syncthreads();
  if (t == 0) s_last = atomicAdd(done, 1u) == (unsigned)(nwg - 1);
  __syncthreads();
  if (s_last) {
    for (int e = t; e < T * T + 2 * T; e += 256)
      __hip_atomic_store(F.flags + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) __hip_atomic_store(F.epoch, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Workgroups of chain_kernel<DERIV, GATHER> the current device keeps resident at once:
// occupancy per CU (its VGPR / LDS footprint) x the CUs this device (or partition) exposes.
int spd_chain_capacity(int deriv, bool gather) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  hipError_t e;
  if (!gather)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, chain_kernel<0, false>, 256, 0);
  else if (deriv == 1)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, chain_kernel<1, true>, 256, 0);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, chain_kernel<2, true>, 256, 0);
  return e == hipSuccess ? per * cus : 0;
}

int spd_chain_multi_capacity(int deriv, bool gather) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  hipError_t e;
  if (!gather)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, chain_multi_kernel<0, false>, 256, 0);
  else if (deriv == 1)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, chain_multi_kernel<1, true>, 256, 0);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, chain_multi_kernel<2, true>, 256, 0);
  return e == hipSuccess ? per * cus : 0;
}

int spd_chain_multi_blocks(const int* p, int nmat) {
  int w = 0;
  for (int m = 0; m < nmat; ++m) w = std::max(w, multi_workgroups(p[m] / 32));
  return w * nmat;
}

int spd_chain_blocks(const int* p, int nmat, bool aug) {
  int blocks = 0, cols = 0;
  for (int m = 0; m < nmat; ++m) cols += p[m] / 32;
  for (int m = 0; m < nmat; ++m) blocks += (p[m] / 32) * (p[m] / 32 + (aug ? cols : 0)) + 1;
  return blocks;
}

hipError_t launch_spd_chain(const ChainArgs* a, int nmat, int deriv, hipStream_t s,
                            const PrepArgs* prep, int q) {
  ChainBatch b{};
  b.nmat = nmat;
  if (prep) {
    b.prep = *prep;
    b.q = q;
  }
  int Tmax = 0;
  bool gather = a[0].cid != nullptr;
  for (int m = 0; m < nmat; ++m) {
    ChainFactor& f = b.f[m];
    f.X = a[m].X; f.PB = a[m].PB; f.piv = a[m].piv; f.ldet = a[m].ldet; f.pst = a[m].pst;
    f.status = a[m].status; f.flags = a[m].flags; f.p = a[m].p; f.n = a[m].n; f.T = a[m].p / 32;
    f.cid = a[m].cid; f.kval = a[m].kval; f.dval = a[m].dval; f.x = a[m].x; f.jitter = a[m].jitter;
    f.Kc = a[m].Kc; f.D = a[m].D;
    f.tu = a[m].tu; f.td = a[m].td; f.Bu = a[m].Bu; f.ldbu = a[m].ldbu; f.bu_t = a[m].bu_t;
    f.Ou = a[m].Ou; f.ldou = a[m].ldou; f.ou_t = a[m].ou_t; f.Od = a[m].Od; f.ldod = a[m].ldod;
    f.PBa = a[m].PBa; f.ldpba = a[m].ldpba;
    f.gran = a[m].gran; f.piv_off = f.T * (f.T + f.tu + f.td);
    f.PB2 = a[m].PB2; f.epoch = a[m].epoch;  // (both null: L^{-1} hand-off by flag + load)
    if ((a[m].cid != nullptr) != gather || !f.gran || !f.PB2 != !f.epoch) return hipErrorInvalidValue;
    Tmax = std::max(Tmax, f.T * (f.T + f.tu + f.td) + 1);  // + the pivot chain's workgroup
  }
  dim3 grid(Tmax, nmat + (prep ? 1 : 0));
  if (!gather)
    hipLaunchKernelGGL((chain_kernel<0, false>), grid, dim3(256), 0, s, b);
  else if (deriv == 1)
    hipLaunchKernelGGL((chain_kernel<1, true>), grid, dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL((chain_kernel<2, true>), grid, dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t launch_spd_chain_multi(const ChainArgs* a, int nmat, int deriv, hipStream_t s,
                                  const PrepArgs* prep, int q) {
  ChainBatch b{};
  b.nmat = nmat;
  if (prep) {
    b.prep = *prep;
    b.q = q;
  }
  int wmax = 0;
  const bool gather = a[0].cid != nullptr;
  for (int m = 0; m < nmat; ++m) {
    ChainFactor& f = b.f[m];
    f.X = a[m].X; f.PB = a[m].PB; f.piv = a[m].piv; f.ldet = a[m].ldet; f.pst = a[m].pst;
    f.status = a[m].status; f.flags = a[m].flags; f.p = a[m].p; f.n = a[m].n; f.T = a[m].p / 32;
    f.cid = a[m].cid; f.kval = a[m].kval; f.dval = a[m].dval; f.x = a[m].x; f.jitter = a[m].jitter;
    f.Kc = a[m].Kc; f.D = a[m].D;
    f.gran = a[m].gran; f.piv_off = f.T * f.T; f.PB2 = a[m].PB2; f.epoch = a[m].epoch;
    if ((a[m].cid != nullptr) != gather || a[m].tu || a[m].td || !f.gran || !f.PB2 || !f.epoch)
      return hipErrorInvalidValue;
    wmax = std::max(wmax, multi_workgroups(f.T));
  }
  // one factor: the pivot chain in the middle of the CUs that hold a single workgroup (the
  // dispatcher deals the first `cus` workgroups one per CU, the rest double up the first CUs
  // again; placement only -- the flags order everything)
  b.mpos = 0;
  int dev = 0, cus = 0;
  if (nmat == 1 && hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      wmax > cus && wmax < 2 * cus)
    b.mpos = wmax - cus + (2 * cus - wmax) / 2;
  dim3 grid(wmax, nmat + (prep ? 1 : 0));
  if (!gather)
    hipLaunchKernelGGL((chain_multi_kernel<0, false>), grid, dim3(256), 0, s, b);
  else if (deriv == 1)
    hipLaunchKernelGGL((chain_multi_kernel<1, true>), grid, dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL((chain_multi_kernel<2, true>), grid, dim3(256), 0, s, b);
  return hipGetLastError();
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
    hipLaunchKernelGGL(sweep_kernel, dim3(nmat, Tmax * Tmax), dim3(256), 0, s, b, stage);
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
    hipLaunchKernelGGL(sweep_kernel, dim3(nmat, Tmax * Tmax), dim3(256), 0, s, b, k);
  return hipGetLastError();
}

}  // namespace gpk
