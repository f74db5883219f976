// spdinv_big.hip — SPD inverse + log-determinant for LARGE covariance factors (gfx950, fp64 MFMA).
//
// Same contract as spdinv.hip (replaces jnp.linalg.solve / slogdet of
// code/model_GP_solver_1d.py:92,135-137, code/model_GP_solver_2d.py:104-105,157-162,
// code/model_GP_solver_advection.py:104-105,153-158): X <- K^{-1} in place, log det K per 32-row
// block, refinement gate, non-PD status.  The 32-wide sweep of spdinv.hip re-reads and rewrites
// the whole matrix once per 32 columns and recomputes its panel in every tile; at p >= ~1024
// that is HBM- and launch-bound.  This path sweeps W = 64 R wide pivot blocks (R = 1 or 2) over
// 64 x 64 tiles and splits each sweep into three pieces of work:
//
//   panel   Z = L^{-1} X_{P,:}   (W x p, small MFMA GEMMs per 64-column block; Z_P = L^{-1})
//   update  X_IJ <- s_IJ (base_IJ - Z_I^T Z_J) on the LOWER tiles only (I >= J), in place:
//             I,J not in P : X_IJ - Z_I^T Z_J          (Schur complement, the SYRK-shaped bulk)
//             one of I,J in P : + Z_I^T Z_J           (= L^{-T} V: the swept panel)
//             I, J in P : - Z_I^T Z_J                 (= -S^{-1})
//   pivot   the next pivot block S = X_{k+1,k+1} (W x W) is factored (Cholesky + L^{-1}) by one
//           extra workgroup of the update launch, right after the workgroups that own its
//           tiles have written them back (write-through stores + counter hand-off, MI355X_MICROARCH
//           inter-workgroup visibility), so the serial pivot chain runs under the bulk of the update.
//
// After ceil(p/W) sweeps X = -K^{-1}; the last sweep flips the sign, mirrors every lower tile into
// the upper triangle (LDS transpose, coalesced stores) and publishes max diag K^{-1} for the
// refinement gate.  Flops: p^3 (potrf + potri equivalent), all on v_mfma_f64_16x16x4.
//
// Sweep width.  Per sweep the update reads and writes the lower triangle once (8 p^2 B) for
// W p^2 flops, i.e. W / 8 flop per byte of X traffic: at W = 64 the 4096^2 update is bound by the
// matrix traffic (~20 TF/s), at W = 128 (R = 2) by MFMA.  Wide sweeps need a 128-pivot; its
// factorisation is exposed where the update is short, so R = 2 is used for the largest factors
// only (SPD_WIDE_MIN) and R = 1 keeps the shorter serial chain at ~2048.
// The 64-pivot factorisation is two 32-pivots (spd_pivot.h) glued by three 32x32 MFMA products:
//   L11^{-1} = chol_inv(S11);  V = L11^{-1} S12;  L22^{-1} = chol_inv(S22 - V^T V);
//   (L^{-1})_21 = -L22^{-1} V^T L11^{-1};
// the 128-pivot is the same recursion one level up with 64-pivots and 64x64 products.
#include <atomic>

#include "gemm_huge_dev.h"
#include "gemm_tile_dev.h"
#include "gpk_internal.h"
#include "spd_pivot.h"
#include "gpk_trace.h"

namespace gpk {

GPK_WAIT_LIMIT_SETTER(wait_limit_spdbig)  // gpk_set_wait_limit

GPK_TRACE_TU(spdbig)

static std::atomic<int> g_big_wgs{0};  // spd_big_set_workgroups override (tests)
void spd_big_set_workgroups(int g) { g_big_wgs.store(g > 0 ? g : 0); }

namespace {

constexpr int BW = 64;   // tile width (and the 64-pivot)
constexpr int SS = 65;   // 64x64 LDS tile stride (doubles)

struct BigSpdBatch {
  double* X[2];      // the matrix, inverted in place
  double* Z[2];      // 3 x [W][p] panel by sweep mod 3 (zbuf: a two-sweep tile update reads
                     // panels k - 1 and k while the launch writes k + 1)
  double* Li[2];     // [W][W] L^{-1} of the current pivot block (row-major, zero upper) + scratch
  double* ldet[2];   // [p/32]
  double* pst[2];    // refinement gate [2]
  int* status[2];
  unsigned int* flag[2];  // [0] hand-off count (64-wide), [1] pivot done (sweep index),
                          // [2] panel-row tiles done (cumulative over the inverse's sweeps)
  int p[2], n[2], T[2];  // T: 64-wide tiles per dimension
  int G;                 // tile workgroups per factor in the update launch
  int nmat;
  int no_quarters;       // (SpdArgs::no_quarters)
  int qfirst;            // (SpdArgs::qfirst)
  const unsigned* sched[2];  // 128-wide update schedule (wide_schedule) per factor, row stride sstride[m]
  int sstride[2];
};

__device__ __forceinline__ int bw(int p, int I) { return min(BW, p - BW * I); }

// S[r][c] = src[r*ld + c] for r < h, c < w (else 0): 64x64 tile, all 16 loads per thread in
// flight before the LDS stores (one wave per row: coalesced)
__device__ __forceinline__ void load_tile(double* S, const double* src, int ld, int h, int w, int t) {
  double v[16];
  const int c = t & 63, r0 = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = r0 + 4 * q;
    v[q] = (r < h && c < w) ? src[(size_t)r * ld + c] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) S[(r0 + 4 * q) * SS + c] = v[q];
}

// acc (16x16 block at rows i0, columns j0) += sa * A B over k < 32, A and B in LDS:
// A(i, k) at a[i * sai + k * sak], B(k, j) at b[k * sbk + j * sbj]
__device__ __forceinline__ d4 mma16s(const double* a, int sai, int sak, const double* b, int sbk, int sbj,
                                     int i0, int j0, int lane, double sa, d4 acc) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = 4 * kk + lk;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sa * a[(i0 + li) * sai + k * sak], b[k * sbk + (j0 + li) * sbj],
                                               acc, 0, 0, 0);
  }
  return acc;
}

constexpr int PB = SP;  // 32x32 LDS block stride (doubles)

// ---- the pivot: blocked Cholesky of the sweep's w x w diagonal block (w <= W = 64 R) -------
// Right-looking over 32-row blocks i: M_i = L_ii^{-1} (Cholesky + L^{-1} of the 32x32 block),
// L_ji = A_ji M_i^T for the blocks below, A_jk -= L_ji L_ki^T on the trailing lower blocks.
// Output Lg (W x W, ld W): the strictly-lower blocks L_ji and, in the diagonal block slots, M_i
// -- exactly what the panel's forward substitution reads (L_ii itself is never needed, and L^{-1}
// of the whole block is never formed).
// Register-resident: wave (bi, bj) keeps the 16x16 quadrant (bi, bj) of every lower 32x32 block
// in an MFMA accumulator for the whole factorisation (at most 10 blocks: 40 doubles per lane),
// loaded with one batch of loads; a block step stages its diagonal block and the column below it
// in LDS, factors the diagonal block on ONE wave (pivot_chol_inv_1w, bitwise the four-wave form),
// forms L_ji in place, and every wave subtracts L_ji L_ki^T from its quadrants of the trailing
// blocks -- no global round trip between block steps (the previous form kept the trailing blocks
// in a global scratch and loaded each 16x16 block's base just before its MFMAs: 46 us per
// 128-pivot).  Same products in the same order: bitwise that form.
// Why this form (tools/gj_accuracy.py, C5's 4096^2 factors vs the long-double inverse): with the
// forward-substitution panel below, a W-wide sweep does the 32-wide sweep's arithmetic -- K^{-1}
// 1.38e-8 relative for W = 64 ... 512 -- where the previous form (L^{-1} of the 64/128 block by
// the recursion -L22^{-1} V^T L11^{-1}, applied as one product) reached 3.4e-8 at W = 128, and
// C5's dL/dU 1.0e-7 instead of 3.4e-8 (the fp64 LU oracle: 4.3e-8).
template <int R>
__device__ __forceinline__ void pivot_blk(const double* src, int ld, int w, double* Lg, double* ldet, int* status,
                                          double* sm) {
  constexpr int W = BW * R, NB = 2 * R;
  double* sP = sm;            // [32][PB] A_ii (clobbered by the factorisation)
  double* sM = sP + 32 * PB;  // [32][PB] M_i
  double* pv = sM + 32 * PB;  // [32]
  double* sL = pv + 32;       // [NB - 1][32][PB] A_ji, then L_ji (j > i)
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int bi = wv >> 1, bj = wv & 1;  // this wave's quadrant of every block
  const int nb = w / 32;
  d4 a[NB][NB];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int k = 0; k <= j; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        a[j][k][r] = j < nb ? src[(size_t)(32 * j + 16 * bi + lk + 4 * r) * ld + 32 * k + 16 * bj + li] : 0.0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    if (i >= nb) break;
    if (i) __syncthreads();  // the previous step's trailing products are done reading sL
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * bi + lk + 4 * r, col = 16 * bj + li;
      sP[row * PB + col] = a[i][i][r];
#pragma unroll
      for (int j = i + 1; j < NB; ++j)
        if (j < nb) sL[(j - i - 1) * 32 * PB + row * PB + col] = a[j][i][r];
    }
    __syncthreads();
    const double ls = pivot_chol_inv_1w(sP, sM, pv, t, status);
    if (t == 0) ldet[i] = ls;
    for (int e = t; e < 1024; e += 256)
      Lg[(size_t)(32 * i + (e >> 5)) * W + 32 * i + (e & 31)] = sM[(e >> 5) * PB + (e & 31)];
    const int nl = nb - 1 - i;  // blocks below the pivot
    if (nl == 0) break;
    // L_ji = A_ji M_i^T (B(k, c) = M_i[c][k]); wave q computes j = i + 1 + q and overwrites its
    // own A_ji in LDS with it (one wave's LDS operations are in order)
    if (wv < nl) {
      double* sA = sL + wv * 32 * PB;
      const int j = i + 1 + wv;
#pragma nounroll
      for (int hb = 0; hb < 2; ++hb) {  // rows 16 hb.. of sA are read, then overwritten
        d4 acc[2];
#pragma unroll
        for (int hc = 0; hc < 2; ++hc)
          acc[hc] = mma16s(sA, PB, 1, sM, 1, PB, 16 * hb, 16 * hc, lane, 1.0, d4{0.0, 0.0, 0.0, 0.0});
#pragma unroll
        for (int hc = 0; hc < 2; ++hc)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * hb + lk + 4 * r, col = 16 * hc + li;
            Lg[(size_t)(32 * j + row) * W + 32 * i + col] = acc[hc][r];
            sA[row * PB + col] = acc[hc][r];
          }
      }
    }
    __syncthreads();
    // trailing lower blocks (j, k), i < k <= j: A_jk -= L_ji L_ki^T (B(x, c) = L_ki[c][x])
#pragma unroll
    for (int j = i + 1; j < NB; ++j)
#pragma unroll
      for (int k = i + 1; k <= j; ++k)
        if (j < nb)
          a[j][k] = mma16s(sL + (j - i - 1) * 32 * PB, PB, 1, sL + (k - i - 1) * 32 * PB, 1, PB, 16 * bi, 16 * bj,
                           lane, -1.0, a[j][k]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int R>
constexpr int pivot_lds() { return 2 * 32 * PB + 32 + (2 * R - 1) * 32 * PB; }
// the panel: X_i (32 x 65) + one row block of L (2R blocks of 32 x PB)
template <int R>
constexpr int panel_lds() { return 32 * 65 + 2 * R * 32 * PB; }
constexpr int PIVOT_LDS = pivot_lds<2>() > panel_lds<2>() ? pivot_lds<2>() : panel_lds<2>();  // doubles

// the panel buffer of sweep k (the update of sweep k reads it -- and panel k - 1, for tiles that
// apply two sweeps -- while the panel of sweep k + 1 is written into the third, by the same launch)
template <int R>
__device__ __forceinline__ double* zbuf(const BigSpdBatch& b, int m, int k) {
  return b.Z[m] + (size_t)(k % 3) * (BW * R) * b.p[m];
}

// inter-workgroup hand-off (MI355X_MICROARCH §inter-workgroup visibility, plain stores + agent
// release / acquire): every storing wave drains, barrier, one lane's release fence + counter
__device__ __forceinline__ void release_add(unsigned int* c, unsigned int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    atomicAdd(c, v);
  }
}
__device__ __forceinline__ void acquire_wait(const unsigned int* c, unsigned int target, int* status) {
  if (threadIdx.x == 0) {
    (void)spin_until_ge<2>(c, target, status);  // bounded: status bit 2 on a lost hand-off
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// the pivot block of sweep k (W = 64 R rows): L and the M_i into Li, log det per 32 rows
template <int R>
__device__ __forceinline__ void pivot_block(const BigSpdBatch& b, int m, int k, double* sm) {
  const int p = b.p[m];
  const int r0 = BW * R * k, w = min(BW * R, p - r0);
  pivot_blk<R>(b.X[m] + (size_t)r0 * p + r0, p, w, b.Li[m], b.ldet[m] + 2 * R * k, b.status[m], sm);
}

template <int R>
__global__ __launch_bounds__(256) void big_pivot_init_kernel(BigSpdBatch b) {
  const int m = blockIdx.x;
  __shared__ double sm[PIVOT_LDS];
  const double x00 = b.X[m][0];
  pivot_block<R>(b, m, 0, sm);
  if (threadIdx.x == 0) {
    b.pst[m][0] = x00;   // K_00 = max diag K (stationary kernel + jitter)
    b.pst[m][1] = 0.0;   // max diag K^{-1}: atomicMax'd by the last sweep
    b.flag[m][0] = 0u;
    b.flag[m][1] = 0u;
    b.flag[m][2] = 0u;
  }
  // the 128-wide update's per-sweep panel-block tickets (wide_update_kernel), one per sweep
  for (int i = threadIdx.x; i < b.p[m] / 32; i += 256) b.flag[m][4 + i] = 0u;
}

// ---- the panel: Z_{:,J} = L^{-1} X_{P,J} by forward substitution over 32-row blocks ---------
// One 256-thread workgroup per 64 columns J of the factor (J < T; the last tile may be 32 wide).
// Stage i: acc = X_i - sum_{j<i} L_ij Z_j, then Z_i = M_i acc (X_i: rows 32 i.. of X_{P,J} in
// the lower storage -- row block P for J < P, the transpose of column block P for J > P -- and
// the identity for the sweep's own columns, whose Z is L^{-1} itself).  Wave w owns columns
// 16 w.. of the block for every row, so each Z_j stays in its registers: a 16x16 MFMA result in
// the C layout (element (lk + 4 r, li) in acc[r]) is the B operand of the next product's k-steps
// (k-step r reads B[4 r + lk][li]).  Row block i of Lg (L_i0 .. L_i,i-1, M_i) is staged in LDS.
// Loads: the first two stages' X values are issued as soon as the panel row is in (wait.rows()),
// before the wait for the pivot, the next ones two stages ahead, and each stage's L row block is
// fetched into registers under the previous stage's products -- about one memory round trip per
// panel instead of two per stage (the standalone C5 panel of sweep 0: 25 -> 15 us).  Same
// products in the same order.
struct NoPanelWait {
  __device__ void rows() const {}
  __device__ void pivot() const {}
};
template <int R, typename Wait = NoPanelWait>
__device__ __forceinline__ void panel_block(const BigSpdBatch& b, int m, int k, int J, double* sm,
                                            Wait wait = Wait()) {
  constexpr int NB = 2 * R, W = BW * R;
  const int p = b.p[m], T = b.T[m];
  const int P0 = R * k;  // first 64-tile of the swept block
  if (P0 >= T || J >= T) return;
  const int nb = min(W, p - BW * P0) / 32;
  const int r0 = BW * P0, c0 = BW * J, wJ = bw(p, J);
  const bool own = J >= P0 && J < P0 + R;
  const double* X = b.X[m];
  const double* Lg = b.Li[m];
  double* Z = zbuf<R>(b, m, k);
  double* sX = sm;            // [32][65]
  double* sL = sm + 32 * 65;  // [NB][32][PB]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int col = c0 + 16 * wv + li;
  wait.rows();
  // X_i element e = t + 256 q: (r, c) = (e >> 6, e & 63) in row block P (J < P: coalesced along
  // c), (e & 31, e >> 5) in column block P (J > P: X_{P,J}[r][c] = X[c0 + c][r0 + 32 i + r],
  // coalesced along r); the identity in the swept columns
  // (two stages in flight: a rolling pair of register sets, stage i + 2's loads issued once
  // stage i is in LDS -- all four at once pushed the update kernel's tile loop into spills)
  double xv[2][8];
  auto xload = [&](double (&v)[8], int i) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = t + 256 * q;
      double x = 0.0;
      if (i < nb) {
        if (own) {
          x = (r0 + 32 * i + (e >> 6) == c0 + (e & 63)) ? 1.0 : 0.0;
        } else if (J < P0) {
          if ((e & 63) < wJ) x = X[(size_t)(r0 + 32 * i + (e >> 6)) * p + c0 + (e & 63)];
        } else {
          if ((e >> 5) < wJ) x = X[(size_t)(c0 + (e >> 5)) * p + r0 + 32 * i + (e & 31)];
        }
      }
      v[q] = x;
    }
  };
  xload(xv[0], 0);
  xload(xv[1], 1);
  wait.pivot();
  // row block i of L: element e = t + 256 q, q < 4 (i + 1): block q >> 2, row (e >> 5) & 31, column e & 31
  double lv[4 * NB];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = t + 256 * q;
    lv[q] = Lg[(size_t)((e >> 5) & 31) * W + (e & 31)];
  }
  d4 z[NB][2];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    if (i >= nb) break;
    if (i) __syncthreads();  // the previous stage's LDS reads are done
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = t + 256 * q;
      if (own || J < P0) sX[(e >> 6) * 65 + (e & 63)] = xv[i & 1][q];
      else sX[(e & 31) * 65 + (e >> 5)] = xv[i & 1][q];
    }
    if (i + 2 < nb) xload(xv[i & 1], i + 2);
#pragma unroll
    for (int q = 0; q < 4 * (i + 1); ++q) {
      const int e = t + 256 * q;
      sL[(e >> 10) * 32 * PB + ((e >> 5) & 31) * PB + (e & 31)] = lv[q];
    }
    if (i + 1 < nb)  // the next stage's row block, in flight under this stage's products
#pragma unroll
      for (int q = 0; q < 4 * (i + 2) && q < 4 * NB; ++q) {
        const int e = t + 256 * q;
        lv[q] = Lg[(size_t)(32 * (i + 1) + ((e >> 5) & 31)) * W + 32 * (e >> 10) + (e & 31)];
      }
    __syncthreads();
    d4 acc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[h][r] = sX[(16 * h + lk + 4 * r) * 65 + 16 * wv + li];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (j >= i) break;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(-sL[j * 32 * PB + (16 * h + li) * PB + 16 * hh + 4 * kk + lk],
                                                          z[j][hh][kk], acc[h], 0, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      z[i][h] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          z[i][h] = __builtin_amdgcn_mfma_f64_16x16x4f64(sL[i * 32 * PB + (16 * h + li) * PB + 16 * hh + 4 * kk + lk],
                                                         acc[hh][kk], z[i][h], 0, 0, 0);
    }
    if (col < p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) Z[(size_t)(32 * i + 16 * h + lk + 4 * r) * p + col] = z[i][h][r];
  }
}

template <int R>
__global__ __launch_bounds__(256) void big_panel_kernel(BigSpdBatch b, int k) {
  __shared__ double sm[PIVOT_LDS];
  panel_block<R>(b, blockIdx.y, k, blockIdx.x, sm);
}

// The next sweep's panel, fused into the update launch of sweep k: it waits for the tiles of the
// next panel row (counted by their workgroups), issues its X loads, then waits for L^{-1} of pivot
// k + 1 (the pivot workgroup), then fills zbuf(k + 1).
struct PanelWait {
  const unsigned int* fl;
  int* status;
  unsigned rows_target, pivot_target;
  __device__ void rows() const { acquire_wait(fl + 2, rows_target, status); }
  __device__ void pivot() const { acquire_wait(fl + 1, pivot_target, status); }
};
// Issue priority over the CU's other workgroup (a tile's product loop): the panel is a chain of
// dependent MFMAs and LDS round trips on the sweep's critical path.
template <int R>
__device__ __forceinline__ void fused_panel(const BigSpdBatch& b, int m, int k, int pj, unsigned int row_tiles, double* sm) {
  __builtin_amdgcn_s_setprio(2);
  panel_block<R>(b, m, k + 1, pj, sm, PanelWait{b.flag[m], b.status[m], (unsigned)(k + 1) * row_tiles, (unsigned)(k + 1)});
  __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void tile_of(int lin, int& I, int& J) {
  int i = (int)((sqrt(8.0 * lin + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= lin) ++i;
  while (i * (i + 1) / 2 > lin) --i;
  I = i;
  J = lin - i * (i + 1) / 2;
}

// The tile list of one update launch: the nh tiles of the next pivot block (hand-off tiles) sit
// at the first position of the runs of workgroups 0, 1, 2 (done first, by different workgroups),
// every other lower tile follows in row-major order.
struct TileList {
  int nt, nh;
  int hlin[3];  // hand-off tiles' row-major lower indices, ascending
  int hpos[3];  // their positions in the list
  __device__ void at(int pos, int& I, int& J) const {
    for (int h = 0; h < nh; ++h)
      if (pos == hpos[h]) {
        tile_of(hlin[h], I, J);
        return;
      }
    int lin = pos;
    for (int h = 0; h < nh; ++h)
      if (hpos[h] < pos) --lin;
    for (int h = 0; h < nh; ++h)
      if (lin >= hlin[h]) ++lin;
    tile_of(lin, I, J);
  }
  __device__ bool handoff(int pos) const {
    for (int h = 0; h < nh; ++h)
      if (pos == hpos[h]) return true;
    return false;
  }
};

// Z panel block in LDS: 64 rows (k) x 64 columns (i), XOR-swizzled instead of padded: element
// (k, i) at k*64 + (i ^ 16(k&1)) -- rows k and k+1 are 32 banks apart for the MFMA fragment
// reads, as with a stride-80 layout, in 32 KB instead of 40
__device__ __forceinline__ int zsw(int k, int i) { return k * 64 + (i ^ ((k & 1) << 4)); }

// 64 x 64 panel block Z[rb..rb+63][c0..c0+63] -> registers (16 per thread, coalesced rows)
__device__ __forceinline__ void zblock_fetch(double (&v)[16], const double* Z, int p, int rb, int c0, int wK,
                                             int t) {
  const int c = t & 63, r0 = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = rb + r0 + 4 * q;
    v[q] = (r < wK && c0 + c < p) ? Z[(size_t)r * p + c0 + c] : 0.0;
  }
}
__device__ __forceinline__ void zblock_store(const double (&v)[16], double* sZ, int t) {
  const int c = t & 63, r0 = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) sZ[zsw(r0 + 4 * q, c)] = v[q];
}

constexpr int UPD_LDS = 2 * 64 * 64;  // sZI, sZJ (doubles); the last sweep's mirror stage reuses them
constexpr int BIG_LDS = UPD_LDS > PIVOT_LDS ? UPD_LDS : PIVOT_LDS;

// One sweep's update of every lower tile (+ the next pivot block, + the final sign flip / mirror).
// Persistent: G tile workgroups per factor each take a contiguous run of the tile list; a tile
// is R units (one per 64 rows of the panel): Z_I and Z_J of the unit sit in LDS, the next unit's
// (and the next tile's X values) are fetched into registers while the current unit's MFMAs run.
// At R = 1 a run stays within a block row mostly and Z_I is staged once per row.
// blockIdx.x: 0 = tile workgroup 0, 1 = the pivot workgroup, 2.. = tile workgroups 1..  The pivot
// workgroup waits for the hand-off tiles only; their workgroups never wait (no deadlock whatever
// the residency).  LDS 67 KB and <= 256 VGPRs: two workgroups per CU.
template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void big_update_kernel(BigSpdBatch b, int k, int skip_pivot) {
  const int m = blockIdx.y;
  const int p = b.p[m], T = b.T[m];
  const int P0 = R * k;
  if (P0 >= T) return;
  const int nsw = (T + R - 1) / R;
  const bool has_next = k + 1 < nsw;
  const bool last = !has_next;
  TileList tl;
  tl.nt = T * (T + 1) / 2;
  const int G = min(tl.nt, b.G);
  const int chunk = (tl.nt + G - 1) / G;
  tl.nh = 0;
  if (has_next) {
    const int Q0 = R * (k + 1);
    tl.hlin[tl.nh++] = Q0 * (Q0 + 1) / 2 + Q0;
    if (R == 2 && Q0 + 1 < T) {
      tl.hlin[tl.nh++] = (Q0 + 1) * (Q0 + 2) / 2 + Q0;
      tl.hlin[tl.nh++] = (Q0 + 1) * (Q0 + 2) / 2 + Q0 + 1;
    }
    for (int h = 0; h < tl.nh; ++h) tl.hpos[h] = h * chunk;
  }
  const int x = blockIdx.x;
  __shared__ double sm[BIG_LDS];
  if (x > G) {  // the next sweep's panel (fused_panel); T - 1 panel-row tiles per sweep
    const int pj = x - G - 1;
    if (!has_next || skip_pivot || pj >= T * R) return;
    fused_panel<R>(b, m, k, pj, (unsigned)(T - 1), sm);
    return;
  }
  if (x == 1) {
    if (!has_next || skip_pivot) return;
    if (threadIdx.x == 0) {  // pivot workgroup for block k+1
      (void)spin_until_ge<2>(b.flag[m], (unsigned)tl.nh, b.status[m]);  // bounded (status bit 2)
      *b.flag[m] = 0u;  // re-arm (next user: the next sweep's update launch)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    pivot_block<R>(b, m, k + 1, sm);
    release_add(b.flag[m] + 1, 1u);  // L^{-1} of pivot k + 1 ready (fused_panel)
    return;
  }
  const int g = x == 0 ? 0 : x - 1;
  if (g >= G) return;
  const int pos0 = g * chunk, pos1 = min(tl.nt, pos0 + chunk);
  if (pos0 >= pos1) return;
  double* X = b.X[m];
  const double* Z = zbuf<R>(b, m, k);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int li = lane & 15, lk = lane >> 4;
  const int wK = min(BW * R, p - BW * P0);  // sweep width
  const int nhalf = (wK + BW - 1) / BW;     // units per tile (<= R)
  double* sZI = sm;
  double* sZJ = sm + 64 * 64;
  double* sT = sm;  // [64][SS] transpose stage of the last sweep's mirror (after a barrier)
  const double fin = last ? -1.0 : 1.0;
  auto inP = [&](int I_) { return I_ >= P0 && I_ < P0 + R; };

  // X tile (I, J) in this wave's MFMA layout; zero base for the swept row / column blocks.
  // Unconditional clamped loads times a 0/1 factor (a guarded load would become an exec-mask
  // branch); rows / columns past p are never stored.
  auto xo_fetch = [&](double (&xv)[2][2][4], int I_, int J_) {
    const double f = (inP(I_) || inP(J_)) ? 0.0 : 1.0;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = min(BW * I_ + 32 * wr + 16 * bi + lk + 4 * r, p - 1);
          const int gj = min(BW * J_ + 32 * wc + 16 * bj + li, p - 1);
          xv[bi][bj][r] = X[(size_t)gi * p + gj] * f;
        }
  };
  int I, J, h = 0, pos = pos0;
  tl.at(pos0, I, J);
  double xo[2][2][4], xn[2][2][4];
  xo_fetch(xn, I, J);
  {
    double v[16];
    zblock_fetch(v, Z, p, 0, BW * I, wK, t);
    zblock_store(v, sZI, t);
    zblock_fetch(v, Z, p, 0, BW * J, wK, t);
    zblock_store(v, sZJ, t);
  }
  __syncthreads();
  d4 acc[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      acc[bi][bj] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) xo[bi][bj][r] = xn[bi][bj][r];
    }
  for (;;) {
    // the next unit: its panel blocks (and, on a tile change, its X values) in flight under
    // this unit's MFMAs
    int hn = h + 1, posn = pos, In = I, Jn = J;
    if (hn >= nhalf) {
      hn = 0;
      posn = pos + 1;
    }
    const bool more = posn < pos1;
    const bool newtile = hn == 0;
    double vj[16], vi[16];
    bool ldI = false;
    if (more) {
      if (newtile) tl.at(posn, In, Jn);
      // Z_I stays staged along a block row (R = 1), except in the last sweep, whose mirror
      // stage overwrites it
      ldI = R > 1 || In != I || last;
      zblock_fetch(vj, Z, p, BW * hn, BW * Jn, wK, t);
      if (ldI) zblock_fetch(vi, Z, p, BW * hn, BW * In, wK, t);
      if (newtile) xo_fetch(xn, In, Jn);
    }
    const int kw = min(BW, wK - BW * h);
    for (int k0 = 0; k0 < kw; k0 += 32) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int kr = k0 + 4 * kk + lk;
        double a[2], bb[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          a[q] = sZI[zsw(kr, 32 * wr + 16 * q + li)];
          bb[q] = sZJ[zsw(kr, 32 * wc + 16 * q + li)];
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
            acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[bi], bb[bj], acc[bi][bj], 0, 0, 0);
      }
    }
    if (h == nhalf - 1) {  // the tile is complete: epilogue
      const int I0 = BW * I, J0 = BW * J;
      const bool inPi = inP(I), inPj = inP(J);
      const double sgn = ((inPi != inPj) ? -1.0 : 1.0) * fin;
      // the next pivot block's tiles go to the pivot workgroup: stored write-through (sc1), so
      // the hand-off needs no L2 write-back (release fence) -- drain, barrier, one counter add
      // (MI355X_MICROARCH §inter-workgroup visibility, "publish-large")
      const bool handoff = has_next && tl.handoff(pos);
      double mx = 0.0;
      double vals[2][2][4];
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 32 * wr + 16 * bi + lk + 4 * r, col = 32 * wc + 16 * bj + li;
            const int gi = I0 + row, gj = J0 + col;
            const double v = sgn * (xo[bi][bj][r] - acc[bi][bj][r]);
            vals[bi][bj][r] = v;
            if (gi < p && gj < p) {
              if (handoff)
                __hip_atomic_store(&X[(size_t)gi * p + gj], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              else
                X[(size_t)gi * p + gj] = v;
              if (last && I == J && gi == gj && gi < b.n[m]) mx = fmax(mx, v);
            }
          }
      if (handoff) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) atomicAdd(b.flag[m], 1u);
      } else if (has_next && (I == R * (k + 1) || J == R * (k + 1))) {  // (R = 1) next panel row
        release_add(b.flag[m] + 2, 1u);
      }
      if (last && I == J) {  // refinement gate: max_i (K^{-1})_ii
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
        if (lane == 0 && mx > 0.0)
          atomicMax(reinterpret_cast<unsigned long long*>(b.pst[m] + 1),
                    (unsigned long long)__double_as_longlong(mx));
      }
      if (last && I != J) {
        __syncthreads();  // every wave is done reading sZI / sZJ: sT reuses them
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              sT[(32 * wr + 16 * bi + lk + 4 * r) * SS + 32 * wc + 16 * bj + li] = vals[bi][bj][r];
        __syncthreads();
        // mirror: X[J0 + r][I0 + c] = tile[c][r], coalesced along c
        const int wI = bw(p, I), wJ = bw(p, J);
#pragma unroll 4
        for (int e = t; e < BW * BW; e += 256) {
          const int r = e >> 6, c = e & 63;
          if (r < wJ && c < wI) X[(size_t)(J0 + r) * p + I0 + c] = sT[c * SS + r];
        }
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4{0.0, 0.0, 0.0, 0.0};
    }
    __syncthreads();  // every wave is done reading sZI / sZJ (and sT)
    if (!more) break;
    zblock_store(vj, sZJ, t);
    if (ldI) zblock_store(vi, sZI, t);
    if (newtile) {
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
          for (int r = 0; r < 4; ++r) xo[bi][bj][r] = xn[bi][bj][r];
    }
    I = In;
    J = Jn;
    h = hn;
    pos = posn;
    __syncthreads();
  }
}

// ---- 128-wide sweeps: the update on 128x128 tiles (the large GEMM's tile loop) ------------
// One workgroup per LOWER 128x128 tile (ti >= tj) computes Z_I^T Z_J with gemm_tile_dev.h's
// pipelined product loop (K = the sweep width, 16-deep K-steps in two LDS stages, 4x4 MFMA
// blocks per wave, stores / loads / reads interleaved with the MFMAs)
// and applies the sweep's epilogue (sign, zero base in the swept row / column).  Diagonal tiles
// keep both triangles of their 128 block, so every lower 64-tile the panel reads is current.
// Workgroup 0 of a factor owns the next pivot block's tile (k+1, k+1): it updates it like the
// others, then factors it in place (pivot_blk: blocked Cholesky) while the other tiles are
// updated -- no hand-off, no workgroup waits on another.  The last sweep flips the sign and
// publishes max diag K^{-1}; big_mirror_kernel then fills the upper triangle.
constexpr int WT = 128;
// the product loops' staging buffers (whole tiles: gemm_tile_dev.h; quarter tiles: [k][64] rows at
// gemm_huge_dev.h's stride)
constexpr int WIDE_LDS = tile::LDS_DOUBLES > 2 * 2 * huge::KS * huge::S ? tile::LDS_DOUBLES : 2 * 2 * huge::KS * huge::S;
static_assert(WIDE_LDS >= PIVOT_LDS, "the pivot reuses the staging LDS");

// position pos of sweep k's tile list of a factor with T2 128-tiles per dimension, with a next
// pivot Q = k + 1: the T2 - 1 tiles the next panel reads first -- row Q left of the diagonal,
// then column Q below it (round 0 of the factor's first XCD slot run: the panel's wait for its
// row ends after one tile time instead of the last round) -- then every other lower tile in
// row-major order; (Q, Q) is the pivot workgroup's, not listed.
__device__ __forceinline__ void wide_tile_at(int pos, int T2, int Q, bool has_next, int& I, int& J) {
  if (!has_next) {
    tile_of(pos, I, J);
    return;
  }
  if (pos < Q) {
    I = Q;
    J = pos;
    return;
  }
  if (pos < T2 - 1) {
    I = pos + 1;
    J = Q;
    return;
  }
  const int r = pos - (T2 - 1);
  int i, j;
  tile_of(r, i, j);
  if (r < Q * (Q + 1) / 2) {  // rows above Q: row-major as they are
    I = i;
    J = j;
    return;
  }
  I = i + 1;  // rows below Q hold I tiles each once column Q is taken out
  J = j < Q ? j : j + 1;
}

__global__ __launch_bounds__(256, 2) void wide_update_kernel(BigSpdBatch b, int k, int skip_pivot, int gx,
                                                          int per_xcd, int nx, int first) {
  using namespace huge;
  // 1-D grid over both factors.  8 nx PERSISTENT tile workgroups, two per CU, in two dispatch
  // passes over the CUs: blocks [0, first) and [first + 8, first + 8 + (8 nx - first)); between
  // them, blocks [first, first + 8) hold the factors' pivot workgroups (the sweep's serial part),
  // in the first pass on CUs the second pass leaves alone (first = CUs - 8).  Tile workgroup t
  // (its ordinal, = its block mod 8) works on XCD slot t & 7's run of per_xcd tiles (blocks t,
  // t+8, ... share an XCD and take consecutive tiles, i.e. runs along block rows whose Z_I / Z_J
  // panels stay in that XCD's L2), tile s + j nx of the run in round j.  A tile workgroup issues
  // the next tile's first K-step loads before its current tile's stores (vector-memory
  // operations complete in issue order): the stores drain under the next tile's product loop.
  // gx = tiles per factor slot.
  __shared__ double sm[WIDE_LDS];
  const int L = blockIdx.x;
  const bool probe = k == BIG_PROBE_SWEEP && threadIdx.x == 0;  // (trace build only)
  if (probe && L == 0) TR_LO(SLOT_BIG_START);
  if (L >= 8 * nx + 8) {  // the next sweep's panel (fused_panel), factors interleaved
    const int m = (L - 8 * nx - 8) % b.nmat;
    const int T2 = (b.p[m] + WT - 1) / WT;
    if (k + 1 >= T2 || skip_pivot) return;
    // Column blocks are claimed from a per-sweep ticket counter (zeroed with the pivot of block 0)
    // instead of one per workgroup: the first panel workgroups find free slots at once (on the
    // pivot workgroups' CUs, which the tile workgroups' second pass leaves with one free slot)
    // and, once the pivot is in, keep taking blocks until the rest get CU slots as tile
    // workgroups exit -- no block waits for a late workgroup.
    __shared__ int s_tk;
    unsigned int* ctr = b.flag[m] + 4 + k;
    for (;;) {
      if (threadIdx.x == 0) s_tk = (int)atomicAdd(ctr, 1u);
      __syncthreads();
      const int pj = s_tk;  // (read by every thread before fused_panel's first barrier)
      if (pj >= b.T[m]) return;
      // T2 - 1 panel-row tiles per sweep, counted in quarter tiles (a whole tile adds 4)
      if (probe && m == 0) TR_LO(SLOT_BIG_PANEL_WAIT);
      fused_panel<2>(b, m, k, pj, 4u * (unsigned)(T2 - 1), sm);
      if (probe && m == 0) TR_HI(SLOT_BIG_PANEL);
    }
  }
  const bool pivot = L >= first && L < first + 8;
  if (pivot && L - first >= b.nmat) return;
  if (probe && pivot && L == first) TR_LO(SLOT_BIG_PIVTILE);
  const int tt = L < first ? L : L - 8;  // tile workgroup ordinal
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  // Rounds: every XCD slot's run of per_xcd tiles is worked in rounds of nx tiles, so a last
  // round of rem < nx tiles would leave most workgroups idle for a whole tile time (C5: 1056
  // tiles on 496 workgroups = 2 rounds + 64 tiles).  When 4 rem <= nx, that last round is split
  // into quarter tiles (64 x 64 outputs of the same 128-deep product; qq = quarter) worked by
  // 4 rem workgroups at once: a quarter of a tile time.  Same MFMA sequence per output block:
  // bitwise the whole-tile result.
  const int full_rounds = per_xcd / nx, rem_tiles = per_xcd - full_rounds * nx;
  const bool quarters = !b.no_quarters && full_rounds >= 1 && rem_tiles > 0 && 4 * rem_tiles <= nx;
  // item j of this workgroup -> (factor m, tile ti, tj, quarter qq: -1 = whole tile); false past
  // its run
  bool skip_q = false;  // (the quarter item was worked first: quarter_first below)
  auto tile_at = [&](int j, int& m, int& ti, int& tj, int& qq, unsigned& ent) -> bool {
    qq = -1;
    ent = 0u;
    if (pivot) {
      if (j > 0) return false;
      m = L - first;
      const int T2 = (b.p[m] + WT - 1) / WT;
      if (k + 1 >= T2 || skip_pivot) return false;
      ti = tj = k + 1;
      if (b.sched[m]) ent = b.sched[m][(size_t)k * b.sstride[m] + 1];
      return true;
    }
    int loc;
    if (quarters && j >= full_rounds) {
      const int w = tt >> 3;
      if (skip_q || j > full_rounds || w >= 4 * rem_tiles) return false;
      loc = full_rounds * nx + (w >> 2);
      qq = w & 3;
    } else {
      loc = (tt >> 3) + j * nx;
      if (loc >= per_xcd) return false;
    }
    const int wi = (tt & 7) * per_xcd + loc;
    if (wi >= b.nmat * gx) return false;
    m = wi / gx;
    const int T2 = (b.p[m] + WT - 1) / WT;
    if (k >= T2) return false;
    const bool has_next = k + 1 < T2;
    const int nt = T2 * (T2 + 1) / 2;
    const int Q = k + 1, qlin = Q * (Q + 1) / 2 + Q;
    int lin = wi % gx;
    if (b.sched[m]) {  // the two-sweep schedule's list of this sweep
      const unsigned* row = b.sched[m] + (size_t)k * b.sstride[m];
      if (lin >= (int)row[0]) return false;
      ent = row[2 + lin];
      ti = (int)((ent >> 8) & 0xffu);
      tj = (int)(ent & 0xffu);
      return true;
    }
    if (lin >= nt - (has_next ? 1 : 0)) return false;
    if (has_next && !skip_pivot) {  // the next panel row's tiles first (wide_tile_at)
      wide_tile_at(lin, T2, Q, true, ti, tj);
      return true;
    }
    if (has_next && lin >= qlin) ++lin;  // (k+1, k+1) belongs to the pivot workgroup
    tile_of(lin, ti, tj);
    return true;
  };
  constexpr int SZ = KS * S;
  double* sA0 = sm;
  double* sB0 = sm + 2 * SZ;
  int m, ti, tj, qq;
  unsigned ent;
  // the quarter item (qq = 2 qi + qj): rows WT ti + 64 qi, columns WT tj + 64 qj; this wave's
  // 32 x 32 block (wr, wc) as 2 x 2 MFMA blocks, 16-deep K-steps through the same double-buffered
  // staging ([k][64] rows of Z at stride S)
  auto quarter_item = [&]() {
    __syncthreads();  // (the whole-tile loop's last reads of the staging buffers)
    if (probe) TR_LO(SLOT_BIG_QUARTER);
    const int p = b.p[m];
    const int T2 = (p + WT - 1) / WT;
    const bool has_next = k + 1 < T2;
    const bool LAST = !has_next;
    const int Q = k + 1;
    double* X = b.X[m];
    const double* Z = zbuf<2>(b, m, k);
    const int i0 = WT * ti + 64 * (qq >> 1), j0 = WT * tj + 64 * (qq & 1);
    const int wK = min(WT, p - WT * k);
    const bool inPi = ti == k, inPj = tj == k;
    const double sgn = ((inPi != inPj) ? -1.0 : 1.0) * (LAST ? -1.0 : 1.0);
    const int li = lane & 15, lk = lane >> 4;
    // schedule (as the whole tiles): v = c0 X + c1 Z_{k-1}^T Z_{k-1} + c2 Z_k^T Z_k
    const bool sch = b.sched[m] != nullptr;
    const bool two = sch && ((ent >> 16) & 1u);
    auto cf = [](unsigned c) { return c == 0u ? 0.0 : c == 1u ? 1.0 : -1.0; };
    const double c0 = cf((ent >> 18) & 3u), c1 = cf((ent >> 20) & 3u), c2 = cf((ent >> 22) & 3u);
    const double* Zp = two ? zbuf<2>(b, m, k - 1) : Z;
    d4 acc[2][2];
    {
      const double f = sch ? -c0 : ((inPi || inPj) ? 0.0 : 1.0);
#pragma unroll
      for (int bx = 0; bx < 2; ++bx)
#pragma unroll
        for (int by = 0; by < 2; ++by)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = min(i0 + 32 * wr + 16 * bx + lk + 4 * r, p - 1);
            const int col = min(j0 + 32 * wc + 16 * by + li, p - 1);
            acc[bx][by][r] = X[(size_t)row * p + col] * f;
          }
    }
    // K-step kt: Z[16 kt + kr][i0 + c] (A, negated) and Z[16 kt + kr][j0 + c] (B), kr < 16,
    // c < 64: two 16-B loads per operand and thread, 512 B per k row (coalesced); the next
    // K-step's loads in flight under the current one's MFMAs.  (All K-steps' loads up front --
    // one round trip per item -- measured slower: 121 vs 113 us per update launch.)
    // (two sweeps: K-steps [0, WT / KS) read panel k - 1 scaled by c1, the rest panel k by c2;
    // the A operand is staged negated: acc = -(c0 X + ...), stored negated back by sgn below)
    const int nk1 = two ? WT / KS : 0;
    auto qfetch = [&](double2 (&ra)[2], double2 (&rb)[2], int kt) {
      const double* Zs = kt < nk1 ? Zp : Z;
      const int k0 = (kt < nk1 ? kt : kt - nk1) * KS;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = t + 256 * q, kr = e >> 5, c = 2 * (e & 31);
        ra[q] = ld2(Zs + (size_t)(k0 + kr) * p + min(i0 + c, p - 2));
        rb[q] = ld2(Zs + (size_t)(k0 + kr) * p + min(j0 + c, p - 2));
      }
    };
    auto qstore = [&](const double2 (&ra)[2], const double2 (&rb)[2], double* sA, double* sB, int kt) {
      const double sa = sch ? (kt < nk1 ? -c1 : -c2) : -1.0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = t + 256 * q, kr = e >> 5, c = 2 * (e & 31);
        *reinterpret_cast<double2*>(sA + kr * S + c) = make_double2(sa * ra[q].x, sa * ra[q].y);
        *reinterpret_cast<double2*>(sB + kr * S + c) = rb[q];
      }
    };
    const int nk = nk1 + wK / KS;
    double2 ra[2], rb[2];
    qfetch(ra, rb, 0);
    qstore(ra, rb, sA0, sB0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) qfetch(ra, rb, kt + 1);
      const double* sA = sA0 + cur * SZ;
      const double* sB = sB0 + cur * SZ;
#pragma unroll
      for (int kk = 0; kk < KS / 4; ++kk) {
        // (tile::product's k order: MFMA kk of a 16-deep step takes k = 8 (kk >> 1) + 2 lk + (kk & 1)
        // in k-slot lk, so every output block sees the whole-tile MFMA sequence: bitwise equal)
        const int kr = 8 * (kk >> 1) + 2 * lk + (kk & 1);
        double a[2], bb[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          a[x] = sA[kr * S + 32 * wr + 16 * x + li];
          bb[x] = sB[kr * S + 32 * wc + 16 * x + li];
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], bb[y], acc[x][y], 0, 0, 0);
      }
      if (kt + 1 < nk) qstore(ra, rb, sA0 + (cur ^ 1) * SZ, sB0 + (cur ^ 1) * SZ, kt + 1);
      __syncthreads();
    }
    double mx = 0.0;
#pragma unroll
    for (int bx = 0; bx < 2; ++bx)
#pragma unroll
      for (int by = 0; by < 2; ++by)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i0 + 32 * wr + 16 * bx + lk + 4 * r;
          const int col = j0 + 32 * wc + 16 * by + li;
          if (row < p && col < p) {
            const double v = sch ? -acc[bx][by][r] : sgn * acc[bx][by][r];
            X[(size_t)row * p + col] = v;
            if (LAST && row == col && row < b.n[m]) mx = fmax(mx, v);
          }
        }
    if (LAST && ti == tj) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
      if (lane == 0 && mx > 0.0)
        atomicMax(reinterpret_cast<unsigned long long*>(b.pst[m] + 1),
                  (unsigned long long)__double_as_longlong(mx));
    }
    if (has_next && (ti == Q || tj == Q)) release_add(b.flag[m] + 2, 1u);  // a quarter of a row tile
    if (probe) TR_HI(SLOT_BIG_QUARTER);
  };
  // Quarter items first (round 6): on most CUs one of the two tile workgroups has a quarter item
  // besides its whole tiles and the other has none; working the quarter FIRST puts the two
  // workgroups' memory phases (base loads, stores) out of step, so one runs its product loop while
  // the other waits on memory, instead of both bursting together.  Not for a workgroup whose first
  // whole tile is in the next panel's row / column (eager: the fused panel waits for those).
  // Every item is computed the same way in either order (bitwise).
  if (quarters && !pivot && !b.no_quarters && (tt >> 3) < 4 * rem_tiles && b.qfirst) {
    bool eager = true;
    if (tile_at(0, m, ti, tj, qq, ent)) {
      const int T2 = (b.p[m] + WT - 1) / WT;
      eager = k + 1 < T2 && (ti == k + 1 || tj == k + 1);
    }
    if (!eager && tile_at(full_rounds, m, ti, tj, qq, ent) && qq >= 0) {
      quarter_item();
      skip_q = true;
      __syncthreads();  // (its staging reads before the whole tiles' first stores)
    }
  }
  if (!tile_at(0, m, ti, tj, qq, ent)) return;
  int j = 0;
  for (; qq < 0; ++j) {
    if (probe && !pivot && j < 2) {  // (trace build) round-0/1 phases over every tile workgroup
      TR_LO(SLOT_BIG_R0START + 3 * j);
      TR_HI(SLOT_BIG_R0START + 3 * j);
    }
    const int p = b.p[m];
    const int T2 = (p + WT - 1) / WT;  // 128-tiles per dimension
    const bool has_next = k + 1 < T2;
    const bool LAST = !has_next;  // (per factor: the factors of a batch may differ in size)
    const int Q = k + 1;
    double* X = b.X[m];
    const double* Z = zbuf<2>(b, m, k);
    const int i0 = WT * ti, j0 = WT * tj;
    const int wK = min(WT, p - WT * k);  // sweep width (a multiple of 32)
    const bool inPi = ti == k, inPj = tj == k;
    const double sgn = ((inPi != inPj) ? -1.0 : 1.0) * (LAST ? -1.0 : 1.0);
    // the workgroup's next item
    int m2 = 0, ti2 = 0, tj2 = 0, q2 = -1;
    unsigned ent2 = 0u;
    const bool next = tile_at(j + 1, m2, ti2, tj2, q2, ent2);
    // The accumulators start at the tile's current values NEGATED (zero base in the swept blocks;
    // clamped addresses: rows / columns past p are never stored) and the product is added; the
    // store negates back: base - Z_I^T Z_J with the rounding of a subtraction (round-to-nearest
    // commutes with negation), and no separate base registers.  The base loads are issued ahead
    // of the product loop's first K-step.
    // Two-sweep schedule (b.sched): new = c0 X + c1 Z_{k-1}^T Z_{k-1} + c2 Z_k^T Z_k, the
    // coefficients (0, +-1) composing the sweeps' rules (wide_schedule); the products scale the
    // A operand by c1 / c2 (exact).  One sweep (c1 = 0): the same operations as the form below,
    // negated throughout -- bitwise the same values.  Without a schedule: the accumulators start
    // at the tile NEGATED (zero base in the swept blocks) and the store negates back.
    const bool sch = b.sched[m] != nullptr;
    const bool two = sch && ((ent >> 16) & 1u);
    auto cf = [](unsigned c) { return c == 0u ? 0.0 : c == 1u ? 1.0 : -1.0; };
    const double c0 = cf((ent >> 18) & 3u), c1 = cf((ent >> 20) & 3u), c2 = cf((ent >> 22) & 3u);
    d4 acc[4][4];
    {
      const double f = sch ? c0 : ((inPi || inPj) ? -0.0 : -1.0);
#pragma unroll
      for (int bx = 0; bx < 4; ++bx)
#pragma unroll
        for (int by = 0; by < 4; ++by)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = min(i0 + 64 * wr + 16 * bx + (lane >> 4) + 4 * r, p - 1);
            const int col = min(j0 + 64 * wc + 16 * by + (lane & 15), p - 1);
            acc[bx][by][r] = X[(size_t)row * p + col] * f;
          }
    }
    // acc += Z_I^T Z_J: op(A) = Z^T (Z[k][i], i contiguous), op(B) = Z (Z[k][j]) -- both
    // mn-contiguous, staged [k][mn] without a transpose (tile::product<1, 0>)
    // (one call for every case -- a second inlined product loop spilled the accumulators: two
    // sweeps read panel k - 1, always 128 deep since it is not the last sweep, then panel k)
    {
      const double* Zp = two ? zbuf<2>(b, m, k - 1) : Z;
      tile::product2<1, 0>(Zp, Zp, two ? WT : 0, c1, Z, Z, wK, sch ? c2 : 1.0, p, p, p, p, i0, j0, sm, t,
                           wr, wc, lane, acc);
    }
    if (probe && !pivot && j < 2) TR_HI(SLOT_BIG_R0START + 3 * j + 2);
    double mx = 0.0;
#pragma unroll
    for (int bx = 0; bx < 4; ++bx) {
#pragma unroll
      for (int by = 0; by < 4; ++by)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i0 + 64 * wr + 16 * bx + (lane >> 4) + 4 * r;
          const int col = j0 + 64 * wc + 16 * by + (lane & 15);
          if (row < p && col < p) {
            const double v = sch ? acc[bx][by][r] : -sgn * acc[bx][by][r];
            X[(size_t)row * p + col] = v;
            if (LAST && row == col && row < b.n[m]) mx = fmax(mx, v);
          }
        }
      asm volatile("" ::: "memory");
    }
    if (LAST && ti == tj) {  // refinement gate: max_i (K^{-1})_ii
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
      if (lane == 0 && mx > 0.0)
        atomicMax(reinterpret_cast<unsigned long long*>(b.pst[m] + 1),
                  (unsigned long long)__double_as_longlong(mx));
    }
    if (pivot) {
      // the next pivot block, factored in place from this workgroup's own stores (one L1 per
      // workgroup: visible after the barrier)
      if (probe && m == 0) TR_HI(SLOT_BIG_PIVTILE);
      __syncthreads();
      const int r0 = WT * Q, w = min(WT, p - r0);
      pivot_blk<2>(X + (size_t)r0 * p + r0, p, w, b.Li[m], b.ldet[m] + 4 * Q, b.status[m], sm);
      release_add(b.flag[m] + 1, 1u);  // L^{-1} of pivot k + 1 ready (fused_panel)
      if (probe && m == 0) TR_HI(SLOT_BIG_PIVOT);
      return;
    }
    if (probe && j < 2) TR_HI(SLOT_BIG_ROUND0 + j);
    if (has_next && (ti == Q || tj == Q)) release_add(b.flag[m] + 2, 4u);  // next panel row
    if (!next) return;
    m = m2;
    ti = ti2;
    tj = tj2;
    qq = q2;
    ent = ent2;
  }
  quarter_item();
}

// After the last 128-wide sweep: upper 64x64 tiles outside the diagonal 128 blocks <- the
// transposed lower ones (LDS transpose, coalesced loads and stores).
__global__ __launch_bounds__(256) void big_mirror_kernel(BigSpdBatch b) {
  const int m = blockIdx.y;
  const int p = b.p[m], T = b.T[m];
  int I, J;
  tile_of(blockIdx.x, I, J);
  if (I >= T || I == J || (I >> 1) == (J >> 1)) return;
  __shared__ double sT[BW * SS];
  double* X = b.X[m];
  const int wI = bw(p, I), wJ = bw(p, J);
  load_tile(sT, X + (size_t)(BW * I) * p + BW * J, p, wI, wJ, threadIdx.x);
  __syncthreads();
  for (int e = threadIdx.x; e < BW * BW; e += 256) {
    const int r = e >> 6, c = e & 63;  // X[J*64 + r][I*64 + c] = tile[c][r]
    if (r < wJ && c < wI) X[(size_t)(BW * J + r) * p + BW * I + c] = sT[c * SS + r];
  }
}

int batch_R(const SpdArgs* a) { return a[0].wide ? 2 : 1; }

}  // namespace

// ---- the two-sweep schedule of the 128-wide update (round 5) -------------------------------
// A sweep's update reads and writes every lower tile once for K = 128 of MFMA work; a tile that
// takes two sweeps in one pass (K = 256) halves that traffic per flop.  Tiles are split into two
// classes by the parity of I + J: class c applies sweeps in pairs (k - 1, k) in the launches with
// k = c (mod 2), so every launch has half the bulk at K = 256 under which the serial part (next
// pivot, next panel) still runs.  A tile the next panel or pivot reads (row / column k + 1) is
// brought fully up to date in launch k whatever its class, and the last launch flushes every tile.
// Every tile is touched at least every other launch, so it never lags by more than one sweep:
// its pending sweeps are {k} or {k - 1, k}.  Per sweep s a tile changes as
//   X <- lam (beta X + gam Z_s^T Z_s):  beta = 0 when I or J = s (its old value is the panel's
//   input), gam = +1 when exactly one of I, J = s, else -1; lam = -1 on the last sweep;
// two sweeps compose to c0 X + c1 Z_{k-1}^T Z_{k-1} + c2 Z_k^T Z_k.  The panels k - 1 and k are
// both live (zbuf: three buffers).
int wide_sched_stride(int T2) { return 2 + T2 * (T2 + 1) / 2; }

void wide_schedule(int T2, bool paired, std::vector<unsigned>& tab) {
  const int S = wide_sched_stride(T2);
  tab.assign((size_t)T2 * S, 0u);
  auto eager = [&](int I, int J, int k) {  // row / column k + 1, the pivot tile included
    const int Q = k + 1;
    return Q < T2 && ((I == Q && J <= Q) || (J == Q && I > Q));
  };
  // Diagonal tile (k + 2, k + 2) is the pivot workgroup's own tile in launch k + 1, the head of
  // that launch's serial chain (tile -> 128-pivot -> panel).  Bringing it up to date in launch k
  // (one more K = 128 tile in the bulk of odd launches) leaves it one sweep, K = 128, in launch
  // k + 1 instead of the pair (K = 256: 50 vs 32 us in the C5 timeline, tools/big_timeline.py).
  auto pre_pivot = [&](int I, int J, int k) { return I == J && I == k + 2 && I < T2; };
  auto updated = [&](int I, int J, int k) {
    if (k < 0) return true;
    return !paired || k == T2 - 1 || eager(I, J, k) || pre_pivot(I, J, k) || ((I + J) & 1) == (k & 1);
  };
  auto code = [](int c) { return c == 0 ? 0u : c > 0 ? 1u : 3u; };
  for (int k = 0; k < T2; ++k) {
    unsigned* row = tab.data() + (size_t)k * S;
    const int Q = k + 1;
    auto entry = [&](int I, int J) -> unsigned {
      const bool two = !updated(I, J, k - 1);  // last touched in launch k - 2: sweeps k - 1, k
      auto rule = [&](int s, int& beta, int& gam, int& lam) {
        const bool pi = I == s, pj = J == s;
        beta = (pi || pj) ? 0 : 1;
        gam = (pi != pj) ? 1 : -1;
        lam = s == T2 - 1 ? -1 : 1;
      };
      int b2, g2, l2;
      rule(k, b2, g2, l2);
      int c0 = l2 * b2, c1 = 0;
      const int c2 = l2 * g2;
      bool t2 = false;
      if (two) {
        int b1, g1, l1;
        rule(k - 1, b1, g1, l1);
        c0 = l2 * b2 * l1 * b1;
        c1 = l2 * b2 * l1 * g1;
        t2 = c1 != 0;  // (beta2 = 0: sweep k overwrites what sweep k - 1 left; it needs only Z_k)
      }
      return (unsigned)J | ((unsigned)I << 8) | ((t2 ? 1u : 0u) << 16) | (code(c0) << 18) |
             (code(t2 ? c1 : 0) << 20) | (code(c2) << 22);
    };
    int n = 0;
    if (Q < T2) {  // the next panel's tiles first: row Q left of the diagonal, column Q below it
      for (int J = 0; J < Q; ++J) row[2 + n++] = entry(Q, J);
      for (int I = Q + 1; I < T2; ++I) row[2 + n++] = entry(I, Q);
      row[1] = entry(Q, Q);
    }
    for (int I = 0; I < T2; ++I)
      for (int J = 0; J <= I; ++J) {
        if (Q < T2 && (I == Q || J == Q)) continue;  // listed above / the pivot workgroup's
        if (updated(I, J, k)) row[2 + n++] = entry(I, J);
      }
    row[0] = (unsigned)n;
  }
}

namespace {

// the host copy of wide_schedule(T2, paired) -- the table gpk_create uploads per factor -- cached
// per T2 (per host thread: handles of an in-process group launch from several threads)
const std::vector<unsigned>& host_wide_schedule(int T2) {
  static thread_local std::vector<std::vector<unsigned>> cache;
  if ((int)cache.size() <= T2) cache.resize(T2 + 1);
  if (cache[T2].empty()) wide_schedule(T2, true, cache[T2]);
  return cache[T2];
}

BigSpdBatch make_batch(SpdArgs* a, int nmat, int& Tmax, int& tiles_max) {
  BigSpdBatch b{};
  Tmax = 0;
  tiles_max = 0;
  // 64-wide update: 255 tile workgroups per factor (+ its pivot workgroup; two fit per CU).
  // Measured at 2048: 1177 us per inverse vs 1243 us with 383 or 511
  b.G = g_big_wgs.load() > 0 ? g_big_wgs.load() : 255;
  b.nmat = nmat;
  b.no_quarters = a[0].no_quarters;
  b.qfirst = a[0].qfirst;
  for (int m = 0; m < nmat; ++m) {
    // every factor keeps its own schedule (built for its own T2 = ceil(p / 128)); the update
    // launch's per-factor item count covers the longest list (launch_stage_r)
    b.sched[m] = a[m].wide ? a[m].sched : nullptr;
    b.sstride[m] = wide_sched_stride((a[m].p + 127) / 128);
    b.X[m] = a[m].X; b.Z[m] = a[m].Z ? a[m].Z : a[m].Y; b.Li[m] = a[m].piv;
    b.ldet[m] = a[m].ldet; b.pst[m] = a[m].pst; b.status[m] = a[m].status; b.flag[m] = a[m].flag;
    b.p[m] = a[m].p; b.n[m] = a[m].n; b.T[m] = (a[m].p + BW - 1) / BW;
    Tmax = std::max(Tmax, b.T[m]);
    tiles_max = std::max(tiles_max, std::min(b.T[m] * (b.T[m] + 1) / 2, b.G) + 1);
  }
  return b;
}

// CUs of the current device (the persistent update's workgroup count; 256 on a full MI355X)
int wide_cus() {
  static int cached = 0;
  if (cached > 0) return cached;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  cached = cus;
  return cached;
}

template <int R>
void launch_stage_r(const BigSpdBatch& b, int nmat, int Tmax, int tiles, int stage, hipStream_t s,
                    int skip_pivot = 0, bool mirror = true) {
  if (stage < 0) {
    hipLaunchKernelGGL(big_pivot_init_kernel<R>, dim3(nmat), dim3(256), 0, s, b);
  } else if ((stage & 1) == 0) {
    hipLaunchKernelGGL(big_panel_kernel<R>, dim3(Tmax, nmat), dim3(256), 0, s, b, stage >> 1);
  } else if (R == 1) {  // + the next sweep's panel workgroups (Tmax per factor)
    hipLaunchKernelGGL(big_update_kernel<1>, dim3(tiles + Tmax, nmat), dim3(256), 0, s, b, stage >> 1,
                       skip_pivot);
  } else {
    const int k = stage >> 1, nsw = (Tmax + 1) / 2;
    // gx = item slots per factor: the longest list of sweep k over the batch's factors (a factor
    // with a schedule: its row's length; without one: every lower tile but the pivot's)
    int gx = 1;
    for (int m = 0; m < nmat; ++m) {
      const int T2 = (b.p[m] + WT - 1) / WT;
      if (k >= T2) continue;
      int items;
      if (b.sched[m]) {
        const std::vector<unsigned>& tab = host_wide_schedule(T2);
        items = (int)tab[(size_t)k * wide_sched_stride(T2)];
      } else {
        items = T2 * (T2 + 1) / 2 - (k + 1 < T2 ? 1 : 0);
      }
      gx = std::max(gx, items);
    }
    const int per_xcd = (nmat * gx + 7) / 8;
    // persistent tile workgroups: two per CU on all but the 8 CUs whose first-pass workgroup is a
    // pivot slot (8 nx in all, nx per XCD slot), never more than the tiles
    const int first = std::max(8, wide_cus() - 8);
    const int nx = std::max(1, std::min(per_xcd, 2 * first / 8));
    const int tile_wgs = 8 * nx;
    const int fst = std::min(first, tile_wgs);  // (fewer tile workgroups than CUs: pivots right after)
    hipLaunchKernelGGL(wide_update_kernel, dim3(tile_wgs + 8 + nmat * Tmax), dim3(256), 0, s, b, k,
                       skip_pivot, gx, per_xcd, nx, fst);
    // after the last sweep of every factor (a smaller factor's last sweep came earlier; later
    // launches leave it alone)
    if (k + 1 == nsw && mirror)
      hipLaunchKernelGGL(big_mirror_kernel, dim3(Tmax * (Tmax + 1) / 2, nmat), dim3(256), 0, s, b);
  }
}

}  // namespace

int spd_big_sweeps(int p, int wide) { return (p + BW * (wide ? 2 : 1) - 1) / (BW * (wide ? 2 : 1)); }

// the pivot's L + M_i (W x W) and its trailing-block scratch (W x W), W <= 128
size_t spd_big_piv_doubles(int p) { return std::max<size_t>((size_t)p * 32, 2 * 128 * 128); }

// stage -1: pivot 0; stage 2k: panel k (standalone; the inverse launches it for k = 0 only);
// stage 2k+1: update k + the fused panel of sweep k + 1 (profiling / bench)
hipError_t launch_spd_big_stage(SpdArgs* a, int nmat, int stage, hipStream_t s, bool mirror) {
  int Tmax, tiles;
  BigSpdBatch b = make_batch(a, nmat, Tmax, tiles);
  if (batch_R(a) == 2) launch_stage_r<2>(b, nmat, Tmax, tiles, stage, s, 0, mirror);
  else launch_stage_r<1>(b, nmat, Tmax, tiles, stage, s, 0, mirror);
  return hipGetLastError();
}

// The MFMA work update launch k (stage 2k + 1) schedules, per the tile lists it walks (bench
// accounting, gpk_bench_kernel): every listed tile's products, 2 w_I w_J (w_k [+ w_{k-1} for a
// tile that takes sweeps k - 1 and k]) -- a diagonal tile whole (the kernel keeps both triangles
// of its block) -- plus, with the pivot workgroup, the next pivot's tile, its blocked Cholesky
// (W^3 / 3) and the fused next panel (forward substitution, W^2 p).  One-sweep forms: every lower
// tile of the sweep.  Summed over the launches of one inverse the tile products are p^3 for the
// one-sweep form (the Gauss-Jordan count).
double spd_big_update_flops(const SpdArgs* a, int nmat, int k, bool with_pivot) {
  const int W = batch_R(a) == 2 ? 128 : 64;
  double fl = 0.0;
  for (int m = 0; m < nmat; ++m) {
    const int p = a[m].p, T = (p + W - 1) / W;
    if (k >= T) continue;
    auto w = [&](int I) { return (double)std::min(W, p - W * I); };
    const bool has_next = k + 1 < T;
    if (W == 128 && a[m].sched) {
      const std::vector<unsigned>& tab = host_wide_schedule(T);
      const unsigned* row = tab.data() + (size_t)k * wide_sched_stride(T);
      auto item = [&](unsigned ent) {
        const int I = (int)((ent >> 8) & 0xffu), J = (int)(ent & 0xffu);
        const bool two = (ent >> 16) & 1u;
        return 2.0 * w(I) * w(J) * (w(k) + (two ? w(k - 1) : 0.0));
      };
      for (unsigned i = 0; i < row[0]; ++i) fl += item(row[2 + i]);
      if (with_pivot && has_next) fl += item(row[1]);
    } else {
      for (int I = 0; I < T; ++I)
        for (int J = 0; J <= I; ++J) {
          if (!with_pivot && has_next && I == k + 1 && J == k + 1) continue;
          fl += 2.0 * w(I) * w(J) * w(k);
        }
    }
    if (with_pivot && has_next) fl += w(k + 1) * w(k + 1) * w(k + 1) / 3.0 + w(k + 1) * w(k + 1) * p;
  }
  return fl;
}

// bench: the update launch of sweep k without its pivot workgroup (the tile work alone)
hipError_t launch_spd_big_tiles(SpdArgs* a, int nmat, int k, hipStream_t s) {
  int Tmax, tiles;
  BigSpdBatch b = make_batch(a, nmat, Tmax, tiles);
  if (batch_R(a) == 2) launch_stage_r<2>(b, nmat, Tmax, tiles, 2 * k + 1, s, 1);
  else launch_stage_r<1>(b, nmat, Tmax, tiles, 2 * k + 1, s, 1);
  return hipGetLastError();
}

hipError_t launch_spd_inverse_big(SpdArgs* a, int nmat, double** final_out, hipStream_t s) {
  int Tmax, tiles;
  BigSpdBatch b = make_batch(a, nmat, Tmax, tiles);
  for (int m = 0; m < nmat; ++m) final_out[m] = a[m].X;
  const int R = batch_R(a);
  const int nsw = (Tmax + R - 1) / R;
  // pivot 0, panel 0, then one update launch per sweep (each also forms the next sweep's panel)
  for (int st = -1; st < 2 * nsw; ++st) {
    if (st > 0 && (st & 1) == 0) continue;
    if (R == 2) launch_stage_r<2>(b, nmat, Tmax, tiles, st, s);
    else launch_stage_r<1>(b, nmat, Tmax, tiles, st, s);
  }
  return hipGetLastError();
}

}  // namespace gpk
