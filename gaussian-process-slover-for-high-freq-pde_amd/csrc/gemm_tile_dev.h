// gemm_tile_dev.h — the software-pipelined 128x128-tile fp64 MFMA product loop (gfx950).
//
// A 128x128 output tile per 256-thread workgroup, each wave a 64x64 quadrant = 4x4
// v_mfma_f64_16x16x4 blocks (16 independent accumulation chains; every fragment feeds 4 MFMAs).
// 16-deep K-steps through two LDS stages; one K-step is two half steps q = 0, 1 of 32 MFMAs.
//
// The operand layouts are chosen per transpose signature so that no operand is transposed on its
// way into LDS (every store is one 16-B ds_write_b128 of a 16-B global load):
//   * k-contiguous operands (A[i][k], B[j][k]) stay [mn][k]: 16 doubles per row, no padding, the
//     eight 16-B chunks of a row XOR-swizzled by (row >> 1) & 7.  A lane's fragment of half step
//     q is ONE ds_read_b128 of chunk 4q + lk: (k = 8q + 2lk, 8q + 2lk + 1) feed the MFMAs of
//     kk = 2q and 2q + 1.  With the swizzle every 16-lane group of the read hits 16 distinct
//     16-B bank slots (conflict-free; checked in tools/probes/gemm_tile_probe.hip).
//   * mn-contiguous operands (A[k][i], B[k][j]) stay [k][mn], rows SM = 136 doubles apart
//     (rows 2 apart are 32 banks apart): two ds_read_b64 per fragment, of rows 8q + 2lk (+1).
//   Both operands use the same k permutation (physical k = 8q + 2lk + e for MFMA kk = 2q + e,
//   k-slot lk), so the sum is the same set of products, in the order of the k slots.
//
// Schedule of K-step s (LDS stage s & 1 holds it; fragments of its half step 0 are in f0 and the
// global data of step s + 1 in g on entry):
//   g -> other stage (ds_write_b128) | global loads of step s + 2 -> g | half step 1 -> f1
//   | 32 MFMAs on f0 | barrier | half step 0 of step s + 1 -> f0 | 32 MFMAs on f1.
// One barrier per K-step, and it sits between the two MFMA blocks: the other stage's stores are
// complete (lgkmcnt(0)) and every wave has read all of this stage, so after it the next step's
// first fragments are read while the 32 MFMAs of half step 1 run (the LDS latency of a K-step's
// start is covered), and global loads have a whole K-step to land.  Stores, loads and reads are
// interleaved with the MFMAs by sched_group_barrier; issue priority is raised over the MFMA
// blocks (the partner workgroup's wave on the SIMD then takes the memory slots).
// LDS: 2 stages x 2 operands x 2176 doubles = 68 KB (two workgroups per CU).
#pragma once
#include "gpk_internal.h"

namespace gpk {

typedef double d4 __attribute__((ext_vector_type(4)));

namespace tile {
constexpr int TM = 128, KS = 16;
constexpr int SM = 136;                 // [k][mn] row stride (doubles)
constexpr int OPSZ = 16 * SM;           // >= 128 * 16 ([mn][k])
constexpr int STAGE = 2 * OPSZ;         // A then B
constexpr int LDS_DOUBLES = 2 * STAGE;  // 8704 doubles = 68 KB

struct Glob { double2 a[4], b[4]; };  // one K-step of the tile, this thread's share
struct Frag { double2 a[4], b[4]; };  // one half step: .x feeds kk = 2q, .y kk = 2q + 1

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ __forceinline__ void st2(double* p, double2 v) { *reinterpret_cast<double2*>(p) = v; }
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

// Global -> registers for K-step k0.  Rows / columns past M, N load a clamped in-bounds address
// (branch-free; those values reach only outputs that are never stored).
template <int ta, int tb>
__device__ __forceinline__ void fetch(Glob& g, const double* A, int lda, const double* B, int ldb, int M,
                                      int N, int i0, int j0, int k0, int t) {
  if (!ta) {  // A[i][k]: row (t>>3) + 32j, chunk t&7
#pragma unroll
    for (int j = 0; j < 4; ++j)
      g.a[j] = ld2(A + (size_t)min(i0 + (t >> 3) + 32 * j, M - 1) * lda + k0 + 2 * (t & 7));
  } else {    // A[k][i]: k row (t>>6) + 4j, column pair t&63
    const int ic = min(i0 + 2 * (t & 63), M - 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) g.a[j] = ld2(A + (size_t)(k0 + (t >> 6) + 4 * j) * lda + ic);
  }
  if (tb) {   // B[j][k]
#pragma unroll
    for (int j = 0; j < 4; ++j)
      g.b[j] = ld2(B + (size_t)min(j0 + (t >> 3) + 32 * j, N - 1) * ldb + k0 + 2 * (t & 7));
  } else {    // B[k][j]
    const int jc = min(j0 + 2 * (t & 63), N - 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) g.b[j] = ld2(B + (size_t)(k0 + (t >> 6) + 4 * j) * ldb + jc);
  }
}

// registers -> LDS stage st (A scaled by sa: the dual product's alpha2 / alpha)
template <int ta, int tb, bool SCALE>
__device__ __forceinline__ void put(const Glob& g, double* st, double sa, int t) {
  double* sA = st;
  double* sB = st + OPSZ;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double2 v = g.a[j];
    if (SCALE) v = double2{sa * v.x, sa * v.y};
    if (!ta) {
      const int r = (t >> 3) + 32 * j;
      st2(sA + r * 16 + 2 * swz(r, t & 7), v);
    } else {
      st2(sA + ((t >> 6) + 4 * j) * SM + 2 * (t & 63), v);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (tb) {
      const int r = (t >> 3) + 32 * j;
      st2(sB + r * 16 + 2 * swz(r, t & 7), g.b[j]);
    } else {
      st2(sB + ((t >> 6) + 4 * j) * SM + 2 * (t & 63), g.b[j]);
    }
  }
}

// LDS stage st -> fragments of half step q for wave quadrant (wr, wc)
template <int ta, int tb>
__device__ __forceinline__ void get(Frag& f, const double* st, int q, int wr, int wc, int lane) {
  const double* sA = st;
  const double* sB = st + OPSZ;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    if (!ta) {
      const int r = 64 * wr + 16 * x + li;
      f.a[x] = ld2(sA + r * 16 + 2 * swz(r, 4 * q + lk));
    } else {
      const int c = 64 * wr + 16 * x + li, k = 8 * q + 2 * lk;
      f.a[x] = double2{sA[k * SM + c], sA[(k + 1) * SM + c]};
    }
  }
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    if (tb) {
      const int r = 64 * wc + 16 * y + li;
      f.b[y] = ld2(sB + r * 16 + 2 * swz(r, 4 * q + lk));
    } else {
      const int c = 64 * wc + 16 * y + li, k = 8 * q + 2 * lk;
      f.b[y] = double2{sB[k * SM + c], sB[(k + 1) * SM + c]};
    }
  }
}

__device__ __forceinline__ void mma(const Frag& f, d4 (&acc)[4][4]) {
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[x].x, f.b[y].x, acc[x][y], 0, 0, 0);
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[x].y, f.b[y].y, acc[x][y], 0, 0, 0);
}

// instructions per wave of each kind: ds_write_b128 per K-step, ds_reads per half step
template <int ta, int tb>
struct Counts {
  static constexpr int writes = 8;
  static constexpr int reads = (ta ? 8 : 4) + (tb ? 4 : 8);
  static constexpr int loads = 8;
};

// Interleave hints for a 32-MFMA block: NW stores, NL global loads, NR LDS reads, one per MFMA gap
// in that order (sched_group_barrier masks: MFMA 0x8, VMEM read 0x20, DS read 0x100, DS write 0x200)
template <int NW, int NL, int NR>
__device__ __forceinline__ void interleave() {
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x008, 32 - NW - NL - NR, 0);
}

// acc += sa * op(A) op(B) over K (a multiple of 32 by the padding contract, so nk >= 2).
// lds: LDS_DOUBLES doubles.  PRIO: raise issue priority over the MFMA blocks.  SCHED: the
// sched_group_barrier interleave.
template <int ta, int tb, bool SCALE, int PRIO = 1, bool SCHED = true>
__device__ __forceinline__ void product(const double* A, int lda, const double* B, int ldb, int K, int M,
                                        int N, int i0, int j0, double sa, double* lds, int t, int wr,
                                        int wc, int lane, d4 (&acc)[4][4]) {
  using C = Counts<ta, tb>;
  const int nk = K / KS;
  Glob g;
  Frag f0, f1;
  fetch<ta, tb>(g, A, lda, B, ldb, M, N, i0, j0, 0, t);
  put<ta, tb, SCALE>(g, lds, sa, t);
  fetch<ta, tb>(g, A, lda, B, ldb, M, N, i0, j0, KS, t);
  __syncthreads();
  get<ta, tb>(f0, lds, 0, wr, wc, lane);
  int s = 0;
  // steady state: the next stage is written and step s + 2 fetched
  for (; s + 2 < nk; ++s) {
    double* cur = lds + (s & 1) * STAGE;
    double* nxt = lds + ((s & 1) ^ 1) * STAGE;
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
    put<ta, tb, SCALE>(g, nxt, sa, t);
    fetch<ta, tb>(g, A, lda, B, ldb, M, N, i0, j0, (s + 2) * KS, t);
    get<ta, tb>(f1, cur, 1, wr, wc, lane);
    mma(f0, acc);
    if (SCHED) interleave<C::writes, C::loads, C::reads>();
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
    get<ta, tb>(f0, nxt, 0, wr, wc, lane);
    mma(f1, acc);
    if (SCHED) interleave<0, 0, C::reads>();
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  // step nk - 2: write the last stage, nothing more to fetch
  {
    double* cur = lds + (s & 1) * STAGE;
    double* nxt = lds + ((s & 1) ^ 1) * STAGE;
    put<ta, tb, SCALE>(g, nxt, sa, t);
    get<ta, tb>(f1, cur, 1, wr, wc, lane);
    mma(f0, acc);
    if (SCHED) interleave<C::writes, 0, C::reads>();
    __syncthreads();
    get<ta, tb>(f0, nxt, 0, wr, wc, lane);
    mma(f1, acc);
    if (SCHED) interleave<0, 0, C::reads>();
    ++s;
  }
  // last step
  {
    double* cur = lds + (s & 1) * STAGE;
    get<ta, tb>(f1, cur, 1, wr, wc, lane);
    mma(f0, acc);
    if (SCHED) interleave<0, 0, C::reads>();
    mma(f1, acc);
  }
  __syncthreads();  // the LDS is reused (a second product, the epilogue's partial sums)
}

// acc += sa1 op(A1) op(B1) [K1] + sa2 op(A2) op(B2) [K2]: product's pipeline over the two
// sources back to back (one prologue and one drain for K1 + K2; the C5 SPD inverse's two-sweep
// tile updates).  A1 / A2 (B1 / B2) share lda (ldb); both K are multiples of 32.
template <int ta, int tb>
__device__ __forceinline__ void product2(const double* A1, const double* B1, int K1, double sa1,
                                         const double* A2, const double* B2, int K2, double sa2,
                                         int lda, int ldb, int M, int N, int i0, int j0, double* lds,
                                         int t, int wr, int wc, int lane, d4 (&acc)[4][4]) {
  using C = Counts<ta, tb>;
  const int nk1 = K1 / KS, nk = nk1 + K2 / KS;
  auto fetch_s = [&](Glob& g, int s) {
    const bool one = s < nk1;
    fetch<ta, tb>(g, one ? A1 : A2, lda, one ? B1 : B2, ldb, M, N, i0, j0, (one ? s : s - nk1) * KS, t);
  };
  auto put_s = [&](const Glob& g, double* st, int s) { put<ta, tb, true>(g, st, s < nk1 ? sa1 : sa2, t); };
  Glob g;
  Frag f0, f1;
  fetch_s(g, 0);
  put_s(g, lds, 0);
  fetch_s(g, 1);
  __syncthreads();
  get<ta, tb>(f0, lds, 0, wr, wc, lane);
  int s = 0;
  for (; s + 2 < nk; ++s) {
    double* cur = lds + (s & 1) * STAGE;
    double* nxt = lds + ((s & 1) ^ 1) * STAGE;
    put_s(g, nxt, s + 1);
    fetch_s(g, s + 2);
    get<ta, tb>(f1, cur, 1, wr, wc, lane);
    mma(f0, acc);
    interleave<C::writes, C::loads, C::reads>();
    __syncthreads();
    get<ta, tb>(f0, nxt, 0, wr, wc, lane);
    mma(f1, acc);
    interleave<0, 0, C::reads>();
  }
  {
    double* cur = lds + (s & 1) * STAGE;
    double* nxt = lds + ((s & 1) ^ 1) * STAGE;
    put_s(g, nxt, s + 1);
    get<ta, tb>(f1, cur, 1, wr, wc, lane);
    mma(f0, acc);
    interleave<C::writes, 0, C::reads>();
    __syncthreads();
    get<ta, tb>(f0, nxt, 0, wr, wc, lane);
    mma(f1, acc);
    interleave<0, 0, C::reads>();
    ++s;
  }
  {
    double* cur = lds + (s & 1) * STAGE;
    get<ta, tb>(f1, cur, 1, wr, wc, lane);
    mma(f0, acc);
    interleave<0, 0, C::reads>();
    mma(f1, acc);
  }
  __syncthreads();
}

}  // namespace tile
}  // namespace gpk
