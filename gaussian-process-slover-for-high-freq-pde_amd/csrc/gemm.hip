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
#include "gpk_trace.h"
#include "gemm_tile_dev.h"

#include <algorithm>

namespace gpk {

GPK_TRACE_TU(gemm)

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

// Epilogue operands of one output element, fetched early (their latency hides under MFMA).
// Loads only -- no arithmetic on the loaded values here: a product formed at fetch time made
// the compiler wait for each element's loads in turn (four serial round trips in wave 0 ahead
// of its MFMA operand loads, ~4 us per latency-bound GEMM launch).
struct EpiIn {
  double pre, pu, q1, q2, ys;
};

__device__ __forceinline__ EpiIn epi_fetch(const GemmDesc& d, int row, int col) {
  EpiIn e{0.0, 0.0, 0.0, 0.0, 0.0};
  const size_t fo = (size_t)row * d.ldf + col;
  if (d.Y) e.ys = d.Ys[(size_t)row * d.ldy + col];
  if ((d.epi == EPI_STORE || d.epi == EPI_QUAD) && d.beta != 0.0)
    e.pre = d.C0[(size_t)row * d.ldc0 + col];
  else if (d.epi == EPI_RESID)
    e.pre = d.F[fo];
  if (d.epi == EPI_QUAD || (d.epi == EPI_RESID && d.ac)) e.pu = d.U[fo];
  if (d.epi == EPI_RESID && d.red2) {
    e.q1 = d.Q1[fo];
    e.q2 = d.Q2[fo];
  }
  return e;
}

// the side output of a stored value c (GemmDesc::Y)
__device__ __forceinline__ void epi_side(const GemmDesc& d, int row, int col, double c, const EpiIn& e,
                                         double v) {
  if (d.Y) d.Y[(size_t)row * d.ldy + col] = 0.5 * e.ys + v * c;
}

// c = alpha*P1 + alpha2*P2 (already formed); returns the stored value, accumulates partials
__device__ __forceinline__ double epi_apply(const GemmDesc& d, double c, const EpiIn& e,
                                            double& part, double& part2) {
  switch (d.epi) {
    case EPI_STORE:
      if (d.beta != 0.0) c += d.beta * e.pre;
      break;
    case EPI_RESID:
      c -= e.pre;
      if (d.ac) c += e.pu * (e.pu * e.pu - 1.0);
      part += c * c;
      part2 += e.q1 * e.q2;
      break;
    case EPI_QUAD:
      if (d.beta != 0.0) c += d.beta * e.pre;
      part += c * e.pu;
      break;
  }
  return c;
}

__global__ __launch_bounds__(256) void gemm_kernel(GemmBatch batch,
                                                   const StepScalars* __restrict__ sc) {
  const GemmDesc& d = batch.d[blockIdx.y];
  const int tn = d.N >> 5;
  const int tiles = (d.M >> 5) * tn;
  if ((int)blockIdx.x >= tiles) return;
  if (!gate_open(d.gate)) return;  // refinement not needed (uniform)
  const int ti = blockIdx.x / tn, tj = blockIdx.x % tn;
  const int i0 = ti * 32, j0 = tj * 32;

  __shared__ double sA[32 * GSA];
  __shared__ double sB[32 * GSB];
  __shared__ double sred[4], sred2[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  EpiIn ein[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    ein[r] = epi_fetch(d, i0 + 16 * wr + (lane >> 4) + 4 * r, j0 + 16 * wc + (lane & 15));

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

  double alpha = d.alpha, alpha2 = d.alpha2;
  if (d.vscale) alpha *= sc->v;
  if (d.vscale2) alpha2 *= sc->v;
  const double vv = d.Y ? sc->v : 0.0;
  double part = 0.0, part2 = 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = i0 + 16 * wr + (lane >> 4) + 4 * r, col = j0 + 16 * wc + (lane & 15);
    double c = alpha * acc1[r];
    if (d.K2) c += alpha2 * acc2[r];
    c = epi_apply(d, c, ein[r], part, part2);
    d.C[(size_t)row * d.ldc + col] = c;
    epi_side(d, row, col, c, ein[r], vv);
  }
  if (d.red) {
    double s = block_sum_256(part, sred);
    if (t == 0) d.red[blockIdx.x] = s;
  }
  if (d.red2) {
    double s = block_sum_256(part2, sred2);
    if (t == 0) d.red2[blockIdx.x] = s;
  }
}

// ---------------------------------------------------------------------------------------
// Latency-oriented variant for small factors (N <= ~512, e.g. the 256^2 headline): one
// 16x16 output tile per workgroup so a 256x256 product fills 256 CUs; the K range (of each
// product) is split over the 4 waves; operands go straight from L2 into registers, 8
// k-substeps of loads in flight per wave; the 4 partial accumulators are summed through LDS
// in fixed order (deterministic) by wave 0, which runs the epilogue.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ d4 mma_chunk(const double* __restrict__ A, int lda, int ta,
                                        const double* __restrict__ B, int ldb, int tb, int i0,
                                        int j0, int kbeg, int kend, int lane, d4 acc) {
  const int li = lane & 15, lk = lane >> 4;
  const int i = i0 + li, j = j0 + li;
  int k0 = kbeg;
  // 64-deep blocks: all 16 k-substeps of operands in flight before the first MFMA
  for (; k0 + 64 <= kend; k0 += 64) {
    double a[16], b[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = k0 + 4 * s + lk;
      a[s] = ta ? A[(size_t)k * lda + i] : A[(size_t)i * lda + k];
      b[s] = tb ? B[(size_t)j * ldb + k] : B[(size_t)k * ldb + j];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
  }
  if (k0 < kend) {  // K ranges are multiples of 32: at most one 32-deep tail
    double a[8], b[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = k0 + 4 * s + lk;
      a[s] = ta ? A[(size_t)k * lda + i] : A[(size_t)i * lda + k];
      b[s] = tb ? B[(size_t)j * ldb + k] : B[(size_t)k * ldb + j];
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
  }
  return acc;
}

// Operands whose contiguous dimension is k (A untransposed, B transposed) read as MFMA
// fragments directly would touch 16 rows x 32 B per load instruction (16 cache lines for 512
// useful bytes, 16 instructions per 64-deep block).  Instead each wave loads its 16 x 64 block
// with 8 coalesced 16-B loads per lane (2 whole 512-B rows per instruction), stages it in its
// own LDS block and reads the fragments back (row stride FS = 66 doubles: the 32 lanes of each
// ds_read_b64 half hit 64 distinct banks).
constexpr int FS = 66;
__device__ __forceinline__ void rowblk_load(const double* M, int ld, int r0, int k0, int lane,
                                            double2* g) {
#pragma unroll
  for (int q = 0; q < 8; ++q)
    g[q] = *reinterpret_cast<const double2*>(M + (size_t)(r0 + 2 * q + (lane >> 5)) * ld + k0 + 2 * (lane & 31));
}
__device__ __forceinline__ void rowblk_frag(double* buf, const double2* g, int lane, double* f) {
#pragma unroll
  for (int q = 0; q < 8; ++q)
    *reinterpret_cast<double2*>(buf + (2 * q + (lane >> 5)) * FS + 2 * (lane & 31)) = g[q];
  // (one wave's LDS operations complete in issue order: the reads see the writes, and the
  // next block's writes land after these reads -- no wait or barrier needed)
#pragma unroll
  for (int s = 0; s < 16; ++s) f[s] = buf[(lane & 15) * FS + 4 * s + (lane >> 4)];
}

// One 64-deep block of op(A) op(B) [+ op(A2) op(B2)] for this wave's 16x16 tile: fragments of
// the k-contiguous operands through LDS (above), the others loaded directly (already coalesced:
// 16 consecutive doubles of one row per 16 lanes); every global load of both products issued
// before the first MFMA.  The staging pattern is a template (SA = A untransposed, SB = B
// transposed): with runtime-selected arrays LLVM kept the operand arrays in scratch.
template <bool K>  // K: k-contiguous rows r0.. (staged) ; else direct fragment loads
__device__ __forceinline__ void frag_issue(const double* M, int ld, int r0, int k0, int lane,
                                           double2 (&g)[8], double (&f)[16]) {
  if constexpr (K) {
    rowblk_load(M, ld, r0, k0, lane, g);
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s) f[s] = M[(size_t)(k0 + 4 * s + (lane >> 4)) * ld + r0 + (lane & 15)];
  }
}
template <bool SA1, bool SB1, bool SA2, bool SB2, bool DUAL>
__device__ __forceinline__ void blk64(const GemmDesc& d, int i0, int j0, int b0, int c0, int lane,
                                      double* bufA, double* bufB, d4& acc1, d4& acc2) {
  double2 ga1[8], gb1[8], ga2[8], gb2[8];
  double a1[16], bb1[16], a2[16], bb2[16];
  frag_issue<SA1>(d.A, d.lda, i0, b0, lane, ga1, a1);
  frag_issue<SB1>(d.B, d.ldb, j0, b0, lane, gb1, bb1);
  if constexpr (DUAL) {
    frag_issue<SA2>(d.A2, d.lda2, i0, c0, lane, ga2, a2);
    frag_issue<SB2>(d.B2, d.ldb2, j0, c0, lane, gb2, bb2);
  }
  if constexpr (SA1) rowblk_frag(bufA, ga1, lane, a1);
  if constexpr (SB1) rowblk_frag(bufB, gb1, lane, bb1);
#pragma unroll
  for (int s = 0; s < 16; ++s) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], bb1[s], acc1, 0, 0, 0);
  if constexpr (DUAL) {
    if constexpr (SA2) rowblk_frag(bufA, ga2, lane, a2);
    if constexpr (SB2) rowblk_frag(bufB, gb2, lane, bb2);
#pragma unroll
    for (int s = 0; s < 16; ++s) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s], bb2[s], acc2, 0, 0, 0);
  }
}
// runtime transpose flags -> one of the 4 (single) / 16 (dual) instantiations (uniform branch)
template <bool DUAL>
__device__ __forceinline__ void blk64_dispatch(const GemmDesc& d, int i0, int j0, int b0, int c0,
                                               int lane, double* bufA, double* bufB, d4& acc1,
                                               d4& acc2) {
  const int code = (!d.ta) | (d.tb << 1) | ((!d.ta2) << 2) | (d.tb2 << 3);
#define GPK_B64(c) blk64<((c) & 1) != 0, ((c) & 2) != 0, ((c) & 4) != 0, ((c) & 8) != 0, true>
#define GPK_B64S(c) blk64<((c) & 1) != 0, ((c) & 2) != 0, false, false, false>
  if (DUAL && d.K2) {
    switch (code) {
      case 0: GPK_B64(0)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 1: GPK_B64(1)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 2: GPK_B64(2)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 3: GPK_B64(3)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 4: GPK_B64(4)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 5: GPK_B64(5)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 6: GPK_B64(6)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 7: GPK_B64(7)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 8: GPK_B64(8)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 9: GPK_B64(9)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 10: GPK_B64(10)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 11: GPK_B64(11)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 12: GPK_B64(12)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 13: GPK_B64(13)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 14: GPK_B64(14)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      default: GPK_B64(15)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
    }
  } else {
    switch (code & 3) {
      case 0: GPK_B64S(0)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 1: GPK_B64S(1)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      case 2: GPK_B64S(2)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
      default: GPK_B64S(3)(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2); break;
    }
  }
#undef GPK_B64
#undef GPK_B64S
}

// DUAL (some descriptor has a second product): waves_per_eu(2) = 256 VGPRs per lane, enough for
// both products' staged operands in flight without spilling.  Batches without one (C4's G_D
// stage: 4 descriptors = 1024 workgroups) get waves_per_eu(4), four workgroups per CU: one
// round over the chip instead of two.
template <bool DUAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DUAL ? 2 : 4, DUAL ? 2 : 4)))
void gemm_small_kernel(GemmBatch batch, const StepScalars* __restrict__ sc) {
  const GemmDesc& d = batch.d[blockIdx.y];
  const int tn = d.N >> 4;
  const int tiles = (d.M >> 4) * tn;
  // XCD-major dealing: blocks b, b + 8, ... share an XCD (and its L2) and take consecutive tiles,
  // i.e. whole 16-row blocks of op(A), so each XCD's L2 holds 1/8 of op(A)'s rows instead of all
  // of them (a bijection of [0, gridDim.x) when it is a multiple of 8; else the identity)
  const int gx = (int)gridDim.x, x = (int)blockIdx.x;
  const int tile = (gx & 7) ? x : (x & 7) * (gx >> 3) + (x >> 3);
  if (tile >= tiles) return;
  // refinement gate: its (scalar) load is issued first and overlaps the epilogue prefetch; a
  // closed gate ends the workgroup before any operand load (launch + one round trip)
  const bool open = gate_open(d.gate);
  const int i0 = (tile / tn) * 16, j0 = (tile % tn) * 16;
  // per-wave operand staging (one 16 x FS block, A then B), reused for the cross-wave partials
  __shared__ double smem[4 * 16 * FS];
  double(*part)[4][256] = reinterpret_cast<double(*)[4][256]>(smem);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  [[maybe_unused]] const int tslot = SLOT_GEMM + 4 * (d.tag & 15);
  if (TR_FIRST) TR_LO(tslot);
  if (TR_LAST) TR_LO(tslot + 3);
  // K ranges are multiples of 32; wave wv takes a contiguous quarter (rounded to 32)
  auto range = [&](int K, int& b0, int& b1) {
    const int nk = K >> 5;
    b0 = ((nk * wv) >> 2) << 5;
    b1 = ((nk * (wv + 1)) >> 2) << 5;
  };
  // wave wv runs the epilogue of the tile's rows lane / 16 + 4 wv (one output per lane): its
  // operands are prefetched now so their latency hides under the MFMAs
  const EpiIn ein = epi_fetch(d, i0 + (lane >> 4) + 4 * wv, j0 + (lane & 15));
  // class partials (d.cpart): this lane's element's class id and, for thread t < CB_SLOTS =
  // (signed diagonal offset dl, variants v = t & 7 and v + 8), the class range of its diagonal
  // -- all fixed by the tile's position, so loaded here with the epilogue operands (loads only:
  // arithmetic on the loaded values here made the compiler wait for them before the operand
  // loads, a whole memory round trip per launch -- epi_fetch's rule)
  int bu = -1, bcb = 0, bc0 = 0, bc1 = 0;
  double bxi = 0.0, bxj = 0.0;
  if (d.cpart) {  // (uniform)
    const int row = i0 + (lane >> 4) + 4 * wv, col = j0 + (lane & 15);
    bu = d.bcid[(size_t)row * d.ldc + col];
    bcb = d.bcbase[min(abs(row - col), d.bn)];
    if (d.bsx) {
      bxi = d.bsx[min(row, d.bn - 1)];
      bxj = d.bsx[min(col, d.bn - 1)];
    }
    const int k = min(abs(16 * ((i0 - j0) >> 4) + (t >> 3) - 15), d.bn - 1);
    bc0 = d.bcbase[k];
    bc1 = d.bcbase[k + 1];
  }
  if (!open) return;  // uniform
  int b0, b1, c0 = 0, c1 = 0;
  range(d.K, b0, b1);
  if (DUAL && d.K2) range(d.K2, c0, c1);
  d4 acc1 = {0.0, 0.0, 0.0, 0.0}, acc2 = {0.0, 0.0, 0.0, 0.0};
  if (b1 - b0 == 64 && (!(DUAL && d.K2) || c1 - c0 == 64)) {
    // one 64-deep block per wave and product (K = 256): every global operand load of both
    // products in flight before the first MFMA (one memory round trip)
    double* bufA = smem + wv * 16 * FS;
    double* bufB = bufA;  // (in-order LDS per wave: B's block lands after A's fragments are read)
    blk64_dispatch<DUAL>(d, i0, j0, b0, c0, lane, bufA, bufB, acc1, acc2);
  } else {  // (per wave: with K = 224 wave 0 takes 32 deep, the others 64)
    acc1 = mma_chunk(d.A, d.lda, d.ta, d.B, d.ldb, d.tb, i0, j0, b0, b1, lane, acc1);
    if (DUAL && d.K2) acc2 = mma_chunk(d.A2, d.lda2, d.ta2, d.B2, d.ldb2, d.tb2, i0, j0, c0, c1, lane, acc2);
  }
  __syncthreads();  // every wave done with its staging block before `part` reuses the LDS
  if (TR_FIRST) TR_HI(tslot + 2);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[0][wv][lane * 4 + r] = acc1[r];
    part[1][wv][lane * 4 + r] = acc2[r];
  }
  __syncthreads();
  if (TR_LAST) TR_HI(tslot + 3);
  // the epilogue on all four waves (one output per lane each; wave 0 used to run all four rows
  // in turn): the K quarters summed in fixed order, then the stage's epilogue and stores
  double alpha = d.alpha, alpha2 = d.alpha2;
  if (d.vscale) alpha *= sc->v;
  if (d.vscale2) alpha2 *= sc->v;
  const double vv = d.Y ? sc->v : 0.0;
  double red = 0.0, red2 = 0.0, c;
  const int row = i0 + (lane >> 4) + 4 * wv, col = j0 + (lane & 15);
  {
    const int q = lane * 4 + wv;
    const double s1 = (part[0][0][q] + part[0][1][q]) + (part[0][2][q] + part[0][3][q]);
    c = alpha * s1;
    if (DUAL && d.K2) c += alpha2 * ((part[1][0][q] + part[1][1][q]) + (part[1][2][q] + part[1][3][q]));
    c = epi_apply(d, c, ein, red, red2);
  }
  // The tile's class sums (d.cpart) and loss partials (d.red / d.red2) go through LDS: their
  // LDS writes and ONE barrier come before this lane's global stores, because a barrier
  // (__syncthreads: a workgroup release) waits for every earlier store of the wave to be
  // acknowledged -- after the C store it cost a memory round trip per launch.
  // class sums: the tile in LDS diagonal-major, element (r, c) at [r - c + 15][r], so the
  // thread of diagonal offset dl reads its row of 16 with 16-byte loads (the 8 threads of one
  // diagonal share it: a broadcast); positions off the diagonal's range are masked by r.  Row
  // strides 18 doubles / 20 ints: the 16 lanes of one tile row write 16 distinct bank pairs
  // (a 16-double stride put them on 2)
  constexpr int BVS = 18, BWS = 20;
  double* bv = smem + 2 * 4 * 256 + 512;              // [31][BVS] values
  int* bvar = reinterpret_cast<int*>(bv + 31 * BVS);  // [31][BWS] variants
  double* sred = smem + 2 * 4 * 256;                 // [2][256] loss partials
  if (d.cpart) {  // (uniform)
    const int r = (lane >> 4) + 4 * wv, dg = r - (lane & 15) + 15;
    bv[dg * BVS + r] = (d.bsx && !(bxi - bxj >= 0.0)) ? -c : c;  // D_x1: s_ij G_D (JAX abs'(0) = +1)
    bvar[dg * BWS + r] = bu >= 0 ? bu - bcb : -1;
  }
  if (d.red || d.red2) {  // (uniform) (past `part`, which other waves may still be reading)
    sred[wv * 64 + lane] = red;
    sred[256 + wv * 64 + lane] = red2;
  }
  if (d.cpart || d.red || d.red2) __syncthreads();  // (uniform)
  d.C[(size_t)row * d.ldc + col] = c;
  epi_side(d, row, col, c, ein, vv);
  if (d.cpart) {  // (uniform) the tile's sums per (signed diagonal, variant), rows in order
    // this thread's slots: class (k, v) [and (k, v + 8)] at (sign, band group, tile row)
    const int dl = (t >> 3) - 15, v = t & 7;
    int bslot = -1, bslot2 = -1;
    {
      const int I = i0 >> 4, b = I - (j0 >> 4), s = 16 * b + dl, k = abs(s);
      const int fb = s >= 0 ? s / 16 : -((15 - s) / 16);  // floor(s / 16)
      const int e = ((s < 0 ? 2 : 0) + (b == fb ? 0 : 1)) * tn + I - max(0, b);
      if (t < CB_SLOTS && k < d.bn) {
        if (v < bc1 - bc0) bslot = e * d.bncls + bc0 + v;
        if (v + 8 < bc1 - bc0) bslot2 = e * d.bncls + bc0 + v + 8;
      }
    }
    if (bslot >= 0) {  // (bslot2 >= 0 only if bslot is)
      typedef double d2v __attribute__((ext_vector_type(2)));
      typedef int i4v __attribute__((ext_vector_type(4)));
      const d2v* rv = reinterpret_cast<const d2v*>(bv + (dl + 15) * BVS);
      const i4v* rw = reinterpret_cast<const i4v*>(bvar + (dl + 15) * BWS);
      double x[16];
      int w[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const d2v a = rv[q];
        x[2 * q] = a.x;
        x[2 * q + 1] = a.y;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const i4v a = rw[q];
        w[4 * q] = a.x; w[4 * q + 1] = a.y; w[4 * q + 2] = a.z; w[4 * q + 3] = a.w;
      }
      double s = 0.0, s2 = 0.0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool in = (unsigned)(r - dl) < 16u;  // column r - dl inside the tile
        if (in && w[r] == v) s += x[r];
        if (in && w[r] == v + 8) s2 += x[r];
      }
      d.cpart[bslot] = s;
      if (bslot2 >= 0) d.cpart[bslot2] = s2;
    }
  }
  if ((d.red || d.red2) && wv == 0) {  // the tile's partials: waves' terms in row order, then lanes
    red = ((sred[lane] + sred[64 + lane]) + sred[128 + lane]) + sred[192 + lane];
    red2 = ((sred[256 + lane] + sred[320 + lane]) + sred[384 + lane]) + sred[448 + lane];
    if (d.red) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) red += __shfl_xor(red, o, 64);
      if (lane == 0) d.red[tile] = red;
    }
    if (d.red2) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) red2 += __shfl_xor(red2, o, 64);
      if (lane == 0) d.red2[tile] = red2;
    }
  }
  if (TR_FIRST) TR_HI(tslot);
}

static void launch_small(const GemmBatch& b, int ndesc, int tiles, const StepScalars* sc, hipStream_t s) {
  bool dual = false;
  for (int i = 0; i < ndesc; ++i) dual |= b.d[i].K2 != 0;
  if (dual)
    hipLaunchKernelGGL(gemm_small_kernel<true>, dim3(tiles, ndesc), dim3(256), 0, s, b, sc);
  else
    hipLaunchKernelGGL(gemm_small_kernel<false>, dim3(tiles, ndesc), dim3(256), 0, s, b, sc);
}

hipError_t launch_gemm_batch(const GemmDesc* descs, int ndesc, int max_tiles,
                             const StepScalars* sc, hipStream_t s, int small) {
  if (ndesc < 1 || ndesc > GEMM_MAX_BATCH) return hipErrorInvalidValue;
  GemmBatch b{};
  for (int i = 0; i < ndesc; ++i) b.d[i] = descs[i];
  if (small)
    launch_small(b, ndesc, max_tiles, sc, s);
  else
    hipLaunchKernelGGL(gemm_kernel, dim3(max_tiles, ndesc), dim3(256), 0, s, b, sc);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Throughput variant for large factors (N >= ~1500, e.g. the 4096^2 advection grid): a 64x64
// output tile per 256-thread workgroup, each wave a 32x32 quadrant (2x2 v_mfma_f64_16x16x4
// blocks, every A/B fragment used twice); K-steps of 32 through double-buffered LDS with one
// barrier per step; the next K-step's operands are fetched global->registers (16-B loads,
// coalesced along the contiguous dimension of each operand) while the current one is
// multiplied.  Tiles are dealt XCD-major (blocks b, b+8, ... share an XCD and get consecutive
// tiles, so they share A row panels in that XCD's L2).  Edge tiles of a 32-padded matrix are
// half-empty: rows/cols >= M/N are skipped at load (zero) and store.
// ---------------------------------------------------------------------------------------
constexpr int BSA = 34;  // A-role LDS stride: [m][k], ds_read_b64 conflict-free (rows 4 banks apart)
constexpr int BSB = 80;  // B-role LDS stride: [k][n], k and k+1 rows 32 banks apart

struct BigRegs {
  double2 a[4], b[4];
};

__device__ __forceinline__ void big_fetch(BigRegs& R, const double* A, int lda, int ta, const double* B,
                                          int ldb, int tb, int M, int N, int i0, int j0, int k0,
                                          int t) {
  const double2 z = {0.0, 0.0};
  if (!ta) {  // op(A)[i][k] = A[i][k]: row r = t>>2, k-chunk 8*(t&3)
    const int r = t >> 2, kc = (t & 3) * 8;
    const bool ok = i0 + r < M;
    const double* p = A + (size_t)(i0 + r) * lda + k0 + kc;
#pragma unroll
    for (int j = 0; j < 4; ++j) R.a[j] = ok ? *reinterpret_cast<const double2*>(p + 2 * j) : z;
  } else {    // op(A)[i][k] = A[k][i]: k-row t>>3, i-chunk 8*(t&7)
    const int kr = t >> 3, ic = (t & 7) * 8;
    const double* p = A + (size_t)(k0 + kr) * lda + i0 + ic;
#pragma unroll
    for (int j = 0; j < 4; ++j) R.a[j] = (i0 + ic + 2 * j < M) ? *reinterpret_cast<const double2*>(p + 2 * j) : z;
  }
  if (!tb) {  // op(B)[k][j] = B[k][j]: k-row t>>3, j-chunk 8*(t&7)
    const int kr = t >> 3, jc = (t & 7) * 8;
    const double* p = B + (size_t)(k0 + kr) * ldb + j0 + jc;
#pragma unroll
    for (int j = 0; j < 4; ++j) R.b[j] = (j0 + jc + 2 * j < N) ? *reinterpret_cast<const double2*>(p + 2 * j) : z;
  } else {    // op(B)[k][j] = B[j][k]: j-row t>>2, k-chunk 8*(t&3)
    const int r = t >> 2, kc = (t & 3) * 8;
    const bool ok = j0 + r < N;
    const double* p = B + (size_t)(j0 + r) * ldb + k0 + kc;
#pragma unroll
    for (int j = 0; j < 4; ++j) R.b[j] = ok ? *reinterpret_cast<const double2*>(p + 2 * j) : z;
  }
}

__device__ __forceinline__ void big_store(const BigRegs& R, double* sA, double* sB, int ta, int tb, int t) {
  if (!ta) {
    const int r = t >> 2, kc = (t & 3) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<double2*>(sA + r * BSA + kc + 2 * j) = R.a[j];
  } else {
    const int kr = t >> 3, ic = (t & 7) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sA[(ic + 2 * j) * BSA + kr] = R.a[j].x;
      sA[(ic + 2 * j + 1) * BSA + kr] = R.a[j].y;
    }
  }
  if (!tb) {
    const int kr = t >> 3, jc = (t & 7) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<double2*>(sB + kr * BSB + jc + 2 * j) = R.b[j];
  } else {
    const int r = t >> 2, kc = (t & 3) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sB[(kc + 2 * j) * BSB + r] = R.b[j].x;
      sB[(kc + 2 * j + 1) * BSB + r] = R.b[j].y;
    }
  }
}

// acc[bi][bj] += the wave's 32x32 quadrant (wr, wc) of one 32-deep K-step
__device__ __forceinline__ void big_mma(const double* sA, const double* sB, int wr, int wc, int lane,
                                        d4 (&acc)[2][2]) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = 4 * kk + lk;
    const double a0 = sA[(32 * wr + li) * BSA + k], a1 = sA[(32 * wr + 16 + li) * BSA + k];
    const double b0 = sB[k * BSB + 32 * wc + li], b1 = sB[k * BSB + 32 * wc + 16 + li];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
}

__device__ __forceinline__ void big_product(const double* A, int lda, int ta, const double* B, int ldb,
                                            int tb, int K, int M, int N, int i0, int j0, double* sA0,
                                            double* sB0, int t, int wr, int wc, int lane,
                                            d4 (&acc)[2][2]) {
  constexpr int SAZ = 64 * BSA, SBZ = 32 * BSB;
  BigRegs R;
  const int nk = K >> 5;
  big_fetch(R, A, lda, ta, B, ldb, tb, M, N, i0, j0, 0, t);
  big_store(R, sA0, sB0, ta, tb, t);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) big_fetch(R, A, lda, ta, B, ldb, tb, M, N, i0, j0, (kt + 1) * 32, t);
    big_mma(sA0 + cur * SAZ, sB0 + cur * SBZ, wr, wc, lane, acc);
    if (kt + 1 < nk) big_store(R, sA0 + (cur ^ 1) * SAZ, sB0 + (cur ^ 1) * SBZ, ta, tb, t);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void gemm_big_kernel(GemmBatch batch, const StepScalars* __restrict__ sc,
                                                       int per_xcd) {
  const GemmDesc& d = batch.d[blockIdx.y];
  const int tn = (d.N + 63) >> 6;
  const int tiles = ((d.M + 63) >> 6) * tn;
  const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);  // XCD-major dealing
  if (tile >= tiles) return;
  if (!gate_open(d.gate)) return;  // refinement not needed (uniform)
  const int i0 = (tile / tn) * 64, j0 = (tile % tn) * 64;
  __shared__ double sA[2 * 64 * BSA], sB[2 * 32 * BSB];
  __shared__ double sred[4], sred2[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc1[2][2], acc2[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      acc1[a][b] = d4{0.0, 0.0, 0.0, 0.0};
      acc2[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    }
  big_product(d.A, d.lda, d.ta, d.B, d.ldb, d.tb, d.K, d.M, d.N, i0, j0, sA, sB, t, wr, wc, lane, acc1);
  if (d.K2) big_product(d.A2, d.lda2, d.ta2, d.B2, d.ldb2, d.tb2, d.K2, d.M, d.N, i0, j0, sA, sB, t, wr, wc, lane, acc2);
  double alpha = d.alpha, alpha2 = d.alpha2;
  if (d.vscale) alpha *= sc->v;
  if (d.vscale2) alpha2 *= sc->v;
  const double vv = d.Y ? sc->v : 0.0;
  double part = 0.0, part2 = 0.0;
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i0 + 32 * wr + 16 * bi + (lane >> 4) + 4 * r;
        const int col = j0 + 32 * wc + 16 * bj + (lane & 15);
        if (row < d.M && col < d.N) {
          const EpiIn e = epi_fetch(d, row, col);
          double c = alpha * acc1[bi][bj][r];
          if (d.K2) c += alpha2 * acc2[bi][bj][r];
          c = epi_apply(d, c, e, part, part2);
          d.C[(size_t)row * d.ldc + col] = c;
          epi_side(d, row, col, c, e, vv);
        }
      }
  if (d.red) {
    double s = block_sum_256(part, sred);
    if (t == 0) d.red[tile] = s;
  }
  if (d.red2) {
    double s = block_sum_256(part2, sred2);
    if (t == 0) d.red2[tile] = s;
  }
}

// ---------------------------------------------------------------------------------------
// Largest-size variant (M, N >= ~2048, e.g. the 4096^2 advection grid): a 128x128 output tile
// per 256-thread workgroup, each wave a 64x64 quadrant = 4x4 v_mfma_f64_16x16x4 blocks, the
// software-pipelined product loop of gemm_tile_dev.h (no operand transposed on its way into LDS,
// one barrier per 16-deep K-step between the two MFMA half steps, stores / loads / reads
// interleaved with the MFMAs).  A dual product is folded into the same accumulators: its A2
// operand is scaled by alpha2 / alpha on the way into LDS, and the epilogue applies alpha once.
// Tiles are dealt XCD-major and walked in groups of 4 tile rows (A/B panel reuse in each XCD's
// L2).  4096^3: 71.8 (NN) / 73.4 (NT) / 73.1 (TN) / 73.4 (TT) TF/s, against 65 TF/s for the
// previous 16-deep-step loop and 66.8 / 73.2 / 73.2 for the library (tools/probes/
// gemm_tile_probe.hip, profiles/r5_tile_probe1.txt).
// ---------------------------------------------------------------------------------------

// one instantiation per transpose signature: the K-loop carries no branches at all (a runtime
// transpose switch makes the compiler shuttle the accumulators between AGPRs and VGPRs every
// K-step).  A dual product runs as two launches (launch_huge): the first stores
// alpha op(A) op(B) [+ beta C0] into C, the second adds alpha2 op(A2) op(B2) to it (Cp) and runs
// the epilogue -- one product loop per kernel keeps the loop's 224 live VGPRs (128 accumulator,
// 64 fragment, 32 global-prefetch) spill-free, for one extra pass over C (at 4096^2 about 35 us
// against the 4.4 ms of the two products).
// waves_per_eu(2): 256 VGPRs per lane and two workgroups per CU (2 x 68 KB of LDS).
template <int TA, int TB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void gemm_huge_kernel(GemmBatch batch, const StepScalars* __restrict__ sc, int per_xcd) {
  using namespace tile;
  constexpr int GROUP_M = 4;
  const GemmDesc& d = batch.d[blockIdx.y];
  const int tm = (d.M + TM - 1) / TM, tn = (d.N + TM - 1) / TM;
  const int o = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);  // XCD-major dealing
  if (o >= tm * tn) return;
  if (!gate_open(d.gate)) return;  // refinement not needed (uniform)
  const int gsz = GROUP_M * tn, grp = o / gsz, first = grp * GROUP_M;
  const int gm = min(GROUP_M, tm - first), in = o - grp * gsz;
  const int ti = first + in % gm, tj = in / gm;
  const int tile = ti * tn + tj;  // partial-sum slot (row-major tile index)
  const int i0 = ti * TM, j0 = tj * TM;
  __shared__ double lds[LDS_DOUBLES];
  __shared__ double sred[4], sred2[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};
  product<TA, TB, false, 0>(d.A, d.lda, d.B, d.ldb, d.K, d.M, d.N, i0, j0, 1.0, lds, t, wr, wc, lane, acc);
  const double alpha = d.vscale ? d.alpha * sc->v : d.alpha;
  const double vv = d.Y ? sc->v : 0.0;
  // Epilogue through LDS, one half tile (64 rows) at a time: the two waves of that half store
  // their accumulators (static indices: a rolled epilogue over the accumulators put them in
  // scratch), then every thread finishes 16 rows x 2 adjacent columns -- whole-row (coalesced)
  // accesses to C and the epilogue operands.
  double part = 0.0, part2 = 0.0;
  constexpr int ES = TM;  // [64][128] doubles = 64 KB of the 68 KB staging array
  for (int h = 0; h < 2; ++h) {
    if (wr == h) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            lds[(16 * x + (lane >> 4) + 4 * r) * ES + 64 * wc + 16 * y + (lane & 15)] = acc[x][y][r];
    }
    __syncthreads();
    const int col0 = j0 + 2 * (t & 63);
    for (int i = 0; i < 16; ++i) {
      const int lr = (t >> 6) + 4 * i, row = i0 + 64 * h + lr;
      if (row >= d.M) break;  // (rows ascend with i)
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        const int col = col0 + e2;
        if (col < d.N) {
          const EpiIn e = epi_fetch(d, row, col);
          double c = alpha * lds[lr * ES + 2 * (t & 63) + e2];
          if (d.Cp) c += d.Cp[(size_t)row * d.ldcp + col];
          c = epi_apply(d, c, e, part, part2);
          d.C[(size_t)row * d.ldc + col] = c;
          epi_side(d, row, col, c, e, vv);
        }
      }
    }
    __syncthreads();
  }
  if (d.red) {
    double s = block_sum_256(part, sred);
    if (t == 0) d.red[tile] = s;
  }
  if (d.red2) {
    double s = block_sum_256(part2, sred2);
    if (t == 0) d.red2[tile] = s;
  }
}

typedef void (*HugeFn)(GemmBatch, const StepScalars*, int);
static HugeFn huge_fn(int ta, int tb) {
  static const HugeFn tab[4] = {gemm_huge_kernel<0, 0>, gemm_huge_kernel<0, 1>, gemm_huge_kernel<1, 0>,
                                gemm_huge_kernel<1, 1>};
  return tab[(ta ? 2 : 0) | (tb ? 1 : 0)];
}

// one launch per transpose signature in each of two passes: pass 0 the first products of the
// dual descriptors (plain stores: C = alpha op(A) op(B) [+ beta C0]), pass 1 every descriptor's
// last product with its epilogue (a dual descriptor's second product reads pass 0's C as Cp).
static hipError_t launch_huge(const GemmDesc* descs, int ndesc, const StepScalars* sc, hipStream_t s) {
  GemmDesc pass[2][GEMM_MAX_BATCH];
  int np[2] = {0, 0};
  for (int i = 0; i < ndesc; ++i) {
    const GemmDesc& d = descs[i];
    if (!d.K2) {
      pass[1][np[1]++] = d;
      continue;
    }
    // the second pass reads C while writing it (same element, same thread: read before write);
    // C must not be an operand of the second product
    if (d.C == d.A2 || d.C == d.B2 || d.C == d.F || d.C == d.U || d.C == d.Q1 || d.C == d.Q2 || d.C == d.Ys)
      return hipErrorInvalidValue;
    // nor may another descriptor of the batch read it (pass 0 writes it before pass 1 runs)
    for (int j = 0; j < ndesc; ++j) {
      const GemmDesc& o = descs[j];
      if (j != i && (o.A == d.C || o.B == d.C || o.A2 == d.C || o.B2 == d.C || o.C0 == d.C || o.F == d.C ||
                     o.U == d.C || o.Q1 == d.C || o.Q2 == d.C || o.Ys == d.C))
        return hipErrorInvalidValue;
    }
    GemmDesc a{};  // alpha op(A) op(B) [+ beta C0] -> C
    a.A = d.A; a.lda = d.lda; a.ta = d.ta; a.B = d.B; a.ldb = d.ldb; a.tb = d.tb;
    a.alpha = d.alpha; a.vscale = d.vscale; a.C = d.C; a.ldc = d.ldc;
    a.M = d.M; a.N = d.N; a.K = d.K; a.epi = EPI_STORE; a.gate = d.gate; a.ngate = d.ngate; a.tag = d.tag;
    if (d.epi != EPI_RESID && d.beta != 0.0) { a.beta = d.beta; a.C0 = d.C0; a.ldc0 = d.ldc0; }
    pass[0][np[0]++] = a;
    GemmDesc b = d;  // alpha2 op(A2) op(B2) + C, then the descriptor's epilogue
    b.A = d.A2; b.lda = d.lda2; b.ta = d.ta2; b.B = d.B2; b.ldb = d.ldb2; b.tb = d.tb2; b.K = d.K2;
    b.alpha = d.alpha2; b.vscale = d.vscale2; b.K2 = 0; b.A2 = b.B2 = nullptr;
    b.Cp = d.C; b.ldcp = d.ldc;
    if (d.epi != EPI_RESID) b.beta = 0.0;
    pass[1][np[1]++] = b;
  }
  for (int p = 0; p < 2; ++p) {
    bool done[GEMM_MAX_BATCH] = {};
    for (int i = 0; i < np[p]; ++i) {
      if (done[i]) continue;
      const int ta = pass[p][i].ta, tb = pass[p][i].tb;
      GemmBatch b{};
      int nb = 0, mt = 0;
      for (int j = i; j < np[p]; ++j)
        if (!done[j] && pass[p][j].ta == ta && pass[p][j].tb == tb) {
          done[j] = true;
          b.d[nb++] = pass[p][j];
          mt = std::max(mt, gemm_tiles(pass[p][j], GEMM_HUGE));
        }
      const int per = (mt + 7) / 8;
      hipLaunchKernelGGL(huge_fn(ta, tb), dim3(8 * per, nb), dim3(256), 0, s, b, sc, per);
    }
  }
  return hipGetLastError();
}

int gemm_tiles(const GemmDesc& d, int variant) {
  if (variant == GEMM_SMALL) return (d.M / 16) * (d.N / 16);
  if (variant == GEMM_HUGE) return ((d.M + 127) / 128) * ((d.N + 127) / 128);
  if (variant == GEMM_BIG) return ((d.M + 63) / 64) * ((d.N + 63) / 64);
  return (d.M / 32) * (d.N / 32);
}

int gemm_variant(const GemmDesc* descs, int ndesc, int force_big) {
  if (force_big == 2) return GEMM_HUGE;
  if (force_big) return GEMM_BIG;
  long tot16 = 0, tot128 = 0;
  for (int i = 0; i < ndesc; ++i) {
    tot16 += (long)(descs[i].M / 16) * (descs[i].N / 16);
    tot128 += (long)((descs[i].M + 127) / 128) * ((descs[i].N + 127) / 128);
  }
  if (gemm_use_small(tot16)) return GEMM_SMALL;
  return tot128 >= GEMM_HUGE_MIN_TILES ? GEMM_HUGE : GEMM_BIG;
}

hipError_t launch_gemm_auto(const GemmDesc* descs, int ndesc, const StepScalars* sc, hipStream_t s,
                            int variant) {
  if (ndesc < 1 || ndesc > GEMM_MAX_BATCH) return hipErrorInvalidValue;
  GemmBatch b{};
  int mt = 0;
  for (int i = 0; i < ndesc; ++i) {
    b.d[i] = descs[i];
    mt = std::max(mt, gemm_tiles(descs[i], variant));
  }
  if (variant == GEMM_SMALL) {
    launch_small(b, ndesc, mt, sc, s);
  } else if (variant == GEMM_BIG) {
    const int per = (mt + 7) / 8;
    hipLaunchKernelGGL(gemm_big_kernel, dim3(8 * per, ndesc), dim3(256), 0, s, b, sc, per);
  } else if (variant == GEMM_HUGE) {
    return launch_huge(descs, ndesc, sc, s);
  } else {
    hipLaunchKernelGGL(gemm_kernel, dim3(mt, ndesc), dim3(256), 0, s, b, sc);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// GEMV (1D solver, code/model_GP_solver_1d.py:92,97): one wave per row, 4 rows per block.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gemv_kernel(GemvDesc d) {
  const bool open = gate_open(d.gate);  // consulted before the stores only
  __shared__ double sred[4], sred2[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int row = blockIdx.x * 4 + wv;
  double acc = 0.0;
  if (row < d.rows && d.cid) {
    // class operand: the same element pairs and summation order as the matrix form below (lane
    // c takes columns 2c, 2c+1), the pair's two ids in one 8-B load, their values gathered from
    // the class table (L2-resident); ids first, then values, then the FMAs
    const int2* ids = reinterpret_cast<const int2*>(d.cid + (size_t)row * d.lda);
    const double2* xv = reinterpret_cast<const double2*>(d.x);
    const int n2 = d.p >> 1;
    auto val = [&](int u, int col) {
      double v = u >= 0 ? d.cv[u] : 0.0;
      if (col == row) v = u >= 0 ? (d.ident ? v + d.cdiag : v) : (d.ident ? 1.0 : 0.0);
      return v;
    };
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    int c = lane;
    if ((n2 & 255) == 0) {
      // whole 256-pair groups: up to 4 groups (16 pairs per lane) per batch -- every id load of
      // the batch, then every value gather, then the FMAs in the loop below's order (two memory
      // round trips per batch instead of two per group)
      for (; c < n2; c += 1024) {
        const int ng = min(4, (n2 - (c - lane)) >> 8);  // (uniform)
        int2 iv[16];
        double2 bv[16], av[16];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (g < ng)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              iv[4 * g + u] = ids[c + 256 * g + 64 * u];
              bv[4 * g + u] = xv[c + 256 * g + 64 * u];
            }
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (g < ng)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int col = 2 * (c + 256 * g + 64 * u);
              av[4 * g + u] = make_double2(val(iv[4 * g + u].x, col), val(iv[4 * g + u].y, col + 1));
            }
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (g < ng)
#pragma unroll
            for (int u = 0; u < 4; ++u)
              s[u] = fma(av[4 * g + u].y, bv[4 * g + u].y, fma(av[4 * g + u].x, bv[4 * g + u].x, s[u]));
      }
    }
    for (; c + 192 < n2; c += 256) {
      int2 iv[4];
      double2 bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        iv[u] = ids[c + 64 * u];
        bv[u] = xv[c + 64 * u];
      }
      double2 av[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int col = 2 * (c + 64 * u);
        av[u] = make_double2(val(iv[u].x, col), val(iv[u].y, col + 1));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] = fma(av[u].y, bv[u].y, fma(av[u].x, bv[u].x, s[u]));
    }
    for (; c < n2; c += 64) {
      const int2 iv = ids[c];
      const double2 bv = xv[c];
      const double ax = val(iv.x, 2 * c), ay = val(iv.y, 2 * c + 1);
      s[0] = fma(ay, bv.y, fma(ax, bv.x, s[0]));
    }
    acc = (s[0] + s[1]) + (s[2] + s[3]);
  } else if (row < d.rows) {
    // 16-B loads (p and lda are multiples of 32), 8 per lane in flight before the FMAs, four
    // independent partial sums (a serial chain held one load round trip per 64 columns)
    const double2* a = reinterpret_cast<const double2*>(d.A + (size_t)row * d.lda);
    const double2* xv = reinterpret_cast<const double2*>(d.x);
    const int n2 = d.p >> 1;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    int c = lane;
    for (; c + 192 < n2; c += 256) {
      double2 av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = a[c + 64 * u];
        bv[u] = xv[c + 64 * u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] = fma(av[u].y, bv[u].y, fma(av[u].x, bv[u].x, s[u]));
    }
    for (; c < n2; c += 64) {
      const double2 av = a[c], bv = xv[c];
      s[0] = fma(av.y, bv.y, fma(av.x, bv.x, s[0]));
    }
    acc = (s[0] + s[1]) + (s[2] + s[3]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  double part = 0.0, part2 = 0.0;
  if (lane == 0 && row < d.rows) {
    double y = d.alpha * acc;
    if (d.beta != 0.0) y += d.beta * d.C0[row];
    if (d.epi == EPI_RESID) {
      y -= d.F[row];
      if (d.ac) {
        const double u = d.U[row] + (d.U0 ? d.U0[row] : 0.0);
        y += u * (u * u - 1.0);
      }
      part = y * y;
    } else if (d.epi == EPI_QUAD) {
      part = y * d.U[row];
    }
    if (d.red2) part2 = d.Q1[row] * d.Q2[row];
    if (open) d.y[row] = y;
  }
  if (d.red || d.red2) {
    if (lane == 0) {
      sred[wv] = part;
      sred2[wv] = part2;
    }
    __syncthreads();
    if (t == 0 && d.red) d.red[blockIdx.x] = (sred[0] + sred[1]) + (sred[2] + sred[3]);
    if (t == 0 && d.red2) d.red2[blockIdx.x] = (sred2[0] + sred2[1]) + (sred2[2] + sred2[3]);
  }
}

int gemv_blocks(int rows) { return (rows + 3) / 4; }

hipError_t launch_gemv(const GemvDesc& d, hipStream_t s) {
  hipLaunchKernelGGL(gemv_kernel, dim3(gemv_blocks(d.rows)), dim3(256), 0, s, d);
  return hipGetLastError();
}

}  // namespace gpk
