// assemble.hip — fused covariance + derivative-covariance block assembly (gfx950).
//
// Replaces, per axis and per step,
//   K  = vmap(kappa)(X1, X2) + jitter*I         code/kernel_matrix.py:21-30
//   D  = vmap(DD_x1_kappa) or vmap(D_x1_kappa)  code/model_GP_solver_2d.py:107-117,
//                                               code/model_GP_solver_advection.py:107-117
// with closed-form fields instead of nested jax.grad.
//
// Design: d = |x_i - x_j| is exactly symmetric, so K and DD are bitwise symmetric and D_x1
// bitwise antisymmetric.  Only the LOWER tile triangle is evaluated and every element is
// written twice (direct + mirror): half the exp/sincos work of a full sweep.  The Q mixture
// components of one element are spread over 4 waves (latency: a 256x256 factor pair is
// ~1150 workgroups) and summed in fixed order through LDS; per-axis constants (w, a, 2*pi*f)
// sit in LDS.  Pads (i or j >= n) are written as identity (K) / zero (D) so the padded SPD
// inverse stays block-diagonal.
#include <algorithm>

#include "gpk_internal.h"
#include "spd_pivot.h"
#include "gpk_trace.h"
#include "prep_dev.h"

namespace gpk {

GPK_WAIT_LIMIT_SETTER(wait_limit_assemble)  // gpk_set_wait_limit

GPK_TRACE_TU(assemble)

// (eval_kd_part, class_value_store: prep_dev.h, shared with the pipelined class values of the
// parameter-gradient launch)

template <bool MATERN, bool COS, int DERIV>
__device__ __forceinline__ void eval_kd(double diff, const double* w, const double* a,
                                        const double* om, const double* oml, int q, double& K,
                                        double& D) {
  eval_kd_part<MATERN, COS, DERIV>(diff, w, a, om, oml, 0, 1, q, K, D);
  // JAX abs JVP: select(x >= 0, g, -g) -> sign(0) = +1
  if (DERIV == 1 && !(diff >= 0.0)) D = -D;
}

constexpr int ASM_SUB = 16;  // workgroups per 32x32 tile: 64 elements (2 rows) each

struct AssembleBatch {
  AssembleArgs ax[2];
  int tiles[2];   // lower-triangle tile count per axis
  int pivot_x;    // blockIdx.x of the pivot-0 workgroup (per axis), or -1
  PrepArgs prep;
};

// Pivot block 0 (rows/cols 0..31) of the SPD inverse, factored inside the assembly launch by
// one extra workgroup per axis.  The 16 workgroups that assemble tile (0,0) release their rows
// (vmcnt drain, agent release, counter add); the pivot workgroup polls (sc1), acquires,
// reads the tile and runs the Cholesky + L^{-1} of pivot_init.  It is dispatched after those
// 16 (highest blockIdx.x), so they are resident or done: no deadlock at any grid size.
__device__ void pivot0(const AssembleArgs& A, unsigned need) {
  __shared__ double P[32 * SP], M[32 * SP], pv[32];
  const int t = threadIdx.x;
  if (t == 0) {
    (void)spin_until_ge<1>(A.flag, need, A.status);  // bounded: status bit 2 on a lost hand-off
    *A.flag = 0u;  // re-arm for the next step (no other user until then)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // see the released tile rows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (blockIdx.x == 0) TR_HI(SLOT_PIVOT0_WAIT);
  }
  __syncthreads();
  for (int e = t; e < 1024; e += 256) P[(e >> 5) * SP + (e & 31)] = A.K[(size_t)(e >> 5) * A.p + (e & 31)];
  __syncthreads();
  const double k00 = P[0];
  if (t == 0 && blockIdx.x == 0) TR_LO(SLOT_PIVOT0);
  const double ls = pivot_chol_inv_block(P, M, pv, t, A.status);  // (four-wave form: the one-wave
  // form's accumulators cost gather_kernel, an HBM-bound launch, one wave per SIMD of occupancy)
  if (t == 0 && blockIdx.x == 0) TR_HI(SLOT_PIVOT0);
  for (int e = t; e < 1024; e += 256) A.piv[e] = M[(e >> 5) * SP + (e & 31)];
  if (t == 0) {
    A.ldet[0] = ls;
    A.pst[0] = k00;   // refinement gate: K_00
    A.pst[1] = 0.0;   // max diag K^{-1}, atomicMax'd by the last sweep
  }
}

template <bool MATERN, bool COS, int DERIV>
__global__ __launch_bounds__(256) void assemble_kernel(AssembleBatch b, int q) {
  const int axis = blockIdx.y;
  const AssembleArgs& A = b.ax[axis];
  const int t = threadIdx.x;
  const bool pivot_wg = (int)blockIdx.x == b.pivot_x;
  const int tile = blockIdx.x / ASM_SUB, sub = blockIdx.x % ASM_SUB;
  if (!pivot_wg && tile >= b.tiles[axis]) return;
  // tile (0,0) feeds the pivot-0 workgroup, the critical path of the launch: its waves get
  // issue priority over the other ~4 waves sharing each SIMD
  if (b.pivot_x >= 0 && (tile == 0 || pivot_wg)) __builtin_amdgcn_s_setprio(3);

  __shared__ double sw[QMAX], sa[QMAX], so[QMAX], sol[QMAX];
  __shared__ double pk[4][64], pd[4][64];
  if (t < q) axis_component(b.prep, axis, q, t, sw[t], sa[t], so[t], sol[t]);
  if (blockIdx.x == 0 && axis == 0) publish_prep(b.prep, q);
  __syncthreads();
  if (pivot_wg) {
    pivot0(A, ASM_SUB);
    return;
  }
  int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= tile) ++I;
  while (I * (I + 1) / 2 > tile) --I;
  const int J = tile - I * (I + 1) / 2;
  const int e = t & 63, g = t >> 6;
  const int i = I * 32 + 2 * sub + (e >> 5), j = J * 32 + (e & 31);
  const bool real = i < A.n && j < A.n;
  double diff = 0.0, kv = 0.0, dv = 0.0;
  if (real) {
    diff = A.x[i] - A.x[j];
    eval_kd_part<MATERN, COS, DERIV>(diff, sw, sa, so, sol, g, 4, q, kv, dv);
  }
  pk[g][e] = kv;
  pd[g][e] = dv;
  __syncthreads();
  if (g != 0) return;
  if (real) {
    kv = (pk[0][e] + pk[1][e]) + (pk[2][e] + pk[3][e]);
    dv = (pd[0][e] + pd[1][e]) + (pd[2][e] + pd[3][e]);
    if (i == j) kv += A.jitter;
  } else {
    kv = (i == j) ? 1.0 : 0.0;  // padded block is the identity
    dv = 0.0;
  }
  const double s_ij = (diff >= 0.0) ? 1.0 : -1.0;         // JAX abs'(0) = +1
  const double s_ji = (-diff >= 0.0) ? 1.0 : -1.0;
  A.K[(size_t)i * A.p + j] = kv;
  if (A.Kc) A.Kc[(size_t)i * A.p + j] = kv;
  if (DERIV == 2) A.D[(size_t)i * A.p + j] = dv;
  if (DERIV == 1) A.D[(size_t)i * A.p + j] = real ? s_ij * dv : 0.0;
  if (I != J) {
    A.K[(size_t)j * A.p + i] = kv;
    if (A.Kc) A.Kc[(size_t)j * A.p + i] = kv;
    if (DERIV == 2) A.D[(size_t)j * A.p + i] = dv;
    if (DERIV == 1) A.D[(size_t)j * A.p + i] = real ? s_ji * dv : 0.0;
  }
  if (tile == 0 && b.pivot_x >= 0) {  // release this sub-block of tile (0,0) to pivot0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (only wave 0 stored)
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicAdd(A.flag, 1u);
    }
  }
}

// ---- class path (gpk_internal.h ClassArgs) -------------------------------------------------
// Launch 1: kappa and its derivative field at every class distance.  One mixture component per
// lane: half-wave h of wave w holds class 8*blockIdx.x + 2w + h, lane c its component c (and
// c + 32, ...); the 32 terms are added by a fixed xor-butterfly (deterministic).  The latency
// of one exp + sincos instead of q/4 of them in sequence.  Workgroup (0, 0) also publishes the
// step constants (prep).
template <bool MATERN, bool COS, int DERIV>
__global__ __launch_bounds__(256) void class_eval_kernel(AssembleBatch b, int q) {
  const int axis = blockIdx.y;
  const ClassArgs& C = b.ax[axis].cls;
  const int t = threadIdx.x;
  __shared__ double sw[QMAX], sa[QMAX], so[QMAX], sol[QMAX];
  if (t < q) axis_component(b.prep, axis, q, t, sw[t], sa[t], so[t], sol[t]);
  if (blockIdx.x == 0 && axis == 0) publish_prep(b.prep, q, false);
  // the boundary gap's parts, one per workgroup of axis 0 (strided: every part is written
  // whatever the grid's width)
  if (axis == 0 && !b.prep.skip && b.prep.bgap)
    for (int w = blockIdx.x; w < b.prep.bgap_parts; w += gridDim.x) bgap_part(b.prep, w);
  __syncthreads();
  if (TR_FIRST) TR_LO(SLOT_CLASS_EVAL);
  if (TR_LAST) TR_LO(SLOT_CEVAL_START);
  const int u = blockIdx.x * 8 + (t >> 5);
  class_value_store<MATERN, COS, DERIV>(C, u, u < C.ncls ? C.dist[u] : 0.0, sw, sa, so, sol, q);
  if (TR_FIRST) TR_HI(SLOT_CLASS_EVAL);
  if (TR_LAST) TR_HI(SLOT_CEVAL_START);
}

// Launch 2: K (+ jitter), its kept copy and D of one 32x32 tile per workgroup, gathered from
// the class values (pads: identity / zero); the workgroup of tile (0, 0) releases it to the
// pivot-0 workgroup (the last one of the grid), which factors it as in assemble_kernel.
// grid (naxes, 1 + tiles [+ 1]): dispatch order = tile (0,0) of every axis, the pivot workgroups
// (which wait for it: dispatched after it, so no deadlock), then the other tiles.
template <int DERIV>
__global__ __launch_bounds__(256) void gather_kernel(AssembleBatch b) {
  const int axis = blockIdx.x;
  const AssembleArgs& A = b.ax[axis];
  const int t = threadIdx.x;
  if (TR_LAST) TR_LO(SLOT_GATHER_START);
  const bool piv = b.pivot_x >= 0;
  if (piv && blockIdx.y == 1) {
    if (t == 0 && axis == 0) TR_LO(SLOT_GATHER);
    pivot0(A, 1u);
    if (t == 0 && axis == 0) TR_HI(SLOT_GATHER);
    return;
  }
  const int T = A.p / 32;
  const int tile = (piv && blockIdx.y > 1) ? (int)blockIdx.y - 1 : (int)blockIdx.y;
  if (tile >= T * T) return;
  if (tile == 0 && b.pivot_x >= 0) __builtin_amdgcn_s_setprio(3);
  const int I = tile / T, J = tile % T;
  const int j = J * 32 + (t & 31);
  const ClassArgs& C = b.ax[axis].cls;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = I * 32 + (t >> 5) + 8 * r;
    const size_t o = (size_t)i * A.p + j;
    const int u = C.cid[o];
    double kv, dv;
    if (u >= 0) {
      kv = C.kval[u];
      if (i == j) kv += A.jitter;
      dv = C.dval[u];
      if (DERIV == 1 && !(A.x[i] - A.x[j] >= 0.0)) dv = -dv;  // JAX abs'(0) = +1
    } else {
      kv = (i == j) ? 1.0 : 0.0;
      dv = 0.0;
    }
    A.K[o] = kv;
    if (A.Kc) A.Kc[o] = kv;
    if (DERIV) A.D[o] = dv;
  }
  if (tile == 0 && b.pivot_x >= 0) {  // release tile (0, 0) to pivot0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicAdd(A.flag, 1u);
    }
  }
  if (TR_LAST) TR_HI(SLOT_GATHER_START);
}

// Launch 2, large factors (no pivot-0 workgroup: the large-factor inverse factors its own
// pivots): the same element values as gather_kernel, laid out for HBM streaming -- a workgroup
// covers 8 rows x 512 columns, each lane two adjacent columns (8-B class-id pairs in, 16-B K / Kc /
// D pairs out, whole 1-KiB row segments per wave instruction), all 8 of a lane's class-id loads
// issued before its gathers and stores (memory-level parallelism), nontemporal stores.  C5 (two
// 4096^2 factors): 940 MB per launch (K, Kc, D written, the ids read).
// GW_H row pairs of 4 per workgroup (one row per wave and pair): 16 rows x 512 columns, every
// class id of the block loaded in one batch (16 int2 per thread) before the dependent class-value
// loads.  In a step the ids come from HBM -- the memory-side cache holds the previous kernels'
// lines, not the ids -- and with 8 rows per workgroup the launch ran at half its back-to-back
// rate (a pure write stream of the same bytes does not slow down: profiles/r4_gather_context.txt)
constexpr int GW_H = 4, GW_ROWS = 4 * GW_H, GW_COLS = 512;
constexpr int GW_WIDE_MIN_TILES = 1024;  // 32x32 tiles: P >= 1024
struct GwIds {  // one block's class ids of a lane: variant bytes (2 columns) + their cbase entries
  unsigned short v[GW_H][4];
  int2 cb[GW_H][4];
};
// Persistent: GW_WGS workgroups walk the blocks (axis, row block, column block) with a stride of
// the grid, and each issues the NEXT block's class ids before it gathers and stores the current
// one, so the store stream does not stall on the id loads' HBM latency.
constexpr int GW_WGS = 2048;
template <int DERIV>
__global__ __launch_bounds__(256) void gather_wide_kernel(AssembleBatch b, int nbx, int nby, int nblk) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // block -> (axis, r0, c0); false past the shorter axis
  auto where = [&](int blk, int& axis, int& r0, int& c0) -> bool {
    axis = blk / (nbx * nby);
    const int rem = blk - axis * nbx * nby;
    r0 = (rem / nbx) * GW_ROWS;
    c0 = (rem % nbx) * GW_COLS;
    const int p = axis ? b.ax[1].p : b.ax[0].p;
    return r0 < p && c0 < p;
  };
  // A pair's class is cbase[|i - j|] + its variant byte: the 2 bytes of a lane's column pair and
  // the two cbase entries (n + 1 ints, cache-resident) are loaded together, the class values
  // after them -- the id stream from HBM is 2 bytes per pair instead of round 4's 4-byte class
  // ids (C5: 33 MB per gather instead of 134 MB)
  auto load_ids = [&](GwIds& id, int axis, int r0, int c0) {
    const ClassArgs& C = axis ? b.ax[1].cls : b.ax[0].cls;
    const int p = axis ? b.ax[1].p : b.ax[0].p, n = axis ? b.ax[1].n : b.ax[0].n;
#pragma unroll
    for (int h = 0; h < GW_H; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = c0 + 128 * q + 2 * lane, i = r0 + w + 4 * h;
        const bool in = col < p;
        id.v[h][q] = in ? *reinterpret_cast<const unsigned short*>(C.vidx + (size_t)i * p + col) : 0xffff;
        const int k0 = min(abs(i - col), n - 1), k1 = min(abs(i - col - 1), n - 1);
        id.cb[h][q] = make_int2(C.cbase[k0], C.cbase[k1]);
      }
  };
  auto process = [&](const GwIds& ids, int axis, int r0, int c0) {
    const AssembleArgs& A = axis ? b.ax[1] : b.ax[0];
    const double* kval = A.cls.kval;
    const double* dval = A.cls.dval;
    const int p = A.p;
    int row[GW_H], col[4];
#pragma unroll
    for (int h = 0; h < GW_H; ++h) row[h] = r0 + w + 4 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q) col[q] = c0 + 128 * q + 2 * lane;
    double xi[GW_H] = {};
    double2 xj[4];
    if (DERIV == 1) {
#pragma unroll
      for (int h = 0; h < GW_H; ++h) xi[h] = A.x[min(row[h], A.n - 1)];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        xj[q] = make_double2(A.x[min(col[q], A.n - 1)], A.x[min(col[q] + 1, A.n - 1)]);
    }
#pragma unroll
    for (int h = 0; h < GW_H; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (col[q] >= p) continue;
        const int i = row[h];
        double kv[2], dv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int vb = (ids.v[h][q] >> (8 * e)) & 0xff;
          const int u = vb == 0xff ? -1 : (e == 0 ? ids.cb[h][q].x : ids.cb[h][q].y) + vb, j = col[q] + e;
          if (u >= 0) {
            kv[e] = kval[u];
            if (i == j) kv[e] += A.jitter;
            dv[e] = dval[u];
            if (DERIV == 1) {
              const double xjj = e == 0 ? xj[q].x : xj[q].y;
              if (!(xi[h] - xjj >= 0.0)) dv[e] = -dv[e];  // JAX abs'(0) = +1
            }
          } else {
            kv[e] = (i == j) ? 1.0 : 0.0;
            dv[e] = 0.0;
          }
        }
        // nontemporal stores: 3.4 -> 7.0 TB/s at C5 size (tools/probes/gather_probe.hip; write-
        // allocating stores held the launch at 3.4-3.7 TB/s whatever the layout); the next readers
        // (the inverse, the GEMMs) run on other XCDs and read from memory anyway
        // (one 16-B store per array and lane: per-element stores interleaved across the arrays
        // were not merged and ran at 1.9 TB/s)
        typedef double d2v __attribute__((ext_vector_type(2)));
        const size_t o = (size_t)i * p + col[q];
        const d2v k2 = {kv[0], kv[1]}, d2 = {dv[0], dv[1]};
        __builtin_nontemporal_store(k2, reinterpret_cast<d2v*>(A.K + o));
        if (A.Kc) __builtin_nontemporal_store(k2, reinterpret_cast<d2v*>(A.Kc + o));
        if (DERIV) __builtin_nontemporal_store(d2, reinterpret_cast<d2v*>(A.D + o));
      }
  };
  GwIds ida, idb;
  int blk = blockIdx.x, ax, r0, c0;
  while (blk < nblk && !where(blk, ax, r0, c0)) blk += gridDim.x;
  if (blk >= nblk) return;
  load_ids(ida, ax, r0, c0);
  for (;;) {  // two blocks per trip: the id arrays alternate (registers, not indexed)
    int nb = blk + gridDim.x, ax2 = 0, r2 = 0, c2 = 0;
    while (nb < nblk && !where(nb, ax2, r2, c2)) nb += gridDim.x;
    if (nb < nblk) load_ids(idb, ax2, r2, c2);
    process(ida, ax, r0, c0);
    if (nb >= nblk) return;
    blk = nb; ax = ax2; r0 = r2; c0 = c2;
    nb = blk + gridDim.x;
    while (nb < nblk && !where(nb, ax2, r2, c2)) nb += gridDim.x;
    if (nb < nblk) load_ids(ida, ax2, r2, c2);
    process(idb, ax, r0, c0);
    if (nb >= nblk) return;
    blk = nb; ax = ax2; r0 = r2; c0 = c2;
  }
}

static hipError_t launch_gather_wide(const AssembleBatch& b, int naxes, int deriv, hipStream_t s) {
  // every axis needs its variant bytes (gpk_create builds them for all axes once max P >= 1024);
  // an axis without them would be left unassembled, so refuse the launch
  for (int k = 0; k < naxes; ++k)
    if (!b.ax[k].cls.vidx) return hipErrorInvalidValue;
  int pmax = 0;
  for (int k = 0; k < naxes; ++k) pmax = std::max(pmax, b.ax[k].p);
  const int nbx = (pmax + GW_COLS - 1) / GW_COLS, nby = (pmax + GW_ROWS - 1) / GW_ROWS, nblk = nbx * nby * naxes;
  const dim3 g(std::min(nblk, GW_WGS));
  if (deriv == 2) hipLaunchKernelGGL((gather_wide_kernel<2>), g, dim3(256), 0, s, b, nbx, nby, nblk);
  else if (deriv == 1) hipLaunchKernelGGL((gather_wide_kernel<1>), g, dim3(256), 0, s, b, nbx, nby, nblk);
  else hipLaunchKernelGGL((gather_wide_kernel<0>), g, dim3(256), 0, s, b, nbx, nby, nblk);
  return hipSuccess;
}

template <bool MATERN, bool COS>
static hipError_t launch_class_t(const AssembleBatch& b, int naxes, int maxc, int maxtiles, int q,
                           int deriv, hipStream_t s, bool eval_only) {
  dim3 ge((maxc + 7) / 8, naxes), gg(naxes, maxtiles + (b.pivot_x >= 0 ? 1 : 0));
  // (no pivot-0 workgroup and large tiles: the streaming layout)
  const bool wide = b.pivot_x < 0 && maxtiles >= GW_WIDE_MIN_TILES;
  if (deriv == 2) {
    hipLaunchKernelGGL((class_eval_kernel<MATERN, COS, 2>), ge, dim3(256), 0, s, b, q);
    if (!eval_only && !wide) hipLaunchKernelGGL((gather_kernel<2>), gg, dim3(256), 0, s, b);
  } else if (deriv == 1) {
    hipLaunchKernelGGL((class_eval_kernel<MATERN, COS, 1>), ge, dim3(256), 0, s, b, q);
    if (!eval_only && !wide) hipLaunchKernelGGL((gather_kernel<1>), gg, dim3(256), 0, s, b);
  } else {
    hipLaunchKernelGGL((class_eval_kernel<MATERN, COS, 0>), ge, dim3(256), 0, s, b, q);
    if (!eval_only && !wide) hipLaunchKernelGGL((gather_kernel<0>), gg, dim3(256), 0, s, b);
  }
  if (!eval_only && wide) return launch_gather_wide(b, naxes, deriv, s);
  return hipSuccess;
}

// the gather launch alone (gpk_bench_kernel "gather": the K-assembly kernel's HBM rate); the
// class values must be current (a class_eval launch ran since the parameters last changed)
hipError_t launch_gather_only(const AssembleArgs* a, int naxes, hipStream_t s) {
  AssembleBatch b{};
  int maxtiles = 0;
  for (int k = 0; k < naxes; ++k) {
    b.ax[k] = a[k];
    if (a[k].piv || a[k].cls.ncls <= 0) return hipErrorInvalidValue;
    maxtiles = std::max(maxtiles, (a[k].p / 32) * (a[k].p / 32));
  }
  b.pivot_x = -1;
  if (maxtiles >= GW_WIDE_MIN_TILES) {  // (what launch_assemble runs at this size)
    const hipError_t e = launch_gather_wide(b, naxes, a[0].deriv, s);
    return e != hipSuccess ? e : hipGetLastError();
  }
  dim3 gg(naxes, maxtiles);
  if (a[0].deriv == 2) hipLaunchKernelGGL((gather_kernel<2>), gg, dim3(256), 0, s, b);
  else if (a[0].deriv == 1) hipLaunchKernelGGL((gather_kernel<1>), gg, dim3(256), 0, s, b);
  else hipLaunchKernelGGL((gather_kernel<0>), gg, dim3(256), 0, s, b);
  return hipGetLastError();
}

// rectangular block (preds' Kmn, gpk_kernel_matrices): no symmetry assumed
template <bool MATERN, bool COS, int DERIV>
__global__ __launch_bounds__(256) void cross_kernel(const double* __restrict__ xr, int nr,
                                                    const double* __restrict__ xc, int nc, int ld,
                                                    const AxisConst* kc, int q, double jitter,
                                                    double* K, double* D) {
  __shared__ double sw[QMAX], sa[QMAX], so[QMAX], sol[QMAX];
  const int t = threadIdx.x;
  if (t < q) {
    sw[t] = kc->w[t];
    sa[t] = kc->a[t];
    so[t] = kc->om[t];
    sol[t] = kc->oml[t];
  }
  __syncthreads();
  const int j = blockIdx.x * 64 + (t & 63);
  const int i = blockIdx.y * 4 + (t >> 6);
  if (i >= nr || j >= nc) return;
  double kv, dv;
  eval_kd<MATERN, COS, DERIV>(xr[i] - xc[j], sw, sa, so, sol, q, kv, dv);
  if (i == j) kv += jitter;
  K[(size_t)i * ld + j] = kv;
  if (DERIV) D[(size_t)i * ld + j] = dv;
}

// elementwise pairs: out[e] = kappa / D_x1 / DD_x1 at (x1[e], x2[e]) -- vmap(kappa) semantics
template <bool MATERN, bool COS, int DERIV>
__global__ __launch_bounds__(256) void pairs_kernel(const double* __restrict__ x1,
                                                    const double* __restrict__ x2, long n,
                                                    const AxisConst* kc, int q, double* out) {
  __shared__ double sw[QMAX], sa[QMAX], so[QMAX], sol[QMAX];
  const int t = threadIdx.x;
  if (t < q) {
    sw[t] = kc->w[t];
    sa[t] = kc->a[t];
    so[t] = kc->om[t];
    sol[t] = kc->oml[t];
  }
  __syncthreads();
  const long e = (long)blockIdx.x * 256 + t;
  if (e >= n) return;
  double kv, dv;
  eval_kd<MATERN, COS, DERIV>(x1[e] - x2[e], sw, sa, so, sol, q, kv, dv);
  out[e] = DERIV ? dv : kv;
}

template <bool MATERN, bool COS>
static void launch_pairs_t(const double* x1, const double* x2, long n, const AxisConst* kc, int q,
                           int deriv, double* out, hipStream_t s) {
  dim3 grid((unsigned)((n + 255) / 256));
  if (deriv == 2)
    hipLaunchKernelGGL((pairs_kernel<MATERN, COS, 2>), grid, dim3(256), 0, s, x1, x2, n, kc, q, out);
  else if (deriv == 1)
    hipLaunchKernelGGL((pairs_kernel<MATERN, COS, 1>), grid, dim3(256), 0, s, x1, x2, n, kc, q, out);
  else
    hipLaunchKernelGGL((pairs_kernel<MATERN, COS, 0>), grid, dim3(256), 0, s, x1, x2, n, kc, q, out);
}

hipError_t launch_pairs(int kind, int q, const double* x1, const double* x2, long n,
                        const AxisConst* kc, int deriv, double* out, hipStream_t s) {
  switch (kind) {
    case SE_COS: launch_pairs_t<false, true>(x1, x2, n, kc, q, deriv, out, s); break;
    case MATERN52_COS: launch_pairs_t<true, true>(x1, x2, n, kc, q, deriv, out, s); break;
    case SE: launch_pairs_t<false, false>(x1, x2, n, kc, q, deriv, out, s); break;
    default: launch_pairs_t<true, false>(x1, x2, n, kc, q, deriv, out, s); break;
  }
  return hipGetLastError();
}

template <bool MATERN, bool COS>
static void launch_assemble_t(const AssembleBatch& b, int naxes, int maxt, int q, int deriv,
                              hipStream_t s) {
  dim3 grid(maxt * ASM_SUB + (b.pivot_x >= 0 ? 1 : 0), naxes);
  if (deriv == 2)
    hipLaunchKernelGGL((assemble_kernel<MATERN, COS, 2>), grid, dim3(256), 0, s, b, q);
  else if (deriv == 1)
    hipLaunchKernelGGL((assemble_kernel<MATERN, COS, 1>), grid, dim3(256), 0, s, b, q);
  else
    hipLaunchKernelGGL((assemble_kernel<MATERN, COS, 0>), grid, dim3(256), 0, s, b, q);
}

hipError_t launch_assemble(int kind, int q, const AssembleArgs* a, int naxes, const PrepArgs& prep,
                           hipStream_t s, bool eval_only) {
  AssembleBatch b{};
  int maxt = 0;
  for (int k = 0; k < naxes; ++k) {
    b.ax[k] = a[k];
    int T = a[k].p / 32;
    b.tiles[k] = T * (T + 1) / 2;
    if (b.tiles[k] > maxt) maxt = b.tiles[k];
  }
  b.prep = prep;
  for (int k = 1; k < naxes; ++k)
    if ((a[k].piv != nullptr) != (a[0].piv != nullptr) ||
        (a[k].cls.ncls > 0) != (a[0].cls.ncls > 0))
      return hipErrorInvalidValue;
  int deriv = a[0].deriv;
  if (a[0].cls.ncls > 0) {  // class path: every 32x32 tile of the full matrix, one per workgroup
    int maxc = 0, maxtiles = 0;
    for (int k = 0; k < naxes; ++k) {
      const int T = a[k].p / 32;
      maxtiles = std::max(maxtiles, T * T);
      maxc = std::max(maxc, a[k].cls.ncls);
    }
    b.pivot_x = a[0].piv ? maxtiles : -1;
    hipError_t e;
    switch (kind) {
      case SE_COS: e = launch_class_t<false, true>(b, naxes, maxc, maxtiles, q, deriv, s, eval_only); break;
      case MATERN52_COS: e = launch_class_t<true, true>(b, naxes, maxc, maxtiles, q, deriv, s, eval_only); break;
      case SE: e = launch_class_t<false, false>(b, naxes, maxc, maxtiles, q, deriv, s, eval_only); break;
      default: e = launch_class_t<true, false>(b, naxes, maxc, maxtiles, q, deriv, s, eval_only); break;
    }
    return e != hipSuccess ? e : hipGetLastError();
  }
  b.pivot_x = a[0].piv ? maxt * ASM_SUB : -1;
  switch (kind) {
    case SE_COS: launch_assemble_t<false, true>(b, naxes, maxt, q, deriv, s); break;
    case MATERN52_COS: launch_assemble_t<true, true>(b, naxes, maxt, q, deriv, s); break;
    case SE: launch_assemble_t<false, false>(b, naxes, maxt, q, deriv, s); break;
    default: launch_assemble_t<true, false>(b, naxes, maxt, q, deriv, s); break;
  }
  return hipGetLastError();
}

template <bool MATERN, bool COS>
static void launch_cross_t(const double* xr, int nr, const double* xc, int nc, int ld,
                           const AxisConst* kc, int q, double jitter, int deriv, double* K,
                           double* D, hipStream_t s) {
  dim3 grid((nc + 63) / 64, (nr + 3) / 4);
  if (deriv == 2)
    hipLaunchKernelGGL((cross_kernel<MATERN, COS, 2>), grid, dim3(256), 0, s, xr, nr, xc, nc, ld,
                       kc, q, jitter, K, D);
  else if (deriv == 1)
    hipLaunchKernelGGL((cross_kernel<MATERN, COS, 1>), grid, dim3(256), 0, s, xr, nr, xc, nc, ld,
                       kc, q, jitter, K, D);
  else
    hipLaunchKernelGGL((cross_kernel<MATERN, COS, 0>), grid, dim3(256), 0, s, xr, nr, xc, nc, ld,
                       kc, q, jitter, K, D);
}

hipError_t launch_cross(int kind, int q, const double* xr, int nr, const double* xc, int nc,
                        int ld, const AxisConst* kc, double jitter, int deriv, double* K,
                        double* D, hipStream_t s) {
  switch (kind) {
    case SE_COS: launch_cross_t<false, true>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
    case MATERN52_COS: launch_cross_t<true, true>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
    case SE: launch_cross_t<false, false>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
    default: launch_cross_t<true, false>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
  }
  return hipGetLastError();
}

}  // namespace gpk
