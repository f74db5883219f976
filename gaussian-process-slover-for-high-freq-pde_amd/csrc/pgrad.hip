// pgrad.hip — kernel-hyperparameter gradient contraction (gfx950).
//
// Replaces the reverse pass that jax.grad pushes through vmap(kappa) and
// vmap(grad(grad(kappa))) (code/kernel_matrix.py:26, :49-57; code/model_GP_solver_2d.py:179):
//
//   dL/dtheta_q = sum_ij G_K[i,j] dK_ij/dtheta_q + G_D[i,j] dD_ij/dtheta_q,
//   theta in {freq, log-ls, log-w},  G_K = dL/dK, G_D = dL/dD   
//
// The fields depend on d = |x_i - x_j| only, so each unordered pair is evaluated once with
// its mirror's weight folded in (D_x1's sign s_ij folded into the weight).  A workgroup
// stages 64 pairs (d, w_K, w_D) in LDS; thread (g = t>>5, q = t&31) walks every 8th pair for
// mixture component q, so each (pair, q) costs one exp + one sincos; 8-way LDS reduction at
// the end leaves 3*Q deterministic partials per workgroup (~1150 workgroups at N = 256).
//
// 2D mode reads materialised G_K / G_D tiles; 1D mode forms them on the fly from K^{-1} and
// the vectors alpha = K^{-1}u, beta = K^{-1}D^T R, R (model_GP_solver_1d.py:80-149):
//   G_K = c/2 K^{-1} - 1/2 alpha alpha^T - v beta alpha^T,   G_D = v R alpha^T.
#include <algorithm>

#include "gpk_internal.h"
#include "gpk_trace.h"
#include "fields_dd.h"
#include "spd_pivot.h"
#include "prep_dev.h"

namespace gpk {
GPK_TRACE_TU(pgrad)
GPK_WAIT_LIMIT_SETTER(wait_limit_pgrad)  // gpk_set_wait_limit
}  // namespace gpk
#define FIN_PROBE(slot) TR_HI(slot)  // finalize_body phases (gpk_trace.h)
#include "stepk_dev.h"

#ifndef GPK_PG_PAIRS
#define GPK_PG_PAIRS 64
#endif

namespace gpk {

constexpr int PAIRS = GPK_PG_PAIRS;  // pairs per workgroup (PAIRS/32 rows x 32 cols of a 32x32 tile)
constexpr int PG_SUB = 1024 / PAIRS;  // workgroups per tile

struct PGradBatch {
  PGradArgs ax[2];
  int tiles[2];
  int naxes, bpa;
  int shard_rank, shard_n;  // row-sharded step: this rank contracts pair tiles t % shard_n == rank
  TailArgs tail;
};

// Fused tail, run by every block of the gradient planes after its partial is stored: the last
// block of each group of `tg` blocks sums the group's partials (block order), the last group
// sums the group partials (group order) into pg and runs finalize_body.  Cross-XCD hand-off per
// MI355X_MICROARCH.md §inter-workgroup visibility: producers store write-through (sc1), every
// storing wave drains (vmcnt 0), a barrier, then ONE lane's agent-scope ticket add; the block
// whose add came last (told by the value its add returned) reads every handed-off byte with sc1
// loads after a barrier -- the guide's sc1 row, no agent acquire (~1.7 us per level saved).
// No __threadfence() per block (its L2 write-back made this tail 4x slower).  Counters are
// re-armed by the blocks that consume them.
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store sc1
}

__device__ __forceinline__ bool arrive_last(unsigned int* counter, unsigned int n, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(counter, 1u);
    *s_flag = prev == n - 1u;
  }
  __syncthreads();
  return *s_flag != 0;
}

// (ld_wt, strided_sum, strided_sum_dd: stepk_dev.h, shared with finalize_body)

__device__ void pgrad_tail(const PGradBatch& b, int axis, int blk, int q) {
  const TailArgs& T = b.tail;
  __shared__ int s_last;
  const int t = threadIdx.x;
  const int gi = blk / T.tg;
  const int gsize = min(T.tg, b.bpa - gi * T.tg);
  if (t == 0 && blk == 0 && axis == 0) TR_HI(SLOT_PG_CONTRACT);
  if (t == 0 && blk == b.bpa - 1 && axis == b.naxes - 1) TR_HI(SLOT_PG_START);
  if (!arrive_last(T.gcount + axis * T.ngpa + gi, (unsigned)gsize, &s_last)) return;
  if (t == 0) {
    TR_LO(SLOT_PG_GARR);
    TR_HI(SLOT_PG_GARR);
  }
  const double* part = b.ax[axis].part;
  const double* part_lo = b.ax[axis].part_lo;
  for (int x = t; x < 3 * QMAX; x += 256) {
    const size_t go = (size_t)(axis * T.ngpa + gi) * (3 * QMAX) + x;
    if (T.gpart_lo) {  // DD: the group's partials summed in double-double
      dd::D acc = {0.0, 0.0};
      if ((x % QMAX) < q)
        acc = strided_sum_dd(part + (size_t)gi * T.tg * (3 * QMAX) + x,
                             part_lo + (size_t)gi * T.tg * (3 * QMAX) + x, 3 * QMAX, gsize);
      st_wt(T.gpart + go, acc.h);
      st_wt(T.gpart_lo + go, acc.l);
      continue;
    }
    double acc = 0.0;
    if ((x % QMAX) < q)
      acc = strided_sum(part + (size_t)gi * T.tg * (3 * QMAX) + x, 3 * QMAX, gsize);
    st_wt(T.gpart + go, acc);
  }
  if (t == 0) T.gcount[axis * T.ngpa + gi] = 0u;  // re-arm (no other user this step)
  if (t == 0) TR_HI(SLOT_PG_GROUP);
  if (!arrive_last(T.top, (unsigned)(b.naxes * T.ngpa), &s_last)) return;
  if (t == 0) TR_LO(SLOT_PG_TOP);
  if (t == 0) *T.top = 0u;
  if (t == 0) TR_HI(SLOT_PG_TOP);
  // the kernel-parameter gradients and Adam: each thread sums its own parameters' pg entries
  // from the group partials (FinalizeArgs::gpart, set by make_tail) together with its other
  // loads -- one round trip (the pg of every live entry used to be summed into global pg first,
  // then re-loaded)
  finalize_body(T.fin, 2);  // (the loss part ran at the start of the launch)
  if (t == 0) TR_HI(SLOT_PG_FINAL);
  if (T.nce_flag) {  // the updated kernel parameters (fin.kp_wt, sc1) -> the next step's class values
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave drains its sc1 stores
    __syncthreads();
    if (t == 0) __hip_atomic_store(T.nce_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Pipelined class values (TailArgs::nce_flag; gpk_api.cpp cls_pipe_ok): plane naxes + 2 + ax of
// the launch evaluates the NEXT step's class values of axis ax -- the same 8 classes per
// workgroup and the same code as class_eval_kernel (class_value_store), from the parameters the
// kernel-parameter Adam of this launch has just written: bitwise the values the next step's
// class-value launch would produce, which that step then skips.  These workgroups are the last
// of the grid: the block they wait for (the last contraction block to arrive) was dispatched
// before them and waits for none of them, so the wait cannot deadlock at any grid size.
template <bool MATERN, bool COS, int DERIV>
__device__ void next_class_values(const PGradBatch& b, int ax, int blk, int q) {
  const ClassArgs& C = b.ax[ax].cls;
  if (blk * 8 >= C.ncls) return;
  __shared__ double sw[QMAX], sa[QMAX], so[QMAX], sol[QMAX];
  const int t = threadIdx.x, u = blk * 8 + (t >> 5);
  const double d = u < C.ncls ? C.dist[u] : 0.0;  // (issued before the wait)
  // the guide's sc1 hand-off (no fences): thread 0 polls the flag with sc1 loads, the barrier,
  // then sc1 loads of the parameters the Adam block stored write-through
  if (t == 0) (void)spin_until_ge<1>(b.tail.nce_flag, 1u, b.tail.nce_status);  // bounded: status bit 2
  __syncthreads();
  if (t < q) {
    const Layout& L = b.tail.fin.L;
    const double* kp = b.tail.fin.kp_wt + ((ax == 0 ? L.off_kp[0] : L.off_kp[1]) - L.off_small);
    axis_component_v(ld_wt(kp + t), ld_wt(kp + q + t), ld_wt(kp + 2 * q + t), sw[t], sa[t], so[t], sol[t]);
  }
  __syncthreads();
  class_value_store<MATERN, COS, DERIV>(C, u, d, sw, sa, so, sol, q);
}

// ---- class path (gpk_internal.h ClassArgs) -------------------------------------------------
// Class sums over one row chunk: part[c][u] = sum_{(i,j) in u, i in chunk c} G_K[i,j] (and
// s_ij G_D[i,j] in the second half).  Workgroup (chunk c, band of 64 diagonals); lane = diagonal
// k.  At row r lane k reads the lower pair (r, r-k) and the upper pair (r, r+k): contiguous row
// segments across the wave (coalesced), and every ordered pair is read exactly once over the
// grid.  The 4 waves take interleaved rows, load 4 rows' operands before accumulating (memory-
// level parallelism), and keep V running sums per lane (one per distance variant of the lane's
// diagonal, selected branch-free); they add them into LDS in wave order: deterministic.
// LDSB: the running sums as lane-private LDS bins instead (dynamic LDS [4 waves][2][vb][64]):
// each pair is one ds_add_f64 per sum into its variant's bin -- O(1) per pair instead of the
// V-way select (grids with many variants per diagonal, C2: 17).  A lane adds only into its own
// bins, in program order, and the waves are added in the same fixed order: the same sums,
// bitwise, as the register form.
template <int V, int DERIV, bool MODE1D, bool LDSB = false>
__global__ __launch_bounds__(256) void class_sum_kernel(PGradBatch b,
                                                       const StepScalars* __restrict__ sc, int vb = 0) {
  const int axis = blockIdx.z, band = blockIdx.y, chunk = blockIdx.x;
  const PGradArgs& A = b.ax[axis];
  const ClassArgs& C = A.cls;
  const int n = A.n, p = A.p;
  if (band * 64 >= n || chunk >= C.nchunk) return;  // shorter axis
  // 1D (lower pairs only): a chunk whose rows all lie above the band's diagonals has no pair; its
  // partials stay the zeros they were allocated with (nobody else writes them), so the ~half of
  // the grid above the diagonal ends here instead of zeroing LDS bins and storing zeros
  if (MODE1D && min(n, chunk * C.rb + C.rb) - 1 < band * 64) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (TR_FIRST) TR_LO(SLOT_CLASS_SUM);
  if (TR_LAST) TR_LO(SLOT_CSUM_START);
  const int k = band * 64 + lane;
  const bool kv = k < n;
  const int cb = kv ? C.cbase[k] : 0;
  const int nvar = kv ? C.cbase[k + 1] - cb : 0;  // distance variants of this lane's diagonal
  const int r0 = chunk * C.rb, r1 = min(n, r0 + C.rb);
  // variants in use by any diagonal of this wave (wave-uniform): the running sums past it are
  // never selected, so the V-way select stops there (C2: V = 32 slots, 3-17 variants per band)
  int nvw = V;
  if constexpr (V > 16) {
    nvw = nvar;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nvw = max(nvw, __shfl_xor(nvw, o, 64));
    nvw = __builtin_amdgcn_readfirstlane(nvw);
  }
  double ak[LDSB ? 1 : V], ad[LDSB ? 1 : V];
#pragma unroll
  for (int x = 0; x < (LDSB ? 1 : V); ++x) ak[x] = ad[x] = 0.0;
  extern __shared__ double lbin[];
  double* mybin = lbin + (size_t)w * 2 * vb * 64;  // [2][vb][64] of this wave
  if constexpr (LDSB) {
    for (int x = 0; x < vb; ++x) {
      mybin[x * 64 + lane] = 0.0;
      mybin[(vb + x) * 64 + lane] = 0.0;
    }
  }
  double vs = 0.0, hc = 0.0;
  if (MODE1D) {
    vs = sc->v;
    hc = A.halfc;
  }
  // 8 ordered pairs per wave per pass (4 rows x lower / upper).  Addresses first, then every
  // load of the pass back to back (cid, then the G operands), then the sums: one memory round
  // trip per pass.  Out-of-range pairs load the clamped element (0, 0) and get v = -1, which
  // matches no variant (bit-masked: a select on the loaded value let LLVM sink the load into an
  // exec-masked branch behind a vmcnt(0) wait).
  // (4 rows per wave and pass, 8 pairs; 8 rows -- twice the loads per round trip -- measured
  // slower with the LDS bins: C2 30 -> 32 us, C4 3.5 -> 4.5 us)
  // 1D (MODE1D): K^{-1} is symmetric (its upper triangle mirrors the lower one) and so are the
  // class ids, so a class's pairs (i, j) and (j, i) are folded into one lower pair:
  // G_K(i,j) + G_K(j,i) = c K^{-1}_ij - a_i a_j - v (b_i a_j + b_j a_i), G_D likewise -- half the
  // loads and bin updates; 8 rows per wave and pass, 8 lower pairs.
  static_assert(!(MODE1D && DERIV == 1), "the 1D fold assumes a symmetric G_D sign");
  constexpr int RP = MODE1D ? 8 : 4, NP = 8;
  for (int base = r0; base < r1; base += 4 * RP) {
    int ii[NP], jj[NP], msk[NP];
    if (MODE1D) {
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        const int r = base + w + 4 * s;
        const bool lo = kv && r < r1 && r >= k;
        ii[s] = lo ? r : 0;
        jj[s] = lo ? r - k : 0;
        msk[s] = -(int)lo;
      }
    } else {
#pragma unroll
      for (int s = 0; s < RP; ++s) {
        const int r = base + w + 4 * s;
        const bool in = kv && r < r1;
        const bool lo = in && r >= k, up = in && k > 0 && r + k < n;
        ii[2 * s] = lo ? r : 0;
        jj[2 * s] = lo ? r - k : 0;
        msk[2 * s] = -(int)lo;
        ii[2 * s + 1] = up ? r : 0;
        jj[2 * s + 1] = up ? r + k : 0;
        msk[2 * s + 1] = -(int)up;
      }
    }
    int cv[NP];
    double g0[NP], g1[NP];
#pragma unroll
    for (int s = 0; s < NP; ++s) cv[s] = C.cid[(size_t)ii[s] * p + jj[s]];
    if (MODE1D) {  // G_K = c/2 K^{-1} - 1/2 alpha alpha^T - v beta alpha^T, G_D = v R alpha^T
      double ai[NP], aj[NP], bi[NP], bj[NP], ri[NP], rj[NP];
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        g0[s] = A.Kinv[(size_t)ii[s] * p + jj[s]];
        ai[s] = A.alpha[ii[s]];
        aj[s] = A.alpha[jj[s]];
        bi[s] = A.beta[ii[s]];
        bj[s] = A.beta[jj[s]];
        ri[s] = A.R[ii[s]];
        rj[s] = A.R[jj[s]];
      }
      if (k == 0) {  // the diagonal: one pair
#pragma unroll
        for (int s = 0; s < NP; ++s) {
          g1[s] = vs * ri[s] * aj[s];
          g0[s] = hc * g0[s] - 0.5 * ai[s] * aj[s] - vs * bi[s] * aj[s];
        }
      } else {
#pragma unroll
        for (int s = 0; s < NP; ++s) {
          g1[s] = vs * (ri[s] * aj[s] + rj[s] * ai[s]);
          g0[s] = 2.0 * hc * g0[s] - ai[s] * aj[s] - vs * (bi[s] * aj[s] + bj[s] * ai[s]);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < NP; ++s) g0[s] = A.GK[(size_t)ii[s] * p + jj[s]];
#pragma unroll
      for (int s = 0; s < NP; ++s) g1[s] = A.GD[(size_t)ii[s] * p + jj[s]];
    }
    if (DERIV == 1) {
      double xi[NP], xj[NP];
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        xi[s] = A.x[ii[s]];
        xj[s] = A.x[jj[s]];
      }
#pragma unroll
      for (int s = 0; s < NP; ++s)
        if (!(xi[s] - xj[s] >= 0.0)) g1[s] = -g1[s];
    }
    if constexpr (LDSB) {
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        const int v = cv[s] - cb;
        if (msk[s] && v >= 0 && v < vb) {
          __hip_atomic_fetch_add(mybin + v * 64 + lane, g0[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(mybin + (vb + v) * 64 + lane, g1[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    } else if constexpr (V > 16) {  // slot-major, bounded by the wave's variant count
      int vv[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) vv[s] = ((cv[s] - cb) & msk[s]) | ~msk[s];
#pragma unroll
      for (int x = 0; x < V; ++x) {
        if (x < nvw) {  // (uniform)
#pragma unroll
          for (int s = 0; s < 8; ++s) {
            ak[x] += (vv[s] == x) ? g0[s] : 0.0;
            ad[x] += (vv[s] == x) ? g1[s] : 0.0;
          }
        }
      }
    } else {  // (V <= 16: the unbounded pair-major form keeps C4's occupancy at 4)
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int v = ((cv[s] - cb) & msk[s]) | ~msk[s];
#pragma unroll
        for (int x = 0; x < V; ++x) {
          ak[x] += (v == x) ? g0[s] : 0.0;
          ad[x] += (v == x) ? g1[s] : 0.0;
        }
      }
    }
  }
  if constexpr (LDSB) {  // wave 0: the four waves' bins added in wave order, per variant
    __syncthreads();
    if (w == 0) {
      double* pk = C.part + (size_t)chunk * C.ncls + cb;
      double* pd = C.part + (size_t)(C.nchunk + chunk) * C.ncls + cb;
      for (int x = 0; x < nvar; ++x) {
        double rk = lbin[x * 64 + lane], rd = lbin[(vb + x) * 64 + lane];
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) {
          rk = rk + lbin[(size_t)ww * 2 * vb * 64 + x * 64 + lane];
          rd = rd + lbin[(size_t)ww * 2 * vb * 64 + (vb + x) * 64 + lane];
        }
        pk[x] = rk;
        pd[x] = rd;
      }
    }
    if (TR_FIRST) TR_HI(SLOT_CLASS_SUM);
    if (TR_LAST) TR_HI(SLOT_CSUM_START);
    return;
  }
  __shared__ double red[2][V][64];
#pragma unroll
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int x = 0; x < V; ++x) {
        if (x < nvw) {
          red[0][x][lane] = ww == 0 ? ak[x] : red[0][x][lane] + ak[x];
          red[1][x][lane] = ww == 0 ? ad[x] : red[1][x][lane] + ad[x];
        }
      }
    }
    __syncthreads();
  }
  // wave 0 writes: lane = diagonal, its class range [cb, cb + nvar) already in registers (the
  // previous form re-read cbase per stored element: a dependent round trip per pass)
  if (w == 0) {
    double* pk = C.part + (size_t)chunk * C.ncls + cb;
    double* pd = C.part + (size_t)(C.nchunk + chunk) * C.ncls + cb;
#pragma unroll
    for (int x = 0; x < V; ++x)
      if (x < nvar) {
        pk[x] = red[0][x][lane];
        pd[x] = red[1][x][lane];
      }
  }
  if (TR_FIRST) TR_HI(SLOT_CLASS_SUM);
  if (TR_LAST) TR_HI(SLOT_CSUM_START);
}

constexpr int PG_CLS = 16;  // classes per contraction workgroup

template <bool MATERN, bool COS, int DERIV, bool MODE1D, bool CLS, bool DD = false>
__global__ __launch_bounds__(256) void pgrad_kernel(PGradBatch b, int q,
                                                    const StepScalars* __restrict__ sc) {
  const int axis = blockIdx.y;
  const int blk = blockIdx.x;
  if (TR_FIRST) TR_LO(SLOT_PGRAD);
  if (axis == b.naxes + 1) {  // fused tail: the loss and log_tau / log_v update, off the chain
    if (blk == 0) finalize_body(b.tail.fin, 1);
    return;
  }
  if (axis >= b.naxes + 2) {  // the next step's class values (pipelined)
    if (CLS && b.tail.nce_flag) next_class_values<MATERN, COS, DERIV>(b, axis - (b.naxes + 2), blk, q);
    return;
  }
  if (axis == b.naxes) {
    if (threadIdx.x == 0 && blk == 0) TR_LO(SLOT_PG_UPLANE);  // fused tail: dL/dU + Adam on U (grid-stride over the solution grid)
    const int nu = tail_nu(b.tail.adam.L);
    for (int e = blk * 256 + threadIdx.x; e < nu; e += gridDim.x * 256) adam_u_elem(b.tail.adam, e);
    if (threadIdx.x == 0 && blk == 0) TR_HI(SLOT_PG_UPLANE);
    if (threadIdx.x == 0 && blk == gridDim.x - 1) TR_HI(SLOT_PG_ULAST);
    return;
  }
  if (blk >= b.bpa) return;  // the U plane is wider than the gradient planes
  const bool trl = threadIdx.x == 0 && blk == b.bpa - 1 && axis == b.naxes - 1;
  if (trl) TR_LO(SLOT_PG_START);
  const PGradArgs& A = b.ax[axis];
  const int tile = CLS ? blk : blk / PG_SUB, chunk = blk % PG_SUB;
  if (CLS ? blk * PG_CLS >= A.cls.ncls : tile >= b.tiles[axis]) {
    // no pairs / classes here (shorter axis); its partial slot stays zero
    if (b.tail.fused) pgrad_tail(b, axis, blk, q);
    return;
  }
  // sharded step (never fused): another rank's pair tile -- this slot is never written, so it
  // stays zero and the cross-rank all-reduce of the reduced partials counts each tile once
  if (b.shard_n > 1 && tile % b.shard_n != b.shard_rank) return;

  __shared__ double sd[PAIRS], swk[PAIRS], swd[PAIRS];
  __shared__ double sw[QMAX], sa[QMAX], so[QMAX], sol[QMAX];
  __shared__ double sacc[8][3][32];
  const int t = threadIdx.x;
  if (t < q) {
    sw[t] = A.kc->w[t];
    sa[t] = A.kc->a[t];
    so[t] = A.kc->om[t];
    sol[t] = A.kc->oml[t];
  }
  constexpr int NP = CLS ? PG_CLS : PAIRS;  // staged (d, w_K, w_D) entries
  if (CLS) {  // class blk * PG_CLS + (t & 15): weights = its chunk partials, added in chunk order
    const ClassArgs& C = A.cls;
    const int ul = t & (PG_CLS - 1), cs = t / PG_CLS;  // 16 chunk slices
    const int u = blk * PG_CLS + ul;
    double sk = 0.0, sdd = 0.0;
    if (u < C.ncls && A.cpK) {  // the GEMM epilogues' class tile partials (class_slots)
      for (int e = cs; e < A.cslots; e += 256 / PG_CLS) {
        sk += A.cpK[(size_t)e * C.ncls + u];
        sdd += A.cpD[(size_t)e * C.ncls + u];
      }
    } else if (u < C.ncls) {
      for (int c = cs; c < C.nchunk; c += 256 / PG_CLS) {
        sk += C.part[(size_t)c * C.ncls + u];
        sdd += C.part[(size_t)(C.nchunk + c) * C.ncls + u];
      }
    }
    sacc[cs >> 1][0][(cs & 1) * PG_CLS + ul] = sk;  // scratch: [16 slices][16 classes] x 2
    sacc[cs >> 1][1][(cs & 1) * PG_CLS + ul] = sdd;
    __syncthreads();
    if (t < PG_CLS) {
      double a = 0.0, d = 0.0;
#pragma unroll
      for (int x = 0; x < 256 / PG_CLS; ++x) {
        a += sacc[x >> 1][0][(x & 1) * PG_CLS + t];
        d += sacc[x >> 1][1][(x & 1) * PG_CLS + t];
      }
      const bool ok = u < C.ncls;
      sd[t] = ok ? C.dist[u] : 0.0;
      swk[t] = ok ? a : 0.0;
      swd[t] = ok ? d : 0.0;
    }
  } else if (t < PAIRS) {  // stage pair t
    int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tile) ++I;
    while (I * (I + 1) / 2 > tile) --I;
    const int J = tile - I * (I + 1) / 2;
    const int i = I * 32 + chunk * (PAIRS / 32) + (t >> 5), j = J * 32 + (t & 31);
    double d = 0.0, wk = 0.0, wd = 0.0;
    if (i < A.n && j < A.n) {
      const double diff = A.x[i] - A.x[j];
      d = fabs(diff);
      const double sij = diff >= 0.0 ? 1.0 : -1.0;
      const double sji = (A.x[j] - A.x[i]) >= 0.0 ? 1.0 : -1.0;
      double gkij, gkji, gdij, gdji;
      if (MODE1D) {
        const double v = sc->v;
        const double ai = A.alpha[i], aj = A.alpha[j];
        gkij = A.halfc * A.Kinv[(size_t)i * A.p + j] - 0.5 * ai * aj - v * A.beta[i] * aj;
        gkji = A.halfc * A.Kinv[(size_t)j * A.p + i] - 0.5 * aj * ai - v * A.beta[j] * ai;
        gdij = v * A.R[i] * aj;
        gdji = v * A.R[j] * ai;
      } else {
        gkij = A.GK[(size_t)i * A.p + j];
        gkji = A.GK[(size_t)j * A.p + i];
        gdij = A.GD[(size_t)i * A.p + j];
        gdji = A.GD[(size_t)j * A.p + i];
      }
      if (DERIV == 1) {
        gdij *= sij;
        gdji *= sji;
      }
      if (I == J) {  // diagonal tile: every ordered pair once
        wk = gkij;
        wd = gdij;
      } else {       // off-diagonal tile: fold in the mirror pair (j, i)
        wk = gkij + gkji;
        wd = gdij + gdji;
      }
    }
    sd[t] = d;
    swk[t] = wk;
    swd[t] = wd;
  }
  __syncthreads();
  if (TR_FIRST) TR_HI(SLOT_PG_STAGED);

  const int g = t >> 5, ql = t & 31;
  double* out = A.part + (size_t)blk * (3 * QMAX);
  __shared__ double slo[DD ? 8 : 1][3][32];  // DD: the low parts of sacc
  for (int q0 = 0; q0 < q; q0 += 32) {
    const int c = q0 + ql;
    double accf = 0.0, accl = 0.0, accw = 0.0;
    dd::D xf = {0.0, 0.0}, xl = {0.0, 0.0}, xw = {0.0, 0.0};
    if (c < q) {
      const double a = sa[c], om = so[c], oml = sol[c];
      for (int e = g; e < NP; e += 8) {
        const double wk = swk[e], wd = swd[e];
        if (wk == 0.0 && wd == 0.0) continue;
        const double d = sd[e];
        if constexpr (DD) {
          dd::D fw, fl, ff, dw, dl, df;
          fields_dd<MATERN, COS, DERIV>(d, a, om, oml, fw, fl, ff, dw, dl, df);
          xw = dd::add(xw, dd::add(dd::mul_d(fw, wk), dd::mul_d(dw, wd)));
          xl = dd::add(xl, dd::add(dd::mul_d(fl, wk), dd::mul_d(dl, wd)));
          xf = dd::add(xf, dd::add(dd::mul_d(ff, wk), dd::mul_d(df, wd)));
          continue;
        }
        double m0, m1, m2, m0l, m1l, m2l;
        radial_l<MATERN>(d, a, m0, m1, m2, m0l, m1l, m2l);
        if (COS) {
          double S, C;
          phase_sincos(om, oml, d, S, C);
          const double c0 = C, c1 = -om * S, c2 = -om * om * C;
          const double c0f = -TWO_PI * d * S;
          const double c1f = -TWO_PI * S - TWO_PI * om * d * C;
          const double c2f = -2.0 * TWO_PI * om * C + TWO_PI * om * om * d * S;
          double fw = m0 * c0, fl = m0l * c0, ff = m0 * c0f;
          double dw, dl, df;
          if (DERIV == 2) {
            dw = m2 * c0 + 2.0 * m1 * c1 + m0 * c2;
            dl = m2l * c0 + 2.0 * m1l * c1 + m0l * c2;
            df = m2 * c0f + 2.0 * m1 * c1f + m0 * c2f;
          } else {
            dw = m1 * c0 + m0 * c1;
            dl = m1l * c0 + m0l * c1;
            df = m1 * c0f + m0 * c1f;
          }
          accw += wk * fw + wd * dw;
          accl += wk * fl + wd * dl;
          accf += wk * ff + wd * df;
        } else {
          const double dw = DERIV == 2 ? m2 : m1, dl = DERIV == 2 ? m2l : m1l;
          accw += wk * m0 + wd * dw;
          accl += wk * m0l + wd * dl;
        }
      }
    }
    if constexpr (DD) {
      sacc[g][0][ql] = xf.h;
      sacc[g][1][ql] = xl.h;
      sacc[g][2][ql] = xw.h;
      slo[g][0][ql] = xf.l;
      slo[g][1][ql] = xl.l;
      slo[g][2][ql] = xw.l;
    } else {
      sacc[g][0][ql] = accf;
      sacc[g][1][ql] = accl;
      sacc[g][2][ql] = accw;
    }
    __syncthreads();
    if (t < 96) {
      const int which = t >> 5, qq = t & 31;
      if constexpr (DD) {  // (only with the fused tail: launch_pg_c)
        dd::D s = {0.0, 0.0};
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) s = dd::add(s, dd::D{sacc[gg][which][qq], slo[gg][which][qq]});
        if (q0 + qq < QMAX) {
          st_wt(out + which * QMAX + q0 + qq, s.h);
          st_wt(A.part_lo + (size_t)blk * (3 * QMAX) + which * QMAX + q0 + qq, s.l);
        }
      } else {
        double s = 0.0;
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) s += sacc[gg][which][qq];
        if (q0 + qq < QMAX) {
          if (b.tail.fused) st_wt(out + which * QMAX + q0 + qq, s);  // write-through: handed off
          else out[which * QMAX + q0 + qq] = s;
        }
      }
    }
    __syncthreads();
  }
  if (b.tail.fused) pgrad_tail(b, axis, blk, q);
}

int pgrad_blocks(int n) {
  int T = pad_up(n) / 32;
  return T * (T + 1) / 2 * PG_SUB;
}

int pgrad_class_blocks(int ncls) { return (ncls + PG_CLS - 1) / PG_CLS; }

template <int V>
static void launch_csum_v(const PGradBatch& b, int nchunk, int nbands, int deriv, int mode1d,
                          const StepScalars* sc, hipStream_t s) {
  dim3 grid(nchunk, nbands, b.naxes);
  if (mode1d)
    hipLaunchKernelGGL((class_sum_kernel<V, 2, true>), grid, dim3(256), 0, s, b, sc);
  else if (deriv == 2)
    hipLaunchKernelGGL((class_sum_kernel<V, 2, false>), grid, dim3(256), 0, s, b, sc);
  else
    hipLaunchKernelGGL((class_sum_kernel<V, 1, false>), grid, dim3(256), 0, s, b, sc);
}

// many variants per diagonal (> 16): LDS bins sized to the variant count
static void launch_csum_lds(const PGradBatch& b, int nchunk, int nbands, int deriv, int mode1d, int vmax,
                            const StepScalars* sc, hipStream_t s) {
  dim3 grid(nchunk, nbands, b.naxes);
  const size_t lds = (size_t)4 * 2 * vmax * 64 * sizeof(double);
  if (mode1d)
    hipLaunchKernelGGL((class_sum_kernel<1, 2, true, true>), grid, dim3(256), lds, s, b, sc, vmax);
  else if (deriv == 2)
    hipLaunchKernelGGL((class_sum_kernel<1, 2, false, true>), grid, dim3(256), lds, s, b, sc, vmax);
  else
    hipLaunchKernelGGL((class_sum_kernel<1, 1, false, true>), grid, dim3(256), lds, s, b, sc, vmax);
}

template <bool MATERN, bool COS, bool CLS>
static void launch_pg_c(const PGradBatch& b, int naxes, int bpa, int q, int deriv, int mode1d,
                        const StepScalars* sc, hipStream_t s) {
  // the U plane (dL/dU + Adam) gets one element per thread when it is wider than bpa blocks
  const int ublocks = b.tail.fused ? (tail_nu(b.tail.adam.L) + 255) / 256 : 0;
  dim3 grid(std::max(bpa, std::min(ublocks, 4096)), naxes + (b.tail.fused ? 2 : 0));
  if (b.tail.fused && b.tail.nce_flag) {  // + one plane per axis: the next step's class values
    for (int k = 0; k < naxes; ++k) grid.x = std::max<unsigned>(grid.x, (b.ax[k].cls.ncls + 7) / 8);
    grid.y += naxes;
  }
  // double-double contraction: class path, 2D, with the fused tail carrying the low parts
  const bool ddc = CLS && b.tail.fused && b.tail.gpart_lo && b.ax[0].part_lo && (naxes < 2 || b.ax[1].part_lo);
  if (ddc) {
    if (mode1d)
      hipLaunchKernelGGL((pgrad_kernel<MATERN, COS, 2, true, CLS, true>), grid, dim3(256), 0, s, b, q, sc);
    else if (deriv == 2)
      hipLaunchKernelGGL((pgrad_kernel<MATERN, COS, 2, false, CLS, true>), grid, dim3(256), 0, s, b, q, sc);
    else
      hipLaunchKernelGGL((pgrad_kernel<MATERN, COS, 1, false, CLS, true>), grid, dim3(256), 0, s, b, q, sc);
    return;
  }
  if (mode1d) {
    hipLaunchKernelGGL((pgrad_kernel<MATERN, COS, 2, true, CLS>), grid, dim3(256), 0, s, b, q, sc);
  } else if (deriv == 2) {
    hipLaunchKernelGGL((pgrad_kernel<MATERN, COS, 2, false, CLS>), grid, dim3(256), 0, s, b, q, sc);
  } else {
    hipLaunchKernelGGL((pgrad_kernel<MATERN, COS, 1, false, CLS>), grid, dim3(256), 0, s, b, q, sc);
  }
}

template <bool MATERN, bool COS>
static void launch_pg_t(const PGradBatch& b, int naxes, int bpa, int q, int deriv, int mode1d,
                        const StepScalars* sc, hipStream_t s) {
  if (b.ax[0].cls.ncls > 0) {
    int nbands = 0, vmax = 0, nchunk = 0;
    for (int k = 0; k < naxes; ++k) {
      nbands = std::max(nbands, (b.ax[k].n + 63) / 64);
      vmax = std::max(vmax, b.ax[k].cls.vmax);
      nchunk = std::max(nchunk, b.ax[k].cls.nchunk);
    }
    // (class tile partials from the G_K / G_D GEMMs: no class-sum launch)
    if (!b.ax[0].cpK) {
      if (vmax <= 8) launch_csum_v<8>(b, nchunk, nbands, deriv, mode1d, sc, s);
      else launch_csum_lds(b, nchunk, nbands, deriv, mode1d, vmax, sc, s);
    }
    launch_pg_c<MATERN, COS, true>(b, naxes, bpa, q, deriv, mode1d, sc, s);
  } else {
    launch_pg_c<MATERN, COS, false>(b, naxes, bpa, q, deriv, mode1d, sc, s);
  }
}

hipError_t launch_pgrad(int kind, int q, int mode1d, const PGradArgs* a, int naxes,
                        int blocks_per_axis, const StepScalars* sc, hipStream_t s,
                        const TailArgs* tail, int shard_rank, int shard_n) {
  PGradBatch b{};
  b.shard_rank = shard_rank;
  b.shard_n = shard_n;
  if (shard_n > 1 && tail && tail->fused) return hipErrorInvalidValue;
  for (int k = 0; k < naxes; ++k) {
    b.ax[k] = a[k];
    int T = a[k].p / 32;
    b.tiles[k] = T * (T + 1) / 2;
    if ((a[k].cls.ncls > 0) != (a[0].cls.ncls > 0) || a[k].cls.vmax > CLS_VMAX) return hipErrorInvalidValue;
    // class tile partials on every axis or none, from GEMM epilogues (2D class path)
    if ((a[k].cpK != nullptr) != (a[0].cpK != nullptr) ||
        (a[k].cpK && (!a[k].cpD || a[k].cslots <= 0 || a[k].cls.ncls <= 0 || mode1d)))
      return hipErrorInvalidValue;
  }
  b.naxes = naxes;
  b.bpa = blocks_per_axis;
  if (tail) b.tail = *tail;
  if (b.tail.fused) {
    // every block of the gradient planes must exist: group sizes are sized on bpa
    if (b.tail.tg <= 0 || b.tail.ngpa * b.tail.tg < blocks_per_axis) return hipErrorInvalidValue;
  }
  // pipelined class values: the class path with the fused tail only (its Adam block raises the flag)
  if (b.tail.nce_flag && (!b.tail.fused || !b.tail.nce_status || !b.tail.fin.kp_wt || a[0].cls.ncls <= 0 ||
                          shard_n > 1))
    return hipErrorInvalidValue;
  int deriv = a[0].deriv;
  switch (kind) {
    case SE_COS: launch_pg_t<false, true>(b, naxes, blocks_per_axis, q, deriv, mode1d, sc, s); break;
    case MATERN52_COS: launch_pg_t<true, true>(b, naxes, blocks_per_axis, q, deriv, mode1d, sc, s); break;
    case SE: launch_pg_t<false, false>(b, naxes, blocks_per_axis, q, deriv, mode1d, sc, s); break;
    default: launch_pg_t<true, false>(b, naxes, blocks_per_axis, q, deriv, mode1d, sc, s); break;
  }
  return hipGetLastError();
}

}  // namespace gpk
