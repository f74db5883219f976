// spdinv_big.hip — SPD inverse + log-determinant for LARGE covariance factors (gfx950, fp64 MFMA).
//
// Same contract as spdinv.hip (replaces jnp.linalg.solve / slogdet of
// code/model_GP_solver_1d.py:92,135-137, code/model_GP_solver_2d.py:104-105,157-162,
// code/model_GP_solver_advection.py:104-105,153-158): X <- K^{-1} in place, log det K per 32-row
// block, refinement gate, non-PD status.  The 32-wide sweep of spdinv.hip re-reads and rewrites
// the whole matrix once per 32 columns and recomputes its panel in every tile; at p >= ~1024
// that is HBM- and launch-bound.  This path sweeps 64-wide pivot blocks and splits each sweep
// into three pieces of work:
//
//   panel   Z = L^{-1} X_{P,:}   (64 x p, one small MFMA GEMM per 64-column block; Z_P = L^{-1})
//   update  X_IJ <- s_IJ (base_IJ - Z_I^T Z_J) on the LOWER tiles only (I >= J), in place:
//             I,J != P : X_IJ - Z_I^T Z_J          (Schur complement, the SYRK-shaped bulk)
//             one of I,J == P : + Z_I^T Z_J        (= L^{-T} V: the swept panel)
//             I = J = P : - Z_P^T Z_P              (= -S^{-1})
//   pivot   the next pivot block S = X_{k+1,k+1} is factored (Cholesky + L^{-1}, in LDS) by one
//           extra workgroup of the update launch, right after the workgroup that owns that tile
//           has written it back (release + counter hand-off, MI355X_MICROARCH inter-workgroup
//           visibility), so the serial pivot chain runs under the bulk of the update.
//
// After T = ceil(p/64) sweeps X = -K^{-1}; the last sweep flips the sign, mirrors every lower
// tile into the upper triangle (LDS transpose, coalesced stores) and publishes max diag K^{-1}
// for the refinement gate.  Flops: p^3 (potrf + potri equivalent), all on v_mfma_f64_16x16x4.
// The 64-pivot factorisation is two 32-pivots (spd_pivot.h) glued by three 32x32 MFMA products:
//   L11^{-1} = chol_inv(S11);  V = L11^{-1} S12;  L22^{-1} = chol_inv(S22 - V^T V);
//   (L^{-1})_21 = -L22^{-1} V^T L11^{-1}.
#include "gpk_internal.h"
#include "spd_pivot.h"

namespace gpk {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int BW = 64;   // pivot / tile width
constexpr int SS = 65;   // 64x64 LDS tile stride (doubles)

struct BigSpdBatch {
  double* X[2];      // the matrix, inverted in place
  double* Z[2];      // [64][p] panel
  double* Li[2];     // [64][64] L^{-1} of the current pivot block (row-major, zero upper)
  double* ldet[2];   // [p/32]
  double* pst[2];    // refinement gate [2]
  int* status[2];
  unsigned int* flag[2];
  int p[2], n[2], T[2];
};

__device__ __forceinline__ int bw(int p, int I) { return min(BW, p - BW * I); }

// 16x16 block of a 32-deep product out of LDS: acc += A(i0.., k) * B(k, j0..)
// element (i,k) of A at a[i*sai + k*sak], (k,j) of B at b[k*sbk + j*sbj]
__device__ __forceinline__ d4 mma16(const double* a, int sai, int sak, const double* b, int sbk,
                                    int sbj, int i0, int j0, int lane, d4 acc) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = 4 * kk + lk;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[(i0 + li) * sai + k * sak],
                                               b[k * sbk + (j0 + li) * sbj], acc, 0, 0, 0);
  }
  return acc;
}

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

// S[r][c] = src[c*ld + r] (r < h, c < w; else 0): transposed 64x64 tile, reads along r
__device__ __forceinline__ void load_tile_t(double* S, const double* src, int ld, int h, int w, int t) {
  double v[16];
  const int r = t & 63, c0 = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int c = c0 + 4 * q;
    v[q] = (r < h && c < w) ? src[(size_t)c * ld + r] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) S[r * SS + c0 + 4 * q] = v[q];
}

// the 32-pivot factorisation as a real call: inlined twice (or in a loop) its fully unrolled
// register blocking blows past 256 VGPRs and spills; as a callee it keeps its own ~130
__device__ __noinline__ double pivot32(lds_ptr A, lds_ptr M, lds_ptr pv, int t, int* status) {
  return pivot_chol_inv_block<4, lds_ptr>(A, M, pv, t, status);
}

// Factor the w x w (w = 32 or 64) diagonal block kb of X (symmetric; both triangles valid):
// writes Li (64x64 row-major, zero-padded), ldet[2kb(+1)], status.  One 256-thread workgroup.
__device__ void pivot64(const double* X, int p, int kb, double* Li, double* ldet, int* status,
                        double* sm) {
  double* S = sm;                   // [64][SS]
  double* A = S + 64 * SS;          // [32][SP] factor scratch, then W
  double* M1 = A + 32 * SP;         // [32][SP]
  double* M2 = M1 + 32 * SP;        // [32][SP]
  double* V = M2 + 32 * SP;         // [32][SP]
  double* pv = V + 32 * SP;         // [32]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int w = bw(p, kb);
  const double* Xs = X + (size_t)(BW * kb) * p + BW * kb;
  load_tile(S, Xs, p, w, w, t);
  __syncthreads();
  for (int e = t; e < 1024; e += 256) A[(e >> 5) * SP + (e & 31)] = S[(e >> 5) * SS + (e & 31)];
  __syncthreads();
  d4 acc;
  const int ro = 16 * wr, co = 16 * wc;
  double ls[2] = {0.0, 0.0};
  // one copy of the (register-heavy) 32-pivot code: half h = 0 factors S11 (L^{-1} into M2, then
  // moved to M1), h = 1 the Schur complement S22 - V^T V of the second half
#pragma nounroll
  for (int h = 0; h < w / 32; ++h) {
    ls[h] = pivot32((lds_ptr)A, (lds_ptr)M2, (lds_ptr)pv, t, status);
    if (h == 0 && w == BW) {
      for (int e = t; e < 32 * SP; e += 256) M1[e] = M2[e];
      __syncthreads();
      // V = M1 S12
      acc = d4{0.0, 0.0, 0.0, 0.0};
      acc = mma16(M1, SP, 1, S + 32, SS, 1, ro, co, lane, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) V[(ro + (lane >> 4) + 4 * r) * SP + co + (lane & 15)] = acc[r];
      __syncthreads();
      // A = S22 - V^T V
      acc = d4{0.0, 0.0, 0.0, 0.0};
      acc = mma16(V, 1, SP, V, SP, 1, ro, co, lane, acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ro + (lane >> 4) + 4 * r, j = co + (lane & 15);
        A[i * SP + j] = S[(32 + i) * SS + 32 + j] - acc[r];
      }
      __syncthreads();
    }
  }
  if (w != BW)
    for (int e = t; e < 32 * SP; e += 256) M1[e] = M2[e];  // read after the barrier below
  __syncthreads();
  const double ls1 = ls[0], ls2 = ls[1];
  if (w == BW) {
    // A = W = V^T M1
    acc = d4{0.0, 0.0, 0.0, 0.0};
    acc = mma16(V, 1, SP, M1, SP, 1, ro, co, lane, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) A[(ro + (lane >> 4) + 4 * r) * SP + co + (lane & 15)] = acc[r];
    __syncthreads();
    // (L^{-1})_21 = -M2 W  -> S rows 32.., cols 0..31 (S is free now)
    acc = d4{0.0, 0.0, 0.0, 0.0};
    acc = mma16(M2, SP, 1, A, SP, 1, ro, co, lane, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) S[(32 + ro + (lane >> 4) + 4 * r) * SS + co + (lane & 15)] = -acc[r];
    __syncthreads();
  }
  for (int e = t; e < BW * BW; e += 256) {
    const int r = e >> 6, c = e & 63;
    double v = 0.0;
    if (r < 32 && c < 32) v = M1[r * SP + c];
    else if (r >= 32 && r < w && c < 32) v = S[r * SS + c];
    else if (r >= 32 && r < w && c >= 32 && c < w) v = M2[(r - 32) * SP + c - 32];
    Li[e] = v;
  }
  if (t == 0) {
    ldet[2 * kb] = ls1;
    if (w == BW) ldet[2 * kb + 1] = ls2;
  }
}

constexpr int PIVOT_LDS = 64 * SS + 4 * 32 * SP + 32;  // doubles

__global__ __launch_bounds__(256) void big_pivot_init_kernel(BigSpdBatch b) {
  const int m = blockIdx.x;
  __shared__ double sm[PIVOT_LDS];
  const double x00 = b.X[m][0];
  pivot64(b.X[m], b.p[m], 0, b.Li[m], b.ldet[m], b.status[m], sm);
  if (threadIdx.x == 0) {
    b.pst[m][0] = x00;   // K_00 = max diag K (stationary kernel + jitter)
    b.pst[m][1] = 0.0;   // max diag K^{-1}: atomicMax'd by the last sweep
    *b.flag[m] = 0u;
  }
}

// Z[:, J-block] = L^{-1} X_{P,J}  (X_{P,J} of the lower storage: row block P for J < P, the
// transpose of column block P for J > P);  Z[:, P-block] = L^{-1}.
__global__ __launch_bounds__(256) void big_panel_kernel(BigSpdBatch b, int k) {
  const int m = blockIdx.y, J = blockIdx.x;
  const int p = b.p[m], T = b.T[m];
  if (k >= T || J >= T) return;
  const double* X = b.X[m];
  double* Z = b.Z[m];
  const double* Li = b.Li[m];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wP = bw(p, k), wJ = bw(p, J);
  if (J == k) {
    for (int e = t; e < wP * wP; e += 256) {
      const int r = e / wP, c = e - r * wP;
      Z[(size_t)r * p + BW * k + c] = Li[r * BW + c];
    }
    return;
  }
  __shared__ double sL[BW * SS], sX[BW * SS];
  load_tile(sL, Li, BW, BW, BW, t);
  if (J < k)  // row block P of the lower storage
    load_tile(sX, X + (size_t)(BW * k) * p + BW * J, p, wP, wJ, t);
  else        // tile (J, k): X_{P,J}[r][c] = X[J*64 + c][k*64 + r]
    load_tile_t(sX, X + (size_t)(BW * J) * p + BW * k, p, wP, wJ, t);
  __syncthreads();
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < wP; k0 += 32)
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
        acc[bi][bj] = mma16(sL + k0, SS, 1, sX + k0 * SS, SS, 1, 32 * wr + 16 * bi, 32 * wc + 16 * bj,
                            lane, acc[bi][bj]);
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 32 * wr + 16 * bi + (lane >> 4) + 4 * r, col = 32 * wc + 16 * bj + (lane & 15);
        if (row < wP && col < wJ) Z[(size_t)row * p + BW * J + col] = acc[bi][bj][r];
      }
}

__device__ __forceinline__ void tile_of(int lin, int& I, int& J) {
  int i = (int)((sqrt(8.0 * lin + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= lin) ++i;
  while (i * (i + 1) / 2 > lin) --i;
  I = i;
  J = lin - i * (i + 1) / 2;
}

constexpr int UPD_WGS = 255;  // tile workgroups per factor (+1 pivot workgroup = one per CU)
constexpr int SZ = 80;        // LDS stride of the Z panels [k][i]: k and k+1 32 banks apart

// The tile list of one update launch: position 0 = (k+1,k+1) when there is a next pivot (so its
// hand-off happens first), then every other lower tile in row-major order.
struct TileList {
  int k, ntiles, dk;
  bool has_next;
  __device__ void at(int pos, int& I, int& J) const {
    if (has_next) {
      if (pos == 0) { I = J = k + 1; return; }
      int lin = pos - 1;
      if (lin >= dk) ++lin;
      tile_of(lin, I, J);
    } else {
      tile_of(pos, I, J);
    }
  }
};

// 64 x 64 panel block Z[0..63][c0..c0+63] -> registers (16 per thread, coalesced rows)
__device__ __forceinline__ void zblock_fetch(double (&v)[16], const double* Z, int p, int c0, int wK, int t) {
  const int c = t & 63, r0 = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = r0 + 4 * q;
    v[q] = (r < wK && c0 + c < p) ? Z[(size_t)r * p + c0 + c] : 0.0;
  }
}
__device__ __forceinline__ void zblock_store(const double (&v)[16], double* sZ, int t) {
  const int c = t & 63, r0 = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) sZ[(r0 + 4 * q) * SZ + c] = v[q];
}

constexpr int UPD_LDS = 2 * 64 * SZ + 64 * SS;  // sZI, sZJ, mirror stage (doubles)
constexpr int BIG_LDS = UPD_LDS > PIVOT_LDS ? UPD_LDS : PIVOT_LDS;

// One sweep's update of every lower tile (+ the next pivot, + the final sign flip / mirror).
// Persistent: G <= 255 tile workgroups each take a contiguous run of the tile list (runs stay
// within a block row, so Z_I is staged once per row); Z_I and Z_J sit in LDS, the next tile's
// Z_J (and Z_I on a row change) is fetched into registers while the current tile's MFMAs run.
// blockIdx.x: 0 = tile workgroup 0 (takes (k+1,k+1) first), 1 = the pivot workgroup,
// 2.. = tile workgroups 1..  The pivot workgroup only waits for workgroup 0, dispatched
// before it (resident or finished: no deadlock).
__global__ __launch_bounds__(256) void big_update_kernel(BigSpdBatch b, int k, int skip_pivot) {
  const int m = blockIdx.y;
  const int p = b.p[m], T = b.T[m];
  if (k >= T) return;
  TileList tl;
  tl.k = k;
  tl.ntiles = T * (T + 1) / 2;
  tl.has_next = k + 1 < T;
  tl.dk = (k + 1) * (k + 2) / 2 + (k + 1);
  const bool last = !tl.has_next;
  const int G = min(tl.ntiles, UPD_WGS);
  const int x = blockIdx.x;
  __shared__ double sm[BIG_LDS];
  if (x == 1) {
    if (!tl.has_next || skip_pivot) return;
    if (threadIdx.x == 0) {  // pivot workgroup for block k+1
      while (__hip_atomic_load(b.flag[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 1u)
        __builtin_amdgcn_s_sleep(2);
      *b.flag[m] = 0u;  // re-arm (next user: the next sweep's update launch)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    pivot64(b.X[m], p, k + 1, b.Li[m], b.ldet[m], b.status[m], sm);
    return;
  }
  const int g = x == 0 ? 0 : x - 1;
  if (g >= G) return;
  const int chunk = (tl.ntiles + G - 1) / G;
  const int pos0 = g * chunk, pos1 = min(tl.ntiles, pos0 + chunk);
  if (pos0 >= pos1) return;
  double* X = b.X[m];
  const double* Z = b.Z[m];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int li = lane & 15, lk = lane >> 4;
  const int wK = bw(p, k);
  double* sZI = sm;
  double* sZJ = sm + 64 * SZ;
  double* sT = sm + 2 * 64 * SZ;  // [64][SS] transpose stage for the final mirror
  const double fin = last ? -1.0 : 1.0;

  // X tile (I, J) in this wave's MFMA layout; zero base for the swept row / column block.
  // Unconditional clamped loads times a 0/1 factor (a guarded load would become an exec-mask
  // branch); rows / columns past p are never stored.
  auto xo_fetch = [&](double (&xv)[2][2][4], int I_, int J_) {
    const double f = (I_ == k || J_ == k) ? 0.0 : 1.0;
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
  int I, J;
  tl.at(pos0, I, J);
  double xo[2][2][4], xn[2][2][4];
  xo_fetch(xn, I, J);
  {
    double v[16];
    zblock_fetch(v, Z, p, BW * I, wK, t);
    zblock_store(v, sZI, t);
    zblock_fetch(v, Z, p, BW * J, wK, t);
    zblock_store(v, sZJ, t);
  }
  __syncthreads();
  for (int pos = pos0; pos < pos1; ++pos) {
    const int I0 = BW * I, J0 = BW * J;
    const bool inPi = I == k, inPj = J == k;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) xo[bi][bj][r] = xn[bi][bj][r];
    // the next tile's panels and X tile in flight under this tile's MFMAs
    const bool more = pos + 1 < pos1;
    int In = I, Jn = J;
    double vj[16], vi[16];
    if (more) {
      tl.at(pos + 1, In, Jn);
      zblock_fetch(vj, Z, p, BW * Jn, wK, t);
      if (In != I) zblock_fetch(vi, Z, p, BW * In, wK, t);
      xo_fetch(xn, In, Jn);
    }
    d4 acc[2][2];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = d4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < wK; k0 += 32) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int kr = (k0 + 4 * kk + lk) * SZ;
        double a[2], bb[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          a[h] = sZI[kr + 32 * wr + 16 * h + li];
          bb[h] = sZJ[kr + 32 * wc + 16 * h + li];
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
            acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[bi], bb[bj], acc[bi][bj], 0, 0, 0);
      }
    }
    const double sgn = ((inPi != inPj) ? -1.0 : 1.0) * fin;
    // tile (k+1,k+1) goes to the pivot workgroup: stored write-through (sc1), so the hand-off
    // needs no L2 write-back (release fence) -- drain, barrier, one flag add (MI355X_MICROARCH
    // §inter-workgroup visibility, "publish-large")
    const bool handoff = tl.has_next && pos == 0;
    double mx = 0.0;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 32 * wr + 16 * bi + lk + 4 * r, col = 32 * wc + 16 * bj + li;
          const int gi = I0 + row, gj = J0 + col;
          const double v = sgn * (xo[bi][bj][r] - acc[bi][bj][r]);
          if (gi < p && gj < p) {
            if (handoff)
              __hip_atomic_store(&X[(size_t)gi * p + gj], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
              X[(size_t)gi * p + gj] = v;
            if (last && I == J && gi == gj && gi < b.n[m]) mx = fmax(mx, v);
          }
          if (last && I != J) sT[row * SS + col] = v;
        }
    if (handoff) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) atomicAdd(b.flag[m], 1u);
    }
    if (last && I == J) {  // refinement gate: max_i (K^{-1})_ii
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
      if (lane == 0 && mx > 0.0)
        atomicMax(reinterpret_cast<unsigned long long*>(b.pst[m] + 1),
                  (unsigned long long)__double_as_longlong(mx));
    }
    __syncthreads();  // every wave is done reading sZI / sZJ (and has staged sT)
    if (last && I != J) {
      // mirror: X[J0 + r][I0 + c] = tile[c][r], coalesced along c
      const int wI = bw(p, I), wJ = bw(p, J);
#pragma unroll 4
      for (int e = t; e < BW * BW; e += 256) {
        const int r = e >> 6, c = e & 63;
        if (r < wJ && c < wI) X[(size_t)(J0 + r) * p + I0 + c] = sT[c * SS + r];
      }
    }
    if (!more) break;
    zblock_store(vj, sZJ, t);
    if (In != I) zblock_store(vi, sZI, t);
    I = In;
    J = Jn;
    __syncthreads();
  }
}

BigSpdBatch make_batch(SpdArgs* a, int nmat, int& Tmax, int& tiles_max) {
  BigSpdBatch b{};
  Tmax = 0;
  tiles_max = 0;
  for (int m = 0; m < nmat; ++m) {
    b.X[m] = a[m].X; b.Z[m] = a[m].Y; b.Li[m] = a[m].piv;
    b.ldet[m] = a[m].ldet; b.pst[m] = a[m].pst; b.status[m] = a[m].status; b.flag[m] = a[m].flag;
    b.p[m] = a[m].p; b.n[m] = a[m].n; b.T[m] = (a[m].p + BW - 1) / BW;
    Tmax = std::max(Tmax, b.T[m]);
    tiles_max = std::max(tiles_max, std::min(b.T[m] * (b.T[m] + 1) / 2, UPD_WGS) + 1);
  }
  return b;
}

}  // namespace

int spd_big_sweeps(int p) { return (p + BW - 1) / BW; }

// stage -1: pivot 0; stage 2k: panel k; stage 2k+1: update k (profiling / bench)
hipError_t launch_spd_big_stage(SpdArgs* a, int nmat, int stage, hipStream_t s) {
  int Tmax, tiles;
  BigSpdBatch b = make_batch(a, nmat, Tmax, tiles);
  if (stage < 0)
    hipLaunchKernelGGL(big_pivot_init_kernel, dim3(nmat), dim3(256), 0, s, b);
  else if ((stage & 1) == 0)
    hipLaunchKernelGGL(big_panel_kernel, dim3(Tmax, nmat), dim3(256), 0, s, b, stage >> 1);
  else
    hipLaunchKernelGGL(big_update_kernel, dim3(tiles, nmat), dim3(256), 0, s, b, stage >> 1, 0);
  return hipGetLastError();
}

// bench: the update launch of sweep k without its pivot workgroup (the tile work alone)
hipError_t launch_spd_big_tiles(SpdArgs* a, int nmat, int k, hipStream_t s) {
  int Tmax, tiles;
  BigSpdBatch b = make_batch(a, nmat, Tmax, tiles);
  hipLaunchKernelGGL(big_update_kernel, dim3(tiles, nmat), dim3(256), 0, s, b, k, 1);
  return hipGetLastError();
}

hipError_t launch_spd_inverse_big(SpdArgs* a, int nmat, double** final_out, hipStream_t s) {
  int Tmax, tiles;
  BigSpdBatch b = make_batch(a, nmat, Tmax, tiles);
  for (int m = 0; m < nmat; ++m) final_out[m] = a[m].X;
  hipLaunchKernelGGL(big_pivot_init_kernel, dim3(nmat), dim3(256), 0, s, b);
  for (int k = 0; k < Tmax; ++k) {
    hipLaunchKernelGGL(big_panel_kernel, dim3(Tmax, nmat), dim3(256), 0, s, b, k);
    hipLaunchKernelGGL(big_update_kernel, dim3(tiles, nmat), dim3(256), 0, s, b, k, 0);
  }
  return hipGetLastError();
}

}  // namespace gpk
