// gpk_internal.h — shared device helpers and launcher declarations for libgpk (gfx950).
//
// Closed-form spectral-mixture kernel fields replacing the
// reference's jax.grad-of-kappa machinery (code/kernel_matrix.py:49-57, :114-193).
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gpk {

constexpr int QMAX = 64;      // max mixture components per axis
constexpr int PADM = 32;      // every device matrix dimension is padded to a multiple of this
constexpr int NB = 32;        // SPD-inverse pivot block (= one 32x32 tile)
constexpr double SQRT5 = 2.23606797749978969641;
constexpr double TWO_PI = 6.28318530717958647692;

enum Kind { SE_COS = 0, MATERN52_COS = 1, SE = 2, MATERN52 = 3 };

__host__ __device__ inline bool kind_matern(int k) { return k == MATERN52_COS || k == MATERN52; }
__host__ __device__ inline bool kind_cos(int k) { return k == SE_COS || k == MATERN52_COS; }
inline int pad_up(int n) { return (n + PADM - 1) / PADM * PADM; }

// Per-axis kernel constants, recomputed on device from the params at the start of a step.
struct AxisConst {
  double w[QMAX];    // e^{log-w}
  double a[QMAX];    // e^{log-ls}   (an inverse lengthscale, kernel_matrix.py:147)
  double om[QMAX];   // 2*pi*freq, rounded
  double oml[QMAX];  // its rounding error: om + oml = 2*pi*freq exactly (om_low)
};

// The kernel fields with the phase and radial arguments as double-doubles.  fp64 rounds the
// phase 2*pi*f*d (~250 rad at C5) and the radial argument sqrt5*a*d / a*d^2 by ~|arg| * eps, and
// cos / sin / exp inherit that as an absolute error: hundreds of ulp in K, D and the derivative
// fields, which the kernel-parameter contraction cancels into ~1e-8 relative at C5
// (tools/c5_kp_split.py).  Carrying the argument's low part and correcting to first order
// (cos(h + l) = cos h - l sin h, e^{-(h + l)} = e^{-h} (1 - l); l^2 ~ 1e-28) leaves the
// sincos / exp rounding only: the fields to a few ulp of exact, for two FMAs per argument.
__host__ __device__ inline double om_low(double freq, double om) { return fma(TWO_PI, freq, -om); }

__device__ __forceinline__ void phase_sincos(double om, double oml, double d, double& S, double& C) {
  const double h = om * d;
  const double l = fma(om, d, -h) + oml * d;
  double s, c;
  sincos(h, &s, &c);
  S = fma(l, c, s);
  C = fma(-l, s, c);
}

// e^{-arg} of the radial factor and the argument's high part: Matern52 arg = sqrt5 a d,
// SE arg = a d^2, both as double-doubles
template <bool MATERN>
__device__ __forceinline__ double radial_exp(double d, double a, double& r) {
  double l;
  if (MATERN) {
    const double p = SQRT5 * a;
    r = p * d;
    l = fma(p, d, -r) + fma(SQRT5, a, -p) * d;
  } else {
    const double d2 = d * d;
    r = a * d2;
    l = fma(a, d2, -r) + a * fma(d, d, -d2);
  }
  const double E = exp(-r);
  return fma(-l, E, E);
}

// Step scalars (device), written by the prep kernel.
struct StepScalars {
  double tau, v;     // e^{log_tau}, e^{log_v}
  double bc1, bc2;   // Adam bias corrections 1-b1^t, 1-b2^t for this step
};

// radial factor m(d) and derivatives; Matern52 (kernel_matrix.py:147-151) or SE (:125)
template <bool MATERN>
__device__ __forceinline__ void radial(double d, double a, double& m0, double& m1, double& m2) {
  double r;
  const double E = radial_exp<MATERN>(d, a, r);
  if (MATERN) {
    m0 = (1.0 + r + r * r * (1.0 / 3.0)) * E;
    m1 = -(SQRT5 / 3.0) * a * r * (1.0 + r) * E;
    m2 = (5.0 / 3.0) * a * a * (r * r - r - 1.0) * E;
  } else {
    const double d2 = d * d, g = E;
    m0 = g;
    m1 = -2.0 * a * d * g;
    m2 = (4.0 * a * a * d2 - 2.0 * a) * g;
  }
}

// radial factor plus its log-ls derivatives
template <bool MATERN>
__device__ __forceinline__ void radial_l(double d, double a, double& m0, double& m1, double& m2,
                                         double& m0l, double& m1l, double& m2l) {
  double r;
  const double E = radial_exp<MATERN>(d, a, r);
  if (MATERN) {
    double ka = (SQRT5 / 3.0) * a, k2 = (5.0 / 3.0) * a * a;
    double r2 = r * r;
    m0 = (1.0 + r + r2 * (1.0 / 3.0)) * E;
    m1 = -ka * r * (1.0 + r) * E;
    m2 = k2 * (r2 - r - 1.0) * E;
    m0l = -(r2 * (1.0 / 3.0)) * (1.0 + r) * E;
    m1l = -ka * r * (2.0 + 2.0 * r - r2) * E;
    m2l = k2 * (-r2 * r + 5.0 * r2 - 2.0 * r - 2.0) * E;
  } else {
    const double d2 = d * d, g = E;
    m0 = g;
    m1 = -2.0 * a * d * g;
    m2 = (4.0 * a * a * d2 - 2.0 * a) * g;
    m0l = -a * d2 * g;
    m1l = (-2.0 * a * d + 2.0 * a * a * d2 * d) * g;
    m2l = (10.0 * a * a * d2 - 2.0 * a - 4.0 * a * a * a * d2 * d2) * g;
  }
}

}  // namespace gpk

// ------------------------------------------------------------------------------------------
// launchers (host side), one TU per kernel family
// ------------------------------------------------------------------------------------------
namespace gpk {

// Per-step constants from the flat params (kernel constants per axis, tau, v, the Adam step
// counter and bias corrections).  Computed inside the assembly kernel: every workgroup derives
// its axis constants itself and workgroup (0, 0) publishes them for the later kernels.
constexpr int BGAP_CHUNK = 2048, BGAP_PARTS_MAX = 16;
struct PrepArgs {
  const double* params;
  int off_kp[2];       // start of (freq, log-ls, log-w) per axis
  int off_tau, off_v;
  int naxes, has_cos;
  AxisConst* kc;       // out [naxes]
  StepScalars* sc;     // out
  int* count;          // Adam step counter (incremented when apply)
  int apply;
  double b1, b2;
  // boundary gap ||u_b - b||^2 of U at the start of the step (model_GP_solver_2d.py:123-128,
  // model_GP_solver_1d.py:101-106), taken here because the fused tail updates U in place
  const double* Up; const double* bvals; const int* bidx;
  int nb, dim, n1, n2, p2;
  // out [bgap_parts]: partial sums over consecutive chunks of BGAP_CHUNK boundary entries,
  // added in order by the step's tail.  A large 2D boundary (C5: 16384 entries) is spread over
  // the first bgap_parts workgroups of the class-value launch -- one load round trip each
  // instead of eight in one workgroup, which held that launch at 28 us
  double* bgap;
  int bgap_parts;      // 1 .. BGAP_PARTS_MAX
  int skip;            // 1: this launch does not publish them (another launch of the step does)
  // first step of a batch, folded in (stepk.h StepBegin; all null otherwise): snap_count <- count
  // before this step's increment, *viol0 = 0, *slot0 = 0 (thread 0 of publish_prep), and the
  // rollback snapshot of (params, m, v) copied by the publishing launch's spare workgroups
  int* snap_count; unsigned int* viol0; int* slot0;
  double* snap; const double* snap_m; const double* snap_v; size_t snap_np;
  // pipelined class values (TailArgs::nce_flag): reset to 0 by thread 0 of publish_prep, i.e.
  // between the previous step's parameter-gradient launch (its waiters are done) and this one's
  unsigned int* nce_flag;
};

// Distance classes.  Every field of a stationary kernel depends on the pair (i, j) only
// through d = |x_i - x_j| (kernel_matrix.py:119-151), and on a collocation grid
// (linspace(0,1,N)*scale, model_GP_solver_2d.py:369-374) the n^2 pairs take only ~5n distinct
// fp64 values of d: each diagonal k = i - j holds a handful of rounding variants of k*h.  The
// host (gpk_create) groups the pairs of each axis by the EXACT value of d, per diagonal: class
// (k, v), k in [0, n), v < nvar(k) <= CLS_VMAX, ids [cbase[k], cbase[k+1]).  The fields are then
// evaluated once per class (bitwise the per-pair values: same d, same code) and the
// hyper-parameter contraction sum_ij G[i,j] f(d_ij) becomes sum_c (sum_{ij in c} G[i,j]) f(d_c).
// Grids whose diagonals carry more than CLS_VMAX distinct distances use the per-pair kernels.
constexpr int CLS_VMAX = 32;
struct ClassArgs {
  int ncls;              // classes of this axis (0: per-pair path)
  int vmax;              // max variants per diagonal (<= CLS_VMAX)
  const double* dist;    // [ncls] d of each class
  const int* cid;        // [p*p] class of pair (i, j); -1 on pads
  const int* cbase;      // [n+1] first class of diagonal k
  // [p*p] bytes: the variant of pair (i, j) on its diagonal, cid - cbase[|i - j|] (< CLS_VMAX),
  // 255 on pads; built for the large-factor gather (p >= 1024), whose id stream it shrinks 4x
  const unsigned char* vidx;
  double* kval;          // [ncls] kappa(d)      (+ jitter is added per element)
  double* dval;          // [ncls] d2k or |dk| (the D_x1 sign s_ij is applied per element)
  // hyper-parameter contraction: row chunk c of the class-sum launch writes its partial sums
  // of G_K[i,j] and s_ij G_D[i,j] over every class to part[c][.] / part[nchunk + c][.]; the
  // contraction launch adds the nchunk partials of each class in chunk order
  int nchunk, rb;        // row chunks of rb rows
  double* part;          // [2][nchunk][ncls]
};

struct AssembleArgs {
  const double* x;       // coords [n] (padded buffer ok)
  int n;                 // true size
  int p;                 // padded size (leading dimension)
  const AxisConst* kc;   // device
  double jitter;
  double* K;             // [p*p]  (consumed in place by the SPD inverse)
  double* Kc;            // [p*p]  kept copy of K for iterative refinement (nullable)
  double* D;             // [p*p]
  int deriv;             // 1 or 2 (0: K only)
  // pivot block 0 of the SPD inverse, factored by one extra workgroup of the assembly launch
  // (nullable piv: not fused).  Same outputs as the sweep's pivot_init.
  double* piv; double* ldet; double* pst; int* status;
  unsigned int* flag;    // zero-initialised counter (re-armed by the pivot workgroup)
  ClassArgs cls;         // ncls > 0: class evaluation + gather instead of per-pair evaluation
};
// the class path's gather launch alone (K, Kc, D from current class values; no pivot 0)
hipError_t launch_gather_only(const AssembleArgs* a, int naxes, hipStream_t s);
// eval_only (class path): the class values (+ prep) only, no gather / pivot-0 launch
hipError_t launch_assemble(int kind, int q, const AssembleArgs* a, int naxes, const PrepArgs& prep,
                           hipStream_t s, bool eval_only = false);
hipError_t launch_pairs(int kind, int q, const double* x1, const double* x2, long n,
                        const AxisConst* kc, int deriv, double* out, hipStream_t s);
hipError_t launch_cross(int kind, int q, const double* xr, int nr, const double* xc, int nc,
                        int ld, const AxisConst* kc, double jitter, int deriv, double* K,
                        double* D, hipStream_t s);

// SPD inverse by blocked Cholesky-Gauss-Jordan sweeps (pivot blocks factored in LDS).
struct SpdArgs {
  double* X;       // [p*p] input (assembled K), ping
  double* Y;       // [p*p] pong
  int p;           // padded dim (multiple of NB)
  int n;           // true dim (pads are identity)
  double* piv;     // [(p/NB) * NB*NB] pivot-block inverse scratch
  double* ldet;    // [p/NB] logdet contribution of each pivot block
  double* pst;     // refinement gate [2]: K_00, bits of max diag K^{-1} (gate_open)
  int* status;     // nonzero => not positive definite
  unsigned int* flag;  // large path: [3] hand-off / pivot-done / panel-row counters
  int wide;        // large path: 128-wide sweeps (else 64)
  int no_quarters; // 128-wide update: keep the last round in whole tiles (tests, GPK_FLAG_NO_QUARTER_TILES)
  int qfirst;      // 128-wide update: quarter items before whole tiles (GPK_FLAG_NO_QUARTER_FIRST: after)
  double* Z;       // large path: panel buffers [3][128][p] by sweep mod 3 (nullable: Y)
  // 128-wide update schedule (wide_schedule): per sweep, the tiles the launch updates and the
  // sweeps (1 or 2) each applies; null: every tile every sweep (the one-sweep form)
  const unsigned* sched;
};
// Two-sweep schedule of the 128-wide update (spdinv_big.hip): per sweep k of a factor with T2
// 128-tiles per dimension, row k of tab (stride wide_sched_stride(T2)) holds [0] the tile count,
// [1] the next pivot tile's entry, [2 + i] tile i's entry: J | I << 8 | two << 16 | c0 << 18 |
// c1 << 20 | c2 << 22 (codes 0, 1 = +1, 3 = -1).  paired = false: every tile every sweep.
int wide_sched_stride(int T2);
void wide_schedule(int T2, bool paired, std::vector<unsigned>& tab);
// Runs the full inverse; returns (via *final) the buffer that holds +K^{-1}.
// pivot0_done: pivot block 0 was already factored (by the assembly launch).
hipError_t launch_spd_inverse(SpdArgs* args, int nmat, double** final_out, hipStream_t s,
                              bool pivot0_done = false);
hipError_t launch_spd_stage(SpdArgs* args, int nmat, int stage, hipStream_t s);

// Persistent ("chain") form of the small-factor inverse (spdinv.hip): every sweep in one launch,
// ordered by flags; K^{-1} ends in X.  Gather mode (cid != nullptr) builds K from the distance
// classes first and writes Kc and D on the way (no assembly launch); otherwise X holds K.
// Augmented form: extra tile columns carry right-hand sides B = [B_u | D^T] through the same
// sweeps (the sweep operator's upper-right block), which end as K^{-1} B_u and K^{-1} D^T --
// the step's first solves (A = K1^{-1} U, Bt^T = K2^{-1} U^T) and the derivative solves
// (K^{-1} D^T) without GEMM launches of their own.
// Every workgroup waits on others, so the grid must be co-resident: gpk_create checks the
// grid against spd_chain_capacity (occupancy per CU x CUs: two per CU on a full MI355X -- 235
// VGPRs, 50 KB LDS each fit twice -- i.e. 512) and caps it at CHAIN_MAX_BLOCKS.
constexpr int CHAIN_MAX_BLOCKS = 512;
struct ChainArgs {
  double* X; double* PB; double* piv; double* ldet; double* pst; int* status;
  unsigned int* flags;  // [T*(T+tu+td) + 2T + 1], zero-initialised
  int p, n;
  const int* cid; const double* kval; const double* dval; const double* x; double jitter;
  double* Kc; double* D;
  int tu, td;                              // augmented tile columns: B_u, D^T (0: none)
  const double* Bu; int ldbu, bu_t;        // B_u[i][j] = bu_t ? Bu[j*ldbu+i] : Bu[i*ldbu+j]
  double* Ou; int ldou, ou_t;              // K^{-1} B_u (stored transposed when ou_t)
  double* Od; int ldod;                    // K^{-1} D^T
  double* PBa; int ldpba;                  // augmented panel buffer [p][32*(tu+td)]
  double* gran;                            // pivot-chain input slots [T][2][1024], CHAIN_SENTINEL
  double* PB2; unsigned int* epoch;        // chain_multi: hand-off slots [2][multi_half(p)]
                                           // (CHAIN_SENTINEL), launch counter (zeroed)
};
// one launch-parity half of chain_multi's hand-off slots: the panel [p*p], then L_k^{-1} of every
// pivot [p/32][1024]
__host__ __device__ inline size_t multi_half(int p) { return (size_t)p * p + (size_t)32 * p; }
// one launch-parity half of a chain handle's hand-off slots: chain_multi_kernel's panel slots +
// L^{-1} slots (multi_half), chain_kernel's L^{-1} slots alone (T x 32 x 32 words)
__host__ __device__ inline size_t chain_half(int p, bool multi) { return multi ? multi_half(p) : (size_t)32 * p; }
// bit pattern of an unwritten hand-off word: a signalling NaN (quiet bit clear), which no
// floating-point operation returns; equal 32-bit halves (hipMemsetD32 fills it)
constexpr unsigned long long CHAIN_SENTINEL = 0x7ff4dead7ff4deadull;
constexpr unsigned int CHAIN_SENTINEL32 = 0x7ff4deadu;
int spd_chain_blocks(const int* p, int nmat, bool aug);
// co-resident workgroups of the chain kernel variant on the current device (0 if unknown)
int spd_chain_capacity(int deriv, bool gather);
// chain_kernel's dispatch slot x of factor m's grid row -> its role: tile index I*TC + J, or
// T*TC for the pivot chain.  With ~390 workgroups on 256 CUs the dispatcher's second pass over
// the CUs doubles up the first ~130; the grid's middle (end of row 0, start of row 1) is alone
// on its CUs.  The pivot chain sits there (last of row 0, first of row 1), and next to it the
// 2(T-1) tiles whose sweep-k updates feed it -- panel (k, k+1) and diagonal (k+1, k+1) -- so
// that their hand-offs reach the chain's prefetch window; the other tiles keep their order.
__host__ __device__ inline int chain_role(int m, int x, int T, int TC) {
  const int nt = T * TC, nc = 2 * (T - 1);
  // critical tiles in ascending order: (0,1), (1,1), (1,2), (2,2), ...
  auto crit = [TC](int i) { return (i & 1) ? ((i >> 1) + 1) * (TC + 1) : (i >> 1) * (TC + 1) + 1; };
  int r;
  if (m == 0) {
    if (x == nt) return nt;
    if (x >= nt - nc) return crit(x - (nt - nc));
    r = x;
  } else {
    if (x == 0) return nt;
    if (x <= nc) return crit(x - 1);
    r = x - 1 - nc;
  }
  int tile = r;  // the r-th non-critical tile
  for (int i = 0; i < nc; ++i)
    if (crit(i) <= tile) ++tile;
  return tile;
}
// Multi-tile form for large factors (1D, p <= 2048 on a full MI355X): 64-row macro tiles of
// the lower triangle per workgroup + the pivot chain; no augmented columns.  Co-residency as
// above: gpk_create compares spd_chain_multi_blocks with spd_chain_multi_capacity.
int spd_chain_multi_blocks(const int* p, int nmat);
int spd_chain_multi_capacity(int deriv, bool gather);
hipError_t launch_spd_chain_multi(const ChainArgs* a, int nmat, int deriv, hipStream_t s,
                                  const PrepArgs* prep = nullptr, int q = 0);
// prep (nullable): the step constants are published by one extra workgroup of this launch
hipError_t launch_spd_chain(const ChainArgs* a, int nmat, int deriv, hipStream_t s,
                            const PrepArgs* prep = nullptr, int q = 0);

// Large-factor path (spdinv_big.hip): 64- or 128-wide pivots (SpdArgs::wide), panel + lower-tile
// MFMA update per sweep, next pivot factored inside the update launch.  In place: K^{-1} ends in
// X.  Y is used as the W x p panel buffer and piv as the W x W L^{-1} buffer + the 128-pivot's
// scratch (spd_big_piv_doubles).
// Chosen when the largest padded factor is >= SPD_BIG_MIN (or forced by a problem flag); the
// 128-wide sweeps from SPD_WIDE_MIN (or forced).
constexpr int SPD_BIG_MIN = 1600;
constexpr int SPD_WIDE_MIN = 3072;
size_t spd_big_piv_doubles(int p);
// tile workgroups per factor of the update launch (0: two per CU); tests use a few to get long
// runs of tiles per workgroup at small sizes
void spd_big_set_workgroups(int g);
// default poll budget of every bounded inter-workgroup wait (spd_pivot.h)
constexpr unsigned SPIN_CAP = 1u << 22;
// the bounded waits' poll budget of each translation unit that waits (spd_pivot.h g_wait_limit)
hipError_t wait_limit_spdinv(unsigned polls);
hipError_t wait_limit_spdbig(unsigned polls);
hipError_t wait_limit_assemble(unsigned polls);
hipError_t wait_limit_pgrad(unsigned polls);
hipError_t launch_spd_inverse_big(SpdArgs* args, int nmat, double** final_out, hipStream_t s);
// stage -1: pivot 0; 2k: panel of sweep k; 2k+1: update of sweep k
// (mirror = false: the last update launch leaves the upper triangle unmirrored -- bench timing)
hipError_t launch_spd_big_stage(SpdArgs* args, int nmat, int stage, hipStream_t s, bool mirror = true);
// MFMA work of update launch k as scheduled (bench accounting; spdinv_big.hip)
double spd_big_update_flops(const SpdArgs* args, int nmat, int k, bool with_pivot);
hipError_t launch_spd_big_tiles(SpdArgs* args, int nmat, int k, hipStream_t s);  // bench only
int spd_big_sweeps(int p, int wide);

// Iterative-refinement gate: a refinement GEMM/GEMV runs only when the factor's condition
// number may be large.  gate[0] = K_00 = max diagonal of K (written with pivot block 0),
// gate[1] = bit pattern of max_i (K^{-1})_ii (atomicMax by the last sweep); their product is a
// lower bound on cond_2(K) (lambda_max >= max K_ii, 1/lambda_min >= max K^{-1}_ii), observed
// 20-60x below cond for these kernels (tools/cond_track.py).  Below REFINE_COND_LB = 100 the
// explicit-inverse products are within ~1e-12 of the LU solves and refinement is skipped.
constexpr double REFINE_COND_LB = 100.0;

// Batched fp64 MFMA GEMM with fused epilogues.
enum Epi {
  EPI_STORE = 0,   // C = alpha*P1 + alpha2*P2 + beta*C0
  EPI_RESID = 1,   // C = alpha*P1 + alpha2*P2 - F (+ U(U^2-1) if ac) ; red += sum C^2
                   //     (+ red2 += sum Q1*Q2 when red2 != NULL)
  EPI_QUAD = 2,    // C = alpha*P1 + beta*C0 ; red += sum C*U
};
struct GemmDesc {
  const double* A; const double* B; int lda, ldb, ta, tb;
  const double* A2; const double* B2; int lda2, ldb2, ta2, tb2;
  double alpha, alpha2, beta;
  const double* C0; int ldc0;
  double* C; int ldc;
  int M, N, K, K2;          // padded (multiples of 32); K2 = 0 when no second product
  int epi;
  int ac;                   // EPI_RESID: Allen-Cahn term
  const double* F; const double* U; int ldf; // epilogue operands
  int vscale, vscale2;      // multiply alpha / alpha2 by v (StepScalars) when 1
  double* red;              // per-tile partial sums, [tiles] (nullable)
  double* red2; const double* Q1; const double* Q2;  // EPI_RESID: sum Q1*Q2 (quad term)
  const double* gate; int ngate;  // refinement gate (gate_open); nullptr = always store
  // side output (EPI_STORE): Y = 0.5 Ys + v C, with C the stored value -- the G_K operand
  // (S/2 + v X) formed where X is produced, so the G_K stage is a single product
  double* Y; const double* Ys; int ldy;
  int tag;                  // step stage (timeline probes only, gpk_trace.h)
  // 128x128-tile kernel only: a partial product added to alpha op(A) op(B) before the epilogue
  // (the first pass of a dual product, launch_gemm_auto's split)
  const double* Cp; int ldcp;
  // 16x16-tile kernel only: class sums of the stored G_K / G_D (cpart != nullptr; see
  // class_slots below).  bcid / bcbase: the axis' ClassArgs cid (leading dimension ldc) and
  // cbase, bn its true size; bsx (nullable): coordinates for the D_x1 sign s_ij
  double* cpart; const int* bcid; const int* bcbase; const double* bsx; int bn, bncls;
};
// Class tile partials (GemmDesc::cpart, round 6): the G_K / G_D producers sum their 16x16
// output tile per (signed diagonal, distance variant) and store each sum into the slot of its
// class, so the contraction adds per class class_slots(T) partials (T = 16x16 tiles per side)
// instead of a class-sum launch's chunk partials.  Diagonal s = i - j of class (k, v) lies in
// tile band b = I - J with |s - 16 b| <= 15: b = floor(s/16) (group 0) or floor(s/16) + 1
// (group 1); slot e = (sign(s) < 0, group, I - max(0, b)).  Layout [e][class]: a tile's slots
// for its ~31 consecutive diagonals are consecutive classes (whole-line stores), and the
// contraction's 16 consecutive classes per slot are one line.  Slots no tile maps to stay zero
// (allocated zeroed, never written).
__host__ __device__ inline int class_slots(int T) { return 4 * T; }
// epilogue threads: (signed diagonal offset in a 16x16 tile, variant v < 8 -- and v + 8: the
// epilogue handles diagonals of up to 16 variants; C4's grid has 9)
constexpr int CB_SLOTS = 31 * 8;
constexpr int CB_VMAX = 16;
constexpr int GEMM_MAX_BATCH = 4;
struct GemmBatch {  // passed by value (kernarg): no dependent descriptor load before the operands
  GemmDesc d[GEMM_MAX_BATCH];
};
// small = 1: 16x16-tile latency kernel (max_tiles counts 16x16 tiles); 0: 32x32 LDS-tiled.
// descs: HOST array of ndesc <= GEMM_MAX_BATCH descriptors (copied into the kernel arguments).
hipError_t launch_gemm_batch(const GemmDesc* descs, int ndesc, int max_tiles,
                             const StepScalars* sc, hipStream_t s, int small);
// heuristic: use the 16x16 latency kernel while the whole stage has few enough tiles
inline bool gemm_use_small(long tiles16_total) { return tiles16_total <= 16384; }
enum { GEMM_TILED32 = 0, GEMM_SMALL = 1, GEMM_BIG = 2, GEMM_HUGE = 3 };
// 128x128 tiles once a launch has this many of them (one round over the 256 CUs)
constexpr long GEMM_HUGE_MIN_TILES = 256;
// variant for a batch (force_big 1: the 64x64 throughput kernel, 2: the 128x128 one, regardless
// of size), tiles of a
// descriptor under a variant (= the entries its red/red2 partials fill), and the launcher
int gemm_variant(const GemmDesc* descs, int ndesc, int force_big);
int gemm_tiles(const GemmDesc& d, int variant);
hipError_t launch_gemm_auto(const GemmDesc* descs, int ndesc, const StepScalars* sc, hipStream_t s,
                            int variant);

__device__ __forceinline__ bool gate_open(const double* gate) {
  if (!gate) return true;
  const double k00 = gate[0];
  const double mx = __longlong_as_double(*reinterpret_cast<const long long*>(gate + 1));
  return mx * k00 > REFINE_COND_LB;
}

// GEMV y = alpha * A x + beta * C0 (A padded, op N), optional epilogues like GEMM
struct GemvDesc {
  const double* A; int lda; const double* x; double* y; int p; int rows;
  double alpha;
  const double* C0; double beta;
  int epi;           // EPI_STORE / EPI_RESID / EPI_QUAD
  int ac;
  const double* F; const double* U;
  const double* U0;  // Allen-Cahn offset: the term uses U + U0 (nullable)
  double* red;       // per-block partials
  double* red2; const double* Q1; const double* Q2;  // per-block partials of sum Q1*Q2
  const double* gate; int ngate;
  // class operand (cid != nullptr, A unused): A[i][j] = cv[cid[i*lda + j]], ident = 1 (K): + cdiag
  // (the jitter) on i == j and the identity on pads (cid < 0); ident = 0 (D): zero on pads --
  // bitwise the Kc / D matrices the inverse launch would have written, read as int32 ids (half
  // the bytes)
  const int* cid; const double* cv; double cdiag; int ident;
};
hipError_t launch_gemv(const GemvDesc& d, hipStream_t s);
int gemv_blocks(int rows);

// parameter-gradient contraction
struct PGradArgs {
  const double* x; int n; int p;
  const AxisConst* kc;
  const double* GK; const double* GD;     // 2D mode: materialised [p*p]
  const double* Kinv;                     // 1D mode
  const double* alpha; const double* beta; const double* R;  // 1D mode vectors
  double halfc;                           // 1D mode: 0.5*logdet flag
  int deriv;
  double* part;                           // [nblocks * 3*QMAX]
  // DD (class path, 2D, fused tail): the derivative fields and every sum after them in
  // double-double; part holds the partials' high parts, part_lo their low parts (null: fp64)
  double* part_lo;
  ClassArgs cls;                          // ncls > 0: class sums + per-class contraction
  // 2D class path: the G_K / G_D GEMM epilogues wrote class tile partials ([cslots][ncls],
  // GemmDesc::cpart) -- no class-sum launch, the contraction adds each class's slots in order
  const double* cpK; const double* cpD; int cslots;
};
struct TailArgs;  // stepk.h
// tail (nullable): the fused step tail carried by the same launch (stepk.h TailArgs)
hipError_t launch_pgrad(int kind, int q, int mode1d, const PGradArgs* a, int naxes,
                        int blocks_per_axis, const StepScalars* sc, hipStream_t s,
                        const TailArgs* tail = nullptr, int shard_rank = 0, int shard_n = 1);
int pgrad_blocks(int n);
int pgrad_class_blocks(int ncls);  // contraction blocks of the class path

}  // namespace gpk
