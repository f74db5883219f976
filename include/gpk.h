/*
 * gpk.h — C ABI of libgpk, the MI355X-native (gfx950, HIP) hot path of the GP-PDE solver.
 *
 * The reference (xuangu-fang/Gaussian-Process-Slover-for-High-Freq-PDE, pure Python + JAX)
 * has no FFI: its "operator surface" is a handful of Python methods.  Each entry point
 * below replaces one of them; the Python mirror in
 * gaussian-process-slover-for-high-freq-pde_amd/gpk/ binds them with ctypes
 * (INTEGRATION.md shows the binding).  References are to /root/reference/code/.
 *
 * Conventions
 *   - every function returns an int status (GPK_OK = 0); on failure gpk_last_error()
 *     returns a thread-local message.  No C++ exception crosses the ABI.
 *   - all pointers are HOST pointers unless a name ends in _dev; the library copies.
 *   - matrices are row-major; x1 indexes rows (kernel_matrix.py:26).
 *   - fp64 throughout (kernel_matrix.py:6-7 enables jax x64).
 *   - one handle = one HIP device + one HIP stream; calls on a handle are synchronous on
 *     return and not re-entrant; distinct handles are independent.
 */
#ifndef GPK_H_
#define GPK_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPK_ABI_VERSION 2  /* 2: gpk_problem.uoff (extra-GP second phase) */

/* status codes */
enum {
  GPK_OK = 0,
  GPK_EINVAL = 1,  /* bad argument (reference: assert / raise Exception('Invalid Kernel')) */
  GPK_ENOTPD = 2,  /* a covariance factor lost positive definiteness in the SPD inverse   */
  GPK_EHIP = 3,    /* HIP runtime error                                                    */
  GPK_ERCCL = 4,   /* RCCL error (sharded handles)                                         */
  GPK_ENOMEM = 5,  /* device allocation failed                                             */
  GPK_ENODEV = 6   /* no gfx950 device visible                                             */
};

/* kernel kinds: kernel_matrix.py:107-193 */
enum { GPK_SE_COS = 0, GPK_MATERN52_COS = 1, GPK_SE = 2, GPK_MATERN52 = 3 };

/* equation families: model_GP_solver_1d.py:108-116, model_GP_solver_2d.py:131-141,
 * model_GP_solver_advection.py:132-134 */
enum { GPK_POISSON = 0, GPK_ALLENCAHN = 1, GPK_ADVECTION = 2 };

/* Problem description = the solver constructor's arguments + trick_paras.
 *   1D (GP_solver_1d_single.__init__, model_GP_solver_1d.py:38-47):
 *       dim=1, n1=N_col, x1=X_col, src=src_col [n1], bvals=y [nb], bidx=Xind [nb]
 *   2D / advection (GP_solver_2d_single.__init__, model_GP_solver_2d.py:40-48):
 *       dim=2, x1=X_col[0] [n1], x2=X_col[1] [n2], src=src_vals [n1*n2],
 *       bvals=hstack(U[0,:],U[-1,:],U[:,0],U[:,-1]) [2*n2+2*n1], bidx=NULL
 */
typedef struct gpk_problem {
  int32_t dim;          /* 1 or 2 */
  int32_t eq;           /* GPK_POISSON | GPK_ALLENCAHN | GPK_ADVECTION (dim 2 only) */
  int32_t kind;         /* GPK_SE_COS .. GPK_MATERN52 */
  int32_t n1, n2;       /* collocation points per axis (n2 ignored for dim 1) */
  int32_t q;            /* mixture components Q (1..64) */
  const double* x1;
  const double* x2;
  const double* src;
  const double* bvals;
  const int32_t* bidx;  /* dim 1 only */
  int32_t nb;           /* dim 1: len(Xind); dim 2: ignored (2*n1+2*n2) */
  double jitter;        /* 1e-6 in the reference (model_GP_solver_2d.py:432) */
  double llk_weight;    /* trick_paras['llk_weight'] */
  double logdet;        /* trick_paras['logdet'] (1.0 / 0.0) */
  double beta;          /* advection speed (advection-sin.yaml:16); ignored otherwise */
  double lr, b1, b2, eps; /* optax.adam(lr) defaults b1=.9, b2=.999, eps=1e-8 */
  int32_t device;       /* HIP device ordinal */
  int32_t flags;        /* GPK_FLAG_* bits, normally 0 */
  /* dim 1 only, nullable [n1]: a frozen field u0 added to u inside the Allen-Cahn term,
   * (u+u0)((u+u0)^2-1) -- the extra GP's second phase, where the first GP's u is frozen
   * (model_GP_solver_1d_extra.py:86-98).  Its u_xx and u0[Xind] enter as shifted src / bvals. */
  const double* uoff;
} gpk_problem;

/* gpk_problem.flags bits */
#define GPK_FLAG_FORCE_BIG_GEMM 1 /* use the 64x64 throughput GEMM at every size (tests/tuning) */
#define GPK_FLAG_FORCE_BIG_SPD 2  /* use the 64-wide panel/update SPD inverse at every size */
#define GPK_FLAG_FORCE_SMALL_SPD 4 /* use the 32-wide sweep SPD inverse at every size */
#define GPK_FLAG_FORCE_HUGE_GEMM 8 /* use the 128x128 throughput GEMM at every size (tests/tuning) */
/* gpk_step / gpk_loss_grad run one of two captured step graphs: the full one, whose iterative-
 * refinement GEMM stages check a device-side cond(K) gate and skip themselves when it is closed,
 * or a fast one without those stages, chosen while the last observed gate value is 2x below its
 * threshold.  The fast graph checks the gate every step; a step that needed refinement makes the
 * call roll its batch back (params, Adam state) and rerun it with the full graph, so results are
 * bitwise those of the full graph. */
#define GPK_FLAG_NO_FAST_GRAPH 16  /* always run the full graph */
#define GPK_FLAG_FAST_FIRST 32     /* start in fast-graph mode (tests: exercises the rollback) */
/* The step evaluates the covariance fields once per distinct pair distance |x_i - x_j| of each
 * axis (exact fp64 classes, built at gpk_create; ~5n classes on a linspace grid instead of n^2
 * pairs) and contracts the hyper-parameter gradient per class.  K and D are bitwise the per-pair
 * evaluation's; the gradient sums differ only in summation order.  Grids with more than 32
 * distinct distances on one diagonal |i - j| = k fall back to the per-pair kernels. */
#define GPK_FLAG_NO_DCLASS 64      /* always use the per-pair kernels */
/* Small factors (sum of (p/32)^2 over the factors <= 256) are inverted by ONE persistent
 * launch whose workgroups order the pivot sweeps through flags; bitwise the per-sweep launches. */
#define GPK_FLAG_NO_CHAIN 128      /* one launch per pivot sweep instead */
/* 2D, unsharded, chain-sized: the inverse launch also carries U, U^T and D^T as augmented
 * columns of the sweep operator and ends with A = K1^{-1} U, Bt = U K2^{-1} and K^{-1} D^T,
 * which replace the step's first GEMM stage and fold the X1/X2 solves into the G_D stage. */
#define GPK_FLAG_NO_CHAIN_AUG 256  /* the chain inverts K only */
/* Large factors (the panel/update inverse): 128-wide sweeps from a padded size of 3072 (the update
 * is MFMA-bound instead of bound by the matrix traffic), 64-wide below (shorter serial pivots). */
#define GPK_FLAG_FORCE_WIDE_SPD 512   /* 128-wide sweeps at every size (with FORCE_BIG_SPD: tests) */
#define GPK_FLAG_FORCE_NARROW_SPD 1024 /* 64-wide sweeps at every size */
/* Row-sharded handles (nranks >= 2): the first half of the ranks inverts K1 only, the second half
 * K2 only, and the inverses (+ their log-det blocks and refinement gates) are broadcast from
 * ranks 0 and nranks/2 -- one Kronecker factor per rank group instead of both on every rank. */
#define GPK_FLAG_SPLIT_FACTORS 2048
/* 1D factors of padded size >= 1600 (the large-factor range): the persistent chain inverse on
 * 64-row macro tiles of the lower triangle, when its grid is co-resident (p <= 2048 on a full
 * MI355X); GPK_FLAG_NO_CHAIN or GPK_FLAG_FORCE_BIG_SPD select the launch-per-sweep path. */
#define GPK_FLAG_FORCE_CHAIN_MULTI 4096 /* the macro-tile chain at every 1D size (tests) */
/* Large 2D factors (P >= 1600): which solves get one (cond-gated) refinement step.  Default: the
 * forward solves A = K1^{-1} U, Bt = U K2^{-1}; REFINE_ALL: also S and X1 / X2 (every solve, as
 * the small-factor path, whose forward solves are refined on every step, ungated); NO_REFINE:
 * none at any size (explicit-inverse products only; accuracy studies). */
#define GPK_FLAG_REFINE_ALL 8192
#define GPK_FLAG_NO_REFINE 16384
/* Large 1D factors on the macro-tile chain: the inverse launch writes Kc and D as matrices and the
 * GEMVs read them (round-2 form; default: the GEMVs read class ids + class values and the
 * inverse writes neither). Bitwise the same results. */
#define GPK_FLAG_MATRIX_GEMV 32768
/* 128-wide SPD inverse: keep the update's last round of tiles whole (default: quarter tiles when
 * that round would leave most workgroups idle). Bitwise the same results. */
#define GPK_FLAG_NO_QUARTER_TILES 65536
/* Kernel-parameter contraction (distance classes): the derivative fields and every sum after
 * them in double-double (default only for factors of >= 3072 points, where the contraction's
 * cancellation amplifies the fields' fp64 rounding ~1e8-fold), at any size (DD_CONTRACTION) or
 * never (NO_DD_CONTRACTION). */
#define GPK_FLAG_DD_CONTRACTION 131072
#define GPK_FLAG_NO_DD_CONTRACTION 262144
/* 128-wide SPD inverse (factors >= 3072): every lower tile takes every sweep in its own pass
 * (default: tiles take sweeps in pairs, K = 256 per pass, half the tiles per launch). */
#define GPK_FLAG_ONE_SWEEP_UPDATE 524288
/* 128-wide SPD inverse: a tile workgroup with a quarter item works it after its whole tiles
 * (default: first, unless its first whole tile is in the next panel's row / column; A/B only).
 * Bitwise the same results. */
#define GPK_FLAG_NO_QUARTER_FIRST 1048576
/* Large 2D factors: refine only the axis-1 forward solve A = K1^{-1} U (not Bt = U K2^{-1}), as
 * the default does when beta >= 16 (advection); diagnostics (tools/c5_refine_diag.py). */
#define GPK_FLAG_REFINE_FWD1_ONLY 2097152
/* 2D factors with distance classes: the class sums of G_K / G_D by a class-sum launch over their
 * rows (default: the 16x16-tile GEMMs that produce them sum each output tile per class in their
 * epilogue, and the contraction adds those partials -- one launch fewer per step). */
#define GPK_FLAG_NO_CLASS_BINS 4194304
/* Chain-inverse handles with distance classes: every step of a multi-step batch evaluates its
 * class values in a launch of its own (default: step s + 1's class values are evaluated at the
 * end of step s's parameter-gradient launch, right after the kernel-parameter Adam, so steps
 * 2.. of a batch start with the inverse launch).  Bitwise the same results; A/B only. */
#define GPK_FLAG_NO_CLASS_PIPE 8388608

typedef struct gpk_handle gpk_handle;

int gpk_abi_version(void);
const char* gpk_last_error(void);
int gpk_device_count(int32_t* n);

/* Kernel_matrix.get_kernel_matrix (kernel_matrix.py:21-30) and the vmap'd derivative
 * covariances (model_GP_solver_2d.py:107-117, model_GP_solver_advection.py:107-117).
 * K_out[n1*n2] = kappa(x1_i, x2_j) + jitter*[i==j]  (pass jitter=0 for the rectangular
 * cross-covariance of preds, model_GP_solver_2d.py:198-202).
 * deriv 1: D_out = D_x1_kappa (kernel_matrix.py:49-52); deriv 2: DD_x1_kappa (:54-57);
 * deriv 0: D_out unused (may be NULL). */
int gpk_kernel_matrices(int32_t kind, int32_t deriv, const double* x1, int32_t n1,
                        const double* x2, int32_t n2, const double* logw, const double* logls,
                        const double* freq, int32_t q, double jitter, double* K_out,
                        double* D_out);

/* vmap(kappa) / vmap(D_x1_kappa) / vmap(DD_x1_kappa) over n elementwise pairs
 * (x1[e], x2[e]) -- the reference's per-pair kernel calls (kernel_matrix.py:26,
 * model_GP_solver_2d.py:107-117): out[e] for deriv 0 / 1 / 2.  No jitter. */
int gpk_kernel_pairs(int32_t kind, int32_t deriv, const double* x1, const double* x2, int64_t n,
                     const double* logw, const double* logls, const double* freq, int32_t q,
                     double* out);

/* Solver object: copies the problem to device memory; params start at the reference init
 * (train(), model_GP_solver_2d.py:245-261 / model_GP_solver_1d.py:203-213) with zero Adam
 * state.  freq_scale sets the initial frequencies linspace(0,1,Q)*freq_scale. */
int gpk_create(const gpk_problem* prob, double freq_scale, gpk_handle** out);
int gpk_destroy(gpk_handle* h);

/* SPD inverse path a handle's step uses (chosen at gpk_create from the factor sizes, the flags
 * and the device): 32-wide per-sweep launches, the persistent chain (K^{-1} only / augmented
 * with the first solves), or the large-factor path. */
enum { GPK_INV_SWEEP = 0, GPK_INV_CHAIN = 1, GPK_INV_CHAIN_AUG = 2, GPK_INV_BIG = 3, GPK_INV_BIG_WIDE = 4,
       GPK_INV_CHAIN_MULTI = 5 };
int gpk_inverse_path(const gpk_handle* h, int32_t* path);
/* The chain's workgroups wait on one another, so gpk_create uses it only when its grid fits the
 * device's co-resident capacity (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs).  This
 * overrides that capacity for handles created afterwards (workgroups > 0; 0 restores the device
 * query) -- tests use it to force the per-sweep fallback. */
int gpk_set_chain_capacity(int32_t workgroups);
/* Tile workgroups per factor of the large-factor inverse's update launch (0: the default, two per
 * CU).  Applies to every later launch; tests use a few to give each workgroup long tile runs. */
int gpk_set_spd_big_workgroups(int32_t workgroups);
/* Poll budget of every inter-workgroup wait of later launches on the current device (polls > 0;
 * 0 restores the default 2^22).  A wait that spends it -- a hand-off that never arrives, e.g. a
 * persistent grid that is not co-resident -- gives up instead of hanging the device, and every
 * other wait of the handle then gives up within 64 polls: the call returns GPK_ENOTPD ("hand-off
 * timed out") and a gpk_step batch is undone (see gpk_step).  Tests force that path with 1 (every
 * wait whose first poll fails gives up). */
int gpk_set_wait_limit(int32_t polls);
/* Tests: apply the poll budget only while gpk_step runs chunk `chunk` (0-based, 64-step chunks)
 * of a later call; polls = 0 clears it. */
int gpk_set_wait_limit_chunk(int32_t polls, int32_t chunk);

/* Graph selection state (see GPK_FLAG_NO_FAST_GRAPH): *fast = 1 if the next gpk_step uses the
 * fast graph, *rollbacks = batches rerun with the full graph so far.  Either pointer may be NULL. */
int gpk_graph_mode(const gpk_handle* h, int32_t* fast, int64_t* rollbacks);

/* Distance classes (GPK_FLAG_NO_DCLASS) of one coordinate axis x[n], host only (no device):
 * *ncls = classes (distinct |x_i - x_j| per diagonal |i - j|), *vmax = the most on one diagonal;
 * *ncls = 0 when that exceeds 32 (the step then uses the per-pair kernels).
 * gpk_class_count: the classes a handle's step uses on axis 0 / 1 (0 = per-pair kernels). */
int gpk_distance_classes(const double* x, int32_t n, int32_t* ncls, int32_t* vmax);
int gpk_class_count(const gpk_handle* h, int32_t axis, int32_t* ncls);
/* How a 2D class-path step sums G_K / G_D per class: *epilogue = 1 when the GEMMs that produce
 * them write class tile partials (GPK_FLAG_NO_CLASS_BINS off, <= 16 variants per diagonal,
 * 16x16-tile GEMM stages, unsharded), 0 when a class-sum launch reads the matrices. */
int gpk_class_sum_path(const gpk_handle* h, int32_t* epilogue);
/* *on = 1 when a multi-step batch evaluates step s + 1's class values at the end of step s's
 * parameter-gradient launch (chain-inverse handles with distance classes, unsharded,
 * GPK_FLAG_NO_CLASS_PIPE off), 0 when every step launches its own class-value evaluation. */
int gpk_class_pipe(const gpk_handle* h, int32_t* on);

/* Latency-tuning probes (libgpk_trace.so, `make trace`; the product library returns GPK_EINVAL):
 * per timeline slot (csrc/gpk_trace.h) the first-arrival / last-departure device clock
 * (100 MHz) since the last gpk_trace_reset.  n >= 128. */
int gpk_trace_reset(void);
int gpk_trace_read(uint64_t* lo, uint64_t* hi, int32_t n);

/* Flat parameter layout = jax's pytree leaf order (dict keys sorted):
 *   2D: [U (n1*n2, row-major), k1.freq[Q], k1.log-ls[Q], k1.log-w[Q],
 *        k2.freq[Q], k2.log-ls[Q], k2.log-w[Q], log_tau, log_v]
 *   1D: [freq[Q], log-ls[Q], log-w[Q], log_tau, log_v, u[n1]]                       */
int gpk_num_params(const gpk_handle* h, int64_t* n);
int gpk_set_params(gpk_handle* h, const double* flat, int64_t n);
int gpk_get_params(gpk_handle* h, double* flat, int64_t n);
/* Adam state (optax ScaleByAdamState: count, mu, nu), same flat layout */
int gpk_set_opt_state(gpk_handle* h, int64_t count, const double* mu, const double* nu, int64_t n);
int gpk_get_opt_state(gpk_handle* h, int64_t* count, double* mu, double* nu, int64_t n);

/* value_and_grad(loss) at the current params (model_GP_solver_2d.py:145-174,179);
 * grad_flat may be NULL. */
int gpk_loss_grad(gpk_handle* h, double* loss, double* grad_flat);

/* n_steps x step() (model_GP_solver_2d.py:176-183): loss + full gradient + Adam update,
 * params and Adam state device-resident.  losses[n_steps] receives the loss evaluated
 * BEFORE each update (as step() returns it); may be NULL.  Returns once the losses and the
 * device status of the call are final: the last step's U update may still be running, like
 * the reference's asynchronously dispatched jax step; every later call on the handle is ordered
 * after it, and gpk_sync waits for it.  Batches: when the handle has a fast graph (every handle
 * but the row-sharded ones and the large 2D factors), a call is split into 64-step chunks + the
 * remainder, on the fast and on the full (refining) graph alike, and every chunk is a batch of
 * its own; otherwise the whole call is one batch.  A batch that fails on the device -- GPK_ENOTPD:
 * a non-positive pivot or a hand-off timeout -- is undone: params, Adam state and step count are
 * restored from the snapshot the batch took at its start.  Earlier chunks of the same call stay
 * applied (their losses are written), so a failed call may have advanced the handle by a
 * multiple of 64 steps. */
int gpk_step(gpk_handle* h, int32_t n_steps, double* losses);

/* Wait until every launch enqueued on the handle has finished (timing). */
int gpk_sync(gpk_handle* h);

/* Capture and instantiate every step graph a gpk_step(n_steps) call can launch (full and fast,
 * single-step and multi-step) without running a step: graph construction is a one-time host
 * cost of the first call otherwise.  Params and Adam state are untouched. */
int gpk_prepare(gpk_handle* h, int32_t n_steps);

/* preds (model_GP_solver_2d.py:185-220 / model_GP_solver_1d.py:160-180) at the current
 * params: 2D out[m1*m2] (row-major, x-test indexes rows); 1D out[m1] (xte2 ignored). */
int gpk_predict(gpk_handle* h, const double* xte1, int32_t m1, const double* xte2, int32_t m2,
                double* out);

/* compute_early_stopping (model_GP_solver_2d.py:222-233): bgap/Nb + egap/Nc */
int gpk_criterion(gpk_handle* h, double* out);

/* value_and_grad_kernel (model_GP_solver_2d.py:87-121 / model_GP_solver_1d.py:80-99) at the
 * current params, computed on the device; `what` selects one field, out gets it unpadded:
 *   2D: 0 K1 [n1*n1], 1 K2 [n2*n2], 2 K1inv_U [n1*n2], 3 K2inv_Ut [n2*n1], 4 U_xx [n1*n2],
 *       5 U_yy [n1*n2]   (advection: U_x, U_y); the reverse pass's kernel-parameter operands
 *       (diagnostics): 6 G_K1, 7 G_D1 [n1*n1], 8 G_K2, 9 G_D2 [n2*n2] (the weights of
 *       sum_ij G_K dK/dtheta + G_D dD/dtheta), 10 K1^{-1} [n1*n1], 11 K2^{-1} [n2*n2],
 *       12 K1^{-1} D1^T [n1*n1], 13 K2^{-1} D2^T [n2*n2] (augmented chain path only), 14 R,
 *       15 X1, 16 X2, 17 S [n1*n2] (model_GP_solver_2d.py:133 residual),
 *       18 Kc1, 19 Kc2 (the step's kept copy of K, refinement residuals), 20 D1, 21 D2 (the
 *       step's derivative blocks) -- the matrices as the last step assembled them; 22 K1,
 *       23 K2, 24 D1, 25 D2 expanded on the host from the distance-class table (class ids +
 *       class values; handles with classes), the gathers' reference
 *   1D: 0 K [n*n], 2 Kinv_u [n], 4 u_xx [n]; 6 K, 7 D [n*n] as the last step assembled them                                                */
int gpk_forward_field(gpk_handle* h, int32_t what, double* out, int64_t n);

/* Per-stage device timings (HIP events on the handle's stream) of one step, averaged over
 * `iters` eager (non-graph) steps run on a saved copy of the state: out_us[stage], names via
 * gpk_stage_name(h, stage).  Returns #stages in *n. */
int gpk_profile_stages(gpk_handle* h, int32_t iters, double* out_us, int32_t cap, int32_t* n);
const char* gpk_stage_name(const gpk_handle* h, int32_t stage);

/* Standalone SPD factor+inverse of the assembled K factor(s) at the current params,
 * `iters` times on the handle's stream; returns average microseconds per call. */
int gpk_time_spd_inverse(gpk_handle* h, int32_t iters, double* avg_us);

/* One kernel of the step, launched `iters` times back to back on the handle's stream
 * between two HIP events (after one full step so its inputs are valid; every listed kernel
 * is idempotent).  name: "assemble" | "sweep" | "gemm_B" | "pgrad" | "spd_chain" | "gather";
 * large-factor inverse: "sweep" / "spd_tiles" (update launch 0 with / without its pivot
 * workgroup), "spd_updates" (every update launch of one inverse, averaged per launch),
 * "spd_pivot" | "spd_panel".  Returns the average device time per launch and the kernel's
 * ALGORITHMIC work per launch (flops, HBM bytes; DESIGN.md §Measurement defines them; the
 * large-factor update launches are credited the tile products their lists schedule). */
int gpk_bench_kernel(gpk_handle* h, const char* name, int32_t iters, double* avg_us,
                     double* alg_flops, double* alg_bytes);

/* The step's fp64 MFMA GEMM kernels on host operands (row-major, device 0), for tests and
 * rate measurements: C = alpha op(A) op(B) + alpha2 op(A2) op(B2) + beta C0, op = transpose
 * when ta / tb / ta2 / tb2; K2 = 0 drops the second product; C0 may equal C (in-place
 * update) or be NULL.  variant: 0 auto (the step's size rule), 1 16x16 latency tiles, 2 64x64
 * tiles, 3 the 128x128 pipelined tile (model_GP_solver_2d.py:104-119's solves and products
 * are these GEMMs here).  M, N, K, K2 multiples of 32 (the step's padding contract); lda etc.
 * in elements.  iters > 0 times that many back-to-back launches with HIP events after the
 * checked one and returns the average microseconds in *avg_us (may be NULL when iters = 0;
 * written only on success).  C receives the checked launch's result; with C0 == C the timed
 * launches keep updating the device copy in place (same work, each on the last one's output). */
int gpk_dgemm(int32_t variant, int32_t M, int32_t N, int32_t K, double alpha, const double* A,
              int32_t lda, int32_t ta, const double* B, int32_t ldb, int32_t tb, int32_t K2,
              double alpha2, const double* A2, int32_t lda2, int32_t ta2, const double* B2,
              int32_t ldb2, int32_t tb2, double beta, const double* C0, double* C, int32_t ldc,
              int32_t iters, double* avg_us);

/* The 128-wide SPD inverse's two-sweep update schedule (host only, no device): for T2 128-tiles
 * per dimension, T2 rows of wide_sched_stride(T2) = 2 + T2 (T2 + 1) / 2 words -- per sweep k the
 * tile count, the next pivot tile's entry, then the entries J | I << 8 | two << 16 | c0 << 18 |
 * c1 << 20 | c2 << 22 (coefficient codes 0, 1 = +1, 3 = -1; the tile's new value is
 * c0 X + c1 Z_{k-1}^T Z_{k-1} + c2 Z_k^T Z_k).  paired = 0: the one-sweep form.  Writes at most
 * cap words; returns GPK_EINVAL when cap is too small.  For tests and tools. */
int gpk_wide_schedule(int32_t T2, int32_t paired, uint32_t* out, int64_t cap);

/* ---- Row-sharded 2D step across GPUs (the reference has no multi-GPU path).
 * Every rank holds the problem, forms both Kronecker factors' K, D, K^{-1} itself, and computes
 * its block of rows of every product of the step (model_GP_solver_2d.py:87-183 /
 * advection :87-179); operands read beyond a rank's rows are completed by in-place all-gathers,
 * the kernel-parameter partials and per-tile loss partials by all-reduces.  Loss, gradients of
 * the small params and their Adam update are identical on every rank; Adam on U updates the
 * rank's rows (gathered after the step).  gpk_step / gpk_loss_grad run this step on a sharded
 * handle; gpk_loss_grad's U gradient is valid on the rank's rows only (gpk_shard_info). */

/* 128-byte RCCL communicator id: rank 0 creates it, every rank passes the same bytes. */
int gpk_comm_unique_id(uint8_t* out, int32_t len);
/* One rank (one process, device = problem.device) of an RCCL (xGMI) group of nranks. */
int gpk_create_sharded(const gpk_problem* p, double freq_scale, int32_t rank, int32_t nranks,
                       const uint8_t* comm_id, gpk_handle** out);
/* nranks handles on ONE device in this process, exchanging through device copies (the same
 * sharded step without RCCL: tests on a single GPU).  Driven by gpk_group_step /
 * gpk_group_loss_grad (one host thread per rank); gpk_step on them returns GPK_EINVAL. */
int gpk_group_create(const gpk_problem* p, double freq_scale, int32_t nranks, gpk_handle** out);
int gpk_group_step(gpk_handle** hs, int32_t nranks, int32_t n_steps, double* losses);
/* loss and the FULL flat gradient (U rows collected from their owners) */
int gpk_group_loss_grad(gpk_handle** hs, int32_t nranks, double* loss, double* grad_flat);
/* this handle's rank, group size and rows [row0, row0 + rows) of U it owns */
int gpk_shard_info(const gpk_handle* h, int32_t* rank, int32_t* nranks, int32_t* row0, int32_t* rows);
/* the sharded step's plan as text (NUL-terminated, <= cap bytes): per GEMM stage "s<k>:" and one
 * mode letter per product -- r = this rank's output rows, k = its share of the contraction
 * index, f = whole (replicated) -- then " g<buffer>" for each all-gather after that stage; the
 * step ends with "ar" (its one all-reduce: status, contraction partials, loss partials) and "gU"
 * (U rows after Adam).  gpk/shard.py shard_plan restates it (tests/test_shard.py). */
int gpk_shard_plan(const gpk_handle* h, char* out, int64_t cap);

/* ---- 3-axis Kronecker solver (the d > 2 generalisation) ------------
 * The reference's GP_solver_2d_single log joint (model_GP_solver_2d.py:87-183) with
 * K = K1 (x) K2 (x) K3 on a tensor grid: prior -1/2 c sum_k (prod_{j!=k} N_j) logdet K_k -
 * 1/2 <U, K^{-1} U> (the 2-axis weights :157-162), residual sum_k (D_k K_k^{-1}) x_k U - F
 * [+ U(U^2-1)], boundary on the six faces.  Flat params (sorted-key pytree order): U
 * [n1*n2*n3 row-major], k1.{freq, log-ls, log-w}[Q], k2..., k3..., log_tau, log_v. */
typedef struct gpk_problem3 {
  int32_t eq;           /* GPK_POISSON | GPK_ALLENCAHN */
  int32_t kind;         /* GPK_SE_COS .. GPK_MATERN52 */
  int32_t n1, n2, n3;   /* collocation points per axis */
  int32_t q;            /* mixture components Q (1..64) */
  const double* x1;
  const double* x2;
  const double* x3;
  const double* src;    /* [n1*n2*n3] row-major */
  const double* bvals;  /* faces U[0], U[-1], U[:,0], U[:,-1], U[:,:,0], U[:,:,-1], each row-major:
                         * [2(n2 n3 + n1 n3 + n1 n2)] */
  double jitter, llk_weight, logdet;
  double lr, b1, b2, eps;
  int32_t device;
  int32_t flags;        /* reserved, 0 */
} gpk_problem3;

typedef struct gpk_handle3 gpk_handle3;
int gpk_create3(const gpk_problem3* p, double freq_scale, gpk_handle3** out);
int gpk_destroy3(gpk_handle3* h);
int gpk_num_params3(const gpk_handle3* h, int64_t* n);
int gpk_set_params3(gpk_handle3* h, const double* flat, int64_t n);
int gpk_get_params3(gpk_handle3* h, double* flat, int64_t n);
/* loss and full gradient at the current params (no update) */
int gpk_loss_grad3(gpk_handle3* h, double* loss, double* grad_flat);
/* n_steps of loss + gradient + Adam, device-resident; losses[n_steps] nullable */
int gpk_step3(gpk_handle3* h, int32_t n_steps, double* losses);

#ifdef __cplusplus
}
#endif
#endif /* GPK_H_ */
