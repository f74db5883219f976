// stepk.h — argument blocks of the step-tail kernels (loss, reductions, Adam).
#pragma once
#include "gpk_internal.h"

namespace gpk {

// Flat-parameter layout (jax pytree order, include/gpk.h) plus padded device geometry.
struct Layout {
  int dim, naxes, q;
  int n1, n2, p1, p2;   // true / padded sizes (1D: n2 = p2 = 1)
  int off_u;            // U (2D) / u (1D)
  int off_kp[2];        // start of (freq, log-ls, log-w) per axis
  int off_tau, off_v;
  int off_small, nsmall;  // contiguous non-U block (kernel params + log_tau + log_v)
  int64_t nparams;
};

struct AdamHyper {
  double lr, b1, b2, eps;
};

// Per-batch bookkeeping around the steps of one host call (gpk_step): begin = the rollback
// snapshot and counter resets before the first step, report = the end-of-batch record.  Graphs
// fold both into step launches where they can (PrepArgs.snap*, FinalizeArgs.report); the
// kernels below run them on their own otherwise.
struct StepBegin {
  double* snap; const double* params; const double* m; const double* v; size_t np;
  int* snap_count; const int* count;
  unsigned int* viol;   // nullable
  int* loss_slot;
};
struct StepReport {
  const int* status; const unsigned int* viol;  // viol nullable
  const double* pst[2];                         // nullable per axis
  const double* losses; int nloss;              // the batch's losses -> out[8 ..]
  double* out;                                  // [8 + nloss], pinned host memory
};
struct FinalizeArgs {
  Layout L;
  AdamHyper hyper;
  double llk_weight, logdet;
  int apply, has_cos;
  const double* red_quad; int nquad;
  const double* red_egap; int negap;
  const double* ldet[2]; int nldet[2];
  const double* pg;          // reduced [naxes][3*QMAX]
  const AxisConst* kc;
  const StepScalars* sc;
  const double* Up;          // padded U (2D, stride p2) / u (1D)
  const double* bvals;
  const int* bidx; int nb;   // 1D
  double* params; double* grad; double* m; double* v;
  double* losses; int* loss_slot;
  double* diag;              // [8]: loss, logdet1, logdet2, quad, egap, bgap
  const double* bgap;        // [bgap_parts] ||u_b - b||^2 at the start of the step (assembly
  int bgap_parts;            // launch, PrepArgs::bgap), added in order
  // fast graph (refinement stages left out): the refinement gate of each axis is checked here
  // and an open one raises *viol, after which the host rolls the batch back and reruns it
  // with the refinement stages (gpk_step).  watch[a] = nullptr: not checked.
  const double* watch[2]; unsigned int* viol;
  // last step of a batch in a captured call: the loss workgroup writes the batch report itself
  // (after this step's loss), in place of a separate step_report launch
  int report; StepReport rep;
  // fused tail (part 2): each thread forms its kernel parameters' pg entries itself from the
  // group partials (gpart [naxes * ngpa][3 QMAX], + gpart_lo: double-double) in group order,
  // with its other loads in the same round trip, and stores them to pg_out; null: read pg
  const double* gpart; const double* gpart_lo; int ngpa; double* pg_out;
  // nullable [nsmall]: the kernel parameters after this step's Adam (index idx - L.off_small),
  // stored write-through (sc1) by the Adam block for the next step's class values (the guide's
  // sc1 hand-off: pgrad.hip pgrad_tail raises TailArgs::nce_flag after them)
  double* kp_wt;
};

struct AdamUArgs {
  Layout L;
  AdamHyper hyper;
  double llk_weight;
  int apply, ac;
  const StepScalars* sc;
  // 2D: gU = S + v (X1 + X2) (X1 includes beta for advection); 1D: gu = X1 + v X2 (alpha, beta)
  const double* S; const double* X1; const double* X2; const double* R;
  double* Up;
  const double* U0;  // 1D Allen-Cahn offset (extra-GP second phase), nullable
  int e0, e1;        // element range [e0, e1) of the solution grid (row-sharded step); e1 = 0: all
  const double* bvals;
  const int* bidx; int nb;
  double* params; double* grad; double* m; double* v;
};

// Fused tail of a step, carried by the parameter-gradient launch (pgrad.hip): one extra grid
// plane of blocks runs dL/dU + Adam on U, and the parameter-gradient partials are reduced by a
// two-level "last block" scheme (fixed summation order: deterministic) whose final block runs
// the loss / small-parameter Adam (finalize_body).
struct TailArgs {
  int fused;                 // 0: pgrad only (separate reduce/finalize/adam launches)
  FinalizeArgs fin;
  AdamUArgs adam;
  unsigned int* gcount;      // [naxes * ngpa] level-1 counters (zero; re-armed in the kernel)
  unsigned int* top;         // level-2 counter
  double* gpart;             // [naxes * ngpa][3*QMAX] group partials
  double* pg;                // [naxes][3*QMAX] reduced parameter gradients (-> fin.pg)
  int tg, ngpa;              // blocks per group, groups per axis
  double* gpart_lo;          // DD contraction: the group partials' low parts (null: fp64)
  // pipelined class values (null: off): the launch carries naxes more planes that evaluate the
  // NEXT step's class values (pgrad.hip next_class_values); the block that runs the kernel-
  // parameter Adam raises *nce_flag after it (agent release), the planes wait for it (bounded,
  // status bit 2 on a lost hand-off) and read the updated parameters
  unsigned int* nce_flag;
  int* nce_status;
};

hipError_t launch_step_begin(const StepBegin& b, hipStream_t s);
hipError_t launch_step_report(const StepReport& r, hipStream_t s);

hipError_t launch_prep2(const double* params, const Layout& L, AxisConst* kc, StepScalars* sc,
                        int* count, int apply, double b1, double b2, hipStream_t s);
hipError_t launch_reduce_parts(const double* part, int bpa, int naxes, int q, double* out,
                               hipStream_t s);
hipError_t launch_finalize(const FinalizeArgs& f, hipStream_t s);
hipError_t launch_adam_u(const AdamUArgs& a, hipStream_t s);
hipError_t launch_sync_u(const double* params, const Layout& L, double* Up, hipStream_t s);
hipError_t launch_params_from_up(const double* Up, const Layout& L, double* params, hipStream_t s);
hipError_t launch_add_into(double* dst, const double* src, size_t n, hipStream_t s);
hipError_t launch_status_f64(int* st, double* x, int mode, hipStream_t s);

}  // namespace gpk
