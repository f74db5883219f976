// gpk_api.cpp — C ABI of libgpk (include/gpk.h): solver handles, device buffers, the
// captured HIP graph of one log-joint step, and the standalone entry points.
//
// One handle = the reference's solver object (GP_solver_1d_single / GP_solver_2d_single /
// GP_solver_2d_single_advection, code/model_GP_solver_{1d,2d,advection}.py) with its params
// and optax state resident in HBM.  step() (model_GP_solver_2d.py:176-183) is one replay of
// a hipGraph that holds every kernel of the step in stream order:
//   prep -> assemble K,D -> SPD inverse (+logdet) -> GEMM stages A..E (2D) | GEMVs (1D)
//   -> hyperparameter-gradient contraction -> deterministic reduction -> loss + Adam.
// A row-sharded handle (gpk_create_sharded / gpk_group_create) runs the 2D step across ranks:
// see "row-sharded multi-GPU step" below.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <sched.h>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <map>
#include <vector>

#include "../../include/gpk.h"
#include "gpk_internal.h"
#include "stepk.h"
#include "gpk_trace.h"

using namespace gpk;

static thread_local std::string g_err;
static std::atomic<int> g_chain_cap{0};  // gpk_set_chain_capacity override (0: query the device)
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail(e_ == hipErrorOutOfMemory ? GPK_ENOMEM : GPK_EHIP,                   \
                  std::string(#x) + ": " + hipGetErrorString(e_));                     \
  } while (0)

namespace {

constexpr int LOSS_CAP = 4096;
const char* kStageNames1D[] = {"prep", "assemble", "spd_inverse", "gemv_alpha", "gemv_alpha_res",
                               "gemv_alpha_fix", "gemv_resid", "gemv_DtR", "gemv_beta",
                               "gemv_beta_res", "gemv_beta_fix", "pgrad_tail"};
const char* kStageNames2D[] = {"prep", "assemble", "spd_inverse", "gemm_A", "gemm_A_res",
                               "gemm_A_fix", "gemm_B", "gemm_B_res", "gemm_B_fix", "gemm_C",
                               "gemm_D", "gemm_D_res", "gemm_D_fix", "gemm_E", "pgrad_tail"};
constexpr int kMaxStages = 18;
constexpr int kGemmStages = 11;  // A, A_res, A_fix, B, B_res, B_fix, C, D, D_res, D_fix, E

struct DevSwitch {  // restore the caller's current device on scope exit
  int prev = -1;
  explicit DevSwitch(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DevSwitch() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

struct Stage {
  int off = 0, n = 0, variant = 0;
  bool gated = false;  // every descriptor is a refinement GEMM (left out of the fast graph)
};

}  // namespace

struct ShardComm;  // collective backend of a row-sharded handle (RCCL, or an in-process group)
struct ShardGather {
  double* buf;
  size_t chunk;     // doubles per rank (a block of rows), rank r's block at buf + r * chunk
};

struct gpk_handle {
  gpk_problem prob{};
  double freq_scale = 0.0;
  Layout L{};
  AdamHyper hyper{};
  int dev = 0;
  hipStream_t s = nullptr;
  std::vector<void*> allocs;

  double *x1 = nullptr, *x2 = nullptr, *F = nullptr, *bvals = nullptr;
  int* bidx = nullptr;
  double *params = nullptr, *grad = nullptr, *m = nullptr, *v = nullptr, *Up = nullptr;
  AxisConst* kc = nullptr;
  StepScalars* sc = nullptr;
  int *count = nullptr, *loss_slot = nullptr, *status = nullptr;
  // batch begin / report folded into the next enqueued step (capture_call, capture_calln): the
  // step that takes one clears its pointer
  const StepBegin* fold_begin = nullptr;
  const StepReport* fold_report = nullptr;
  double *losses = nullptr, *diag = nullptr;
  double* stat_x = nullptr;  // [2] status bits as doubles (split-factor group all-reduce)

  double *K[2] = {}, *Kb[2] = {}, *D[2] = {}, *Kinv[2] = {}, *piv[2] = {}, *ldet[2] = {};
  int nldet[2] = {0, 0};
  // 2D work
  double *A = nullptr, *Bt = nullptr, *S = nullptr, *R = nullptr, *T1 = nullptr, *T2 = nullptr,
         *X1 = nullptr, *X2 = nullptr, *W1 = nullptr, *W2 = nullptr;  // W: refinement residuals
  double *Y1 = nullptr, *Y2 = nullptr;  // S/2 + v X1, S/2 + v X2 (the G_K operands)
  double *GK[2] = {}, *GD[2] = {};
  // 2D class path: class tile partials of G_K / G_D written by their GEMM epilogues
  // ([class_slots(P/16)][ncls] per axis; GemmDesc::cpart); cp_on: the stages use them
  double *cpK[2] = {}, *cpD[2] = {};
  bool cp_on = false;
  // 1D work
  double *alpha = nullptr, *tvec = nullptr, *beta = nullptr;
  double *red_quad = nullptr, *red_egap = nullptr;
  int nquad = 0, negap = 0;
  double *pgpart = nullptr, *pg = nullptr;
  double *pgpart_lo = nullptr, *tgpart_lo = nullptr;  // DD contraction (pg_dd): low parts
  bool pg_dd = false;                 // kernel-parameter contraction in double-double
  int bpa = 0;
  // fused step tail (pgrad launch): group counters / partials, boundary gap
  unsigned int *tcount = nullptr, *ttop = nullptr;
  double *tgpart = nullptr, *bgap = nullptr;
  int bgap_parts = 1;                 // PrepArgs::bgap_parts
  int ttg = 0, tngpa = 0;
  std::vector<GemmDesc> hdescs;  // per-stage GEMM descriptors (kernel arguments)
  Stage st[kGemmStages];
  double *Kc[2] = {}, *pst[2] = {};  // kept K (refinement residuals), pivot stats (gate)
  unsigned int* aflag[2] = {};        // assembly -> pivot-0 hand-off counters (small path) /
                                      // update -> pivot hand-off counters (large path)
  bool bigspd = false;                // large-factor SPD inverse (spdinv_big.hip)
  bool bigwide = false;               // ... with 128-wide sweeps
  bool chain_multi = false;           // persistent inverse on macro tiles (large 1D factors)
  // large 1D factors with distance classes: the GEMVs read Kc and D as class ids + class values
  // (GemvDesc::cid), so the inverse launch's gather writes neither matrix (64 MB at C2)
  bool cls_gemv = false;
  double* Zp[2] = {};                 // ... its panel buffers [3][128][P] (by sweep mod 3)
  unsigned* wsched[2] = {};           // ... its two-sweep update schedule (wide_schedule)
  bool chain = false;                 // small factors: persistent one-launch inverse (chain_kernel)
  bool chain_aug = false;             // ... which also solves A, Bt^T and K^{-1} D^T (2D, unsharded)
  unsigned int* cflags[2] = {};       // its hand-off flags [T*(T+taug) + 2T + 1] per factor
  double* cgran[2] = {};              // its pivot-chain input slots [T][2][1024] per factor
  double* PB2[2] = {};                // chain_multi: panel slots [2][P*P] by launch parity
  unsigned int* cepoch[2] = {};       // chain_multi: launch counter per factor
  double *PD[2] = {}, *PBa[2] = {};   // K_a^{-1} D_a^T; augmented panel buffers
  ClassArgs cls[2] = {};              // distance classes per axis (ncls = 0: per-pair path)
  double* rvec = nullptr;            // 1D refinement residual
  double* uoff = nullptr;            // 1D Allen-Cahn offset (gpk_problem.uoff), or null
  // predict scratch
  GemmDesc* pdescs = nullptr;

  // row-sharded step: this rank computes rows [rank*h, (rank+1)*h) of every GEMM output
  bool shard = false;
  int rank = 0, nranks = 1;
  int split_axis = -1;                // GPK_FLAG_SPLIT_FACTORS: the factor this rank inverts
  int h1 = 0, h2 = 0;                 // row-block heights of the P1- and P2-row outputs
  ShardComm* comm = nullptr;
  std::vector<GemmDesc> sdescs;       // row slices of hdescs
  Stage sst[kGemmStages];
  std::vector<ShardGather> sgather[kGemmStages];
  // the one per-step all-reduce of a sharded handle: [status (2) | pg | egap | quad] contiguous
  double* sred = nullptr;
  std::string splan;                  // the step's shard plan (gpk_shard_plan; gpk/shard.py)

  hipGraphExec_t g_exec[2] = {nullptr, nullptr};  // [apply] full step graph
  hipGraphExec_t g_fast[2] = {nullptr, nullptr};  // [apply] without the refinement stages
  // STEP_GRAPH_REPS training steps back to back in one graph ([0] fast, [1] full): one host
  // launch per group of steps (a graph launch boundary costs ~5-9 us of idle GPU)
  hipGraphExec_t g_multi[2] = {nullptr, nullptr};
  // batch graphs of exactly `reps` steps ([0] fast, [1] full), captured by gpk_prepare for the
  // chunk sizes a call of its step count runs (FAST_CHUNK and the remainder): a prepared call is
  // one graph launch per chunk
  std::map<int, hipGraphExec_t> g_batch[2];
  // fast chunks of a prepared step(n) call as whole-call graphs: batch begin (the rollback
  // snapshot) + `reps` steps + the pinned-memory report -- one launch and one synchronisation
  // per chunk (capture_call's form for step(1))
  std::map<int, hipGraphExec_t> g_calln;
  // one step(1) call as one graph ([0] fast, [1] full): batch begin (snapshot, counters), the
  // step, and the pinned-memory report -- the reference's one-call-per-iteration loop shape
  hipGraphExec_t g_call[2] = {nullptr, nullptr};
  bool fast_ok = false;    // the fast graph exists for this handle (not row-sharded)
  int fast_mode = 0;       // next step(s) run the fast graph (gate closed with margin last time)
  long long rollbacks = 0;
  double* snap = nullptr;  // [3 * nparams] params, m, v at the start of a fast batch
  int* snap_count = nullptr;
  unsigned int* viol = nullptr;  // the fast graph met an open refinement gate
  // pipelined class values (TailArgs::nce_flag): the parameter-gradient launch of step s of a
  // captured batch evaluates step s + 1's class values after the kernel-parameter Adam.
  // cls_next: the step being enqueued does that; cls_have: the previous enqueued step did, so
  // this one needs no class-value launch.  Both false outside a multi-step capture.
  unsigned int* nce_flag = nullptr;  // raised by the Adam block, reset by the next publish_prep
  double* nce_kp = nullptr;          // [nsmall] the kernel parameters it hands over (sc1)
  bool cls_next = false, cls_have = false;
  double* rep_host = nullptr;    // [8 + LOSS_CAP] pinned: status, viol, gates, losses (step_report)
  double* pend_losses = nullptr; // caller's buffer for the last batch's losses (finish_batch)
  int pend_n = 0;
  hipEvent_t ev[kMaxStages + 1] = {};
  bool profiling = false;
  int nstage = 0;
  const char* sname[kMaxStages] = {};  // name of each launched (profiled) stage

  template <class T>
  int alloc(T** p, size_t count_) {
    void* q = nullptr;
    size_t bytes = std::max<size_t>(count_ * sizeof(T), 16);
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) return fail(GPK_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    e = hipMemsetAsync(q, 0, bytes, s);
    if (e != hipSuccess) return fail(GPK_EHIP, hipGetErrorString(e));
    allocs.push_back(q);
    *p = static_cast<T*>(q);
    return GPK_OK;
  }
};

#define TRY(x)                  \
  do {                          \
    int r_ = (x);               \
    if (r_ != GPK_OK) return r_; \
  } while (0)

static int check_launch(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(GPK_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  return GPK_OK;
}

static void mark(gpk_handle* h, int stage) {
  if (h->profiling) (void)hipEventRecord(h->ev[stage + 1], h->s);
}

// ------------------------------------------------------------------------------------------
// the step, in stream order
// ------------------------------------------------------------------------------------------
static PrepArgs make_prep(gpk_handle* h, int apply) {
  const Layout& L = h->L;
  PrepArgs P{};
  P.params = h->params;
  P.off_kp[0] = L.off_kp[0];
  P.off_kp[1] = L.off_kp[1];
  P.off_tau = L.off_tau;
  P.off_v = L.off_v;
  P.naxes = L.naxes;
  P.has_cos = (h->prob.kind == GPK_SE_COS || h->prob.kind == GPK_MATERN52_COS) ? 1 : 0;
  P.kc = h->kc;
  P.sc = h->sc;
  P.count = h->count;
  P.apply = apply;
  P.b1 = h->hyper.b1;
  P.b2 = h->hyper.b2;
  P.Up = h->Up; P.bvals = h->bvals; P.bidx = h->bidx; P.nb = h->prob.nb;
  P.dim = L.dim; P.n1 = L.n1; P.n2 = L.n2; P.p2 = L.p2;
  P.bgap = h->bgap;
  P.bgap_parts = h->bgap_parts;
  P.nce_flag = h->nce_flag;
  return P;
}

// Pipelined class values (gpk.h GPK_FLAG_NO_CLASS_PIPE): chain-inverse handles with distance
// classes, unsharded -- the class-value launch is then the step's only user of the kernel
// parameters before the inverse, so it can run at the end of the previous step's parameter-
// gradient launch, which has just updated them.
static bool cls_pipe_ok(const gpk_handle* h) {
  return !h->shard && h->chain && h->cls[0].ncls > 0 && h->nce_flag &&
         !(h->prob.flags & GPK_FLAG_NO_CLASS_PIPE);
}

static void fill_spd(gpk_handle* h, SpdArgs* sa) {
  const Layout& L = h->L;
  for (int a = 0; a < L.naxes; ++a) {
    sa[a] = SpdArgs{};
    sa[a].X = h->K[a];
    sa[a].Y = h->Kb[a];
    sa[a].p = a == 0 ? L.p1 : L.p2;
    sa[a].n = a == 0 ? L.n1 : L.n2;
    sa[a].piv = h->piv[a];
    sa[a].ldet = h->ldet[a];
    sa[a].status = h->status;
    sa[a].pst = h->pst[a];
    sa[a].flag = h->aflag[a];
    sa[a].wide = h->bigwide ? 1 : 0;
    sa[a].no_quarters = (h->prob.flags & GPK_FLAG_NO_QUARTER_TILES) ? 1 : 0;
    sa[a].qfirst = (h->prob.flags & GPK_FLAG_NO_QUARTER_FIRST) ? 0 : 1;
    sa[a].Z = h->Zp[a];
    sa[a].sched = h->wsched[a];
  }
}

// the persistent small-factor inverse; gather: K (+ Kc, D) straight from the distance classes
static hipError_t launch_chain(gpk_handle* h, bool gather, double** fin, bool aug = true,
                               const PrepArgs* prep = nullptr) {
  const Layout& L = h->L;
  ChainArgs ca[2] = {};
  for (int a = 0; a < L.naxes; ++a) {
    ChainArgs& c = ca[a];
    c.X = h->K[a]; c.PB = h->Kb[a]; c.piv = h->piv[a]; c.ldet = h->ldet[a]; c.pst = h->pst[a];
    c.status = h->status; c.flags = h->cflags[a]; c.gran = h->cgran[a];
    c.PB2 = h->PB2[a]; c.epoch = h->cepoch[a];
    c.p = a == 0 ? L.p1 : L.p2;
    c.n = a == 0 ? L.n1 : L.n2;
    if (gather) {
      c.cid = h->cls[a].cid; c.kval = h->cls[a].kval; c.dval = h->cls[a].dval;
      c.x = a == 0 ? h->x1 : h->x2; c.jitter = h->prob.jitter; c.Kc = h->Kc[a];
    }
    c.D = h->D[a];  // gather: written; read mode: the augmented D^T columns read it
    if (gather && h->cls_gemv) c.Kc = c.D = nullptr;  // (the GEMVs read them as classes)
    if (h->chain_aug && aug) {  // axis 0: [U | D1^T] -> A, K1^{-1} D1^T;  axis 1: [U^T | D2^T] -> Bt^T, P2
      const int Po = a == 0 ? L.p2 : L.p1;
      c.tu = Po / 32; c.td = c.p / 32;
      c.Bu = h->Up; c.ldbu = L.p2; c.bu_t = a;
      c.Ou = a == 0 ? h->A : h->Bt; c.ldou = L.p2; c.ou_t = a;
      c.Od = h->PD[a]; c.ldod = c.p;
      c.PBa = h->PBa[a]; c.ldpba = L.p1 + L.p2;
    }
    fin[a] = h->K[a];
  }
  if (h->chain_multi)
    return launch_spd_chain_multi(ca, L.naxes, h->prob.eq == GPK_ADVECTION ? 1 : 2, h->s, prep, L.q);
  return launch_spd_chain(ca, L.naxes, h->prob.eq == GPK_ADVECTION ? 1 : 2, h->s, prep, L.q);
}

// the SPD inverse of every factor (small: 32-wide sweeps, pivot 0 possibly fused into the
// assembly launch; large: 64-wide panel/update sweeps)
static hipError_t launch_inverse(gpk_handle* h, SpdArgs* sa, double** fin, bool pivot0_done) {
  if (h->bigspd) return launch_spd_inverse_big(sa, h->L.naxes, fin, h->s);
  if (h->chain) return launch_chain(h, false, fin, false);  // K^{-1} only (timing, predict)
  return launch_spd_inverse(sa, h->L.naxes, fin, h->s, pivot0_done);
}

static int split_broadcast(gpk_handle* h);  // (after ShardComm)

// assemble K, D (+ step constants, + pivot block 0) and invert K: the first part of a step
static int enqueue_assemble_inverse(gpk_handle* h, int apply, bool have_cls = false) {
  const Layout& L = h->L;
  AssembleArgs aa[2] = {};
  int deriv = (h->prob.eq == GPK_ADVECTION) ? 1 : 2;
  for (int a = 0; a < L.naxes; ++a) {
    aa[a].x = a == 0 ? h->x1 : h->x2;
    aa[a].n = a == 0 ? L.n1 : L.n2;
    aa[a].p = a == 0 ? L.p1 : L.p2;
    aa[a].kc = h->kc + a;
    aa[a].jitter = h->prob.jitter;
    aa[a].K = h->K[a];
    aa[a].D = h->D[a];
    aa[a].deriv = deriv;
    aa[a].Kc = h->Kc[a];
    aa[a].cls = h->cls[a];
    if (!h->bigspd && !h->chain) {  // pivot block 0 factored inside the assembly launch
      aa[a].piv = h->piv[a];
      aa[a].ldet = h->ldet[a];
      aa[a].pst = h->pst[a];
      aa[a].status = h->status;
      aa[a].flag = h->aflag[a];
    }
  }
  // chain + classes: the class values only; the inverse launch gathers K, Kc, D itself and
  // publishes the step constants from one extra workgroup (off the critical path)
  const bool eval_only = h->chain && h->cls[0].ncls > 0;
  PrepArgs prep = make_prep(h, apply), prep_eval = prep;
  prep_eval.skip = eval_only ? 1 : 0;
  if (eval_only && h->fold_begin) {  // the batch begin rides on the chain launch's prep row
    const StepBegin& b = *h->fold_begin;
    prep.snap = b.snap; prep.snap_m = b.m; prep.snap_v = b.v; prep.snap_np = b.np;
    prep.snap_count = b.snap ? b.snap_count : nullptr;
    prep.viol0 = b.viol; prep.slot0 = b.loss_slot;
    h->fold_begin = nullptr;
  }
  // (have_cls: the previous step's parameter-gradient launch evaluated them, cls_pipe_ok)
  if (!(eval_only && have_cls))
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, prep_eval, h->s, eval_only),
                     "assemble"));
  mark(h, 1);
  SpdArgs sa[2];
  fill_spd(h, sa);
  double* fin[2] = {nullptr, nullptr};
  if (h->chain) {
    TRY(check_launch(launch_chain(h, eval_only, fin, true, eval_only ? &prep : nullptr), "spd_chain"));
  } else if (h->split_axis >= 0) {
    // one factor per rank group: invert this rank's factor, then every factor's K^{-1}, log-det
    // blocks and refinement gate from its group's first rank (the other factor's buffers on
    // this rank are overwritten; the sweep path's output buffer is fixed per factor size)
    const int a = h->split_axis;
    double* f1[1] = {nullptr};
    if (h->bigspd)
      TRY(check_launch(launch_spd_inverse_big(sa + a, 1, f1, h->s), "spd_inverse"));
    else
      TRY(check_launch(launch_spd_inverse(sa + a, 1, f1, h->s, true), "spd_inverse"));
    TRY(split_broadcast(h));
    for (int b = 0; b < L.naxes; ++b) fin[b] = h->Kinv[b];
  } else {
    TRY(check_launch(launch_inverse(h, sa, fin, true), "spd_inverse"));
  }
  for (int a = 0; a < L.naxes; ++a) h->Kinv[a] = fin[a];
  mark(h, 2);
  return GPK_OK;
}

// the step tail (loss, small-parameter Adam, dL/dU + Adam on U) fused into the pgrad launch
static TailArgs make_tail(gpk_handle* h, int apply, bool refine = true) {
  const Layout& L = h->L;
  const int ac = h->prob.eq == GPK_ALLENCAHN;
  TailArgs T{};
  T.fused = 1;
  FinalizeArgs& f = T.fin;
  f.L = L; f.hyper = h->hyper; f.llk_weight = h->prob.llk_weight; f.logdet = h->prob.logdet;
  f.apply = apply; f.has_cos = kind_cos(h->prob.kind);
  f.red_quad = h->red_quad; f.nquad = h->nquad; f.red_egap = h->red_egap; f.negap = h->negap;
  for (int a = 0; a < L.naxes; ++a) { f.ldet[a] = h->ldet[a]; f.nldet[a] = h->nldet[a]; }
  f.pg = h->pg; f.kc = h->kc; f.sc = h->sc; f.Up = h->Up; f.bvals = h->bvals;
  f.bidx = h->bidx; f.nb = h->prob.nb;
  f.params = h->params; f.grad = h->grad; f.m = h->m; f.v = h->v;
  f.losses = h->losses; f.loss_slot = h->loss_slot; f.diag = h->diag;
  f.bgap = h->bgap;
  f.bgap_parts = h->bgap_parts;
  if (!refine) {  // fast graph: check that no refinement was needed
    for (int a = 0; a < L.naxes; ++a) f.watch[a] = h->pst[a];
    f.viol = h->viol;
  }
  if (h->fold_report) {
    f.report = 1;
    f.rep = *h->fold_report;
    h->fold_report = nullptr;
  }
  AdamUArgs& au = T.adam;
  au.L = L; au.hyper = h->hyper; au.llk_weight = h->prob.llk_weight; au.apply = apply; au.ac = ac;
  au.sc = h->sc; au.Up = h->Up; au.bvals = h->bvals; au.bidx = h->bidx; au.nb = h->prob.nb;
  au.params = h->params; au.grad = h->grad; au.m = h->m; au.v = h->v;
  if (L.dim == 2) { au.S = h->S; au.X1 = h->X1; au.X2 = h->X2; au.R = h->R; }
  else { au.S = nullptr; au.X1 = h->alpha; au.X2 = h->beta; au.R = h->R; au.U0 = h->uoff; }
  T.gcount = h->tcount; T.top = h->ttop; T.gpart = h->tgpart; T.pg = h->pg;
  T.tg = h->ttg; T.ngpa = h->tngpa;
  T.gpart_lo = h->pg_dd ? h->tgpart_lo : nullptr;
  // the fused tail's Adam block forms pg from the group partials itself (the sharded path's
  // standalone finalize reads pg: enqueue_step_shard clears these)
  f.gpart = T.gpart; f.gpart_lo = T.gpart_lo; f.ngpa = T.ngpa; f.pg_out = h->pg;
  if (h->cls_next && cls_pipe_ok(h)) {  // the next step's class values, after the Adam
    T.nce_flag = h->nce_flag;
    T.nce_status = h->status;
    f.kp_wt = h->nce_kp;
  }
  return T;
}

// A GEMV operand that is Kc or D of axis 0: as class ids + class values on a cls_gemv handle
static void gemv_operand(const gpk_handle* h, GemvDesc& g) {
  if (!h->cls_gemv || !(g.A == h->Kc[0] || g.A == h->D[0])) return;
  const bool k = g.A == h->Kc[0];
  g.cid = h->cls[0].cid;
  g.cv = k ? h->cls[0].kval : h->cls[0].dval;
  g.cdiag = k ? h->prob.jitter : 0.0;
  g.ident = k ? 1 : 0;
  g.A = nullptr;
}

static int enqueue_step_shard(gpk_handle* h, int apply);

static int launch_stage(gpk_handle* h, int k) {
  return check_launch(launch_gemm_auto(h->hdescs.data() + h->st[k].off, h->st[k].n, h->sc, h->s, h->st[k].variant),
                      "gemm");
}

static int enqueue_step(gpk_handle* h, int apply, bool refine = true) {
  if (h->shard) return enqueue_step_shard(h, apply);
  const Layout& L = h->L;
  // pipelined class values: this step's were evaluated by the previous step (have); this step
  // evaluates the next one's when its caller asked for it (cls_next, make_tail)
  const bool have = h->cls_have && cls_pipe_ok(h);
  h->cls_have = false;
  if (h->profiling) (void)hipEventRecord(h->ev[0], h->s);
  mark(h, 0);  // "prep" is fused into the assembly launch (stage kept for the name table)
  TRY(enqueue_assemble_inverse(h, apply, have));
  int stage = 3;
  const char* const* names = L.dim == 2 ? kStageNames2D : kStageNames1D;
  for (int k = 0; k < 3; ++k) h->sname[k] = names[k];
  auto stamp = [&](const char* nm) {  // a launched stage: its name and end event
    if (stage < kMaxStages) {
      h->sname[stage] = nm;
      mark(h, stage++);
    }
  };
  const int ac = h->prob.eq == GPK_ALLENCAHN;
  if (L.dim == 2) {
    for (int k = 0; k < kGemmStages; ++k) {
      if (h->st[k].n == 0 || (!refine && h->st[k].gated)) continue;
      TRY(launch_stage(h, k));
      stamp(kStageNames2D[3 + k]);
    }
    PGradArgs pa[2];
    for (int a = 0; a < 2; ++a) {
      pa[a] = PGradArgs{};
      pa[a].x = a == 0 ? h->x1 : h->x2;
      pa[a].n = a == 0 ? L.n1 : L.n2;
      pa[a].p = a == 0 ? L.p1 : L.p2;
      pa[a].kc = h->kc + a;
      pa[a].GK = h->GK[a];
      pa[a].GD = h->GD[a];
      pa[a].deriv = (h->prob.eq == GPK_ADVECTION) ? 1 : 2;
      pa[a].part = h->pgpart + (size_t)a * h->bpa * 3 * QMAX;
      pa[a].part_lo = h->pg_dd ? h->pgpart_lo + (size_t)a * h->bpa * 3 * QMAX : nullptr;
      pa[a].cls = h->cls[a];
      if (h->cp_on) {
        pa[a].cpK = h->cpK[a];
        pa[a].cpD = h->cpD[a];
        pa[a].cslots = class_slots(pa[a].p / 16);
      }
    }
    TailArgs tail = make_tail(h, apply, refine);
    TRY(check_launch(launch_pgrad(h->prob.kind, L.q, 0, pa, 2, h->bpa, h->sc, h->s, &tail), "pgrad"));
    h->cls_have = tail.nce_flag != nullptr;
    stamp("pgrad_tail");
  } else {
    const int P = L.p1;
    // every K^{-1} application gets one step of iterative refinement x += K^{-1}(b - K x),
    // gated on a cond(K) lower bound (gemv skips itself when K is well conditioned)
    GemvDesc g{};
    g.lda = P; g.p = P; g.rows = P; g.alpha = 1.0; g.ac = ac; g.F = h->F; g.U = h->Up; g.U0 = h->uoff;
    auto gemv = [&](const char* nm, const double* A, const double* x, double* y, double alpha,
                    const double* C0, double beta, int epi, double* red, bool gated) -> int {
      if (gated && !refine) return GPK_OK;
      GemvDesc q = g;
      q.A = A; q.x = x; q.y = y; q.alpha = alpha; q.C0 = C0; q.beta = beta; q.epi = epi; q.red = red;
      q.gate = gated ? h->pst[0] : nullptr;
      gemv_operand(h, q);
      TRY(check_launch(launch_gemv(q, h->s), "gemv"));
      stamp(nm);
      return GPK_OK;
    };
    // alpha = K^{-1} u (refined), quad = <u, alpha>          (model_GP_solver_1d.py:92,137)
    TRY(gemv("gemv_alpha", h->Kinv[0], h->Up, h->alpha, 1.0, nullptr, 0.0, EPI_STORE, nullptr, false));
    TRY(gemv("gemv_alpha_res", h->Kc[0], h->alpha, h->rvec, -1.0, h->Up, 1.0, EPI_STORE, nullptr, true));
    TRY(gemv("gemv_alpha_fix", h->Kinv[0], h->rvec, h->alpha, 1.0, h->alpha, 1.0, EPI_STORE, nullptr, true));
    // R = D alpha - f (+u(u^2-1)): egap = ||R||^2 and quad = <u, alpha> in one pass
    {
      GemvDesc q = g;
      q.A = h->D[0]; q.x = h->alpha; q.y = h->R; q.epi = EPI_RESID; q.red = h->red_egap;
      q.red2 = h->red_quad; q.Q1 = h->Up; q.Q2 = h->alpha;
      gemv_operand(h, q);
      TRY(check_launch(launch_gemv(q, h->s), "gemv"));
      stamp("gemv_resid");
    }
    // t = D^T R (DD_x1 is bitwise symmetric, so D^T = D)
    TRY(gemv("gemv_DtR", h->D[0], h->R, h->tvec, 1.0, nullptr, 0.0, EPI_STORE, nullptr, false));
    // beta = K^{-1} t (refined)
    TRY(gemv("gemv_beta", h->Kinv[0], h->tvec, h->beta, 1.0, nullptr, 0.0, EPI_STORE, nullptr, false));
    TRY(gemv("gemv_beta_res", h->Kc[0], h->beta, h->rvec, -1.0, h->tvec, 1.0, EPI_STORE, nullptr, true));
    TRY(gemv("gemv_beta_fix", h->Kinv[0], h->rvec, h->beta, 1.0, h->beta, 1.0, EPI_STORE, nullptr, true));
    PGradArgs pa{};
    pa.x = h->x1; pa.n = L.n1; pa.p = P; pa.kc = h->kc;
    pa.Kinv = h->Kinv[0]; pa.alpha = h->alpha; pa.beta = h->beta; pa.R = h->R;
    pa.halfc = 0.5 * h->prob.logdet; pa.deriv = 2; pa.part = h->pgpart; pa.cls = h->cls[0];
    pa.part_lo = h->pg_dd ? h->pgpart_lo : nullptr;
    TailArgs tail = make_tail(h, apply, refine);
    TRY(check_launch(launch_pgrad(h->prob.kind, L.q, 1, &pa, 1, h->bpa, h->sc, h->s, &tail), "pgrad"));
    h->cls_have = tail.nce_flag != nullptr;
    stamp("pgrad_tail");
  }
  h->nstage = stage;
  return GPK_OK;
}

// Distance classes of one axis (gpk_internal.h ClassArgs): per diagonal k the distinct exact
// values of d = |x_{j+k} - x_j| (= |x_j - x_{j+k}| bitwise), in order of first appearance.
// false: some diagonal has more than CLS_VMAX of them (the step keeps the per-pair kernels).
static bool build_classes(const double* x, int n, int P, std::vector<double>& dist,
                          std::vector<int>& cid, std::vector<int>& cbase, int& vmax) {
  cid.assign((size_t)P * P, -1);
  cbase.assign((size_t)n + 1, 0);
  dist.clear();
  vmax = 0;
  double vals[CLS_VMAX];
  for (int k = 0; k < n; ++k) {
    int nv = 0;
    cbase[k] = (int)dist.size();
    for (int j = 0; j + k < n; ++j) {
      const double d = std::fabs(x[j + k] - x[j]);
      int v = 0;
      while (v < nv && !(vals[v] == d)) ++v;
      if (v == nv) {
        if (nv == CLS_VMAX) return false;
        vals[nv++] = d;
        dist.push_back(d);
      }
      const int c = cbase[k] + v;
      cid[(size_t)(j + k) * P + j] = c;
      cid[(size_t)j * P + j + k] = c;
    }
    vmax = std::max(vmax, nv);
  }
  cbase[n] = (int)dist.size();
  return true;
}

static int gemm_force(int flags) {
  return (flags & GPK_FLAG_FORCE_HUGE_GEMM) ? 2 : (flags & GPK_FLAG_FORCE_BIG_GEMM) ? 1 : 0;
}

static int build_descs(gpk_handle* h) {
  const Layout& L = h->L;
  const int P1 = L.p1, P2 = L.p2;
  const double beta = (h->prob.eq == GPK_ADVECTION) ? h->prob.beta : 1.0;
  const int ac = h->prob.eq == GPK_ALLENCAHN;
  std::vector<GemmDesc> d;
  auto mk = [](const double* A, int lda, int ta, const double* B, int ldb, int tb, double* C,
               int ldc, int M, int N, int K) {
    GemmDesc g{};
    g.A = A; g.lda = lda; g.ta = ta; g.B = B; g.ldb = ldb; g.tb = tb;
    g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.K = K; g.alpha = 1.0; g.epi = EPI_STORE;
    return g;
  };
  auto begin = [&](int k) { h->st[k].off = (int)d.size(); };
  const int force_big = gemm_force(h->prob.flags);
  auto end = [&](int k) {
    h->st[k].n = (int)d.size() - h->st[k].off;
    for (int i = h->st[k].off; i < (int)d.size(); ++i) d[i].tag = k;
    h->st[k].gated = h->st[k].n > 0;
    for (int i = h->st[k].off; i < (int)d.size(); ++i) h->st[k].gated &= d[i].gate != nullptr;
    h->st[k].variant = gemm_variant(d.data() + h->st[k].off, h->st[k].n, force_big);
  };
  // Every solve against K (JAX: LU solves, model_GP_solver_2d.py:104-105 and the reverse
  // pass) is X = K^{-1} B (MFMA) plus one refinement X += K^{-1}(B - K X), whose two GEMMs are
  // gated on a lower bound of cond(K) (refine_gate_open) (skipped when K is well conditioned, e.g. 256^2).
  const int n1 = L.n1, n2 = L.n2;
  auto gate = [&](GemmDesc g, int axis) {
    g.gate = h->pst[axis];
    return g;
  };
  // Refinement GEMMs (X += K^{-1}(B - K X)) are gated on device on a lower bound of cond(K): a
  // closed gate ends each of their workgroups before any load (a launch).  Small factors: every
  // solve is refined.  Large 2D factors (P >= 1600), where each refinement is two N^3 GEMMs
  // (C5: ~2.2 ms each), by default the FORWARD solves A = K1^{-1} U and Bt = U K2^{-1}: the
  // residual R = beta D1 A + Bt D2^T - F differentiates them (D amplifies the unstructured
  // error of an explicit-inverse product) and ||R||^2 feeds the loss and the log_v gradient;
  // GPK_FLAG_REFINE_ALL adds S and X1 / X2, GPK_FLAG_NO_REFINE drops all (round 2's path).
  // Accuracy of each choice against the long-double yardstick: tests/test_gpu_accuracy.py,
  // profiles/r3_parity.json, DESIGN.md §5.
  const int rfl = h->prob.flags;
  const bool ref_fwd = !(rfl & GPK_FLAG_NO_REFINE);
  const bool ref_rev = (!h->bigspd || (rfl & GPK_FLAG_REFINE_ALL)) && !(rfl & GPK_FLAG_NO_REFINE);
  // Large 2D factors, the axis-2 forward solve Bt = U K2^{-1} (round 6): it enters the residual
  // R = beta D1 A + Bt D2^T - F with weight 1 against beta for A, so at beta >= 16 (advection;
  // C5: beta = 200) refining A alone leaves R's error ~1/beta of the unrefined one.  Measured at
  // C5 against the exact-field yardstick (tools/c5_refine_diag.py, profiles/r6_c5_refine_fwd1.txt):
  // log_v (||R||^2) 3.3e-12 with A refined alone, 1.1e-12 with both, 8.3e-9 with neither (the LU
  // oracle: 2.9e-10); every other key within 0.3x of the LU oracle's distance either way -- and
  // the step 37.3 -> 33.5 ms (two 4096^3 products fewer).  GPK_FLAG_REFINE_ALL refines both.
  const bool ref_fwd2 = ref_fwd && !(rfl & GPK_FLAG_REFINE_FWD1_ONLY) &&
                        (!h->bigspd || beta < 16.0 || (rfl & GPK_FLAG_REFINE_ALL));
  bool ref_now = ref_fwd;
  auto pushg = [&](const GemmDesc& g) {
    if (ref_now) d.push_back(g);
  };
  // X1 / X2 producers also write Y = S/2 + v X (GemmDesc::Y): G_K's left operand
  auto side = [&](GemmDesc g, double* Y) {
    g.Y = Y; g.Ys = h->S; g.ldy = P2;
    return g;
  };
  // Stage A: A = K1^{-1} U, Bt = U K2^{-1}                       (2d.py:104-105)
  // (augmented chain: both come out of the inverse launch itself -- no stage)
  begin(0);
  if (!h->chain_aug) {
    d.push_back(mk(h->Kinv[0], P1, 0, h->Up, P2, 0, h->A, P2, P1, P2, P1));
    d.push_back(mk(h->Up, P2, 0, h->Kinv[1], P2, 0, h->Bt, P2, P1, P2, P2));
  }
  end(0);
  // (Measured in C4's training regime, tools/train_regime_parity.py, profiles/r5_train_regime_
  // parity.json: with the gate closed -- cond(K) <= 1.4e3, bound < 21 -- the unrefined step is
  // within 0.45 of the parity bar on its own K and D after 200-2000 Adam steps; refining the
  // forward solves every step took that to 0.05-0.25 for ~12 us per step, so the gate stays.)
  begin(1);  // residuals W1 = U - K1 A, W2 = U - Bt K2
  {
    GemmDesc g = mk(h->Kc[0], P1, 0, h->A, P2, 0, h->W1, P2, P1, P2, P1);
    g.alpha = -1.0; g.beta = 1.0; g.C0 = h->Up; g.ldc0 = P2;
    pushg(gate(g, 0));
    GemmDesc g2 = mk(h->Bt, P2, 0, h->Kc[1], P2, 0, h->W2, P2, P1, P2, P2);
    g2.alpha = -1.0; g2.beta = 1.0; g2.C0 = h->Up; g2.ldc0 = P2;
    if (ref_fwd2) pushg(gate(g2, 1));
  }
  end(1);
  begin(2);  // A += K1^{-1} W1, Bt += W2 K2^{-1}  (in place)
  {
    GemmDesc g = mk(h->Kinv[0], P1, 0, h->W1, P2, 0, h->A, P2, P1, P2, P1);
    g.beta = 1.0; g.C0 = h->A; g.ldc0 = P2;
    pushg(gate(g, 0));
    GemmDesc g2 = mk(h->W2, P2, 0, h->Kinv[1], P2, 0, h->Bt, P2, P1, P2, P2);
    g2.beta = 1.0; g2.C0 = h->Bt; g2.ldc0 = P2;
    if (ref_fwd2) pushg(gate(g2, 1));
  }
  end(2);
  // Stage B: S = A K2^{-1};  R = beta D1 A + Bt D2^T - F (+AC), ||R||^2 and the prior's
  // quadratic term sum(A * Bt) (2d.py:112-143, :161) from the same tile loop
  begin(3);
  {
    d.push_back(mk(h->A, P2, 0, h->Kinv[1], P2, 0, h->S, P2, P1, P2, P2));
    GemmDesc r = mk(h->D[0], P1, 0, h->A, P2, 0, h->R, P2, P1, P2, P1);
    r.alpha = beta;
    r.A2 = h->Bt; r.lda2 = P2; r.ta2 = 0; r.B2 = h->D[1]; r.ldb2 = P2; r.tb2 = 1; r.K2 = P2;
    r.alpha2 = 1.0;
    r.epi = EPI_RESID; r.F = h->F; r.U = h->Up; r.ldf = P2; r.ac = ac; r.red = h->red_egap;
    r.red2 = h->red_quad; r.Q1 = h->A; r.Q2 = h->Bt;
    d.push_back(r);
  }
  end(3);
  ref_now = ref_rev;  // (the reverse-pass solves from here on)
  begin(4);  // W1 = A - S K2
  {
    GemmDesc g = mk(h->S, P2, 0, h->Kc[1], P2, 0, h->W1, P2, P1, P2, P2);
    g.alpha = -1.0; g.beta = 1.0; g.C0 = h->A; g.ldc0 = P2;
    pushg(gate(g, 1));
  }
  end(4);
  begin(5);  // S += W1 K2^{-1}
  {
    GemmDesc g = mk(h->W1, P2, 0, h->Kinv[1], P2, 0, h->S, P2, P1, P2, P2);
    g.beta = 1.0; g.C0 = h->S; g.ldc0 = P2;
    pushg(gate(g, 1));
  }
  end(5);
  // Stage C: T1 = beta D1^T R, T2 = R D2, G_D1 = v beta R A^T, G_D2 = v R^T Bt  (Appendix A)
  // (augmented chain: X1 = beta (K1^{-1} D1^T) R and X2 = R (K2^{-1} D2^T)^T directly, from the
  // inverse launch's K^{-1} D^T -- stage D's solves fold into this stage)
  begin(6);
  if (h->chain_aug) {
    GemmDesc x1 = mk(h->PD[0], P1, 0, h->R, P2, 0, h->X1, P2, P1, P2, P1);
    x1.alpha = beta;
    d.push_back(side(x1, h->Y1));
    d.push_back(side(mk(h->R, P2, 0, h->PD[1], P2, 1, h->X2, P2, P1, P2, P2), h->Y2));
  } else {
    GemmDesc t1 = mk(h->D[0], P1, 1, h->R, P2, 0, h->T1, P2, P1, P2, P1);
    t1.alpha = beta;
    d.push_back(t1);
    d.push_back(mk(h->R, P2, 0, h->D[1], P2, 0, h->T2, P2, P1, P2, P2));
  }
  {
    GemmDesc g = mk(h->R, P2, 0, h->A, P2, 1, h->GD[0], P1, P1, P1, P2);
    g.alpha = beta; g.vscale = 1;
    d.push_back(g);
    GemmDesc g2 = mk(h->R, P2, 1, h->Bt, P2, 0, h->GD[1], P2, P2, P2, P1);
    g2.vscale = 1;
    d.push_back(g2);
  }
  end(6);
  // Stage D: X1 = K1^{-1} T1, X2 = T2 K2^{-1} (refined)
  begin(7);
  if (!h->chain_aug) {
    d.push_back(side(mk(h->Kinv[0], P1, 0, h->T1, P2, 0, h->X1, P2, P1, P2, P1), h->Y1));
    d.push_back(side(mk(h->T2, P2, 0, h->Kinv[1], P2, 0, h->X2, P2, P1, P2, P2), h->Y2));
  }
  end(7);
  begin(8);  // refinement residuals W1 = beta D1^T R - K1 X1, W2 = R D2 - X2 K2
  if (h->chain_aug) {  // (T1, T2 never formed: dual products)
    GemmDesc g = mk(h->D[0], P1, 1, h->R, P2, 0, h->W1, P2, P1, P2, P1);
    g.alpha = beta;
    g.A2 = h->Kc[0]; g.lda2 = P1; g.B2 = h->X1; g.ldb2 = P2; g.K2 = P1; g.alpha2 = -1.0;
    pushg(gate(g, 0));
    GemmDesc g2 = mk(h->R, P2, 0, h->D[1], P2, 0, h->W2, P2, P1, P2, P2);
    g2.A2 = h->X2; g2.lda2 = P2; g2.B2 = h->Kc[1]; g2.ldb2 = P2; g2.K2 = P2; g2.alpha2 = -1.0;
    pushg(gate(g2, 1));
  } else {
    GemmDesc g = mk(h->Kc[0], P1, 0, h->X1, P2, 0, h->W1, P2, P1, P2, P1);
    g.alpha = -1.0; g.beta = 1.0; g.C0 = h->T1; g.ldc0 = P2;
    pushg(gate(g, 0));
    GemmDesc g2 = mk(h->X2, P2, 0, h->Kc[1], P2, 0, h->W2, P2, P1, P2, P2);
    g2.alpha = -1.0; g2.beta = 1.0; g2.C0 = h->T2; g2.ldc0 = P2;
    pushg(gate(g2, 1));
  }
  end(8);
  begin(9);
  {
    GemmDesc g = mk(h->Kinv[0], P1, 0, h->W1, P2, 0, h->X1, P2, P1, P2, P1);
    g.beta = 1.0; g.C0 = h->X1; g.ldc0 = P2;
    pushg(side(gate(g, 0), h->Y1));
    GemmDesc g2 = mk(h->W2, P2, 0, h->Kinv[1], P2, 0, h->X2, P2, P1, P2, P2);
    g2.beta = 1.0; g2.C0 = h->X2; g2.ldc0 = P2;
    pushg(side(gate(g2, 1), h->Y2));
  }
  end(9);
  // Stage E: G_K1 = c N2/2 K1^{-1} - Y1 A^T;  G_K2 = c N1/2 K2^{-1} - Y2^T Bt, with
  // Y = S/2 + v X written by the X producers above (one product each instead of two)
  begin(10);
  {
    GemmDesc g = mk(h->Y1, P2, 0, h->A, P2, 1, h->GK[0], P1, P1, P1, P2);
    g.alpha = -1.0;
    g.beta = 0.5 * h->prob.logdet * n2; g.C0 = h->Kinv[0]; g.ldc0 = P1;
    d.push_back(g);
    GemmDesc g2 = mk(h->Y2, P2, 1, h->Bt, P2, 0, h->GK[1], P2, P2, P2, P1);
    g2.alpha = -1.0;
    g2.beta = 0.5 * h->prob.logdet * n1; g2.C0 = h->Kinv[1]; g2.ldc0 = P2;
    d.push_back(g2);
  }
  end(10);
  // class tile partials (GemmDesc::cpart) from the G_D (stage C) and G_K (stage E) epilogues
  // when both stages run the 16x16-tile kernel (its epilogue forms them)
  h->cp_on = h->cpK[0] && h->st[6].variant == GEMM_SMALL && h->st[10].variant == GEMM_SMALL;
  if (h->cp_on) {
    for (int k : {6, 10})
      for (int i = h->st[k].off; i < h->st[k].off + h->st[k].n; ++i)
        for (int a = 0; a < 2; ++a) {
          GemmDesc& g = d[i];
          if (g.C != (k == 6 ? h->GD[a] : h->GK[a])) continue;
          g.cpart = k == 6 ? h->cpD[a] : h->cpK[a];
          g.bcid = h->cls[a].cid;
          g.bcbase = h->cls[a].cbase;
          g.bn = a == 0 ? n1 : n2;
          g.bncls = h->cls[a].ncls;
          g.bsx = (k == 6 && h->prob.eq == GPK_ADVECTION) ? (a == 0 ? h->x1 : h->x2) : nullptr;
        }
  }
  {  // the residual descriptor of stage B carries the egap / quad partials: one per tile
    int nq = 0;
    for (int i = h->st[3].off; i < h->st[3].off + h->st[3].n; ++i)
      if (d[i].red) nq = gemm_tiles(d[i], h->st[3].variant);
    h->nquad = h->negap = nq;
  }
  for (int k = 0; k < kGemmStages; ++k)
    if (h->st[k].n > GEMM_MAX_BATCH) return fail(GPK_EINVAL, "internal: GEMM stage batch too large");
  h->hdescs = d;
  return GPK_OK;
}


// ------------------------------------------------------------------------------------------
// row-sharded multi-GPU step (the reference has no multi-GPU path)
//
// Every rank holds the whole problem, assembles and inverts both Kronecker factors itself
// (replicated: O(N^2 Q) + O(N^3) per factor), and computes rows [r*h, (r+1)*h) of every
// product of the step -- the GEMM stages are ~26 N^3 of the ~28 N^3 flops (C5: 1.9 TFLOP).
// A row slice of C = op(A) op(B) needs only the same rows of op(A); every operand a later
// stage reads beyond its own rows (a B operand, or an A operand read transposed) is completed
// by an in-place all-gather of its row blocks.  The kernel-parameter contraction runs over a
// 1/P share of the pair tiles; its partials, the per-tile loss partials (||R||^2, <A,Bt>) and
// nothing else are all-reduced (6Q+2 tile vectors); the loss and the small-parameter Adam are
// then identical on every rank; Adam on U updates the rank's rows, which are all-gathered.
// Collectives: RCCL in the handle's stream (captured into the step's hipGraph), or -- for tests
// on one GPU -- an in-process group of handles, one host thread per rank.
// ------------------------------------------------------------------------------------------
struct ShardComm {
  virtual ~ShardComm() {}
  virtual int allgather(gpk_handle* h, double* buf, size_t chunk) = 0;  // in place
  virtual int allreduce(gpk_handle* h, double* buf, size_t n) = 0;      // in place, sum
  virtual int broadcast(gpk_handle* h, double* buf, size_t n, int root) = 0;  // in place
  virtual bool capturable() const = 0;
};

namespace {

struct RcclComm : ShardComm {
  ncclComm_t c = nullptr;
  ~RcclComm() override {
    if (c) (void)ncclCommDestroy(c);
  }
  int allgather(gpk_handle* h, double* buf, size_t chunk) override {
    ncclResult_t r = ncclAllGather(buf + (size_t)h->rank * chunk, buf, chunk, ncclDouble, c, h->s);
    return r == ncclSuccess ? GPK_OK : fail(GPK_ERCCL, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  }
  int allreduce(gpk_handle* h, double* buf, size_t n) override {
    ncclResult_t r = ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, c, h->s);
    return r == ncclSuccess ? GPK_OK : fail(GPK_ERCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  }
  int broadcast(gpk_handle* h, double* buf, size_t n, int root) override {
    ncclResult_t r = ncclBroadcast(buf, buf, n, ncclDouble, root, c, h->s);
    return r == ncclSuccess ? GPK_OK : fail(GPK_ERCCL, std::string("ncclBroadcast: ") + ncclGetErrorString(r));
  }
  bool capturable() const override { return true; }
};

// In-process group (one device, one host thread per rank): collectives meet at a host barrier;
// rank 0 moves the blocks with device copies (and sums in rank order: deterministic).
struct LocalGroup {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  bool broken = false;
  std::vector<double*> slot;
  bool barrier() {  // false if another rank failed
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const long g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || broken; });
    }
    return !broken;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    broken = true;
    cv.notify_all();
  }
};

struct LocalComm : ShardComm {
  std::shared_ptr<LocalGroup> g;
  int allgather(gpk_handle* h, double* buf, size_t chunk) override {
    HIPCHK(hipStreamSynchronize(h->s));
    g->slot[h->rank] = buf;
    if (!g->barrier()) return fail(GPK_EHIP, "rank group aborted");
    int rc = GPK_OK;
    if (h->rank == 0) {
      for (int src = 0; src < g->n && rc == GPK_OK; ++src)
        for (int dst = 0; dst < g->n; ++dst)
          if (dst != src &&
              hipMemcpyAsync(g->slot[dst] + (size_t)src * chunk, g->slot[src] + (size_t)src * chunk,
                             chunk * sizeof(double), hipMemcpyDeviceToDevice, h->s) != hipSuccess)
            rc = fail(GPK_EHIP, "group all-gather copy");
      if (hipStreamSynchronize(h->s) != hipSuccess) rc = fail(GPK_EHIP, "group all-gather sync");
    }
    if (!g->barrier()) return fail(GPK_EHIP, "rank group aborted");
    return rc;
  }
  int allreduce(gpk_handle* h, double* buf, size_t n) override {
    HIPCHK(hipStreamSynchronize(h->s));
    g->slot[h->rank] = buf;
    if (!g->barrier()) return fail(GPK_EHIP, "rank group aborted");
    int rc = GPK_OK;
    if (h->rank == 0) {
      for (int src = 1; src < g->n && rc == GPK_OK; ++src)
        rc = check_launch(launch_add_into(g->slot[0], g->slot[src], n, h->s), "add_into");
      for (int dst = 1; dst < g->n && rc == GPK_OK; ++dst)
        if (hipMemcpyAsync(g->slot[dst], g->slot[0], n * sizeof(double), hipMemcpyDeviceToDevice, h->s) != hipSuccess)
          rc = fail(GPK_EHIP, "group all-reduce copy");
      if (hipStreamSynchronize(h->s) != hipSuccess) rc = fail(GPK_EHIP, "group all-reduce sync");
    }
    if (!g->barrier()) return fail(GPK_EHIP, "rank group aborted");
    return rc;
  }
  int broadcast(gpk_handle* h, double* buf, size_t n, int root) override {
    HIPCHK(hipStreamSynchronize(h->s));
    g->slot[h->rank] = buf;
    if (!g->barrier()) return fail(GPK_EHIP, "rank group aborted");
    int rc = GPK_OK;
    if (h->rank == 0) {
      for (int dst = 0; dst < g->n && rc == GPK_OK; ++dst)
        if (dst != root && hipMemcpyAsync(g->slot[dst], g->slot[root], n * sizeof(double),
                                          hipMemcpyDeviceToDevice, h->s) != hipSuccess)
          rc = fail(GPK_EHIP, "group broadcast copy");
      if (hipStreamSynchronize(h->s) != hipSuccess) rc = fail(GPK_EHIP, "group broadcast sync");
    }
    if (!g->barrier()) return fail(GPK_EHIP, "rank group aborted");
    return rc;
  }
  bool capturable() const override { return false; }
};

int tile_rows(int variant) { return variant == GEMM_SMALL ? 16 : variant == GEMM_BIG ? 64 : variant == GEMM_HUGE ? 128 : 32; }
int tile_cols_count(const GemmDesc& d, int variant) {
  const int tc = tile_rows(variant);
  return (d.N + tc - 1) / tc;
}

// rows [r0, r0 + rows) of C = op(A) op(B) [+ dual] with every row-indexed operand offset
GemmDesc slice_rows(const GemmDesc& d, int r0, int rows, int variant) {
  GemmDesc s = d;
  s.M = rows;
  s.A = d.ta ? d.A + r0 : d.A + (size_t)r0 * d.lda;
  if (d.K2) s.A2 = d.ta2 ? d.A2 + r0 : d.A2 + (size_t)r0 * d.lda2;
  s.C = d.C + (size_t)r0 * d.ldc;
  if (d.C0) s.C0 = d.C0 + (size_t)r0 * d.ldc0;
  if (d.F) s.F = d.F + (size_t)r0 * d.ldf;
  if (d.U) s.U = d.U + (size_t)r0 * d.ldf;
  if (d.Q1) s.Q1 = d.Q1 + (size_t)r0 * d.ldf;
  if (d.Q2) s.Q2 = d.Q2 + (size_t)r0 * d.ldf;
  if (d.Y) {
    s.Y = d.Y + (size_t)r0 * d.ldy;
    s.Ys = d.Ys + (size_t)r0 * d.ldy;
  }
  const size_t toff = (size_t)(r0 / tile_rows(variant)) * tile_cols_count(d, variant);
  if (d.red) s.red = d.red + toff;
  if (d.red2) s.red2 = d.red2 + toff;
  return s;
}

// rows [r0, r0 + rows) of the CONTRACTION index of C = op(A) op(B) (single product): this rank's
// partial of a full-size C, summed over ranks only through the linear parameter contraction.
// The C0 term is carried by rank 0 alone.
GemmDesc slice_k(const GemmDesc& d, int r0, int rows, int rank) {
  GemmDesc s = d;
  s.K = rows;
  s.A = d.ta ? d.A + (size_t)r0 * d.lda : d.A + r0;
  s.B = d.tb ? d.B + r0 : d.B + (size_t)r0 * d.ldb;
  if (rank != 0) {
    s.C0 = nullptr;
    s.beta = 0.0;
  }
  return s;
}

}  // namespace

// GPK_FLAG_SPLIT_FACTORS: factor b's K^{-1}, log-det blocks and gate from its group's first rank
static int split_broadcast(gpk_handle* h) {
  const Layout& L = h->L;
  for (int b = 0; b < 2; ++b) {
    const int P = b == 0 ? L.p1 : L.p2, root = b == 0 ? 0 : h->nranks / 2;
    TRY(h->comm->broadcast(h, h->Kinv[b], (size_t)P * P, root));
    TRY(h->comm->broadcast(h, h->ldet[b], (size_t)P / 32, root));
    TRY(h->comm->broadcast(h, h->pst[b], 2, root));
  }
  return GPK_OK;
}

// Row slices of the step's GEMM stages for this rank, the variant per stage (its tile rows must
// divide the slice height so that the per-tile loss partials land in the full-grid slots), and
// the all-gathers after each stage: exactly the outputs a later stage reads beyond its rows.
// Every descriptor runs in one of three modes: 'r' its output rows [r h, (r + 1) h) (slice_rows),
// 'k' this rank's share of its contraction index (slice_k: G_K2, G_D2, summed through the
// linear parameter contraction) or 'f' whole (replicated on every rank).  The plan -- modes per
// stage, then the collectives -- is kept as text (gpk_shard_plan) and restated by gpk/shard.py
// shard_plan(), whose host stand-in runs it across gloo processes (tests/test_shard.py).
//   augmented chain (small factors, C4): every rank's inverse launch yields the whole A, Bt and
//   K^{-1} D^T, so the forward refinement (stages 1, 2: the gate's two GEMMs) and X1 =
//   beta (K1^{-1} D1^T) R with its refinement (stages 6, 8, 9: one P1^3 product each, cheap at
//   these sizes) run whole: the step's collectives are the R gather, ONE all-reduce and the U
//   gather.
//   otherwise (large factors, C5; the factor split): A is gathered after stage 0 and 2 (W1
//   after the refinement's residual), R, T1 (and X1 / W1 of the reverse refinement) after their
//   stages -- each a 4096^2 row block exchange instead of a replicated 4096^3 product.
static int build_shard(gpk_handle* h) {
  const Layout& L = h->L;
  const int P1 = L.p1, P2 = L.p2;
  h->h1 = P1 / h->nranks;
  h->h2 = P2 / h->nranks;
  const int force = gemm_force(h->prob.flags);
  const bool aug = h->chain_aug;
  h->sdescs.clear();
  auto mode_of = [&](int k, const GemmDesc& d) -> char {
    // G_K2 = c N1/2 K2^{-1} - Y2^T Bt and G_D2 = v R^T Bt contract over the P1 rows: each rank
    // forms the full matrix from its own rows of Y2 / R and Bt (no all-gather of those operands)
    if (d.C == h->GK[1] || d.C == h->GD[1]) return 'k';
    if (aug && (k == 1 || k == 2)) return 'f';
    if (aug && (k == 6 || k == 8 || k == 9) && (d.C == h->X1 || d.C == h->W1)) return 'f';
    return 'r';
  };
  auto slice = [&](char mode, const GemmDesc& d, int variant) {
    const int rows = d.M == P1 ? h->h1 : h->h2;
    if (mode == 'k') return slice_k(d, h->rank * h->h1, h->h1, h->rank);
    if (mode == 'f') return d;
    return slice_rows(d, h->rank * rows, rows, variant);
  };
  for (int k = 0; k < kGemmStages; ++k) {
    const GemmDesc* full = h->hdescs.data() + h->st[k].off;
    const int n = h->st[k].n;
    std::vector<GemmDesc> tmp;
    for (int i = 0; i < n; ++i) {
      const GemmDesc& d = full[i];
      if (d.M != P1 && d.M != P2) return fail(GPK_EINVAL, "shard: unexpected GEMM row count");
      tmp.push_back(slice(mode_of(k, d), d, GEMM_SMALL));
    }
    int variant = gemm_variant(tmp.data(), n, force);
    for (int i = 0; i < n; ++i)
      while (mode_of(k, full[i]) == 'r' && (full[i].M == P1 ? h->h1 : h->h2) % tile_rows(variant) != 0)
        variant = variant == GEMM_HUGE ? GEMM_BIG : GEMM_SMALL;
    h->sst[k].off = (int)h->sdescs.size();
    h->sst[k].n = n;
    h->sst[k].variant = variant;
    for (int i = 0; i < n; ++i) {
      h->sdescs.push_back(slice(mode_of(k, full[i]), full[i], variant));
      if (full[i].red) h->nquad = h->negap = gemm_tiles(full[i], variant);
    }
  }
  // All-gathers: exactly the operands a later product reads beyond this rank's rows.  G_K / G_D
  // are never gathered: axis 1's are row slices (the other rows stay zero on this rank), axis
  // 2's this rank's partials (slice_k); the parameter contraction is linear in them, so every
  // rank contracts what it holds and the partials are all-reduced (enqueue_step_shard).
  auto g1 = [&](double* b) { return ShardGather{b, (size_t)h->h1 * P2}; };
  for (auto& v : h->sgather) v.clear();
  std::string gplan[kGemmStages];
  auto gather = [&](int k, double* b, const char* name) {
    h->sgather[k].push_back(g1(b));
    gplan[k] += std::string(" g") + name;
  };
  if (aug) {
    gather(3, h->R, "R");                                      // X1 = beta P1 R, T = D1^T R (W1)
  } else {
    // (the refinement stages this handle has: build_descs, GPK_FLAG_REFINE_ALL / NO_REFINE)
    if (h->st[1].n > 0) {
      gather(0, h->A, "A");                                    // A_res: K1 A
      gather(1, h->W1, "W1");                                  // A_fix: K1^{-1} W1
    }
    gather(2, h->A, "A");                                      // R: D1 A;  G_K1 = Y1 A^T
    gather(3, h->R, "R");                                      // T1 = D1^T R
    gather(6, h->T1, "T1");                                    // X1 = K1^{-1} T1
    if (h->st[8].n > 0) {
      gather(7, h->X1, "X1");                                  // D_res: K1 X1
      gather(8, h->W1, "W1");                                  // D_fix: K1^{-1} W1
    }
  }
  // the plan: per stage its descriptors' modes, then the gathers that follow it
  std::string out;
  for (int k = 0; k < kGemmStages; ++k) {
    const GemmDesc* full = h->hdescs.data() + h->st[k].off;
    if (h->st[k].n) {
      out += (out.empty() ? "" : " ") + std::string("s") + std::to_string(k) + ":";
      for (int i = 0; i < h->st[k].n; ++i) out += mode_of(k, full[i]);
    }
    out += gplan[k];
  }
  h->splan = out + " ar gU";  // + the step's one all-reduce and the U rows after Adam
  return GPK_OK;
}

static int enqueue_step_shard(gpk_handle* h, int apply) {
  const Layout& L = h->L;
  TRY(enqueue_assemble_inverse(h, apply));  // replicated: K, D, K^{-1}, log det, step constants
  for (int k = 0; k < kGemmStages; ++k) {
    if (h->sst[k].n)  // (empty: a refinement stage of a path without refinement)
      TRY(check_launch(launch_gemm_auto(h->sdescs.data() + h->sst[k].off, h->sst[k].n, h->sc, h->s,
                                        h->sst[k].variant), "gemm"));
    for (const ShardGather& g : h->sgather[k]) TRY(h->comm->allgather(h, g.buf, g.chunk));
  }
  PGradArgs pa[2];
  for (int a = 0; a < 2; ++a) {
    pa[a] = PGradArgs{};
    pa[a].x = a == 0 ? h->x1 : h->x2;
    pa[a].n = a == 0 ? L.n1 : L.n2;
    pa[a].p = a == 0 ? L.p1 : L.p2;
    pa[a].kc = h->kc + a;
    pa[a].GK = h->GK[a];
    pa[a].GD = h->GD[a];
    pa[a].deriv = (h->prob.eq == GPK_ADVECTION) ? 1 : 2;
    pa[a].part = h->pgpart + (size_t)a * h->bpa * 3 * QMAX;
    pa[a].cls = h->cls[a];
  }
  // every rank contracts its own G_K / G_D rows (axis 1) and partials (axis 2) in full
  TRY(check_launch(launch_pgrad(h->prob.kind, L.q, 0, pa, 2, h->bpa, h->sc, h->s, nullptr), "pgrad"));
  TRY(check_launch(launch_reduce_parts(h->pgpart, h->bpa, 2, L.q, h->pg, h->s), "reduce_parts"));
  // the step's one all-reduce: [status bits | parameter-contraction partials | per-tile ||R||^2 |
  // per-tile <A, Bt>], contiguous (h->sred).  The status rides in it: a failed inverse (or a
  // rank-local hand-off timeout) fails every rank's batch before the loss is formed -- every rank
  // runs the same collectives whatever its status, so none waits alone
  TRY(check_launch(launch_status_f64(h->status, h->stat_x, 0, h->s), "status_pack"));
  TRY(h->comm->allreduce(h, h->sred, (size_t)(h->red_quad + h->nquad - h->sred)));
  TRY(check_launch(launch_status_f64(h->status, h->stat_x, 1, h->s), "status_unpack"));
  TailArgs T = make_tail(h, apply);
  T.fin.gpart = T.fin.gpart_lo = nullptr;  // (pg all-reduced above)
  T.fin.pg_out = nullptr;
  TRY(check_launch(launch_finalize(T.fin, h->s), "finalize"));
  // this rank's tile slots are rewritten next step; the summed copies must not leak into it
  HIPCHK(hipMemsetAsync(h->red_egap, 0, (size_t)h->negap * sizeof(double), h->s));
  HIPCHK(hipMemsetAsync(h->red_quad, 0, (size_t)h->nquad * sizeof(double), h->s));
  AdamUArgs au = T.adam;
  const int r0 = h->rank * h->h1, r1 = std::min(L.n1, r0 + h->h1);
  const int nu = L.n1 * L.n2;
  au.e0 = r0 < r1 ? r0 * L.n2 : nu;
  au.e1 = r0 < r1 ? r1 * L.n2 : nu;
  TRY(check_launch(launch_adam_u(au, h->s), "adam_u"));
  TRY(h->comm->allgather(h, h->Up, (size_t)h->h1 * L.p2));
  return GPK_OK;
}

constexpr int STEP_GRAPH_REPS = 8;
static int capture(gpk_handle* h, int apply, bool refine = true, int reps = 1, bool batch = false) {
  hipGraphExec_t* slot = batch ? &h->g_batch[refine ? 1 : 0][reps]
                       : reps > 1 ? &h->g_multi[refine ? 1 : 0]
                                  : refine ? &h->g_exec[apply] : &h->g_fast[apply];
  if (*slot) return GPK_OK;
  if (h->shard && !h->comm->capturable())
    return fail(GPK_EINVAL, "handle belongs to an in-process rank group: use gpk_group_step / gpk_group_loss_grad");
  hipGraph_t g = nullptr;
  HIPCHK(hipStreamBeginCapture(h->s, hipStreamCaptureModeThreadLocal));
  int rc = GPK_OK;
  h->cls_have = false;
  for (int r = 0; r < reps && rc == GPK_OK; ++r) {
    h->cls_next = r + 1 < reps;  // (cls_pipe_ok decides)
    rc = enqueue_step(h, apply, refine);
  }
  h->cls_next = h->cls_have = false;
  hipError_t e = hipStreamEndCapture(h->s, &g);
  if (rc != GPK_OK) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("capture: ") + hipGetErrorString(e));
  e = hipGraphInstantiate(slot, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("instantiate: ") + hipGetErrorString(e));
  return GPK_OK;
}

static StepReport make_report(gpk_handle* h, bool fast, int nloss) {
  StepReport r{};
  r.status = h->status;
  r.viol = fast ? h->viol : nullptr;
  for (int a = 0; a < h->L.naxes; ++a) r.pst[a] = h->pst[a];
  r.out = h->rep_host;
  r.losses = h->losses;
  r.nloss = nloss;
  return r;
}

// Batch begin for the graph being captured: folded into the first step's chain launch when
// that launch publishes the step constants (publish_prep, copy_snapshot), else its own launch.
static int begin_batch(gpk_handle* h, const StepBegin* b) {
  if (!h->shard && h->chain && h->cls[0].ncls > 0) {
    h->fold_begin = b;
    return GPK_OK;
  }
  return check_launch(launch_step_begin(*b, h->s), "step_begin");
}

// Batch end: the last step's loss workgroup wrote the report (make_tail took fold_report), or
// the report kernel runs after it.  Leaves no fold pending (also when the capture failed: rc).
static int end_batch(gpk_handle* h, const StepReport* r, int rc) {
  const bool pending_begin = h->fold_begin != nullptr, pending_report = h->fold_report != nullptr;
  h->fold_begin = nullptr;
  h->fold_report = nullptr;
  if (rc != GPK_OK) return rc;
  if (pending_begin) return fail(GPK_EINVAL, "internal: the batch begin was not folded into a step");
  if (pending_report || h->shard) return check_launch(launch_step_report(*r, h->s), "step_report");
  return GPK_OK;
}

// one step(1) call: begin (snapshot when fast) + step + report, captured once per graph kind
static int capture_call(gpk_handle* h, bool fast) {
  hipGraphExec_t* slot = &h->g_call[fast ? 0 : 1];
  if (*slot) return GPK_OK;
  const size_t np = (size_t)h->L.nparams;
  hipGraph_t g = nullptr;
  HIPCHK(hipStreamBeginCapture(h->s, hipStreamCaptureModeThreadLocal));
  StepBegin b{};  // every batch takes the snapshot: a failed one is undone (read_report)
  b.snap = h->snap; b.params = h->params; b.m = h->m; b.v = h->v; b.np = np;
  b.snap_count = h->snap_count; b.count = h->count;
  if (fast) b.viol = h->viol;
  b.loss_slot = h->loss_slot;
  const StepReport r = make_report(h, fast, 1);
  int rc = begin_batch(h, &b);
  if (rc == GPK_OK) {
    if (!h->shard) h->fold_report = &r;
    rc = enqueue_step(h, 1, !fast);
  }
  rc = end_batch(h, &r, rc);
  hipError_t e = hipStreamEndCapture(h->s, &g);
  if (rc != GPK_OK) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("capture: ") + hipGetErrorString(e));
  e = hipGraphInstantiate(slot, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("instantiate: ") + hipGetErrorString(e));
  return GPK_OK;
}

// a fast chunk of `reps` steps as one graph: begin (snapshot, counters) + steps + report
static int capture_calln(gpk_handle* h, int reps) {
  hipGraphExec_t* slot = &h->g_calln[reps];
  if (*slot) return GPK_OK;
  const size_t np = (size_t)h->L.nparams;
  hipGraph_t g = nullptr;
  HIPCHK(hipStreamBeginCapture(h->s, hipStreamCaptureModeThreadLocal));
  StepBegin b{};
  b.snap = h->snap; b.params = h->params; b.m = h->m; b.v = h->v; b.np = np;
  b.snap_count = h->snap_count; b.count = h->count; b.viol = h->viol;
  b.loss_slot = h->loss_slot;
  const StepReport rep = make_report(h, true, reps);
  int rc = begin_batch(h, &b);
  h->cls_have = false;
  for (int r = 0; r < reps && rc == GPK_OK; ++r) {
    if (r == reps - 1 && !h->shard) h->fold_report = &rep;
    h->cls_next = r + 1 < reps;  // (cls_pipe_ok decides)
    rc = enqueue_step(h, 1, false);
  }
  h->cls_next = h->cls_have = false;
  rc = end_batch(h, &rep, rc);
  hipError_t e = hipStreamEndCapture(h->s, &g);
  if (rc != GPK_OK) {
    if (g) (void)hipGraphDestroy(g);
    h->g_calln.erase(reps);
    return rc;
  }
  if (e != hipSuccess) {
    h->g_calln.erase(reps);
    return fail(GPK_EHIP, std::string("capture: ") + hipGetErrorString(e));
  }
  e = hipGraphInstantiate(slot, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    h->g_calln.erase(reps);
    return fail(GPK_EHIP, std::string("instantiate: ") + hipGetErrorString(e));
  }
  return GPK_OK;
}

// After a launch whose hand-off wait gave up (status bit 2), a late producer may still have
// stored real words into hand-off slots the consumer had already consumed and reset: restore
// every slot, flag and counter to its create-time state (the stream is synchronised, so every
// launch has drained) before the handle is used again -- stale words would otherwise pass for
// the next launch's inputs.
static int reset_handoffs(gpk_handle* h) {
  const Layout& L = h->L;
  for (int a = 0; a < L.naxes; ++a) {
    const size_t P = a == 0 ? L.p1 : L.p2, T = P / 32;
    const size_t nflags = T * (T + (L.p1 + L.p2) / 32) + 2 * T + 1;
    HIPCHK(hipMemsetD32Async(h->cgran[a], CHAIN_SENTINEL32, T * 4096, h->s));
    if (h->PB2[a]) HIPCHK(hipMemsetD32Async(h->PB2[a], CHAIN_SENTINEL32, 4 * chain_half((int)P, h->chain_multi), h->s));
    if (h->cepoch[a]) HIPCHK(hipMemsetAsync(h->cepoch[a], 0, 4 * sizeof(unsigned int), h->s));
    HIPCHK(hipMemsetAsync(h->cflags[a], 0, nflags * sizeof(unsigned int), h->s));
    HIPCHK(hipMemsetAsync(h->aflag[a], 0, (4 + P / 32) * sizeof(unsigned int), h->s));
  }
  HIPCHK(hipMemsetAsync(h->nce_flag, 0, sizeof(unsigned int), h->s));
  HIPCHK(hipStreamSynchronize(h->s));
  return GPK_OK;
}

static int read_status(gpk_handle* h) {
  int st = 0;
  HIPCHK(hipMemcpyAsync(&st, h->status, sizeof(int), hipMemcpyDeviceToHost, h->s));
  HIPCHK(hipStreamSynchronize(h->s));
  if (st) {
    HIPCHK(hipMemsetAsync(h->status, 0, sizeof(int), h->s));
    if (st & 2) TRY(reset_handoffs(h));
    return fail(GPK_ENOTPD, (st & 2) ? "SPD inverse: a pivot-chain hand-off timed out (device status 2)"
                                      : "covariance factor is not positive definite (non-positive pivot in SPD inverse)");
  }
  return GPK_OK;
}

// End of a batch (one synchronisation): non-positive-definite status, the fast graph's gate
// violation flag, and the refinement gate of the last step, which picks the next batch's graph:
// the fast one once max_a K00 * max diag K_a^{-1} is 2x below REFINE_COND_LB, and it stays
// the fast one while that bound stays below REFINE_COND_LB itself (hysteresis: a fast batch
// that crosses the gate is caught by the check in the fast graph's tail (viol) and rerun, which
// costs one FAST_CHUNK; leaving the fast graph at the margin cost ~15% on every later step of
// C4's training, whose bound drifts to ~21 (tools/train_regime_parity.py): round 4's 8x entry
// margin (12.5) kept a handle that had left the fast graph off it for ~2000 steps).
constexpr double FAST_GRAPH_MARGIN = 2.0;
static int read_report(gpk_handle* h, bool fast, bool* violated);

// params, Adam state and step count back to the snapshot the current batch's begin took (every
// gpk_step batch takes one), U's padded copy rebuilt from params: a fast batch that met an open
// refinement gate is rerun from there, a batch that failed on the device is undone
static int restore_snapshot(gpk_handle* h) {
  const size_t np = (size_t)h->L.nparams, nb = np * sizeof(double);
  HIPCHK(hipMemcpyAsync(h->params, h->snap, nb, hipMemcpyDeviceToDevice, h->s));
  HIPCHK(hipMemcpyAsync(h->m, h->snap + np, nb, hipMemcpyDeviceToDevice, h->s));
  HIPCHK(hipMemcpyAsync(h->v, h->snap + 2 * np, nb, hipMemcpyDeviceToDevice, h->s));
  HIPCHK(hipMemcpyAsync(h->count, h->snap_count, sizeof(int), hipMemcpyDeviceToDevice, h->s));
  return check_launch(launch_sync_u(h->params, h->L, h->Up, h->s), "sync_u");
}

static int finish_batch(gpk_handle* h, bool fast, bool* violated) {
  TRY(check_launch(launch_step_report(make_report(h, fast, h->pend_losses ? h->pend_n : 0), h->s),
                   "step_report"));
  HIPCHK(hipStreamSynchronize(h->s));
  return read_report(h, fast, violated);
}

// the report written by step_report_kernel (the stream has been synchronised)
static int read_report(gpk_handle* h, bool fast, bool* violated) {
  if (h->pend_losses) std::memcpy(h->pend_losses, h->rep_host + 8, h->pend_n * sizeof(double));
  h->pend_losses = nullptr;
  h->pend_n = 0;
  const int st = (int)h->rep_host[0];
  const unsigned int vi = (unsigned int)h->rep_host[1];
  double ps[2][2] = {{h->rep_host[2], h->rep_host[3]}, {h->rep_host[4], h->rep_host[5]}};
  *violated = false;
  if (st) {  // undo the batch (its begin took the snapshot), then report
    HIPCHK(hipMemsetAsync(h->status, 0, sizeof(int), h->s));
    if (st & 2) TRY(reset_handoffs(h));
    TRY(restore_snapshot(h));
    HIPCHK(hipStreamSynchronize(h->s));
    return fail(GPK_ENOTPD, (st & 2) ? "SPD inverse: a pivot-chain hand-off timed out (device status 2); "
                                       "the batch was undone"
                                     : "covariance factor is not positive definite (non-positive pivot in SPD inverse); "
                                       "the batch was undone");
  }
  *violated = fast && vi;
  if (h->fast_ok) {
    double lb = 0.0;  // pst[a][1] holds max diag K^{-1} (positive, atomicMax'd as its bits)
    for (int a = 0; a < h->L.naxes; ++a) lb = std::max(lb, ps[a][0] * ps[a][1]);
    const double margin = (fast && !*violated) ? 1.0 : FAST_GRAPH_MARGIN;
    h->fast_mode = !*violated && lb * margin < REFINE_COND_LB;
  }
  return GPK_OK;
}

// ------------------------------------------------------------------------------------------
// extern "C"
// ------------------------------------------------------------------------------------------
extern "C" {

int gpk_abi_version(void) { return GPK_ABI_VERSION; }

const char* gpk_last_error(void) { return g_err.c_str(); }

int gpk_device_count(int32_t* n) {
  if (!n) return fail(GPK_EINVAL, "n is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *n = c;
  return GPK_OK;
}

static int check_device(int dev) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || c == 0) return fail(GPK_ENODEV, "no HIP device visible");
  if (dev < 0 || dev >= c) return fail(GPK_EINVAL, "device ordinal out of range");
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(GPK_ENODEV, std::string("libgpk is built for gfx950, device is ") + prop.gcnArchName);
  return GPK_OK;
}

static void host_axis_const(const double* logw, const double* logls, const double* freq, int q,
                            AxisConst* kc) {
  std::memset(kc, 0, sizeof(AxisConst));
  for (int c = 0; c < q; ++c) {
    kc->w[c] = std::exp(logw[c]);
    kc->a[c] = std::exp(logls[c]);
    kc->om[c] = TWO_PI * freq[c];
    kc->oml[c] = om_low(freq[c], kc->om[c]);
  }
}

int gpk_kernel_matrices(int32_t kind, int32_t deriv, const double* x1, int32_t n1,
                        const double* x2, int32_t n2, const double* logw, const double* logls,
                        const double* freq, int32_t q, double jitter, double* K_out,
                        double* D_out) {
  if (kind < 0 || kind > 3) return fail(GPK_EINVAL, "Invalid Kernel");
  if (deriv < 0 || deriv > 2) return fail(GPK_EINVAL, "deriv must be 0, 1 or 2");
  if (n1 <= 0 || n2 <= 0 || q <= 0 || q > QMAX) return fail(GPK_EINVAL, "bad sizes (0 < q <= 64)");
  if (!x1 || !x2 || !logw || !logls || !freq || !K_out || (deriv && !D_out))
    return fail(GPK_EINVAL, "NULL pointer argument");
  int dev = 0;
  (void)hipGetDevice(&dev);
  TRY(check_device(dev));
  AxisConst hk;
  host_axis_const(logw, logls, freq, q, &hk);
  double *dx1, *dx2, *dK, *dD = nullptr;
  AxisConst* dkc;
  size_t nn = (size_t)n1 * n2;
  HIPCHK(hipMalloc(&dx1, n1 * sizeof(double)));
  HIPCHK(hipMalloc(&dx2, n2 * sizeof(double)));
  HIPCHK(hipMalloc(&dK, nn * sizeof(double)));
  if (deriv) HIPCHK(hipMalloc(&dD, nn * sizeof(double)));
  HIPCHK(hipMalloc(&dkc, sizeof(AxisConst)));
  HIPCHK(hipMemcpy(dx1, x1, n1 * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx2, x2, n2 * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dkc, &hk, sizeof(AxisConst), hipMemcpyHostToDevice));
  TRY(check_launch(launch_cross(kind, q, dx1, n1, dx2, n2, n2, dkc, jitter, deriv, dK, dD, 0), "cross"));
  HIPCHK(hipMemcpy(K_out, dK, nn * sizeof(double), hipMemcpyDeviceToHost));
  if (deriv) HIPCHK(hipMemcpy(D_out, dD, nn * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(dx1); (void)hipFree(dx2); (void)hipFree(dK); (void)hipFree(dkc);
  if (dD) (void)hipFree(dD);
  return GPK_OK;
}

// padm: padding multiple of the matrix dimensions (32; 32 * nranks for a row-sharded handle so
// that every rank's row block is a whole number of 32-row tiles)
static Layout make_layout(const gpk_problem* p, int padm = PADM) {
  auto pad_up = [padm](int n) { return (n + padm - 1) / padm * padm; };
  Layout L{};
  L.dim = p->dim;
  L.q = p->q;
  L.n1 = p->n1;
  L.p1 = pad_up(p->n1);
  if (p->dim == 2) {
    L.naxes = 2;
    L.n2 = p->n2;
    L.p2 = pad_up(p->n2);
    const int nu = p->n1 * p->n2;
    L.off_u = 0;
    L.off_kp[0] = nu;
    L.off_kp[1] = nu + 3 * p->q;
    L.off_tau = nu + 6 * p->q;
    L.off_v = L.off_tau + 1;
    L.off_small = nu;
    L.nsmall = 6 * p->q + 2;
    L.nparams = (int64_t)nu + 6 * p->q + 2;
  } else {
    L.naxes = 1;
    L.n2 = 1;
    L.p2 = 1;
    L.off_kp[0] = 0;
    L.off_kp[1] = 0;
    L.off_tau = 3 * p->q;
    L.off_v = 3 * p->q + 1;
    L.off_u = 3 * p->q + 2;
    L.off_small = 0;
    L.nsmall = 3 * p->q + 2;
    L.nparams = (int64_t)p->n1 + 3 * p->q + 2;
  }
  return L;
}

static std::vector<double> init_params(const gpk_problem* p, const Layout& L, double freq_scale) {
  // train(): log_tau = log_v = 0; log-w = log(1/Q); log-ls = 0; freq = linspace(0,1,Q)*fs; U = 0
  std::vector<double> h((size_t)L.nparams, 0.0);
  const int q = p->q;
  for (int a = 0; a < L.naxes; ++a) {
    const int off = L.off_kp[a];
    for (int c = 0; c < q; ++c) {
      const double lin = (q == 1) ? 0.0 : (double)c / (double)(q - 1);  // np.linspace(0,1,Q)
      h[off + c] = lin * freq_scale;
      h[off + q + c] = 0.0;
      h[off + 2 * q + c] = std::log(1.0 / q);
    }
  }
  return h;
}

static int create_impl(const gpk_problem* p, double freq_scale, int rank, int nranks, bool shard,
                       gpk_handle** out, bool local_group = false) {
  if (!p || !out) return fail(GPK_EINVAL, "NULL argument");
  *out = nullptr;
  if (p->dim != 1 && p->dim != 2) return fail(GPK_EINVAL, "dim must be 1 or 2");
  if (p->kind < 0 || p->kind > 3) return fail(GPK_EINVAL, "Invalid Kernel");
  if (p->eq < 0 || p->eq > 2 || (p->eq == GPK_ADVECTION && p->dim != 2))
    return fail(GPK_EINVAL, "equation type not supported for this dimension");
  if (p->q <= 0 || p->q > QMAX) return fail(GPK_EINVAL, "Q must be in [1, 64]");
  if (p->n1 < 2 || (p->dim == 2 && p->n2 < 2)) return fail(GPK_EINVAL, "need >= 2 collocation points per axis");
  if (!p->x1 || !p->src || !p->bvals || (p->dim == 2 && !p->x2) || (p->dim == 1 && (!p->bidx || p->nb <= 0)))
    return fail(GPK_EINVAL, "NULL problem array");
  if (p->dim == 1)
    for (int k = 0; k < p->nb; ++k)
      if (p->bidx[k] < 0 || p->bidx[k] >= p->n1) return fail(GPK_EINVAL, "Xind out of range");
  TRY(check_device(p->device));
  DevSwitch ds(p->device);
  gpk_handle* h = new gpk_handle();
  h->prob = *p;
  h->prob.x1 = h->prob.x2 = h->prob.src = h->prob.bvals = nullptr;
  h->prob.bidx = nullptr;
  h->prob.uoff = nullptr;
  if (p->dim == 2) h->prob.nb = 2 * p->n1 + 2 * p->n2;
  h->freq_scale = freq_scale;
  h->dev = p->device;
  h->shard = shard;
  h->rank = rank;
  h->nranks = nranks;
  h->L = make_layout(p, shard ? PADM * nranks : PADM);
  h->hyper = AdamHyper{p->lr, p->b1, p->b2, p->eps};
  const Layout& L = h->L;
  {
    const int pmax = std::max(L.p1, L.dim == 2 ? L.p2 : 0);
    h->bigspd = (p->flags & GPK_FLAG_FORCE_BIG_SPD) != 0 ||
                (!(p->flags & GPK_FLAG_FORCE_SMALL_SPD) && pmax >= SPD_BIG_MIN);
    h->bigwide = h->bigspd && !(p->flags & GPK_FLAG_FORCE_NARROW_SPD) &&
                 ((p->flags & GPK_FLAG_FORCE_WIDE_SPD) || pmax >= SPD_WIDE_MIN);
    // The persistent chain inverse needs its whole grid co-resident: the grid (workgroups of
    // every factor's row, the widest row times the factors) must fit the device's capacity for
    // the chain variant the step launches (occupancy per CU x CUs, so a CU-partitioned device
    // falls back to the per-sweep launches), and handles of an in-process rank group -- which
    // launch concurrently on one device from several host threads -- never use it.
    const int pp[2] = {L.p1, L.p2};
    const int deriv = p->eq == GPK_ADVECTION ? 1 : 2;
    int cap = g_chain_cap.load();
    if (cap <= 0) {
      DevSwitch dsw(p->device);
      const bool gather = !(p->flags & GPK_FLAG_NO_DCLASS);  // (gather mode needs classes; the
      cap = std::min(spd_chain_capacity(deriv, gather),       //  per-pair mode's footprint is
                     spd_chain_capacity(deriv, false));        //  bounded by the same check)
    }
    cap = std::min(cap, CHAIN_MAX_BLOCKS);
    auto grid_blocks = [&](bool aug) {  // launch_spd_chain's grid: (max_a T_a TC_a + 1) x factors
      const int cols = (L.p1 + (L.naxes == 2 ? L.p2 : 0)) / 32;
      int wide = 0;
      for (int a = 0; a < L.naxes; ++a) wide = std::max(wide, (pp[a] / 32) * (pp[a] / 32 + (aug ? cols : 0)) + 1);
      return wide * L.naxes;
    };
    const bool in_group = shard && local_group && nranks > 1;
    if (shard && nranks >= 2 && (p->flags & GPK_FLAG_SPLIT_FACTORS)) h->split_axis = rank < nranks / 2 ? 0 : 1;
    // (the chain inverts every factor in one launch: a split rank inverts one, per sweep)
    // (an in-process group's ranks launch their chains concurrently on the one device: all of
    // them must be co-resident together -- the 2-rank group is how the tests exercise the exact
    // chain + row-sharded step an RCCL rank runs)
    const int chains_on_device = in_group ? nranks : 1;
    h->chain = !h->bigspd && h->split_axis < 0 && !(p->flags & GPK_FLAG_NO_CHAIN) &&
               grid_blocks(false) * chains_on_device <= cap;
    // (row-sharded handles too: the augmented chain gives every rank the whole A, Bt and
    // K^{-1} D^T from its replicated inverse, so the forward solves need no all-gather -- the
    // sharded step's plan, build_shard)
    h->chain_aug = h->chain && L.dim == 2 && !(p->flags & GPK_FLAG_NO_CHAIN_AUG) &&
                   grid_blocks(true) * chains_on_device <= cap;
    // large 1D factors: the persistent inverse on 64-row macro tiles (chain_multi_kernel), when
    // its grid is co-resident (else the 64/128-wide launch-per-sweep path)
    if (L.dim == 1 && !in_group && h->split_axis < 0 &&
        !(p->flags & (GPK_FLAG_NO_CHAIN | GPK_FLAG_FORCE_BIG_SPD | GPK_FLAG_FORCE_SMALL_SPD)) &&
        (pmax >= SPD_BIG_MIN || (p->flags & GPK_FLAG_FORCE_CHAIN_MULTI))) {
      int mcap = g_chain_cap.load();
      if (mcap <= 0) {
        DevSwitch dsw(p->device);
        const bool gather = !(p->flags & GPK_FLAG_NO_DCLASS);
        mcap = std::min(spd_chain_multi_capacity(deriv, gather), spd_chain_multi_capacity(deriv, false));
      }
      if (spd_chain_multi_blocks(pp, L.naxes) <= mcap) {
        h->chain_multi = h->chain = true;
        h->chain_aug = h->bigspd = h->bigwide = false;
      }
    }
  }
  auto bail = [&](int rc) {
    gpk_destroy(h);
    return rc;
  };
  if (hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(GPK_EHIP, "hipStreamCreate failed"));
  const int P1 = L.p1, P2 = L.p2;
  const size_t nup = (size_t)P1 * P2;
  int rc = GPK_OK;
#define A_(ptr, n) \
  if ((rc = h->alloc(&(ptr), (n))) != GPK_OK) return bail(rc)
  A_(h->x1, P1);
  A_(h->x2, std::max(P2, 1));
  A_(h->F, nup);
  A_(h->bvals, h->prob.nb);
  A_(h->bidx, std::max(p->nb, 1));
  A_(h->params, L.nparams);
  A_(h->grad, L.nparams);
  A_(h->m, L.nparams);
  A_(h->v, L.nparams);
  A_(h->Up, nup);
  A_(h->kc, 2);
  A_(h->sc, 1);
  A_(h->count, 1);
  A_(h->loss_slot, 1);
  A_(h->status, 1);
  A_(h->stat_x, 2);
  A_(h->losses, LOSS_CAP);
  A_(h->diag, 8);
  for (int a = 0; a < L.naxes; ++a) {
    const int P = a == 0 ? P1 : P2;
    A_(h->K[a], (size_t)P * P);
    A_(h->Kb[a], (size_t)P * P);
    A_(h->D[a], (size_t)P * P);
    A_(h->piv[a], spd_big_piv_doubles(P));  // large path: W x W L^{-1} + 128-pivot scratch
    A_(h->ldet[a], P / 32);
    A_(h->Kc[a], (size_t)P * P);
    A_(h->pst[a], 2);
    A_(h->aflag[a], 4 + P / 32);  // + the 128-wide update's per-sweep panel tickets
    if (h->bigspd) A_(h->Zp[a], (size_t)3 * 128 * P);
    if (h->bigspd && h->bigwide && !(p->flags & GPK_FLAG_ONE_SWEEP_UPDATE)) {
      const int T2 = (int)((P + 127) / 128);
      std::vector<unsigned> tab;
      wide_schedule(T2, true, tab);
      A_(h->wsched[a], tab.size());
      if (hipMemcpyAsync(h->wsched[a], tab.data(), tab.size() * sizeof(unsigned), hipMemcpyHostToDevice, h->s) != hipSuccess ||
          hipStreamSynchronize(h->s) != hipSuccess)
        return bail(fail(GPK_EHIP, "upload the update schedule"));
    }
    A_(h->cflags[a], (size_t)(P / 32) * (P / 32 + (P1 + P2) / 32) + 2 * (P / 32) + 1);
    A_(h->cgran[a], (size_t)(P / 32) * 2048);
    // every hand-off slot starts unwritten (spdinv.hip chain_master / chain_multi_kernel)
    if (hipMemsetD32Async(h->cgran[a], CHAIN_SENTINEL32, (size_t)(P / 32) * 4096, h->s) != hipSuccess)
      return bail(fail(GPK_EHIP, "initialise the pivot-chain input slots"));
    if (h->chain) {  // chain_multi: panel + L^{-1} slots; chain_kernel: the L^{-1} slots
      A_(h->PB2[a], 2 * chain_half(P, h->chain_multi));
      A_(h->cepoch[a], 4);
      if (hipMemsetD32Async(h->PB2[a], CHAIN_SENTINEL32, 4 * chain_half(P, h->chain_multi), h->s) != hipSuccess)
        return bail(fail(GPK_EHIP, "initialise the panel slots"));
    }
    if (h->chain_aug) {
      A_(h->PD[a], (size_t)P * P);
      A_(h->PBa[a], (size_t)P * (P1 + P2));
    }
    h->nldet[a] = P / 32;
  }
  if (L.dim == 2) {
    A_(h->A, nup); A_(h->Bt, nup); A_(h->S, nup); A_(h->R, nup);
    A_(h->T1, nup); A_(h->T2, nup); A_(h->X1, nup); A_(h->X2, nup);
    A_(h->W1, nup); A_(h->W2, nup); A_(h->Y1, nup); A_(h->Y2, nup);
    for (int a = 0; a < 2; ++a) {
      const int P = a == 0 ? P1 : P2;
      A_(h->GK[a], (size_t)P * P);
      A_(h->GD[a], (size_t)P * P);
    }
    h->nquad = h->negap = (P1 / 16) * (P2 / 16);  // upper bound (16x16 tiles); set in build_descs
  } else {
    A_(h->alpha, P1); A_(h->R, P1); A_(h->tvec, P1); A_(h->beta, P1); A_(h->rvec, P1);
    if (p->uoff) A_(h->uoff, P1);
    h->nquad = h->negap = gemv_blocks(P1);
  }
  if (shard) {  // one all-reduce per sharded step: [status | pg | egap | quad] (enqueue_step_shard)
    const size_t npg = (size_t)L.naxes * 3 * QMAX;
    A_(h->sred, 2 + npg + (size_t)h->negap + (size_t)h->nquad);
    h->stat_x = h->sred;
    h->pg = h->sred + 2;
    h->red_egap = h->pg + npg;
    h->red_quad = h->red_egap + h->negap;
  } else {
    A_(h->red_quad, h->nquad);
    A_(h->red_egap, h->negap);
  }
  // distance classes (both axes or none), uploaded once: the coordinates never change
  std::vector<double> cdist[2];
  std::vector<int> ccid[2], cbase[2];
  bool use_cls = !(p->flags & GPK_FLAG_NO_DCLASS);
  int vmax[2] = {0, 0};
  for (int a = 0; a < L.naxes && use_cls; ++a)
    use_cls = build_classes(a == 0 ? p->x1 : p->x2, a == 0 ? L.n1 : L.n2, a == 0 ? P1 : P2,
                            cdist[a], ccid[a], cbase[a], vmax[a]);
  if (use_cls) {
    for (int a = 0; a < L.naxes; ++a) {
      const int P = a == 0 ? P1 : P2, U = (int)cdist[a].size();
      ClassArgs& c = h->cls[a];
      double *dist = nullptr, *kval = nullptr, *dval = nullptr, *part = nullptr;
      int *cid = nullptr, *cb = nullptr;
      // class-sum row chunks: <= 64 chunks of >= 16 rows (one 4-row group per wave and pass);
      // with the LDS bins (> 8 variants per diagonal: 70 KB per workgroup, two per CU) <= 32
      // chunks -- C2: 0.693 -> 0.688 ms/step (64 rows; 128 the same, 256 slower)
      const int n = a == 0 ? L.n1 : L.n2;
      const int maxchunks = vmax[a] > 8 ? 32 : 64;
      const int rb = std::max(16, (n + maxchunks - 1) / maxchunks + 15) / 16 * 16;
      const int nchunk = (n + rb - 1) / rb;
      A_(dist, U); A_(kval, U); A_(dval, U); A_(part, (size_t)2 * nchunk * U);
      A_(cid, (size_t)P * P); A_(cb, cbase[a].size());
      if (hipMemcpyAsync(dist, cdist[a].data(), U * sizeof(double), hipMemcpyHostToDevice, h->s) != hipSuccess ||
          hipMemcpyAsync(cid, ccid[a].data(), ccid[a].size() * sizeof(int), hipMemcpyHostToDevice, h->s) != hipSuccess ||
          hipMemcpyAsync(cb, cbase[a].data(), cbase[a].size() * sizeof(int), hipMemcpyHostToDevice, h->s) != hipSuccess)
        return bail(fail(GPK_EHIP, "upload distance classes"));
      c.ncls = U; c.vmax = vmax[a]; c.dist = dist; c.cid = cid; c.cbase = cb;
      c.kval = kval; c.dval = dval; c.nchunk = nchunk; c.rb = rb; c.part = part;
      // the large-factor gather's variant bytes (ClassArgs::vidx), for EVERY axis once the
      // largest one takes gather_wide_kernel (assemble.hip: (P/32)^2 >= GW_WIDE_MIN_TILES, i.e.
      // max P >= 1024) -- that launch assembles all axes at once
      if (std::max(P1, L.naxes == 2 ? P2 : 0) >= 1024) {
        std::vector<unsigned char> vb((size_t)P * P, 0xff);
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < n; ++j) {
            const int u = ccid[a][(size_t)i * P + j];
            if (u >= 0) vb[(size_t)i * P + j] = (unsigned char)(u - cbase[a][std::abs(i - j)]);
          }
        unsigned char* dv = nullptr;
        if (hipMalloc(&dv, vb.size()) != hipSuccess) return bail(fail(GPK_ENOMEM, "hipMalloc (class variants)"));
        h->allocs.push_back(dv);
        if (hipMemcpyAsync(dv, vb.data(), vb.size(), hipMemcpyHostToDevice, h->s) != hipSuccess ||
            hipStreamSynchronize(h->s) != hipSuccess)
          return bail(fail(GPK_EHIP, "upload class variants"));
        c.vidx = dv;
      }
    }
    h->bpa = std::max(pgrad_class_blocks(h->cls[0].ncls), L.dim == 2 ? pgrad_class_blocks(h->cls[1].ncls) : 0);
    // 2D, <= CB_VMAX variants per diagonal, unsharded: the G_K / G_D GEMMs sum their tiles per
    // class (build_descs turns it on when both stages take the 16x16-tile kernel)
    if (L.dim == 2 && !shard && !(p->flags & GPK_FLAG_NO_CLASS_BINS) && vmax[0] <= CB_VMAX &&
        vmax[1] <= CB_VMAX) {
      for (int a = 0; a < 2; ++a) {
        const size_t ns = (size_t)h->cls[a].ncls * class_slots((a == 0 ? P1 : P2) / 16);
        A_(h->cpK[a], ns);
        A_(h->cpD[a], ns);
      }
    }
    h->cls_gemv = h->chain_multi && L.dim == 1 && !(p->flags & GPK_FLAG_MATRIX_GEMV);
  } else {
    h->bpa = std::max(pgrad_blocks(L.n1), L.dim == 2 ? pgrad_blocks(L.n2) : 0);
  }
  A_(h->pgpart, (size_t)L.naxes * h->bpa * 3 * QMAX);
  if (!shard) A_(h->pg, (size_t)L.naxes * 3 * QMAX);
  h->ttg = std::max(16, (int)std::ceil(std::sqrt((double)h->bpa)));  // one 16-load batch per level at C4
  h->tngpa = (h->bpa + h->ttg - 1) / h->ttg;
  A_(h->tcount, (size_t)L.naxes * h->tngpa);
  A_(h->ttop, 1);
  A_(h->tgpart, (size_t)L.naxes * h->tngpa * 3 * QMAX);
  // The kernel-parameter contraction in double-double on the large 2D factors (C5): there the
  // sum over classes cancels ~1e8-fold and the fp64 rounding of the derivative fields sets its
  // accuracy; at C4 it would cost the latency-bound step ~1 us and buys nothing
  h->pg_dd = use_cls && !shard && !(p->flags & GPK_FLAG_NO_DD_CONTRACTION) &&
             ((L.dim == 2 && std::max(P1, P2) >= SPD_WIDE_MIN) || (p->flags & GPK_FLAG_DD_CONTRACTION));
  if (h->pg_dd) {
    A_(h->pgpart_lo, (size_t)L.naxes * h->bpa * 3 * QMAX);
    A_(h->tgpart_lo, (size_t)L.naxes * h->tngpa * 3 * QMAX);
  }
  // boundary-gap parts (PrepArgs::bgap): one per BGAP_CHUNK entries of a 2D boundary
  h->bgap_parts = L.dim == 2 ? std::min(BGAP_PARTS_MAX, std::max(1, (2 * L.n1 + 2 * L.n2 + BGAP_CHUNK - 1) / BGAP_CHUNK)) : 1;
  A_(h->bgap, BGAP_PARTS_MAX);
  A_(h->snap, (size_t)3 * L.nparams);
  A_(h->snap_count, 1);
  A_(h->viol, 1);
  A_(h->nce_flag, 1);
  A_(h->nce_kp, (size_t)L.nsmall);
  if (hipHostMalloc(reinterpret_cast<void**>(&h->rep_host), (8 + LOSS_CAP) * sizeof(double),
                    hipHostMallocCoherent) != hipSuccess)
    return bail(fail(GPK_ENOMEM, "hipHostMalloc (step report)"));
  std::memset(h->rep_host, 0, (8 + LOSS_CAP) * sizeof(double));
#undef A_
  // upload the problem
  if (hipMemcpyAsync(h->x1, p->x1, L.n1 * sizeof(double), hipMemcpyHostToDevice, h->s) != hipSuccess)
    return bail(fail(GPK_EHIP, "upload x1"));
  if (L.dim == 2) {
    (void)hipMemcpyAsync(h->x2, p->x2, L.n2 * sizeof(double), hipMemcpyHostToDevice, h->s);
    for (int i = 0; i < L.n1; ++i)
      (void)hipMemcpyAsync(h->F + (size_t)i * P2, p->src + (size_t)i * L.n2, L.n2 * sizeof(double),
                           hipMemcpyHostToDevice, h->s);
  } else {
    (void)hipMemcpyAsync(h->F, p->src, L.n1 * sizeof(double), hipMemcpyHostToDevice, h->s);
    (void)hipMemcpyAsync(h->bidx, p->bidx, p->nb * sizeof(int), hipMemcpyHostToDevice, h->s);
    if (p->uoff)
      (void)hipMemcpyAsync(h->uoff, p->uoff, L.n1 * sizeof(double), hipMemcpyHostToDevice, h->s);
  }
  (void)hipMemcpyAsync(h->bvals, p->bvals, h->prob.nb * sizeof(double), hipMemcpyHostToDevice, h->s);
  std::vector<double> init = init_params(p, L, freq_scale);
  (void)hipMemcpyAsync(h->params, init.data(), init.size() * sizeof(double), hipMemcpyHostToDevice, h->s);
  if (hipStreamSynchronize(h->s) != hipSuccess) return bail(fail(GPK_EHIP, "upload failed"));
  for (int k = 0; k <= kMaxStages; ++k)
    if (hipEventCreate(&h->ev[k]) != hipSuccess) return bail(fail(GPK_EHIP, "hipEventCreate"));
  // Kinv buffer identity is static (parity of the sweep count): resolve it by a dry enqueue
  // of the inverse into a throwaway capture is unnecessary -- compute it directly.
  for (int a = 0; a < L.naxes; ++a) {
    const int T = (a == 0 ? P1 : P2) / 32;
    h->Kinv[a] = (h->bigspd || h->chain) ? h->K[a] : ((T & 1) ? h->Kb[a] : h->K[a]);
  }
  if (L.dim == 2 && (rc = build_descs(h)) != GPK_OK) return bail(rc);
  if (shard && (rc = build_shard(h)) != GPK_OK) return bail(rc);
  // (the 2D large-factor path has no refinement stages: its one graph is the fast one)
  h->fast_ok = !shard && !(h->bigspd && L.dim == 2) && !(p->flags & GPK_FLAG_NO_FAST_GRAPH);
  h->fast_mode = h->fast_ok && (p->flags & GPK_FLAG_FAST_FIRST);
  *out = h;
  return GPK_OK;
}

int gpk_create(const gpk_problem* p, double freq_scale, gpk_handle** out) {
  return create_impl(p, freq_scale, 0, 1, false, out);
}

int gpk_comm_unique_id(uint8_t* out, int32_t len) {
  if (!out || len < (int32_t)sizeof(ncclUniqueId)) return fail(GPK_EINVAL, "need a 128-byte buffer");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(GPK_ERCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out, &id, sizeof(id));
  return GPK_OK;
}

int gpk_create_sharded(const gpk_problem* p, double freq_scale, int32_t rank, int32_t nranks,
                       const uint8_t* comm_id, gpk_handle** out) {
  if (!p || !out || !comm_id) return fail(GPK_EINVAL, "NULL argument");
  if (p->dim != 2) return fail(GPK_EINVAL, "row-sharded handles are 2D (Kronecker) only");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(GPK_EINVAL, "bad rank / nranks");
  gpk_handle* h = nullptr;
  TRY(create_impl(p, freq_scale, rank, nranks, true, &h));
  DevSwitch ds(h->dev);
  RcclComm* c = new RcclComm();
  ncclUniqueId id;
  std::memcpy(&id, comm_id, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&c->c, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    gpk_destroy(h);
    return fail(GPK_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  h->comm = c;
  *out = h;
  return GPK_OK;
}

int gpk_group_create(const gpk_problem* p, double freq_scale, int32_t nranks, gpk_handle** out) {
  if (!p || !out) return fail(GPK_EINVAL, "NULL argument");
  if (p->dim != 2) return fail(GPK_EINVAL, "row-sharded handles are 2D (Kronecker) only");
  if (nranks < 1 || nranks > 64) return fail(GPK_EINVAL, "nranks must be in [1, 64]");
  auto g = std::make_shared<LocalGroup>();
  g->n = nranks;
  g->slot.assign(nranks, nullptr);
  for (int r = 0; r < nranks; ++r) out[r] = nullptr;
  for (int r = 0; r < nranks; ++r) {
    int rc = create_impl(p, freq_scale, r, nranks, true, &out[r], true);
    if (rc != GPK_OK) {
      for (int k = 0; k < r; ++k) gpk_destroy(out[k]);
      return rc;
    }
    LocalComm* c = new LocalComm();
    c->g = g;
    out[r]->comm = c;
  }
  return GPK_OK;
}

// one host thread per rank, eager launches (an in-process group cannot be graph-captured)
static int group_run(gpk_handle** hs, int nranks, int apply, int n_steps) {
  if (!hs || nranks < 1) return fail(GPK_EINVAL, "bad group");
  for (int r = 0; r < nranks; ++r)
    if (!hs[r] || !hs[r]->shard || hs[r]->comm->capturable() || hs[r]->rank != r || hs[r]->nranks != nranks)
      return fail(GPK_EINVAL, "not the handles of one gpk_group_create group, in rank order");
  std::vector<int> rcs(nranks, GPK_OK);
  std::vector<std::string> errs(nranks);
  std::vector<std::thread> th;
  for (int r = 0; r < nranks; ++r)
    th.emplace_back([&, r]() {
      gpk_handle* h = hs[r];
      DevSwitch ds(h->dev);
      // the batch begin: loss slot reset and the snapshot a failed batch is undone to
      StepBegin b{};
      b.snap = h->snap; b.params = h->params; b.m = h->m; b.v = h->v; b.np = (size_t)h->L.nparams;
      b.snap_count = h->snap_count; b.count = h->count; b.loss_slot = h->loss_slot;
      int rc = check_launch(launch_step_begin(b, h->s), "step_begin");
      for (int i = 0; i < n_steps && rc == GPK_OK; ++i) rc = enqueue_step_shard(h, apply);
      if (rc == GPK_OK && hipStreamSynchronize(h->s) != hipSuccess) rc = fail(GPK_EHIP, "group step sync");
      if (rc != GPK_OK) {
        errs[r] = g_err;
        static_cast<LocalComm*>(h->comm)->g->abort();
      }
      rcs[r] = rc;
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < nranks; ++r)
    if (rcs[r] != GPK_OK) return fail(rcs[r], "rank " + std::to_string(r) + ": " + errs[r]);
  // every rank's status: the step makes it group-wide (its one all-reduce), so ranks that disagree
  // are an internal error.  A failed batch (non-PD factor, or a hand-off timeout: bit 2, raised by
  // one rank's wait and summed over the group) fails the whole group with GPK_ENOTPD; every rank
  // resets its hand-off slots and restores the batch's snapshot.
  std::vector<int> st(nranks, 0);
  int any = 0, bad = 0;
  for (int r = 0; r < nranks; ++r) {
    DevSwitch ds(hs[r]->dev);
    HIPCHK(hipMemcpy(&st[r], hs[r]->status, sizeof(int), hipMemcpyDeviceToHost));
    any |= st[r];
    bad += st[r] != 0;
  }
  if (!any) return GPK_OK;
  for (int r = 0; r < nranks; ++r) {  // every rank undoes the batch (gpk.h: failed batches are undone)
    DevSwitch ds(hs[r]->dev);
    HIPCHK(hipMemsetAsync(hs[r]->status, 0, sizeof(int), hs[r]->s));
    if (any & 2) TRY(reset_handoffs(hs[r]));
    TRY(restore_snapshot(hs[r]));
    HIPCHK(hipStreamSynchronize(hs[r]->s));
  }
  if (any & 2) {
    int r0 = 0;
    while (!(st[r0] & 2)) ++r0;
    return fail(GPK_ENOTPD, "SPD inverse: a pivot-chain hand-off timed out (device status 2, rank " +
                                std::to_string(r0) + ")");
  }
  if (bad != nranks)
    return fail(GPK_EINVAL, "internal: device status differs across the ranks of the group (" +
                                std::to_string(bad) + " of " + std::to_string(nranks) + ")");
  return fail(GPK_ENOTPD, "covariance factor is not positive definite (non-positive pivot in SPD inverse)");
}

int gpk_group_step(gpk_handle** hs, int32_t nranks, int32_t n_steps, double* losses) {
  if (n_steps < 0 || n_steps > LOSS_CAP) return fail(GPK_EINVAL, "n_steps must be in [0, 4096]");
  TRY(group_run(hs, nranks, 1, n_steps));
  if (losses && n_steps > 0) {
    DevSwitch ds(hs[0]->dev);
    HIPCHK(hipMemcpy(losses, hs[0]->losses, n_steps * sizeof(double), hipMemcpyDeviceToHost));
  }
  return GPK_OK;
}

int gpk_group_loss_grad(gpk_handle** hs, int32_t nranks, double* loss, double* grad_flat) {
  if (!loss) return fail(GPK_EINVAL, "NULL argument");
  TRY(group_run(hs, nranks, 0, 1));
  const Layout& L = hs[0]->L;
  DevSwitch ds(hs[0]->dev);
  HIPCHK(hipMemcpy(loss, hs[0]->diag, sizeof(double), hipMemcpyDeviceToHost));
  if (grad_flat) {  // small params from rank 0 (identical on every rank), U rows from their owner
    HIPCHK(hipMemcpy(grad_flat, hs[0]->grad, L.nparams * sizeof(double), hipMemcpyDeviceToHost));
    for (int r = 1; r < nranks; ++r) {
      const int r0 = r * hs[r]->h1, r1 = std::min(L.n1, r0 + hs[r]->h1);
      if (r0 >= r1) continue;
      HIPCHK(hipMemcpy(grad_flat + L.off_u + (size_t)r0 * L.n2, hs[r]->grad + L.off_u + (size_t)r0 * L.n2,
                       (size_t)(r1 - r0) * L.n2 * sizeof(double), hipMemcpyDeviceToHost));
    }
  }
  return GPK_OK;
}

int gpk_shard_plan(const gpk_handle* h, char* out, int64_t cap) {
  if (!h || !out || cap < 1) return fail(GPK_EINVAL, "NULL argument");
  if (!h->shard) return fail(GPK_EINVAL, "gpk_shard_plan: not a row-sharded handle");
  if ((int64_t)h->splan.size() + 1 > cap) return fail(GPK_EINVAL, "gpk_shard_plan: cap too small");
  std::memcpy(out, h->splan.c_str(), h->splan.size() + 1);
  return GPK_OK;
}

int gpk_shard_info(const gpk_handle* h, int32_t* rank, int32_t* nranks, int32_t* row0, int32_t* rows) {
  if (!h || !rank || !nranks || !row0 || !rows) return fail(GPK_EINVAL, "NULL argument");
  *rank = h->rank;
  *nranks = h->nranks;
  if (!h->shard) {
    *row0 = 0;
    *rows = h->L.n1;
    return GPK_OK;
  }
  *row0 = h->rank * h->h1;
  *rows = std::max(0, std::min(h->L.n1, *row0 + h->h1) - *row0);
  return GPK_OK;
}

int gpk_destroy(gpk_handle* h) {
  if (!h) return GPK_OK;
  DevSwitch ds(h->dev);
  if (h->s) (void)hipStreamSynchronize(h->s);
  for (int k = 0; k < 2; ++k) {
    if (h->g_exec[k]) (void)hipGraphExecDestroy(h->g_exec[k]);
    if (h->g_fast[k]) (void)hipGraphExecDestroy(h->g_fast[k]);
    if (h->g_multi[k]) (void)hipGraphExecDestroy(h->g_multi[k]);
    for (auto& kv : h->g_batch[k])
      if (kv.second) (void)hipGraphExecDestroy(kv.second);
    if (k == 0)
      for (auto& kv : h->g_calln)
        if (kv.second) (void)hipGraphExecDestroy(kv.second);
    if (h->g_call[k]) (void)hipGraphExecDestroy(h->g_call[k]);
  }
  for (int k = 0; k <= kMaxStages; ++k)
    if (h->ev[k]) (void)hipEventDestroy(h->ev[k]);
  if (h->rep_host) (void)hipHostFree(h->rep_host);
  for (void* p : h->allocs) (void)hipFree(p);
  if (h->s) (void)hipStreamDestroy(h->s);
  delete h->comm;
  delete h;
  return GPK_OK;
}

int gpk_num_params(const gpk_handle* h, int64_t* n) {
  if (!h || !n) return fail(GPK_EINVAL, "NULL argument");
  *n = h->L.nparams;
  return GPK_OK;
}

int gpk_set_params(gpk_handle* h, const double* flat, int64_t n) {
  if (!h || !flat) return fail(GPK_EINVAL, "NULL argument");
  if (n != h->L.nparams) return fail(GPK_EINVAL, "parameter count mismatch");
  DevSwitch ds(h->dev);
  HIPCHK(hipMemcpyAsync(h->params, flat, n * sizeof(double), hipMemcpyHostToDevice, h->s));
  TRY(check_launch(launch_sync_u(h->params, h->L, h->Up, h->s), "sync_u"));
  HIPCHK(hipStreamSynchronize(h->s));
  // new parameters: the next batch runs the full graph until their gate value has been seen
  h->fast_mode = h->fast_ok && (h->prob.flags & GPK_FLAG_FAST_FIRST);
  return GPK_OK;
}

int gpk_get_params(gpk_handle* h, double* flat, int64_t n) {
  if (!h || !flat) return fail(GPK_EINVAL, "NULL argument");
  if (n != h->L.nparams) return fail(GPK_EINVAL, "parameter count mismatch");
  DevSwitch ds(h->dev);
  if (h->shard)  // U rows are gathered into Up each step; the flat params hold only this rank's
    TRY(check_launch(launch_params_from_up(h->Up, h->L, h->params, h->s), "params_from_up"));
  HIPCHK(hipMemcpyAsync(flat, h->params, n * sizeof(double), hipMemcpyDeviceToHost, h->s));
  HIPCHK(hipStreamSynchronize(h->s));
  return GPK_OK;
}

int gpk_set_opt_state(gpk_handle* h, int64_t count, const double* mu, const double* nu, int64_t n) {
  if (!h || !mu || !nu) return fail(GPK_EINVAL, "NULL argument");
  if (n != h->L.nparams) return fail(GPK_EINVAL, "parameter count mismatch");
  if (count < 0 || count > 0x7fffffff) return fail(GPK_EINVAL, "bad count");
  DevSwitch ds(h->dev);
  int c = (int)count;
  HIPCHK(hipMemcpyAsync(h->m, mu, n * sizeof(double), hipMemcpyHostToDevice, h->s));
  HIPCHK(hipMemcpyAsync(h->v, nu, n * sizeof(double), hipMemcpyHostToDevice, h->s));
  HIPCHK(hipMemcpyAsync(h->count, &c, sizeof(int), hipMemcpyHostToDevice, h->s));
  HIPCHK(hipStreamSynchronize(h->s));
  return GPK_OK;
}

int gpk_get_opt_state(gpk_handle* h, int64_t* count, double* mu, double* nu, int64_t n) {
  if (!h || !count || !mu || !nu) return fail(GPK_EINVAL, "NULL argument");
  if (n != h->L.nparams) return fail(GPK_EINVAL, "parameter count mismatch");
  DevSwitch ds(h->dev);
  int c = 0;
  HIPCHK(hipMemcpyAsync(mu, h->m, n * sizeof(double), hipMemcpyDeviceToHost, h->s));
  HIPCHK(hipMemcpyAsync(nu, h->v, n * sizeof(double), hipMemcpyDeviceToHost, h->s));
  HIPCHK(hipMemcpyAsync(&c, h->count, sizeof(int), hipMemcpyDeviceToHost, h->s));
  HIPCHK(hipStreamSynchronize(h->s));
  *count = c;
  return GPK_OK;
}

int gpk_loss_grad(gpk_handle* h, double* loss, double* grad_flat) {
  if (!h || !loss) return fail(GPK_EINVAL, "NULL argument");
  DevSwitch ds(h->dev);
  h->pend_losses = nullptr;
  bool fast = h->fast_ok && h->fast_mode, viol = false;
  for (int pass = 0; pass < 2; ++pass) {
    TRY(capture(h, 0, !fast));
    {
      StepBegin b{};
      b.viol = fast ? h->viol : nullptr;
      b.loss_slot = h->loss_slot;
      TRY(check_launch(launch_step_begin(b, h->s), "step_begin"));
    }
    HIPCHK(hipGraphLaunch(fast ? h->g_fast[0] : h->g_exec[0], h->s));
    HIPCHK(hipMemcpyAsync(loss, h->diag, sizeof(double), hipMemcpyDeviceToHost, h->s));
    if (grad_flat)
      HIPCHK(hipMemcpyAsync(grad_flat, h->grad, h->L.nparams * sizeof(double), hipMemcpyDeviceToHost, h->s));
    TRY(finish_batch(h, fast, &viol));
    if (!viol) break;
    ++h->rollbacks;  // nothing to restore: apply = 0 leaves params and Adam state alone
    fast = false;
  }
  return GPK_OK;
}

static int run_steps(gpk_handle* h, int n_steps, double* losses, bool fast, bool reset_slot = true) {
  hipGraphExec_t ge = fast ? h->g_fast[1] : h->g_exec[1];
  const bool multi = !h->shard && n_steps >= STEP_GRAPH_REPS;
  if (multi) TRY(capture(h, 1, !fast, STEP_GRAPH_REPS));
  hipGraphExec_t gm = multi ? h->g_multi[fast ? 0 : 1] : nullptr;
  int done = 0;
  while (done < n_steps) {
    const int nb = std::min(LOSS_CAP, n_steps - done);
    if (reset_slot || done > 0) HIPCHK(hipMemsetAsync(h->loss_slot, 0, sizeof(int), h->s));
    int i = 0;
    const auto& bg = h->g_batch[fast ? 0 : 1];
    while (i < nb) {  // prepared batch graphs: the whole rest, else the largest that fits
      auto it = bg.find(nb - i);
      if (it == bg.end() || !it->second) {
        it = bg.upper_bound(nb - i);
        if (it == bg.begin()) break;
        --it;
        if (!it->second || it->first <= STEP_GRAPH_REPS) break;
      }
      HIPCHK(hipGraphLaunch(it->second, h->s));
      i += it->first;
    }
    if (multi)
      for (; i + STEP_GRAPH_REPS <= nb; i += STEP_GRAPH_REPS) HIPCHK(hipGraphLaunch(gm, h->s));
    for (; i < nb; ++i) HIPCHK(hipGraphLaunch(ge, h->s));
    if (losses && done + nb < n_steps) {
      HIPCHK(hipMemcpyAsync(losses + done, h->losses, nb * sizeof(double), hipMemcpyDeviceToHost, h->s));
    } else if (losses) {  // the last batch's losses come back with finish_batch's report
      h->pend_losses = losses + done;
      h->pend_n = nb;
    }
    done += nb;
  }
  return GPK_OK;
}

// Fast batches run in chunks of FAST_CHUNK steps, each checked at its end: a step that met an
// open refinement gate costs a rerun of its chunk only (not of the whole call -- at C3 the
// gate opens mid-training, and a 300-step call used to run twice).
constexpr int FAST_CHUNK = 64;
constexpr int kBatchMax = FAST_CHUNK;  // largest prepared batch graph

// A whole-call graph (capture_call / capture_calln) ends its report with the ready word
// rep_host[7] (stepk_dev.h report_ready): the host waits for that word instead of the stream, so
// gpk_step returns as soon as the call's losses and status are final -- the last step's dL/dU and
// Adam on U may still run, ordered before anything later enqueued on the handle's stream.  The
// wait polls the stream every few thousand reads, so a faulted or finished-without-report stream
// ends it.
static void arm_report(gpk_handle* h) {
  reinterpret_cast<volatile double*>(h->rep_host)[7] = 0.0;
}

static int wait_report(gpk_handle* h) {
  volatile double* ready = reinterpret_cast<volatile double*>(h->rep_host) + 7;
  for (unsigned it = 1;; ++it) {
    if (*ready != 0.0) break;
    // back-off: tight for the first 2^14 reads (a C4 step's report lands within ~100 us), then
    // a pause per read, then a yield per read past 2^20 (a C5 call waits tens of ms: the host
    // core is left to others instead of spinning flat out)
    if (it > (1u << 20)) sched_yield();
    else if (it > (1u << 14)) __builtin_ia32_pause();
    if ((it & 4095u) == 0) {
      const hipError_t e = hipStreamQuery(h->s);
      if (e == hipErrorNotReady) continue;
      if (e != hipSuccess) return fail(GPK_EHIP, std::string("step graph: ") + hipGetErrorString(e));
      if (*ready != 0.0) break;
      return fail(GPK_EHIP, "internal: the step graph finished without its report");
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return GPK_OK;
}

int gpk_sync(gpk_handle* h) {
  if (!h) return fail(GPK_EINVAL, "NULL handle");
  DevSwitch ds(h->dev);
  HIPCHK(hipStreamSynchronize(h->s));
  return GPK_OK;
}

// gpk_set_wait_limit_chunk: the poll budget applied while gpk_step runs one chunk of a call
// (tests: a failure in a later chunk leaves the earlier chunks applied)
static std::atomic<int> g_chunk_limit_polls{0}, g_chunk_limit_at{-1};
struct ChunkWaitLimit {
  bool on = false;
  ChunkWaitLimit(gpk_handle* h, int chunk) {
    if (g_chunk_limit_polls.load() <= 0 || chunk != g_chunk_limit_at.load()) return;
    // (the previous chunk's tail may still run: the limit must not reach its waits)
    on = hipStreamSynchronize(h->s) == hipSuccess && gpk_set_wait_limit(g_chunk_limit_polls.load()) == GPK_OK;
  }
  ~ChunkWaitLimit() {
    if (on) gpk_set_wait_limit(0);
  }
};

int gpk_set_wait_limit_chunk(int32_t polls, int32_t chunk) {
  if (polls < 0) return fail(GPK_EINVAL, "polls must be >= 0");
  g_chunk_limit_polls.store(polls);
  g_chunk_limit_at.store(polls > 0 ? chunk : -1);
  return GPK_OK;
}

int gpk_step(gpk_handle* h, int32_t n_steps, double* losses) {
  if (!h) return fail(GPK_EINVAL, "NULL handle");
  if (n_steps < 0) return fail(GPK_EINVAL, "n_steps < 0");
  DevSwitch ds(h->dev);
  h->pend_losses = nullptr;  // (a failed earlier call may have left one)
  const size_t np = (size_t)h->L.nparams;
  int done = 0;
  if (n_steps == 1 && !h->shard) {  // one graph launch per call (a rollback takes the path below)
    const bool fast = h->fast_ok && h->fast_mode;
    TRY(capture_call(h, fast));
    arm_report(h);
    HIPCHK(hipGraphLaunch(h->g_call[fast ? 0 : 1], h->s));
    TRY(wait_report(h));
    if (losses) std::memcpy(losses, h->rep_host + 8, sizeof(double));
    bool viol = false;
    TRY(read_report(h, fast, &viol));
    if (!viol) return GPK_OK;
    ++h->rollbacks;  // restore the snapshot the call graph took and rerun with the full graph
    TRY(restore_snapshot(h));
    TRY(capture_call(h, false));
    arm_report(h);
    HIPCHK(hipGraphLaunch(h->g_call[1], h->s));
    TRY(wait_report(h));
    if (losses) std::memcpy(losses, h->rep_host + 8, sizeof(double));
    return read_report(h, false, &viol);
  }
  for (int chunk = 0; done < n_steps; ++chunk) {
    ChunkWaitLimit chunk_limit(h, chunk);  // (tests: gpk_set_wait_limit_chunk)
    // (both graphs run in FAST_CHUNK chunks while the fast graph is available, so the mode is
    // re-decided every 64 steps: a long first call on the full graph used to keep its whole
    // length there, and the training that followed, until the gate bound fell below the entry
    // margin -- round 4's W = 200 line at 8100 it/s)
    const bool fast = h->fast_ok && h->fast_mode;
    const int n = h->fast_ok ? std::min(FAST_CHUNK, n_steps - done) : n_steps - done;
    double* lo = losses ? losses + done : nullptr;
    bool viol = false;
    auto cg = fast && !h->shard ? h->g_calln.find(n) : h->g_calln.end();
    if (cg != h->g_calln.end() && cg->second) {  // a prepared whole-chunk graph
      arm_report(h);
      HIPCHK(hipGraphLaunch(cg->second, h->s));
      TRY(wait_report(h));
      h->pend_losses = lo;
      h->pend_n = n;
      TRY(read_report(h, true, &viol));
    } else {
      TRY(capture(h, 1, !fast));
      {  // the snapshot of everything a fast batch carries forward (Up is rebuilt from params),
         // the violation flag and the loss slot: one launch
        StepBegin b{};
        b.snap = h->snap; b.params = h->params; b.m = h->m; b.v = h->v; b.np = np;
        b.snap_count = h->snap_count; b.count = h->count;
        if (fast) b.viol = h->viol;
        b.loss_slot = h->loss_slot;
        TRY(check_launch(launch_step_begin(b, h->s), "step_begin"));
      }
      TRY(run_steps(h, n, lo, fast, false));
      TRY(finish_batch(h, fast, &viol));
    }
    if (viol) {  // a step of the chunk needed refinement: roll back and rerun with the full graph
      ++h->rollbacks;
      TRY(restore_snapshot(h));
      TRY(capture(h, 1, true));
      TRY(run_steps(h, n, lo, false));
      TRY(finish_batch(h, false, &viol));
    }
    done += n;
  }
  return GPK_OK;
}

int gpk_prepare(gpk_handle* h, int32_t n_steps) {
  if (!h) return fail(GPK_EINVAL, "NULL handle");
  if (n_steps < 0) return fail(GPK_EINVAL, "n_steps < 0");
  if (h->shard && !h->comm->capturable()) return GPK_OK;  // in-process groups run eagerly
  DevSwitch ds(h->dev);
  for (int refine = 0; refine < 2; ++refine) {
    if (!refine && !h->fast_ok) continue;
    TRY(capture(h, 1, refine != 0));
    if (!h->shard) TRY(capture_call(h, refine == 0));
    if (!h->shard && n_steps >= STEP_GRAPH_REPS) TRY(capture(h, 1, refine != 0, STEP_GRAPH_REPS));
    // the chunks of a call of n_steps: FAST_CHUNK-step chunks + the remainder whenever the fast
    // graph exists (fast_ok), on either graph -- each chunk is a batch of its own (snapshot,
    // report, undo on failure); without a fast graph the whole call is one batch, run as
    // kBatchMax-step graphs + the remainder.  One graph each
    if (!h->shard && n_steps > STEP_GRAPH_REPS) {
      const int full = std::min(n_steps, kBatchMax), rest = n_steps % kBatchMax;
      TRY(capture(h, 1, refine != 0, full, true));
      if (rest > STEP_GRAPH_REPS && rest != full) TRY(capture(h, 1, refine != 0, rest, true));
    }
    // fast chunks as whole-call graphs (begin + steps + report)
    if (!refine && !h->shard && n_steps > 1) {
      const int full = std::min(n_steps, FAST_CHUNK), rest = n_steps % FAST_CHUNK;
      TRY(capture_calln(h, full));
      if (rest > 1 && rest != full) TRY(capture_calln(h, rest));
    }
  }
  HIPCHK(hipStreamSynchronize(h->s));
  return GPK_OK;
}

int gpk_trace_reset(void) {
  trace_reset_assemble();
  trace_reset_spdinv();
  trace_reset_pgrad();
  trace_reset_gemm();
  trace_reset_spdbig();
  return GPK_OK;
}

int gpk_trace_read(uint64_t* lo, uint64_t* hi, int32_t n) {
  if (!lo || !hi || n < TRACE_SLOTS) return fail(GPK_EINVAL, "need TRACE_SLOTS (256) slots");
  uint64_t l[5][TRACE_SLOTS], h[5][TRACE_SLOTS];
  trace_fetch_assemble(l[0], h[0]);
  trace_fetch_spdinv(l[1], h[1]);
  trace_fetch_pgrad(l[2], h[2]);
  trace_fetch_gemm(l[3], h[3]);
  trace_fetch_spdbig(l[4], h[4]);
  for (int i = 0; i < TRACE_SLOTS; ++i) {
    lo[i] = l[0][i];
    hi[i] = h[0][i];
    for (int u = 1; u < 5; ++u) {
      lo[i] = std::min(lo[i], l[u][i]);
      hi[i] = std::max(hi[i], h[u][i]);
    }
  }
#ifdef GPK_TRACE
  return GPK_OK;
#else
  return fail(GPK_EINVAL, "built without GPK_TRACE (make trace -> libgpk_trace.so)");
#endif
}

int gpk_distance_classes(const double* x, int32_t n, int32_t* ncls, int32_t* vmax) {
  if (!x || n <= 0 || !ncls) return fail(GPK_EINVAL, "bad argument");
  std::vector<double> dist;
  std::vector<int> cid, cbase;
  int vm = 0;
  const bool ok = build_classes(x, n, pad_up(n), dist, cid, cbase, vm);
  *ncls = ok ? (int32_t)dist.size() : 0;
  if (vmax) *vmax = ok ? vm : CLS_VMAX + 1;
  return GPK_OK;
}

int gpk_class_count(const gpk_handle* h, int32_t axis, int32_t* ncls) {
  if (!h || !ncls || axis < 0 || axis >= h->L.naxes) return fail(GPK_EINVAL, "bad argument");
  *ncls = h->cls[axis].ncls;
  return GPK_OK;
}

int gpk_class_sum_path(const gpk_handle* h, int32_t* epilogue) {
  if (!h || !epilogue) return fail(GPK_EINVAL, "bad argument");
  *epilogue = h->cp_on ? 1 : 0;
  return GPK_OK;
}

int gpk_class_pipe(const gpk_handle* h, int32_t* on) {
  if (!h || !on) return fail(GPK_EINVAL, "bad argument");
  *on = cls_pipe_ok(h) ? 1 : 0;
  return GPK_OK;
}

int gpk_set_spd_big_workgroups(int32_t workgroups) {
  if (workgroups < 0) return fail(GPK_EINVAL, "workgroups must be >= 0");
  spd_big_set_workgroups(workgroups);
  return GPK_OK;
}

int gpk_set_chain_capacity(int32_t workgroups) {
  g_chain_cap.store(workgroups > 0 ? workgroups : 0);
  return GPK_OK;
}

int gpk_set_wait_limit(int32_t polls) {
  if (polls < 0) return fail(GPK_EINVAL, "polls must be >= 0");
  const unsigned v = polls > 0 ? (unsigned)polls : SPIN_CAP;
  if (wait_limit_spdinv(v) != hipSuccess || wait_limit_spdbig(v) != hipSuccess ||
      wait_limit_assemble(v) != hipSuccess || wait_limit_pgrad(v) != hipSuccess)
    return fail(GPK_EHIP, "set the wait limit");
  return GPK_OK;
}

int gpk_inverse_path(const gpk_handle* h, int32_t* path) {
  if (!h || !path) return fail(GPK_EINVAL, "NULL argument");
  *path = h->bigspd ? (h->bigwide ? GPK_INV_BIG_WIDE : GPK_INV_BIG)
          : h->chain_multi ? GPK_INV_CHAIN_MULTI
          : h->chain_aug ? GPK_INV_CHAIN_AUG : h->chain ? GPK_INV_CHAIN : GPK_INV_SWEEP;
  return GPK_OK;
}

int gpk_graph_mode(const gpk_handle* h, int32_t* fast, int64_t* rollbacks) {
  if (!h) return fail(GPK_EINVAL, "NULL handle");
  if (fast) *fast = (h->fast_ok && h->fast_mode) ? 1 : 0;
  if (rollbacks) *rollbacks = h->rollbacks;
  return GPK_OK;
}

int gpk_criterion(gpk_handle* h, double* out) {
  if (!h || !out) return fail(GPK_EINVAL, "NULL argument");
  double loss;
  TRY(gpk_loss_grad(h, &loss, nullptr));
  DevSwitch ds(h->dev);
  double diag[8];
  HIPCHK(hipMemcpy(diag, h->diag, sizeof(diag), hipMemcpyDeviceToHost));
  const Layout& L = h->L;
  const double Nb = (double)h->prob.nb;
  const double Nc = L.dim == 2 ? (double)L.n1 * L.n2 : (double)L.n1;
  *out = diag[5] / Nb + diag[4] / Nc;  // boundary_gap/Nb + eq_gap/Nc
  return GPK_OK;
}

int gpk_predict(gpk_handle* h, const double* xte1, int32_t m1, const double* xte2, int32_t m2,
                double* out) {
  if (!h || !xte1 || !out || m1 <= 0) return fail(GPK_EINVAL, "bad argument");
  const Layout& L = h->L;
  if (L.dim == 2 && (!xte2 || m2 <= 0)) return fail(GPK_EINVAL, "2D predict needs xte2");
  DevSwitch ds(h->dev);
  // K^{-1} at the current params
  bool prof = h->profiling;
  h->profiling = false;
  int rc = enqueue_assemble_inverse(h, 0);
  h->profiling = prof;
  TRY(rc);
  const int M1p = pad_up(m1), P1 = L.p1;
  std::vector<void*> tmp;
  auto dalloc = [&](double** p, size_t n) -> int {
    HIPCHK(hipMalloc((void**)p, std::max<size_t>(n, 2) * sizeof(double)));
    tmp.push_back(*p);
    HIPCHK(hipMemsetAsync(*p, 0, std::max<size_t>(n, 2) * sizeof(double), h->s));
    return GPK_OK;
  };
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(h->s);
    for (void* p : tmp) (void)hipFree(p);
  };
  double *dx1, *Kmn1, *res;
  int r = GPK_OK;
  if ((r = dalloc(&dx1, m1)) || (r = dalloc(&Kmn1, (size_t)M1p * P1))) { cleanup(); return r; }
  (void)hipMemcpyAsync(dx1, xte1, m1 * sizeof(double), hipMemcpyHostToDevice, h->s);
  // Kmn = kappa(xte_i, x_j) (no jitter), zero-padded to M1p x P1   (model_GP_solver_2d.py:198-202)
  r = check_launch(launch_cross(h->prob.kind, L.q, dx1, m1, h->x1, L.n1, P1, h->kc, 0.0, 0, Kmn1, nullptr, h->s), "cross");
  if (r) { cleanup(); return r; }
  if (L.dim == 1) {
    double* alpha;
    if ((r = dalloc(&alpha, P1)) || (r = dalloc(&res, M1p))) { cleanup(); return r; }
    double* rv;
    if ((r = dalloc(&rv, P1))) { cleanup(); return r; }
    auto gv = [&](const double* A, const double* x, double* y, int rows, double al, const double* C0,
                  double be) {
      GemvDesc g{};
      g.A = A; g.lda = P1; g.x = x; g.y = y; g.p = P1; g.rows = rows; g.alpha = al;
      g.C0 = C0; g.beta = be; g.epi = EPI_STORE;
      gemv_operand(h, g);
      (void)launch_gemv(g, h->s);
    };
    // alpha = K^{-1} u with one refinement step (matches solve() accuracy; 1d.py:176-179)
    gv(h->Kinv[0], h->Up, alpha, P1, 1.0, nullptr, 0.0);
    gv(h->Kc[0], alpha, rv, P1, -1.0, h->Up, 1.0);
    gv(h->Kinv[0], rv, alpha, P1, 1.0, alpha, 1.0);
    gv(Kmn1, alpha, res, m1, 1.0, nullptr, 0.0);  // preds = Kmn K^{-1} u
    (void)hipMemcpyAsync(out, res, m1 * sizeof(double), hipMemcpyDeviceToHost, h->s);
  } else {
    // U_pred = Kmn2 (K2^{-1} (Kmn1 K1^{-1} U)^T), associated exactly as the reference does
    // (model_GP_solver_2d.py:185-220: M1 = Kmn K1inv_U, M2 = solve(K2, M1^T), Kmn2 M2): every
    // intermediate stays O(|U_pred|) after its Kmn product.  (Forming S = K1^{-1} U K2^{-1}
    // first, as rounds 1-2 did, builds entries ~ |U| / jitter^2 whose cancellation in
    // Kmn1 S Kmn2^T cost up to 0.37 relative L2 at C5 with a random field.)
    const int M2p = pad_up(m2), P2 = L.p2;
    double *dx2, *Kmn2, *Aw, *Rw, *Mw, *Nw, *Rm;
    if ((r = dalloc(&dx2, m2)) || (r = dalloc(&Kmn2, (size_t)M2p * P2)) || (r = dalloc(&Aw, (size_t)P1 * P2)) ||
        (r = dalloc(&Rw, (size_t)P1 * P2)) || (r = dalloc(&Mw, (size_t)M1p * P2)) ||
        (r = dalloc(&Nw, (size_t)M1p * P2)) || (r = dalloc(&Rm, (size_t)M1p * P2)) ||
        (r = dalloc(&res, (size_t)M1p * M2p))) { cleanup(); return r; }
    (void)hipMemcpyAsync(dx2, xte2, m2 * sizeof(double), hipMemcpyHostToDevice, h->s);
    (void)launch_cross(h->prob.kind, L.q, dx2, m2, h->x2, L.n2, P2, h->kc + 1, 0.0, 0, Kmn2, nullptr, h->s);
    GemmDesc d[8] = {};
    auto mk = [](GemmDesc& g, const double* A, int lda, int ta, const double* B, int ldb, int tb,
                 double* C, int ldc, int M, int N, int K) {
      g.A = A; g.lda = lda; g.ta = ta; g.B = B; g.ldb = ldb; g.tb = tb; g.C = C; g.ldc = ldc;
      g.M = M; g.N = N; g.K = K; g.alpha = 1.0; g.epi = EPI_STORE;
    };
    // A = K1^{-1} U and N = M1 K2^{-1}, each with one refinement step (solve() accuracy)
    mk(d[0], h->Kinv[0], P1, 0, h->Up, P2, 0, Aw, P2, P1, P2, P1);
    mk(d[1], h->Kc[0], P1, 0, Aw, P2, 0, Rw, P2, P1, P2, P1);          // Rw = U - K1 A
    d[1].alpha = -1.0; d[1].beta = 1.0; d[1].C0 = h->Up; d[1].ldc0 = P2;
    mk(d[2], h->Kinv[0], P1, 0, Rw, P2, 0, Aw, P2, P1, P2, P1);        // A += K1^{-1} Rw
    d[2].beta = 1.0; d[2].C0 = Aw; d[2].ldc0 = P2;
    mk(d[3], Kmn1, P1, 0, Aw, P2, 0, Mw, P2, M1p, P2, P1);             // M1 = Kmn1 A
    mk(d[4], Mw, P2, 0, h->Kinv[1], P2, 0, Nw, P2, M1p, P2, P2);       // N = M1 K2^{-1} = M2^T
    mk(d[5], Nw, P2, 0, h->Kc[1], P2, 0, Rm, P2, M1p, P2, P2);         // Rm = M1 - N K2
    d[5].alpha = -1.0; d[5].beta = 1.0; d[5].C0 = Mw; d[5].ldc0 = P2;
    mk(d[6], Rm, P2, 0, h->Kinv[1], P2, 0, Nw, P2, M1p, P2, P2);       // N += Rm K2^{-1}
    d[6].beta = 1.0; d[6].C0 = Nw; d[6].ldc0 = P2;
    mk(d[7], Nw, P2, 0, Kmn2, P2, 1, res, M2p, M1p, M2p, P2);       // U_pred = N Kmn2^T
    const int force_big = gemm_force(h->prob.flags);
    for (int k = 0; k < 8; ++k)
      (void)launch_gemm_auto(d + k, 1, h->sc, h->s, gemm_variant(d + k, 1, force_big));
    for (int i = 0; i < m1; ++i)
      (void)hipMemcpyAsync(out + (size_t)i * m2, res + (size_t)i * M2p, m2 * sizeof(double),
                           hipMemcpyDeviceToHost, h->s);
  }
  hipError_t e = hipStreamSynchronize(h->s);
  cleanup();
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("predict: ") + hipGetErrorString(e));
  return read_status(h);
}

int gpk_profile_stages(gpk_handle* h, int32_t iters, double* out_us, int32_t cap, int32_t* n) {
  if (!h || !out_us || !n || iters <= 0) return fail(GPK_EINVAL, "bad argument");
  DevSwitch ds(h->dev);
  std::vector<double> acc(kMaxStages, 0.0);
  // run on a copy of the state: save params + opt state, restore afterwards
  const int64_t np = h->L.nparams;
  std::vector<double> p(np), mu(np), nu(np);
  int64_t cnt = 0;
  TRY(gpk_get_params(h, p.data(), np));
  TRY(gpk_get_opt_state(h, &cnt, mu.data(), nu.data(), np));
  h->profiling = true;
  for (int it = 0; it < iters; ++it) {
    HIPCHK(hipMemsetAsync(h->loss_slot, 0, sizeof(int), h->s));
    int rc = enqueue_step(h, 1);
    if (rc) { h->profiling = false; return rc; }
    HIPCHK(hipStreamSynchronize(h->s));
    for (int k = 0; k < h->nstage; ++k) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1]));
      acc[k] += ms * 1000.0;
    }
  }
  h->profiling = false;
  TRY(gpk_set_params(h, p.data(), np));
  TRY(gpk_set_opt_state(h, cnt, mu.data(), nu.data(), np));
  const int ns = std::min<int>(h->nstage, cap);
  for (int k = 0; k < ns; ++k) out_us[k] = acc[k] / iters;
  *n = ns;
  return read_status(h);
}

const char* gpk_stage_name(const gpk_handle* h, int32_t stage) {
  if (!h || stage < 0) return "?";
  if (stage >= h->nstage || stage >= kMaxStages || !h->sname[stage]) return "?";
  return h->sname[stage];
}

int gpk_time_spd_inverse(gpk_handle* h, int32_t iters, double* avg_us) {
  if (!h || !avg_us || iters <= 0) return fail(GPK_EINVAL, "bad argument");
  DevSwitch ds(h->dev);
  const Layout& L = h->L;
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  double total = 0.0;
  for (int it = 0; it < iters; ++it) {
    // re-assemble K (the inverse consumes it), time only the inverse
    AssembleArgs aa[2] = {};
    const int deriv = (h->prob.eq == GPK_ADVECTION) ? 1 : 2;
    for (int a = 0; a < L.naxes; ++a) {
      aa[a].x = a == 0 ? h->x1 : h->x2; aa[a].n = a == 0 ? L.n1 : L.n2; aa[a].p = a == 0 ? L.p1 : L.p2;
      aa[a].kc = h->kc + a; aa[a].jitter = h->prob.jitter; aa[a].K = h->K[a]; aa[a].D = h->D[a];
      aa[a].deriv = deriv; aa[a].Kc = nullptr;
    }
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s), "assemble"));
    SpdArgs sa[2];
    fill_spd(h, sa);
    double* fin[2];
    HIPCHK(hipEventRecord(e0, h->s));
    TRY(check_launch(launch_inverse(h, sa, fin, false), "spd_inverse"));
    HIPCHK(hipEventRecord(e1, h->s));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    total += ms * 1000.0;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *avg_us = total / iters;
  return read_status(h);
}

int gpk_kernel_pairs(int32_t kind, int32_t deriv, const double* x1, const double* x2, int64_t n,
                     const double* logw, const double* logls, const double* freq, int32_t q,
                     double* out) {
  if (kind < 0 || kind > 3) return fail(GPK_EINVAL, "Invalid Kernel");
  if (deriv < 0 || deriv > 2) return fail(GPK_EINVAL, "deriv must be 0, 1 or 2");
  if (n <= 0 || q <= 0 || q > QMAX) return fail(GPK_EINVAL, "bad sizes (0 < q <= 64)");
  if (!x1 || !x2 || !logw || !logls || !freq || !out) return fail(GPK_EINVAL, "NULL pointer argument");
  int dev = 0;
  (void)hipGetDevice(&dev);
  TRY(check_device(dev));
  AxisConst hk;
  host_axis_const(logw, logls, freq, q, &hk);
  double *d1 = nullptr, *d2 = nullptr, *dout = nullptr;
  AxisConst* dkc = nullptr;
  auto cleanup = [&]() {
    if (d1) (void)hipFree(d1);
    if (d2) (void)hipFree(d2);
    if (dout) (void)hipFree(dout);
    if (dkc) (void)hipFree(dkc);
  };
  const size_t bytes = (size_t)n * sizeof(double);
  if (hipMalloc(&d1, bytes) != hipSuccess || hipMalloc(&d2, bytes) != hipSuccess ||
      hipMalloc(&dout, bytes) != hipSuccess || hipMalloc(&dkc, sizeof(AxisConst)) != hipSuccess) {
    cleanup();
    return fail(GPK_ENOMEM, "hipMalloc failed");
  }
  hipError_t e = hipMemcpy(d1, x1, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d2, x2, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dkc, &hk, sizeof(AxisConst), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_pairs(kind, q, d1, d2, n, dkc, deriv, dout, 0);
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("kernel_pairs: ") + hipGetErrorString(e));
  return GPK_OK;
}

int gpk_forward_field(gpk_handle* h, int32_t what, double* out, int64_t n) {
  if (!h || !out) return fail(GPK_EINVAL, "NULL argument");
  const Layout& L = h->L;
  const int64_t n1 = L.n1, n2 = L.n2;
  int64_t want;
  if (L.dim == 2) {
    const int64_t sizes[26] = {n1 * n1, n2 * n2, n1 * n2, n2 * n1, n1 * n2, n1 * n2,
                               n1 * n1, n1 * n1, n2 * n2, n2 * n2, n1 * n1, n2 * n2,
                               n1 * n1, n2 * n2, n1 * n2, n1 * n2, n1 * n2, n1 * n2,
                               n1 * n1, n2 * n2, n1 * n1, n2 * n2, n1 * n1, n2 * n2, n1 * n1, n2 * n2};
    if (what < 0 || what > 25) return fail(GPK_EINVAL, "what must be 0..25 (2D)");
    if (what >= 22 && h->cls[0].ncls <= 0) return fail(GPK_EINVAL, "this handle does not use distance classes");
    if ((what == 18 || what == 19) && !h->Kc[what - 18])
      return fail(GPK_EINVAL, "this handle keeps no copy of K");
    if ((what == 12 || what == 13) && !h->PD[what - 12])
      return fail(GPK_EINVAL, "K^{-1} D^T is formed on the augmented chain path only");
    want = sizes[what];
  } else {
    if (what != 0 && what != 2 && what != 4 && what != 6 && what != 7)
      return fail(GPK_EINVAL, "what must be 0, 2, 4, 6 or 7 (1D)");
    want = (what == 0 || what >= 6) ? n1 * n1 : n1;
  }
  if (n != want) return fail(GPK_EINVAL, "output size mismatch");
  DevSwitch ds(h->dev);
  std::vector<double> host;
  double* tmp = nullptr;
  auto cleanup = [&]() {
    if (tmp) (void)hipFree(tmp);
  };
  if (what <= 1) {  // K factor: assemble at the current params (kappa + jitter I)
    const int a = what;
    const int na = a == 0 ? L.n1 : L.n2;
    TRY(check_launch(launch_prep2(h->params, L, h->kc, h->sc, h->count, 0, h->hyper.b1, h->hyper.b2, h->s), "prep"));
    HIPCHK(hipMalloc(&tmp, (size_t)na * na * sizeof(double)));
    const double* xa = a == 0 ? h->x1 : h->x2;
    int rc = check_launch(launch_cross(h->prob.kind, L.q, xa, na, xa, na, na, h->kc + a, h->prob.jitter,
                                       0, tmp, nullptr, h->s), "cross");
    if (rc == GPK_OK && hipMemcpyAsync(out, tmp, n * sizeof(double), hipMemcpyDeviceToHost, h->s) != hipSuccess)
      rc = fail(GPK_EHIP, "copy");
    if (rc == GPK_OK && hipStreamSynchronize(h->s) != hipSuccess) rc = fail(GPK_EHIP, "sync");
    cleanup();
    return rc;
  }
  double loss = 0.0;
  TRY(gpk_loss_grad(h, &loss, nullptr));  // device buffers now hold the forward quantities
  if (L.dim == 1 && what >= 6) {  // the step's K (6) and D (7), as its last step assembled them
    const int P = L.p1, na = L.n1;
    const ClassArgs& C = h->cls[0];
    if (C.ncls > 0) {  // class ids + class values (K and D are never materialised on this path)
      std::vector<int> cid((size_t)P * P);
      std::vector<double> cv(C.ncls);
      HIPCHK(hipMemcpy(cid.data(), C.cid, cid.size() * sizeof(int), hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(cv.data(), what == 6 ? C.kval : C.dval, cv.size() * sizeof(double), hipMemcpyDeviceToHost));
      for (int i = 0; i < na; ++i)
        for (int j = 0; j < na; ++j) {
          double v = cv[cid[(size_t)i * P + j]];
          if (what == 6 && i == j) v += h->prob.jitter;  // (the gather adds it per element)
          out[(size_t)i * na + j] = v;
        }
      return GPK_OK;
    }
    const double* m = what == 6 ? h->Kc[0] : h->D[0];
    if (!m) return fail(GPK_EINVAL, "this handle keeps no copy of K / D");
    host.resize((size_t)P * P);
    HIPCHK(hipMemcpy(host.data(), m, host.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int i = 0; i < na; ++i)
      for (int j = 0; j < na; ++j) out[(size_t)i * na + j] = host[(size_t)i * P + j];
    return GPK_OK;
  }
  if (L.dim == 1) {
    const int P = L.p1;
    const double* src = h->alpha;
    if (what == 4) {  // u_xx = D alpha
      HIPCHK(hipMalloc(&tmp, P * sizeof(double)));
      GemvDesc g{};
      g.A = h->D[0]; g.lda = P; g.x = h->alpha; g.y = tmp; g.p = P; g.rows = P; g.alpha = 1.0;
      g.epi = EPI_STORE;
      gemv_operand(h, g);
      int rc = check_launch(launch_gemv(g, h->s), "gemv");
      if (rc) { cleanup(); return rc; }
      src = tmp;
    }
    hipError_t e = hipMemcpyAsync(out, src, n * sizeof(double), hipMemcpyDeviceToHost, h->s);
    if (e == hipSuccess) e = hipStreamSynchronize(h->s);
    cleanup();
    if (e != hipSuccess) return fail(GPK_EHIP, hipGetErrorString(e));
    return GPK_OK;
  }
  const int P1 = L.p1, P2 = L.p2;
  if (what >= 22) {  // K (22, 23) / D (24, 25) expanded on the host from the class table (cid + values)
    const int a = (what == 22 || what == 24) ? 0 : 1;
    const ClassArgs& C = h->cls[a];
    const int P = a == 0 ? P1 : P2, na = a == 0 ? L.n1 : L.n2;
    std::vector<int> cid((size_t)P * P);
    std::vector<double> cv(C.ncls), x(na);
    HIPCHK(hipMemcpy(cid.data(), C.cid, cid.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cv.data(), what <= 23 ? C.kval : C.dval, cv.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(x.data(), a == 0 ? h->x1 : h->x2, na * sizeof(double), hipMemcpyDeviceToHost));
    const bool sgn = what >= 24 && h->prob.eq == GPK_ADVECTION;  // D_x1: s_ij (JAX abs'(0) = +1)
    for (int i = 0; i < na; ++i)
      for (int j = 0; j < na; ++j) {
        double v = cv[cid[(size_t)i * P + j]];
        if (what <= 23 && i == j) v += h->prob.jitter;
        if (sgn && !(x[i] - x[j] >= 0.0)) v = -v;
        out[(size_t)i * na + j] = v;
      }
    return GPK_OK;
  }
  if ((what >= 6 && what <= 13) || what >= 18) {  // work matrices, K^{-1}, K^{-1} D^T, Kc, D (P x P)
    const int a = (what == 6 || what == 7 || what == 10 || what == 12 || what == 18 || what == 20) ? 0 : 1;
    const int P = a == 0 ? P1 : P2, na = a == 0 ? L.n1 : L.n2;
    const double* m = what >= 20 ? h->D[a] : what >= 18 ? h->Kc[a] : what >= 12 ? h->PD[a]
                    : what >= 10 ? h->Kinv[a] : (what == 6 || what == 8) ? h->GK[a] : h->GD[a];
    host.resize((size_t)P * P);
    hipError_t e = hipMemcpyAsync(host.data(), m, host.size() * sizeof(double), hipMemcpyDeviceToHost, h->s);
    if (e == hipSuccess) e = hipStreamSynchronize(h->s);
    if (e != hipSuccess) return fail(GPK_EHIP, hipGetErrorString(e));
    for (int i = 0; i < na; ++i)
      for (int j = 0; j < na; ++j) out[(size_t)i * na + j] = host[(size_t)i * P + j];
    return GPK_OK;
  }
  if (what >= 14) {  // grid work matrices R, X1, X2, S (P1 x P2)
    const double* m = what == 14 ? h->R : what == 15 ? h->X1 : what == 16 ? h->X2 : h->S;
    host.resize((size_t)P1 * P2);
    hipError_t e = hipMemcpyAsync(host.data(), m, host.size() * sizeof(double), hipMemcpyDeviceToHost, h->s);
    if (e == hipSuccess) e = hipStreamSynchronize(h->s);
    if (e != hipSuccess) return fail(GPK_EHIP, hipGetErrorString(e));
    for (int64_t i = 0; i < n1; ++i)
      for (int64_t j = 0; j < n2; ++j) out[i * n2 + j] = host[(size_t)i * P2 + j];
    return GPK_OK;
  }
  const double* src = (what == 3) ? h->Bt : h->A;
  if (what >= 4) {  // U_xx = D1 A  /  U_yy = Bt D2^T
    HIPCHK(hipMalloc(&tmp, (size_t)P1 * P2 * sizeof(double)));
    GemmDesc g{};
    if (what == 4) {
      g.A = h->D[0]; g.lda = P1; g.B = h->A; g.ldb = P2; g.K = P1;
    } else {
      g.A = h->Bt; g.lda = P2; g.B = h->D[1]; g.ldb = P2; g.tb = 1; g.K = P2;
    }
    g.C = tmp; g.ldc = P2; g.M = P1; g.N = P2; g.alpha = 1.0; g.epi = EPI_STORE;
    hipError_t e = launch_gemm_auto(&g, 1, h->sc, h->s,
                                    gemm_variant(&g, 1, gemm_force(h->prob.flags)));
    if (e != hipSuccess) { cleanup(); return fail(GPK_EHIP, hipGetErrorString(e)); }
    src = tmp;
  }
  host.resize((size_t)P1 * P2);
  hipError_t e = hipMemcpyAsync(host.data(), src, host.size() * sizeof(double), hipMemcpyDeviceToHost, h->s);
  if (e == hipSuccess) e = hipStreamSynchronize(h->s);
  cleanup();
  if (e != hipSuccess) return fail(GPK_EHIP, hipGetErrorString(e));
  for (int64_t i = 0; i < n1; ++i)
    for (int64_t j = 0; j < n2; ++j) {
      const double v = host[(size_t)i * P2 + j];
      if (what == 3)
        out[j * n1 + i] = v;  // K2inv_Ut = (U K2^{-1})^T
      else
        out[i * n2 + j] = v;
    }
  return GPK_OK;
}

int gpk_bench_kernel(gpk_handle* h, const char* name, int32_t iters, double* avg_us,
                     double* alg_flops, double* alg_bytes) {
  if (!h || !name || !avg_us || !alg_flops || !alg_bytes || iters <= 0)
    return fail(GPK_EINVAL, "bad argument");
  const std::string nm(name);
  const Layout& L = h->L;
  // one full step (no update) so every kernel's inputs are valid
  double loss = 0.0;
  TRY(gpk_loss_grad(h, &loss, nullptr));
  DevSwitch ds(h->dev);
  const int deriv = (h->prob.eq == GPK_ADVECTION) ? 1 : 2;
  AssembleArgs aa[2] = {};
  SpdArgs sa[2];
  for (int a = 0; a < L.naxes; ++a) {
    aa[a].x = a == 0 ? h->x1 : h->x2; aa[a].n = a == 0 ? L.n1 : L.n2; aa[a].p = a == 0 ? L.p1 : L.p2;
    aa[a].kc = h->kc + a; aa[a].jitter = h->prob.jitter; aa[a].K = h->K[a]; aa[a].D = h->D[a];
    aa[a].deriv = deriv; aa[a].Kc = nullptr;
  }
  fill_spd(h, sa);
  std::function<hipError_t()> launch;
  double flops = 0.0, bytes = 0.0;
  const double n1 = L.n1, n2 = L.dim == 2 ? L.n2 : 0.0;
  if (nm == "spd_chain") {
    // the step's persistent inverse launch as the step runs it (gather mode after the class
    // values; idempotent: it rebuilds K from the classes each time)
    if (!h->chain) return fail(GPK_EINVAL, "spd_chain: this handle does not use the chain inverse");
    const bool gather = h->cls[0].ncls > 0;
    for (int a = 0; a < L.naxes; ++a) aa[a].cls = h->cls[a];
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s, gather),
                     "assemble"));
    launch = [&, gather]() {
      double* fin[2];
      return launch_chain(h, gather, fin);
    };
    // potrf + potri = n^3 per factor; each augmented column a triangular solve pair, 2 n^2
    // bytes: K^{-1}, Kc, D written (24 n^2), augmented outputs written (8 n m), U read
    for (int a = 0; a < L.naxes; ++a) {
      const double n = a == 0 ? n1 : n2, m = h->chain_aug ? n1 + n2 : 0.0;
      flops += n * n * n + 2.0 * n * n * m;
      bytes += 24.0 * n * n + 8.0 * n * m + (h->chain_aug ? 8.0 * n1 * n2 : 0.0);
    }
  } else if (nm == "sweep" && h->bigspd) {
    // large path: time the update launch of sweep 0 (in place, so every timed launch gets a
    // freshly assembled K, pivot 0 and panel 0 first; only the update is between the events)
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    double tot = 0.0;
    for (int it = 0; it < iters; ++it) {
      TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s), "assemble"));
      TRY(check_launch(launch_spd_big_stage(sa, L.naxes, -1, h->s), "pivot_init"));
      TRY(check_launch(launch_spd_big_stage(sa, L.naxes, 0, h->s), "panel"));
      HIPCHK(hipEventRecord(e0, h->s));
      TRY(check_launch(launch_spd_big_stage(sa, L.naxes, 1, h->s), "update"));
      HIPCHK(hipEventRecord(e1, h->s));
      HIPCHK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms * 1000.0;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    // the MFMA work launch 0 schedules (its tile lists: under the two-sweep schedule launch 0
    // updates only its own parity class + the eager row / column, all at K = 128), + the next
    // pivot and panel; HBM: read + write the lower triangle
    flops = spd_big_update_flops(sa, L.naxes, 0, true);
    for (int a = 0; a < L.naxes; ++a) {
      const double n = a == 0 ? n1 : n2;
      bytes += 8.0 * n * n;
    }
    *avg_us = tot / iters;
    *alg_flops = flops;
    *alg_bytes = bytes;
    return read_status(h);
  } else if (nm == "spd_tiles" && h->bigspd) {
    // the update launch's tile work alone (no pivot workgroup), sweep 0; idempotent enough for
    // timing (each launch re-reads X and Z; values drift but stay finite over a few launches)
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s), "assemble"));
    TRY(check_launch(launch_spd_big_stage(sa, L.naxes, -1, h->s), "pivot_init"));
    TRY(check_launch(launch_spd_big_stage(sa, L.naxes, 0, h->s), "panel"));
    launch = [&]() { return launch_spd_big_tiles(sa, L.naxes, 0, h->s); };
    // the tile products launch 0's lists schedule (no pivot workgroup) -- the work actually done
    flops = spd_big_update_flops(sa, L.naxes, 0, false);
    for (int a = 0; a < L.naxes; ++a) {
      const double n = a == 0 ? n1 : n2;
      bytes += 8.0 * n * n;
    }
  } else if (nm == "spd_updates" && h->bigspd) {
    // every update launch of one inverse (sweeps 0 .. last, each with its fused next pivot and
    // panel; the final mirror left out), between two events after pivot 0 and panel 0: the
    // average update launch as the step runs it, even and odd launches of the two-sweep schedule
    // alike, credited with the work their tile lists schedule (spd_big_update_flops)
    int nsw = 0;
    for (int a = 0; a < L.naxes; ++a) nsw = std::max(nsw, spd_big_sweeps(a == 0 ? L.p1 : L.p2, h->bigwide));
    for (int k = 0; k < nsw; ++k) flops += spd_big_update_flops(sa, L.naxes, k, true);
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    double tot = 0.0;
    for (int it = 0; it < iters; ++it) {
      TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s), "assemble"));
      TRY(check_launch(launch_spd_big_stage(sa, L.naxes, -1, h->s), "pivot_init"));
      TRY(check_launch(launch_spd_big_stage(sa, L.naxes, 0, h->s), "panel"));
      HIPCHK(hipEventRecord(e0, h->s));
      for (int k = 0; k < nsw; ++k)
        TRY(check_launch(launch_spd_big_stage(sa, L.naxes, 2 * k + 1, h->s, false), "update"));
      HIPCHK(hipEventRecord(e1, h->s));
      HIPCHK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms * 1000.0;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (int a = 0; a < L.naxes; ++a) {  // read + write the lower triangle per sweep
      const double n = a == 0 ? n1 : n2;
      bytes += 8.0 * n * n * spd_big_sweeps(a == 0 ? L.p1 : L.p2, h->bigwide);
    }
    *avg_us = tot / iters / nsw;  // per update launch
    *alg_flops = flops / nsw;
    *alg_bytes = bytes / nsw;
    return read_status(h);
  } else if ((nm == "spd_pivot" || nm == "spd_panel") && h->bigspd) {
    // large path pieces (idempotent): the 64-pivot factorisation of block 0, the panel of sweep 0
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s), "assemble"));
    TRY(check_launch(launch_spd_big_stage(sa, L.naxes, -1, h->s), "pivot_init"));
    const int stage = nm == "spd_pivot" ? -1 : 0;
    launch = [&, stage]() { return launch_spd_big_stage(sa, L.naxes, stage, h->s); };
  } else if (nm == "sweep") {
    // re-assemble K and factor pivot 0, then time sweep 0 (idempotent: X -> Y, piv[1]).
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s), "assemble"));
    TRY(check_launch(launch_spd_stage(sa, L.naxes, -1, h->s), "pivot_init"));
    launch = [&]() { return launch_spd_stage(sa, L.naxes, 0, h->s); };
    // potrf+potri-equivalent flops (n^3 per factor) spread over the T = p/32 sweeps;
    // HBM bytes: read X + write Y per factor
    for (int a = 0; a < L.naxes; ++a) {
      const double n = a == 0 ? n1 : n2;
      flops += n * n * n / ((a == 0 ? L.p1 : L.p2) / 32);
      bytes += 16.0 * n * n;
    }
  } else if (nm == "gather") {
    // the K-assembly launch of the class path (the large-factor step's, gpk_api.cpp
    // enqueue_assemble_inverse): K (+ jitter), its kept copy Kc (when the handle keeps one) and D
    // written, the class id of every element read (its variant byte ClassArgs::vidx where the
    // handle built them, p >= 1024; else the int32 id) -- the bytes it really moves; the class
    // values and cbase entries are L2-resident gathers and not counted
    if (h->cls[0].ncls <= 0) return fail(GPK_EINVAL, "gather: this handle does not use distance classes");
    for (int a = 0; a < L.naxes; ++a) {
      aa[a].cls = h->cls[a];
      aa[a].Kc = h->Kc[a];
    }
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s, true),
                     "class_eval"));
    launch = [&]() { return launch_gather_only(aa, L.naxes, h->s); };
    for (int a = 0; a < L.naxes; ++a) {
      const double P = a == 0 ? L.p1 : L.p2;
      bytes += P * P * ((h->cls[a].vidx ? 1.0 : 4.0) + 8.0 + (h->Kc[a] ? 8.0 : 0.0) + (deriv ? 8.0 : 0.0));
    }
  } else if ((nm == "write_stream" || nm == "write_stream_after_copy") && L.dim == 2) {
    // a pure write stream of the gather's bytes (hipMemsetD32 of K, Kc, D of both factors),
    // back to back or right after an HBM-bound copy of other buffers: whether the gather's
    // in-step rate is the write-heavy HBM rate once the memory-side cache holds other lines
    const bool after = nm == "write_stream_after_copy";
    const size_t nb = (size_t)L.p1 * L.p2 * sizeof(double);
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    double tot = 0.0;
    for (int it = 0; it <= iters; ++it) {
      if (after)
        for (int c = 0; c < 2; ++c) HIPCHK(hipMemcpyAsync(h->S, h->R, nb, hipMemcpyDeviceToDevice, h->s));
      HIPCHK(hipEventRecord(e0, h->s));
      for (int a = 0; a < L.naxes; ++a) {
        const size_t P = a == 0 ? L.p1 : L.p2;
        for (double* q : {h->K[a], h->Kc[a], h->D[a]}) HIPCHK(hipMemsetD32Async(q, 0, 2 * P * P, h->s));
      }
      HIPCHK(hipEventRecord(e1, h->s));
      HIPCHK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0) tot += ms * 1000.0;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (int a = 0; a < L.naxes; ++a) {
      const double P = a == 0 ? L.p1 : L.p2;
      bytes += 24.0 * P * P;
    }
    *avg_us = tot / iters;
    *alg_flops = 0.0;
    *alg_bytes = bytes;
    return read_status(h);
  } else if ((nm == "gather_after_gemm" || nm == "gather_after_copy") && L.dim == 2) {
    // the gather timed alone (events around it) right after a C5-size GEMM stage (gemm_B: an
    // MFMA-bound launch writing 2 x 134 MB) or after an HBM-bound copy of the same bytes: which
    // state makes the in-step gather run at half its back-to-back rate
    if (h->cls[0].ncls <= 0) return fail(GPK_EINVAL, "gather: this handle does not use distance classes");
    for (int a = 0; a < L.naxes; ++a) {
      aa[a].cls = h->cls[a];
      aa[a].Kc = h->Kc[a];
    }
    TRY(check_launch(launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s, true),
                     "class_eval"));
    const bool gemm = nm == "gather_after_gemm";
    const size_t nb = (size_t)L.p1 * L.p2 * sizeof(double);
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    double tot = 0.0;
    for (int it = 0; it <= iters; ++it) {
      if (gemm)
        HIPCHK(launch_gemm_auto(h->hdescs.data() + h->st[3].off, h->st[3].n, h->sc, h->s, h->st[3].variant));
      else
        for (int c = 0; c < 2; ++c) HIPCHK(hipMemcpyAsync(h->S, h->R, nb, hipMemcpyDeviceToDevice, h->s));
      HIPCHK(hipEventRecord(e0, h->s));
      HIPCHK(launch_gather_only(aa, L.naxes, h->s));
      HIPCHK(hipEventRecord(e1, h->s));
      HIPCHK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0) tot += ms * 1000.0;  // (the first is a warm-up)
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (int a = 0; a < L.naxes; ++a) {
      const double P = a == 0 ? L.p1 : L.p2;
      bytes += P * P * ((h->cls[a].vidx ? 1.0 : 4.0) + 8.0 + (h->Kc[a] ? 8.0 : 0.0) + (deriv ? 8.0 : 0.0));
    }
    *avg_us = tot / iters;
    *alg_flops = 0.0;
    *alg_bytes = bytes;
    return read_status(h);
  } else if (nm == "class_eval") {
    // the class-value launch (every field at every class distance + the step constants): it
    // reads the U class distances and writes K and D values per class (24 B per class and axis)
    if (h->cls[0].ncls <= 0) return fail(GPK_EINVAL, "class_eval: this handle does not use distance classes");
    for (int a = 0; a < L.naxes; ++a) aa[a].cls = h->cls[a];
    launch = [&]() {
      return launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s, true);
    };
    for (int a = 0; a < L.naxes; ++a) bytes += 24.0 * h->cls[a].ncls;
  } else if (nm == "assemble") {
    // the step's assembly launch(es): class values only when the chain gathers K itself
    const bool eval_only = h->chain && h->cls[0].ncls > 0;
    for (int a = 0; a < L.naxes; ++a) aa[a].cls = h->cls[a];
    launch = [&, eval_only]() {
      return launch_assemble(h->prob.kind, L.q, aa, L.naxes, make_prep(h, 0), h->s, eval_only);
    };
    // the bytes the launch really moves: with classes and the chain, the class values (24 B per
    // class: distance read, K and D value written); otherwise K and D written per element (P^2
    // per axis, 8 B each); flops not counted (transcendental-bound)
    for (int a = 0; a < L.naxes; ++a) {
      const double P = a == 0 ? L.p1 : L.p2;
      bytes += eval_only ? 24.0 * h->cls[a].ncls : 16.0 * P * P;
    }
  } else if (nm == "gemm_B" && L.dim == 2) {
    launch = [&]() {
      return launch_gemm_auto(h->hdescs.data() + h->st[3].off, h->st[3].n, h->sc, h->s, h->st[3].variant);
    };
    // S = A K2^{-1} (2 n1 n2^2); R = D1 A + Bt D2^T (2 n1^2 n2 + 2 n1 n2^2)
    flops = 2 * n1 * n2 * n2 + 2 * n1 * n1 * n2 + 2 * n1 * n2 * n2;
    // reads A, K2^{-1}, D1, Bt, D2, F, U; writes S, R
    bytes = 8.0 * (n1 * n2 + n2 * n2 + n1 * n1 + n1 * n2 + n2 * n2 + 2 * n1 * n2 + 2 * n1 * n2);
  } else if (nm == "pgrad" && L.dim == 2) {
    PGradArgs pa[2];
    for (int a = 0; a < 2; ++a) {
      pa[a] = PGradArgs{};
      pa[a].x = a == 0 ? h->x1 : h->x2; pa[a].n = a == 0 ? L.n1 : L.n2; pa[a].p = a == 0 ? L.p1 : L.p2;
      pa[a].kc = h->kc + a; pa[a].GK = h->GK[a]; pa[a].GD = h->GD[a]; pa[a].deriv = deriv;
      pa[a].part = h->pgpart + (size_t)a * h->bpa * 3 * QMAX;
      pa[a].cls = h->cls[a];
    }
    launch = [&, pa]() mutable { return launch_pgrad(h->prob.kind, L.q, 0, pa, 2, h->bpa, h->sc, h->s); };
    bytes = 16.0 * (n1 * n1 + n2 * n2);  // G_K, G_D read
  } else {
    return fail(GPK_EINVAL, "unknown kernel name (spd_chain | sweep | assemble | gemm_B | pgrad[2D])");
  }
  HIPCHK(launch());  // warm
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipEventRecord(e0, h->s));
  for (int it = 0; it < iters; ++it) HIPCHK(launch());
  HIPCHK(hipEventRecord(e1, h->s));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *avg_us = ms * 1000.0 / iters;
  *alg_flops = flops;
  *alg_bytes = bytes;
  return read_status(h);
}

int gpk_dgemm(int32_t variant, int32_t M, int32_t N, int32_t K, double alpha, const double* A,
              int32_t lda, int32_t ta, const double* B, int32_t ldb, int32_t tb, int32_t K2,
              double alpha2, const double* A2, int32_t lda2, int32_t ta2, const double* B2,
              int32_t ldb2, int32_t tb2, double beta, const double* C0, double* C, int32_t ldc,
              int32_t iters, double* avg_us) {
  if (variant < 0 || variant > 3 || M <= 0 || N <= 0 || K <= 0 || K2 < 0 || (M | N | K | K2) & 31 ||
      !A || !B || !C || (K2 && (!A2 || !B2)) || iters < 0 || (iters && !avg_us))
    return fail(GPK_EINVAL, "gpk_dgemm: bad argument (M, N, K, K2 multiples of 32)");
  // stored extents of op(A) = M x K etc.: rows x row length, each row length <= its ld
  auto ext = [](int rows, int cols, int t, int ld, size_t* n) {
    const int r = t ? cols : rows, c = t ? rows : cols;
    *n = (size_t)(r - 1) * ld + c;
    return ld >= c;
  };
  size_t na = 0, nb = 0, na2 = 0, nb2 = 0, nc = 0;
  if (!ext(M, K, ta, lda, &na) || !ext(K, N, tb, ldb, &nb) || !ext(M, N, 0, ldc, &nc) ||
      (K2 && (!ext(M, K2, ta2, lda2, &na2) || !ext(K2, N, tb2, ldb2, &nb2))))
    return fail(GPK_EINVAL, "gpk_dgemm: leading dimension shorter than a row");
  TRY(check_device(0));
  DevSwitch dsw(0);
  std::vector<void*> mem;
  auto cleanup = [&]() { for (void* p : mem) (void)hipFree(p); };
  auto up = [&](const double* src, size_t n, double** dst) -> hipError_t {
    hipError_t e = hipMalloc(dst, n * 8);
    if (e != hipSuccess) return e;
    mem.push_back(*dst);
    return src ? hipMemcpy(*dst, src, n * 8, hipMemcpyHostToDevice) : hipSuccess;
  };
  GemmDesc d{};
  double *dA = nullptr, *dB = nullptr, *dA2 = nullptr, *dB2 = nullptr, *dC = nullptr, *dC0 = nullptr;
  hipError_t e = up(A, na, &dA);
  if (e == hipSuccess) e = up(B, nb, &dB);
  if (e == hipSuccess && K2) e = up(A2, na2, &dA2);
  if (e == hipSuccess && K2) e = up(B2, nb2, &dB2);
  if (e == hipSuccess) e = up(C0 == C ? C : nullptr, nc, &dC);
  if (e == hipSuccess && C0 && C0 != C) e = up(C0, nc, &dC0);
  if (e != hipSuccess) {
    cleanup();
    return fail(e == hipErrorOutOfMemory ? GPK_ENOMEM : GPK_EHIP, std::string("gpk_dgemm: ") + hipGetErrorString(e));
  }
  d.A = dA; d.lda = lda; d.ta = ta ? 1 : 0; d.B = dB; d.ldb = ldb; d.tb = tb ? 1 : 0;
  d.A2 = dA2; d.lda2 = lda2; d.ta2 = ta2 ? 1 : 0; d.B2 = dB2; d.ldb2 = ldb2; d.tb2 = tb2 ? 1 : 0;
  d.alpha = alpha; d.alpha2 = alpha2; d.K2 = K2;
  d.beta = C0 ? beta : 0.0; d.C0 = C0 ? (C0 == C ? dC : dC0) : nullptr; d.ldc0 = ldc;
  d.C = dC; d.ldc = ldc; d.M = M; d.N = N; d.K = K; d.epi = EPI_STORE;
  const int v = variant ? variant : gemm_variant(&d, 1, 0);
  auto launch = [&]() { return launch_gemm_auto(&d, 1, nullptr, 0, v); };
  // (an in-place C0 == C update is checked once; timed launches then repeat it on their own output)
  e = launch();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(C, dC, nc * 8, hipMemcpyDeviceToHost);
  if (e == hipSuccess && iters) {
    hipEvent_t e0, e1;
    e = hipEventCreate(&e0);
    if (e == hipSuccess) {
      e = hipEventCreate(&e1);
      if (e == hipSuccess) {
        // (timing only: with C0 == C every timed launch updates dC in place, so each one reads
        // the previous launch's output as its C0 -- same shapes and work, different values; the
        // result copied back above is the first launch's)
        e = launch();  // warm
        if (e == hipSuccess) e = hipEventRecord(e0, 0);
        for (int it = 0; it < iters && e == hipSuccess; ++it) e = launch();
        if (e == hipSuccess) e = hipEventRecord(e1, 0);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (e == hipSuccess) *avg_us = ms * 1000.0 / iters;  // (untouched on failure)
        (void)hipEventDestroy(e1);
      }
      (void)hipEventDestroy(e0);
    }
  }
  cleanup();
  if (e != hipSuccess) return fail(GPK_EHIP, std::string("gpk_dgemm: ") + hipGetErrorString(e));
  return GPK_OK;
}

}  // extern "C"

int gpk_wide_schedule(int32_t T2, int32_t paired, uint32_t* out, int64_t cap) {
  if (T2 < 1 || T2 > 255 || !out) return fail(GPK_EINVAL, "gpk_wide_schedule: T2 in [1, 255], out non-null");
  std::vector<unsigned> tab;
  wide_schedule(T2, paired != 0, tab);
  if ((int64_t)tab.size() > cap) return fail(GPK_EINVAL, "gpk_wide_schedule: cap too small");
  std::memcpy(out, tab.data(), tab.size() * sizeof(unsigned));
  return GPK_OK;
}

// error / device helpers for the other C-ABI translation units (gpk_kron3.cpp)
namespace gpk {
int api_fail(int code, const std::string& msg) { return fail(code, msg); }
int api_check_device(int dev) { return check_device(dev); }
}  // namespace gpk
