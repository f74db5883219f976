// gpk_kron3.cpp — C ABI of the 3-axis Kronecker solver (include/gpk.h gpk_*3; SURVEY.md §8(f)
// row 4, the d > 2 generalisation of GP_solver_2d_single, code/model_GP_solver_2d.py:87-183).
//
// One step (one captured hipGraph) on a tensor grid U[i1][i2][i3], K = K1 (x) K2 (x) K3:
//   prep -> K_k, D_k (the 2-axis assembly kernel, per axis) -> K_k^{-1} + log det (the per-sweep
//   SPD inverse) -> mode-k products as fp64 MFMA GEMMs over unfoldings -> R, S, partials ->
//   reverse-mode products -> G_K, G_D per axis -> the 2-axis parameter contraction -> loss +
//   Adam.  Unfoldings: mode 1 is U as P1 x (P2 P3), mode 3 is U as (P1 P2) x P3 -- both plain
//   row-major views -- and mode 2 goes through the permuted copy [i2][i1][i3] (k3_permute),
//   whose rows are the mode-2 unfolding.  With A_k = K_k^{-1} x_k U, X_k = (K_k^{-1} D_k^T) x_k R:
//     S = K^{-1} U,  R = sum_k D_k x_k A_k - F,  dL/dU = S + v sum_k X_k  (+ AC, boundary)
//     G_Kk = c/2 (N / N_k) K_k^{-1} - (S/2 + v X_k)_(k) A_k,(k)^T,   G_Dk = v R_(k) A_k,(k)^T
// (the 2-axis adjoints of SURVEY.md Appendix A, one per axis).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpk.h"
#include "gpk_internal.h"
#include "gpk_kron3.h"
#include "stepk.h"

namespace gpk {
int api_fail(int code, const std::string& msg);
int api_check_device(int dev);
}  // namespace gpk

using namespace gpk;

#define K3TRY(x)                   \
  do {                             \
    int r_ = (x);                  \
    if (r_ != GPK_OK) return r_;   \
  } while (0)
#define K3HIP(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      return api_fail(e_ == hipErrorOutOfMemory ? GPK_ENOMEM : GPK_EHIP,                  \
                      std::string(#x) + ": " + hipGetErrorString(e_));                    \
  } while (0)

namespace {
constexpr int K3_LOSS_CAP = 4096;
constexpr int K3_MAX_N = 1024;  // per axis (the per-sweep inverse; a 3-axis grid of 1024^3 is 8 GB)
}  // namespace

struct gpk_handle3 {
  gpk_problem3 prob{};
  K3Geom g{};
  int q = 0;
  long nu = 0, nparams = 0;
  int off_kp[3] = {}, off_tau = 0, off_v = 0, nsmall = 0;
  int dev = 0;
  hipStream_t s = nullptr;
  std::vector<void*> allocs;
  double* x[3] = {};
  double *F = nullptr, *bvals = nullptr, *params = nullptr, *grad = nullptr, *m = nullptr,
         *v = nullptr, *Up = nullptr;
  AxisConst* kc = nullptr;
  StepScalars* sc = nullptr;
  int *count = nullptr, *loss_slot = nullptr, *status = nullptr;
  double *losses = nullptr, *diag = nullptr, *bgap = nullptr;
  double *K[3] = {}, *Kb[3] = {}, *D[3] = {}, *piv[3] = {}, *ldet[3] = {}, *pst[3] = {}, *Kinv[3] = {};
  unsigned int* aflag[3] = {};
  // grid tensors (natural [p1][p2][p3] or, suffix p, mode-2 permuted [p2][p1][p3])
  double *Upp = nullptr, *A1 = nullptr, *A2p = nullptr, *A3 = nullptr, *Tm = nullptr, *Tp = nullptr,
         *Sp = nullptr, *S = nullptr, *Rx = nullptr, *Rz = nullptr, *Ryp = nullptr, *R = nullptr,
         *Rp = nullptr, *T1 = nullptr, *X1 = nullptr, *T2p = nullptr, *X2p = nullptr, *T3 = nullptr,
         *X3 = nullptr, *Y1 = nullptr, *Y2p = nullptr, *Y3 = nullptr;
  double *GK[3] = {}, *GD[3] = {};
  double *red_egap = nullptr, *red_quad = nullptr;
  int nred = 0;
  double *pgpart = nullptr, *pg = nullptr;
  int bpa = 0;
  std::vector<std::vector<GemmDesc>> stages;  // GEMM launches in stream order
  hipGraphExec_t exec[2] = {nullptr, nullptr};

  template <class T>
  int alloc(T** p, size_t count_) {
    void* q_ = nullptr;
    const size_t bytes = std::max<size_t>(count_ * sizeof(T), 16);
    hipError_t e = hipMalloc(&q_, bytes);
    if (e != hipSuccess) return api_fail(GPK_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    e = hipMemsetAsync(q_, 0, bytes, s);
    if (e != hipSuccess) return api_fail(GPK_EHIP, hipGetErrorString(e));
    allocs.push_back(q_);
    *p = static_cast<T*>(q_);
    return GPK_OK;
  }
};

namespace {

GemmDesc mk(const double* A, int lda, int ta, const double* B, int ldb, int tb, double* C, int ldc,
            int M, int N, int K) {
  GemmDesc d{};
  d.A = A; d.lda = lda; d.ta = ta;
  d.B = B; d.ldb = ldb; d.tb = tb;
  d.C = C; d.ldc = ldc;
  d.M = M; d.N = N; d.K = K;
  d.alpha = 1.0;
  d.epi = EPI_STORE;
  return d;
}

GemmDesc side(GemmDesc d, double* Y, const double* Ys, int ldy) {  // Y = Ys / 2 + v C
  d.Y = Y; d.Ys = Ys; d.ldy = ldy;
  return d;
}

// the step's GEMM launches (stream order; independent products of one launch batched)
void build_stages(gpk_handle3* h) {
  const int P1 = h->g.p[0], P2 = h->g.p[1], P3 = h->g.p[2];
  const int M1 = P2 * P3, M2 = P1 * P3, M3 = P1 * P2;
  const double n1 = h->g.n[0], n2 = h->g.n[1], n3 = h->g.n[2], c = h->prob.logdet;
  double* const* Ki = h->Kinv;
  double* const* D = h->D;
  auto& st = h->stages;
  st.clear();
  // forward: A1 = K1^{-1} x1 U, A3 = K3^{-1} x3 U
  st.push_back({mk(Ki[0], P1, 0, h->Up, M1, 0, h->A1, M1, P1, M1, P1),
                mk(h->Up, P3, 0, Ki[2], P3, 0, h->A3, P3, M3, P3, P3)});
  // (U permuted) A2 = K2^{-1} x2 U;  T = A1 x3 K3^{-1}
  st.push_back({mk(Ki[1], P2, 0, h->Upp, M2, 0, h->A2p, M2, P2, M2, P2),
                mk(h->A1, P3, 0, Ki[2], P3, 0, h->Tm, P3, M3, P3, P3)});
  // (T permuted) S = K2^{-1} x2 T;  U_xx = D1 x1 A1, U_yy = D2 x2 A2, U_zz = D3 x3 A3
  st.push_back({mk(Ki[1], P2, 0, h->Tp, M2, 0, h->Sp, M2, P2, M2, P2),
                mk(D[0], P1, 0, h->A1, M1, 0, h->Rx, M1, P1, M1, P1),
                mk(D[1], P2, 0, h->A2p, M2, 0, h->Ryp, M2, P2, M2, P2),
                mk(h->A3, P3, 0, D[2], P3, 1, h->Rz, P3, M3, P3, P3)});
  // (R, S combined) reverse: D_k^T x_k R;  G_D1 = v R_(1) A1_(1)^T
  {
    GemmDesc gd = mk(h->R, M1, 0, h->A1, M1, 1, h->GD[0], P1, P1, P1, M1);
    gd.vscale = 1;
    st.push_back({mk(D[0], P1, 1, h->R, M1, 0, h->T1, M1, P1, M1, P1),
                  mk(D[1], P2, 1, h->Rp, M2, 0, h->T2p, M2, P2, M2, P2),
                  mk(h->R, P3, 0, D[2], P3, 0, h->T3, P3, M3, P3, P3), gd});
  }
  // X_k = K_k^{-1} x_k (D_k^T x_k R) with the side outputs Y_k = S/2 + v X_k;  G_D2
  {
    GemmDesc gd = mk(h->Rp, M2, 0, h->A2p, M2, 1, h->GD[1], P2, P2, P2, M2);
    gd.vscale = 1;
    st.push_back({side(mk(Ki[0], P1, 0, h->T1, M1, 0, h->X1, M1, P1, M1, P1), h->Y1, h->S, M1),
                  side(mk(Ki[1], P2, 0, h->T2p, M2, 0, h->X2p, M2, P2, M2, P2), h->Y2p, h->Sp, M2),
                  side(mk(h->T3, P3, 0, Ki[2], P3, 0, h->X3, P3, M3, P3, P3), h->Y3, h->S, P3), gd});
  }
  // G_K_k = c/2 (N / N_k) K_k^{-1} - Y_k,(k) A_k,(k)^T;  G_D3
  {
    GemmDesc g1 = mk(h->Y1, M1, 0, h->A1, M1, 1, h->GK[0], P1, P1, P1, M1);
    g1.alpha = -1.0; g1.beta = 0.5 * c * n2 * n3; g1.C0 = Ki[0]; g1.ldc0 = P1;
    GemmDesc g2 = mk(h->Y2p, M2, 0, h->A2p, M2, 1, h->GK[1], P2, P2, P2, M2);
    g2.alpha = -1.0; g2.beta = 0.5 * c * n1 * n3; g2.C0 = Ki[1]; g2.ldc0 = P2;
    GemmDesc g3 = mk(h->Y3, P3, 1, h->A3, P3, 0, h->GK[2], P3, P3, P3, M3);
    g3.alpha = -1.0; g3.beta = 0.5 * c * n1 * n2; g3.C0 = Ki[2]; g3.ldc0 = P3;
    GemmDesc gd = mk(h->R, P3, 1, h->A3, P3, 0, h->GD[2], P3, P3, P3, M3);
    gd.vscale = 1;
    st.push_back({g1, g2, g3, gd});
  }
}

int launch_stage(gpk_handle3* h, int k) {
  const auto& d = h->stages[k];
  const int variant = gemm_variant(d.data(), (int)d.size(), 0);
  hipError_t e = launch_gemm_auto(d.data(), (int)d.size(), h->sc, h->s, variant);
  if (e != hipSuccess) return api_fail(GPK_EHIP, std::string("gemm: ") + hipGetErrorString(e));
  return GPK_OK;
}

int chk(hipError_t e, const char* what) {
  if (e != hipSuccess) return api_fail(GPK_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  return GPK_OK;
}

int enqueue_step3(gpk_handle3* h, int apply) {
  const K3Geom& g = h->g;
  const int q = h->q, kind = h->prob.kind;
  K3Prep P{};
  P.g = g; P.params = h->params; P.q = q;
  for (int a = 0; a < 3; ++a) P.off_kp[a] = h->off_kp[a];
  P.off_tau = h->off_tau; P.off_v = h->off_v;
  P.kc = h->kc; P.sc = h->sc; P.count = h->count; P.apply = apply;
  P.b1 = h->prob.b1; P.b2 = h->prob.b2;
  P.Up = h->Up; P.bvals = h->bvals; P.nb = (int)(2 * ((long)g.n[1] * g.n[2] + (long)g.n[0] * g.n[2] + (long)g.n[0] * g.n[1]));
  P.bgap = h->bgap;
  K3TRY(chk(k3_launch_prep(P, h->s), "k3_prep"));
  // K_k, D_k: the 2-axis assembly kernel (per-pair path), its axis constants from the params
  AssembleArgs aa[3] = {};
  for (int a = 0; a < 3; ++a) {
    aa[a].x = h->x[a]; aa[a].n = g.n[a]; aa[a].p = g.p[a]; aa[a].kc = h->kc + a;
    aa[a].jitter = h->prob.jitter; aa[a].K = h->K[a]; aa[a].D = h->D[a]; aa[a].deriv = 2;
  }
  // (skip = 1: the constants are published by k3_prep; each workgroup derives its axis's own)
  PrepArgs p12{};
  p12.params = h->params; p12.off_kp[0] = h->off_kp[0]; p12.off_kp[1] = h->off_kp[1];
  p12.naxes = 2; p12.skip = 1;
  PrepArgs p3 = p12;
  p3.off_kp[0] = h->off_kp[2];
  p3.naxes = 1;
  K3TRY(chk(launch_assemble(kind, q, aa, 2, p12, h->s), "assemble"));
  K3TRY(chk(launch_assemble(kind, q, aa + 2, 1, p3, h->s), "assemble"));
  // K_k^{-1} and log det K_k (per-sweep Cholesky-Gauss-Jordan inverse; the output buffer of
  // each factor is fixed by its sweep count)
  SpdArgs sa[3] = {};
  for (int a = 0; a < 3; ++a) {
    sa[a].X = h->K[a]; sa[a].Y = h->Kb[a]; sa[a].p = g.p[a]; sa[a].n = g.n[a];
    sa[a].piv = h->piv[a]; sa[a].ldet = h->ldet[a]; sa[a].pst = h->pst[a];
    sa[a].status = h->status; sa[a].flag = h->aflag[a];
  }
  double* fin[3] = {};
  K3TRY(chk(launch_spd_inverse(sa, 2, fin, h->s, false), "spd_inverse"));
  K3TRY(chk(launch_spd_inverse(sa + 2, 1, fin + 2, h->s, false), "spd_inverse"));
  // forward products
  K3TRY(launch_stage(h, 0));
  K3TRY(chk(k3_launch_permute(h->Up, h->Upp, g, h->s), "k3_permute"));
  K3TRY(launch_stage(h, 1));
  K3TRY(chk(k3_launch_permute(h->Tm, h->Tp, g, h->s), "k3_permute"));
  K3TRY(launch_stage(h, 2));
  K3Combine C{};
  C.g = g; C.Rx = h->Rx; C.Rz = h->Rz; C.Ryp = h->Ryp; C.F = h->F; C.Up = h->Up; C.Sp = h->Sp;
  C.ac = h->prob.eq == GPK_ALLENCAHN; C.R = h->R; C.Rp = h->Rp; C.S = h->S;
  C.red_egap = h->red_egap; C.red_quad = h->red_quad;
  K3TRY(chk(k3_launch_combine(C, h->s), "k3_combine"));
  // reverse products and G_K, G_D
  for (int k = 3; k < (int)h->stages.size(); ++k) K3TRY(launch_stage(h, k));
  // kernel-parameter contraction (the 2-axis kernels: axes 1-2, then axis 3)
  PGradArgs pg[3] = {};
  for (int a = 0; a < 3; ++a) {
    pg[a].x = h->x[a]; pg[a].n = g.n[a]; pg[a].p = g.p[a]; pg[a].kc = h->kc + a;
    pg[a].GK = h->GK[a]; pg[a].GD = h->GD[a]; pg[a].deriv = 2;
    pg[a].part = h->pgpart + (size_t)a * h->bpa * 3 * QMAX;
  }
  K3TRY(chk(launch_pgrad(kind, q, 0, pg, 2, h->bpa, h->sc, h->s), "pgrad"));
  K3TRY(chk(launch_pgrad(kind, q, 0, pg + 2, 1, h->bpa, h->sc, h->s), "pgrad"));
  K3TRY(chk(launch_reduce_parts(h->pgpart, h->bpa, 3, q, h->pg, h->s), "reduce_parts"));
  // loss + small-parameter Adam, then dL/dU + Adam on U (U is read by nothing after this)
  K3Final F{};
  F.g = g; F.hyper = AdamHyper{h->prob.lr, h->prob.b1, h->prob.b2, h->prob.eps};
  F.llk_weight = h->prob.llk_weight; F.logdet = h->prob.logdet; F.apply = apply;
  F.has_cos = kind_cos(kind) ? 1 : 0; F.q = q;
  F.red_quad = h->red_quad; F.red_egap = h->red_egap; F.nred = h->nred;
  for (int a = 0; a < 3; ++a) { F.ldet[a] = h->ldet[a]; F.nldet[a] = g.p[a] / 32; F.off_kp[a] = h->off_kp[a]; }
  F.pg = h->pg; F.kc = h->kc; F.sc = h->sc; F.bgap = h->bgap;
  F.off_tau = h->off_tau; F.off_v = h->off_v; F.off_small = (int)h->nu; F.nsmall = h->nsmall;
  F.params = h->params; F.grad = h->grad; F.m = h->m; F.v = h->v;
  F.losses = h->losses; F.loss_slot = h->loss_slot; F.diag = h->diag;
  K3TRY(chk(k3_launch_finalize(F, h->s), "k3_finalize"));
  K3AdamU A{};
  A.g = g; A.hyper = F.hyper; A.llk_weight = h->prob.llk_weight; A.apply = apply; A.ac = C.ac;
  A.sc = h->sc; A.S = h->S; A.X1 = h->X1; A.X2p = h->X2p; A.X3 = h->X3; A.R = h->R; A.Up = h->Up;
  A.bvals = h->bvals; A.off_u = 0; A.params = h->params; A.grad = h->grad; A.m = h->m; A.v = h->v;
  K3TRY(chk(k3_launch_adam_u(A, h->s), "k3_adam_u"));
  return GPK_OK;
}

int capture3(gpk_handle3* h, int apply) {
  if (h->exec[apply]) return GPK_OK;
  hipGraph_t gr = nullptr;
  K3HIP(hipStreamBeginCapture(h->s, hipStreamCaptureModeThreadLocal));
  const int rc = enqueue_step3(h, apply);
  hipError_t e = hipStreamEndCapture(h->s, &gr);
  if (rc != GPK_OK) {
    if (gr) (void)hipGraphDestroy(gr);
    return rc;
  }
  if (e != hipSuccess) return api_fail(GPK_EHIP, std::string("capture: ") + hipGetErrorString(e));
  e = hipGraphInstantiate(&h->exec[apply], gr, nullptr, nullptr, 0);
  (void)hipGraphDestroy(gr);
  if (e != hipSuccess) return api_fail(GPK_EHIP, std::string("instantiate: ") + hipGetErrorString(e));
  return GPK_OK;
}

int read_status3(gpk_handle3* h) {
  int st = 0;
  K3HIP(hipMemcpyAsync(&st, h->status, sizeof(int), hipMemcpyDeviceToHost, h->s));
  K3HIP(hipStreamSynchronize(h->s));
  if (st) {
    (void)hipMemsetAsync(h->status, 0, sizeof(int), h->s);
    return api_fail(GPK_ENOTPD, "covariance factor is not positive definite (non-positive pivot in SPD inverse)");
  }
  return GPK_OK;
}

struct Dev3 {  // restore the caller's current device on scope exit
  int prev = -1;
  explicit Dev3(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(d);
  }
  ~Dev3() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

int gpk_destroy3(gpk_handle3* h) {
  if (!h) return GPK_OK;
  Dev3 ds(h->dev);
  if (h->s) (void)hipStreamSynchronize(h->s);
  for (auto& e : h->exec)
    if (e) (void)hipGraphExecDestroy(e);
  for (void* p : h->allocs) (void)hipFree(p);
  if (h->s) (void)hipStreamDestroy(h->s);
  delete h;
  return GPK_OK;
}

int gpk_create3(const gpk_problem3* p, double freq_scale, gpk_handle3** out) {
  if (!p || !out) return api_fail(GPK_EINVAL, "NULL argument");
  *out = nullptr;
  if (p->kind < 0 || p->kind > 3) return api_fail(GPK_EINVAL, "Invalid Kernel");
  if (p->eq != GPK_POISSON && p->eq != GPK_ALLENCAHN)
    return api_fail(GPK_EINVAL, "equation type not supported for the 3-axis solver");
  if (p->q <= 0 || p->q > QMAX) return api_fail(GPK_EINVAL, "Q must be in [1, 64]");
  const int ns[3] = {p->n1, p->n2, p->n3};
  for (int a = 0; a < 3; ++a)
    if (ns[a] < 2 || ns[a] > K3_MAX_N) return api_fail(GPK_EINVAL, "need 2..1024 collocation points per axis");
  if (!p->x1 || !p->x2 || !p->x3 || !p->src || !p->bvals) return api_fail(GPK_EINVAL, "NULL problem array");
  K3TRY(api_check_device(p->device));
  Dev3 ds(p->device);
  gpk_handle3* h = new gpk_handle3();
  h->prob = *p;
  h->prob.x1 = h->prob.x2 = h->prob.x3 = h->prob.src = h->prob.bvals = nullptr;
  h->dev = p->device;
  h->q = p->q;
  for (int a = 0; a < 3; ++a) {
    h->g.n[a] = ns[a];
    h->g.p[a] = pad_up(ns[a]);
  }
  const K3Geom& g = h->g;
  h->nu = g.real();
  for (int a = 0; a < 3; ++a) h->off_kp[a] = (int)h->nu + 3 * p->q * a;
  h->off_tau = (int)h->nu + 9 * p->q;
  h->off_v = h->off_tau + 1;
  h->nsmall = 9 * p->q + 2;
  h->nparams = h->nu + h->nsmall;
  auto bail = [&](int rc) {
    gpk_destroy3(h);
    return rc;
  };
  if (hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking) != hipSuccess)
    return bail(api_fail(GPK_EHIP, "hipStreamCreate failed"));
  const size_t np = (size_t)g.padded();
  const long nb = 2 * ((long)ns[1] * ns[2] + (long)ns[0] * ns[2] + (long)ns[0] * ns[1]);
  int rc = GPK_OK;
#define A3_(ptr, n) \
  if ((rc = h->alloc(&(ptr), (n))) != GPK_OK) return bail(rc)
  for (int a = 0; a < 3; ++a) {
    const int P = g.p[a];
    A3_(h->x[a], P);
    A3_(h->K[a], (size_t)P * P);
    A3_(h->Kb[a], (size_t)P * P);
    A3_(h->D[a], (size_t)P * P);
    A3_(h->piv[a], (size_t)P * 32);
    A3_(h->ldet[a], P / 32);
    A3_(h->pst[a], 2);
    A3_(h->aflag[a], 1);
    A3_(h->GK[a], (size_t)P * P);
    A3_(h->GD[a], (size_t)P * P);
    const int T = P / 32;  // sweep k reads (k even ? K : Kb): T sweeps end in
    h->Kinv[a] = (T & 1) ? h->Kb[a] : h->K[a];
  }
  A3_(h->F, np); A3_(h->bvals, nb);
  A3_(h->params, h->nparams); A3_(h->grad, h->nparams); A3_(h->m, h->nparams); A3_(h->v, h->nparams);
  A3_(h->Up, np);
  A3_(h->kc, 3); A3_(h->sc, 1); A3_(h->count, 1); A3_(h->loss_slot, 1); A3_(h->status, 1);
  A3_(h->losses, K3_LOSS_CAP); A3_(h->diag, 8); A3_(h->bgap, 1);
  double** tens[] = {&h->Upp, &h->A1, &h->A2p, &h->A3, &h->Tm, &h->Tp, &h->Sp, &h->S, &h->Rx,
                     &h->Rz, &h->Ryp, &h->R, &h->Rp, &h->T1, &h->X1, &h->T2p, &h->X2p, &h->T3,
                     &h->X3, &h->Y1, &h->Y2p, &h->Y3};
  for (double** t : tens) A3_(*t, np);
  h->nred = k3_combine_blocks(g);
  A3_(h->red_egap, h->nred); A3_(h->red_quad, h->nred);
  h->bpa = std::max(pgrad_blocks(ns[0]), std::max(pgrad_blocks(ns[1]), pgrad_blocks(ns[2])));
  A3_(h->pgpart, (size_t)3 * h->bpa * 3 * QMAX);
  A3_(h->pg, (size_t)3 * 3 * QMAX);
#undef A3_
  // upload: coordinates, the padded source, boundary values, the initial params
  // (model_GP_solver_2d.py:245-261: U = 0, freq = linspace(0,1,Q) freq_scale, log-ls = 0,
  // log-w = log(1/Q), log_tau = log_v = 0)
  const double* xs[3] = {p->x1, p->x2, p->x3};
  for (int a = 0; a < 3; ++a)
    if (hipMemcpyAsync(h->x[a], xs[a], ns[a] * sizeof(double), hipMemcpyHostToDevice, h->s) != hipSuccess)
      return bail(api_fail(GPK_EHIP, "upload x"));
  {
    std::vector<double> Fp(np, 0.0);
    for (int i1 = 0; i1 < ns[0]; ++i1)
      for (int i2 = 0; i2 < ns[1]; ++i2)
        std::memcpy(&Fp[g.at(i1, i2, 0)], p->src + ((size_t)i1 * ns[1] + i2) * ns[2], ns[2] * sizeof(double));
    std::vector<double> init(h->nparams, 0.0);
    for (int a = 0; a < 3; ++a)
      for (int c = 0; c < p->q; ++c) {
        init[h->off_kp[a] + c] = p->q > 1 ? (double)c / (p->q - 1) * freq_scale : 0.0;
        init[h->off_kp[a] + 2 * p->q + c] = std::log(1.0 / p->q);
      }
    if (hipMemcpyAsync(h->F, Fp.data(), np * sizeof(double), hipMemcpyHostToDevice, h->s) != hipSuccess ||
        hipMemcpyAsync(h->bvals, p->bvals, nb * sizeof(double), hipMemcpyHostToDevice, h->s) != hipSuccess ||
        hipMemcpyAsync(h->params, init.data(), init.size() * sizeof(double), hipMemcpyHostToDevice, h->s) != hipSuccess ||
        hipStreamSynchronize(h->s) != hipSuccess)
      return bail(api_fail(GPK_EHIP, "upload failed"));
  }
  build_stages(h);
  *out = h;
  return GPK_OK;
}

int gpk_num_params3(const gpk_handle3* h, int64_t* n) {
  if (!h || !n) return api_fail(GPK_EINVAL, "NULL argument");
  *n = h->nparams;
  return GPK_OK;
}

int gpk_set_params3(gpk_handle3* h, const double* flat, int64_t n) {
  if (!h || !flat) return api_fail(GPK_EINVAL, "NULL argument");
  if (n != h->nparams) return api_fail(GPK_EINVAL, "flat parameter vector has the wrong length");
  Dev3 ds(h->dev);
  K3HIP(hipMemcpyAsync(h->params, flat, n * sizeof(double), hipMemcpyHostToDevice, h->s));
  K3TRY(chk(k3_launch_sync_u(h->params, 0, h->g, h->Up, h->s), "k3_sync_u"));
  K3HIP(hipStreamSynchronize(h->s));
  return GPK_OK;
}

int gpk_get_params3(gpk_handle3* h, double* flat, int64_t n) {
  if (!h || !flat) return api_fail(GPK_EINVAL, "NULL argument");
  if (n != h->nparams) return api_fail(GPK_EINVAL, "flat parameter vector has the wrong length");
  Dev3 ds(h->dev);
  K3HIP(hipMemcpyAsync(flat, h->params, n * sizeof(double), hipMemcpyDeviceToHost, h->s));
  K3HIP(hipStreamSynchronize(h->s));
  return GPK_OK;
}

int gpk_loss_grad3(gpk_handle3* h, double* loss, double* grad_flat) {
  if (!h || !loss) return api_fail(GPK_EINVAL, "NULL argument");
  Dev3 ds(h->dev);
  K3TRY(capture3(h, 0));
  K3HIP(hipMemsetAsync(h->loss_slot, 0, sizeof(int), h->s));
  K3HIP(hipGraphLaunch(h->exec[0], h->s));
  K3TRY(read_status3(h));
  K3HIP(hipMemcpy(loss, h->diag, sizeof(double), hipMemcpyDeviceToHost));
  if (grad_flat) K3HIP(hipMemcpy(grad_flat, h->grad, h->nparams * sizeof(double), hipMemcpyDeviceToHost));
  return GPK_OK;
}

int gpk_step3(gpk_handle3* h, int32_t n_steps, double* losses) {
  if (!h) return api_fail(GPK_EINVAL, "NULL handle");
  if (n_steps < 0 || n_steps > K3_LOSS_CAP) return api_fail(GPK_EINVAL, "n_steps must be in [0, 4096]");
  Dev3 ds(h->dev);
  K3TRY(capture3(h, 1));
  K3HIP(hipMemsetAsync(h->loss_slot, 0, sizeof(int), h->s));
  for (int i = 0; i < n_steps; ++i) K3HIP(hipGraphLaunch(h->exec[1], h->s));
  K3TRY(read_status3(h));
  if (losses && n_steps > 0)
    K3HIP(hipMemcpy(losses, h->losses, n_steps * sizeof(double), hipMemcpyDeviceToHost));
  return GPK_OK;
}

}  // extern "C"
