// stepk_dev.h — device bodies of the step tail (loss, small-parameter Adam, U Adam), shared by
// the standalone kernels (stepk.hip) and the fused tail of the parameter-gradient launch
// (pgrad.hip).  References: code/model_GP_solver_2d.py:145-183, code/model_GP_solver_1d.py:123-158.
#pragma once
#include "gpk_internal.h"
#include "stepk.h"
#include "dd_dev.h"

#ifndef FIN_PROBE
#define FIN_PROBE(slot) ((void)0)
#endif

namespace gpk {

__device__ __forceinline__ void adam1(double g, double& p, double& m, double& v, const AdamHyper& h,
                                      double bc1, double bc2) {
  m = (1.0 - h.b1) * g + h.b1 * m;
  v = (1.0 - h.b2) * (g * g) + h.b2 * v;
  const double mh = m / bc1, vh = v / bc2;
  const double u = (mh / (sqrt(vh) + h.eps)) * (-h.lr);
  p = p + u;
}

__device__ inline double block_sum(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int t = threadIdx.x;
  __syncthreads();
  if ((t & 63) == 0) sh[t >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sh[w];
  return s;  // valid in every thread
}

__device__ __forceinline__ double ld_wt(const double* p) {  // global_load sc1 (L2-served)
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum_{k<n} p[k*stride] in index order (sc1 loads), 16 in flight per batch (latency-bound chain)
__device__ __forceinline__ double strided_sum(const double* p, int stride, int n) {
  double acc = 0.0;
  if (n > 16 && n <= 32) {  // (C2's levels: 25-26 partials) every load in flight at once, same order
    double v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = ld_wt(p + (size_t)(j < n ? j : 0) * stride);
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (j < n) acc += v[j];
    return acc;
  }
  int k = 0;
  for (; k + 16 <= n; k += 16) {
    double v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = ld_wt(p + (size_t)(k + j) * stride);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += v[j];
  }
  if (k < n) {  // remainder: one masked batch (a scalar loop here ran one round trip per load)
    double v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = ld_wt(p + (size_t)(k + j < n ? k + j : k) * stride);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (k + j < n) acc += v[j];
  }
  return acc;
}

// the same sum of double-double values (high parts at ph, low parts at pl), in index order
__device__ __forceinline__ dd::D strided_sum_dd(const double* ph, const double* pl, int stride, int n) {
  dd::D acc = {0.0, 0.0};
  for (int k = 0; k < n; k += 16) {
    double vh[16], vl[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const size_t o = (size_t)(k + j < n ? k + j : k) * stride;
      vh[j] = ld_wt(ph + o);
      vl[j] = ld_wt(pl + o);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (k + j < n) acc = dd::add(acc, dd::D{vh[j], vl[j]});
  }
  return acc;
}

// Single-workgroup tail of the step: scalars, loss, small-parameter gradients + Adam.
// Latency-bound (one workgroup on the step's critical path): every global load it needs is
// issued up front (one memory round trip), and the small parameters' gradients and Adam updates
// stay in the registers of the thread that owns them (no store / barrier / reload).
// part: 0 = everything; 1 = the loss, the log_tau / log_v gradients and their Adam (needs no
// kernel-parameter gradient: the fused tail runs it in a workgroup of its own at the start of
// the launch); 2 = the kernel-parameter gradients from f.pg and their Adam (the tail's last
// workgroup, right after it has reduced pg).
// The report's ready word (out[7]), stored last at system scope: the host returns from gpk_step
// once it reads 1 (the rest of the launch -- dL/dU and Adam on U -- is stream-ordered before any
// later call on the handle)
__device__ __forceinline__ void report_ready(double* out) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(out + 7), 0x3ff0000000000000ull,
                     __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void finalize_body(const FinalizeArgs& f, int part = 0) {
  const bool do_loss = part != 2, do_kp = part != 1;
  __shared__ double sh[4], sld[2], sg[2];
  const int t = threadIdx.x;
  const Layout& L = f.L;
  // ---- phase 0: loads.  The first pass of each partial sum is one unconditional load per
  // thread (clamped index, masked value), so the quad / egap / log-det loads issue together;
  // per-axis kernel-argument fields are chosen by uniform selects, not a dynamic index (which
  // reads the kernarg block through memory, one more round trip).
  const double* lp = ((t >> 6) == 1 && L.naxes > 1) ? f.ldet[1] : f.ldet[0];  // never null
  const int nl = (t >> 6) >= L.naxes ? 0 : (t >> 6) == 1 ? f.nldet[1] : f.nldet[0];
  const int lk = t & 63;
  double quad = 0.0, egap = 0.0, ldx = 0.0, bgap = 0.0;
  if (do_loss) {  // (uniform)
    const double q0 = f.red_quad[t < f.nquad ? t : 0], e0 = f.red_egap[t < f.negap ? t : 0];
    const double l0 = lp[lk < nl ? lk : 0];
    // boundary gap of U at the start of the step (assembly launch): its parts, in order
    double bg[BGAP_PARTS_MAX];
#pragma unroll
    for (int i = 0; i < BGAP_PARTS_MAX; ++i) bg[i] = i < f.bgap_parts ? f.bgap[i] : 0.0;
    bgap = bg[0];
#pragma unroll
    for (int i = 1; i < BGAP_PARTS_MAX; ++i)
      if (i < f.bgap_parts) bgap += bg[i];
    quad = t < f.nquad ? q0 : 0.0;
    egap = t < f.negap ? e0 : 0.0;
    for (int i = t + 256; i < f.nquad; i += 256) quad += f.red_quad[i];
    for (int i = t + 256; i < f.negap; i += 256) egap += f.red_egap[i];
    ldx = (t < 128 && lk < nl) ? l0 : 0.0;  // log det of factor t >> 6: its pivot blocks
    if (t < 128)
      for (int k = lk + 64; k < nl; k += 64) ldx += lp[k];
  }
  const double tau = f.sc->tau, v = f.sc->v, bc1 = f.sc->bc1, bc2 = f.sc->bc2;
  const double log_tau = f.params[L.off_tau], log_v = f.params[L.off_v];
  int slot = 0;
  bool gate = false;
  if (t == 0 && do_loss) {
    slot = *f.loss_slot;
    if (f.viol)
      for (int a = 0; a < L.naxes; ++a) gate |= f.watch[a] && gate_open(f.watch[a]);
  }
  // this thread's small parameters (kernel params of both axes, log_tau, log_v): value, Adam
  // moments, and for kernel params the contracted field sum and the weight w_q
  constexpr int PER = 2;  // nsmall <= 6 QMAX + 2 <= 2 * 256
  double pp[PER], pm[PER], pv2[PER], pgx[PER], pw[PER];
  int pidx[PER], pkind[PER];  // kind: 0 = kernel param, 1 = log_tau, 2 = log_v, -1 = none
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int k = t + 256 * r;
    pidx[r] = L.off_small + k;
    pkind[r] = -1;
    pp[r] = pm[r] = pv2[r] = pgx[r] = 0.0;
    pw[r] = 1.0;
    if (k >= L.nsmall) continue;
    const int idx = pidx[r];
    pp[r] = f.params[idx];
    pm[r] = f.m[idx];
    pv2[r] = f.v[idx];
    if (idx == L.off_tau || idx == L.off_v) {
      pkind[r] = do_loss ? (idx == L.off_tau ? 1 : 2) : -1;
      continue;
    }
    if (!do_kp) continue;
    const int a = (L.naxes == 2 && idx >= L.off_kp[1]) ? 1 : 0;
    const int rr = idx - L.off_kp[a], ty = rr / L.q, c = rr % L.q;  // ty: freq, log-ls, log-w
    pkind[r] = 0;
    pw[r] = f.kc[a].w[c];
    const int x = ty * QMAX + c;
    double pgv;
    if (f.gpart && f.gpart_lo) {  // (pgrad.hip pg_reduced's sums, in this thread)
      const dd::D acc = strided_sum_dd(f.gpart + (size_t)a * f.ngpa * (3 * QMAX) + x,
                                       f.gpart_lo + (size_t)a * f.ngpa * (3 * QMAX) + x, 3 * QMAX, f.ngpa);
      pgv = acc.h + acc.l;
    } else if (f.gpart) {
      pgv = strided_sum(f.gpart + (size_t)a * f.ngpa * (3 * QMAX) + x, 3 * QMAX, f.ngpa);
    } else {
      pgv = f.pg[a * 3 * QMAX + x];
    }
    if (f.pg_out) f.pg_out[a * 3 * QMAX + x] = pgv;
    pgx[r] = (ty == 0 && !f.has_cos) ? 0.0 : pgv;
  }
  // ---- phase 1: reductions, loss (thread 0)
  if (t == 0) FIN_PROBE(55);
  if (do_loss) {
  if (t < 128) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ldx += __shfl_xor(ldx, o, 64);
    if ((t & 63) == 0) sld[t >> 6] = ldx;
  }
  quad = block_sum(quad, sh);
  egap = block_sum(egap, sh);  // (its barriers also publish sld)
  }
  if (t == 0) FIN_PROBE(56);
  const double wb = f.llk_weight, c = f.logdet;
  if (t == 0 && do_loss) {
    if (gate) atomicOr(f.viol, 1u);
    const double ld[2] = {sld[0], L.naxes > 1 ? sld[1] : 0.0};
    const double Nb = (L.dim == 2) ? (double)(2 * L.n2 + 2 * L.n1) : (double)f.nb;
    const double Nc = (L.dim == 2) ? (double)L.n1 * (double)L.n2 : (double)L.n1;
    double log_prior;
    if (L.dim == 2)  // model_GP_solver_2d.py:157-162
      log_prior = -0.5 * L.n2 * ld[0] * c - 0.5 * L.n1 * ld[1] * c - 0.5 * quad;
    else             // model_GP_solver_1d.py:135-137
      log_prior = -0.5 * ld[0] * c - 0.5 * quad;
    const double log_b = 0.5 * Nb * log_tau - 0.5 * tau * bgap;
    const double eq_ll = 0.5 * Nc * log_v - 0.5 * v * egap;
    const double loss = -(log_prior + log_b * wb + eq_ll);
    sg[0] = wb * (-0.5 * Nb + 0.5 * tau * bgap);  // dL/dlog_tau
    sg[1] = -0.5 * Nc + 0.5 * v * egap;           // dL/dlog_v
    f.losses[slot] = loss;
    *f.loss_slot = slot + 1;
    double* diag = f.diag;
    diag[0] = loss; diag[1] = ld[0]; diag[2] = ld[1]; diag[3] = quad; diag[4] = egap; diag[5] = bgap;
    if (f.report) {  // this step's loss and the batch header (stepk.hip step_report_kernel's record)
      const StepReport& r = f.rep;
      r.out[8 + slot] = loss;
      r.out[0] = (double)__hip_atomic_load(const_cast<int*>(r.status), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r.out[1] = r.viol ? (double)__hip_atomic_load(const_cast<unsigned int*>(r.viol), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0.0;
      for (int a = 0; a < 2; ++a) {
        r.out[2 + 2 * a] = r.pst[a] ? r.pst[a][0] : 0.0;
        r.out[3 + 2 * a] = r.pst[a] ? r.pst[a][1] : 0.0;
      }
    }
  }
  if (do_loss && f.report) {  // the batch's earlier losses (written by earlier launches)
    for (int k = t; k < f.rep.nloss - 1; k += blockDim.x) f.rep.out[8 + k] = f.rep.losses[k];
    __threadfence_system();
  }
  __syncthreads();
  if (t == 0 && do_loss && f.report) report_ready(f.rep.out);  // after every thread's fence
  if (t == 0) FIN_PROBE(57);
  // ---- phase 2: gradients (kernel params: the fields were contracted without the weight w_q)
  // and Adam on the small parameters
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    if (pkind[r] < 0) continue;
    const double g = pkind[r] == 0 ? pgx[r] * pw[r] : sg[pkind[r] - 1];
    const int idx = pidx[r];
    f.grad[idx] = g;
    if (f.apply) {
      adam1(g, pp[r], pm[r], pv2[r], f.hyper, bc1, bc2);
      f.params[idx] = pp[r]; f.m[idx] = pm[r]; f.v[idx] = pv2[r];
    }
    if (f.kp_wt && pkind[r] == 0)  // global_store sc1 (write-through hand-off)
      __hip_atomic_store(f.kp_wt + (idx - L.off_small), pp[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// dL/dU and Adam on the solution grid.  2D: gU = S + v(X1 + X2)
//   [+ v(3U^2-1)R for Allen-Cahn] + w*tau*scatter(u_b - b);  1D: gu = alpha + v*beta [+...].
__device__ __forceinline__ void adam_u_elem(const AdamUArgs& A, int e) {
  const Layout& L = A.L;
  const double tau = A.sc->tau, v = A.sc->v, wt = A.llk_weight * tau;
  double g, u;
  size_t pi;
  if (L.dim == 2) {
    const int i = e / L.n2, j = e % L.n2;
    pi = (size_t)i * L.p2 + j;
    u = A.Up[pi];
    g = A.S[pi] + v * (A.X1[pi] + A.X2[pi]);
    if (A.ac) g += v * (3.0 * u * u - 1.0) * A.R[pi];
    const int n1 = L.n1, n2 = L.n2;
    if (i == 0) g += wt * (u - A.bvals[j]);
    if (i == n1 - 1) g += wt * (u - A.bvals[n2 + j]);
    if (j == 0) g += wt * (u - A.bvals[2 * n2 + i]);
    if (j == n2 - 1) g += wt * (u - A.bvals[2 * n2 + n1 + i]);
  } else {
    pi = e;
    u = A.Up[pi];
    g = A.X1[pi] + v * A.X2[pi];  // alpha + v*beta
    if (A.ac) {
      const double ua = u + (A.U0 ? A.U0[pi] : 0.0);
      g += v * (3.0 * ua * ua - 1.0) * A.R[pi];
    }
    for (int k = 0; k < A.nb; ++k)
      if (A.bidx[k] == e) g += wt * (u - A.bvals[k]);
  }
  const int idx = L.off_u + e;
  A.grad[idx] = g;
  if (A.apply) {
    double p = A.params[idx], m = A.m[idx], vv = A.v[idx];
    adam1(g, p, m, vv, A.hyper, A.sc->bc1, A.sc->bc2);
    A.params[idx] = p; A.m[idx] = m; A.v[idx] = vv;
    A.Up[pi] = p;
  }
}


__host__ __device__ inline int tail_nu(const Layout& L) { return (L.dim == 2) ? L.n1 * L.n2 : L.n1; }

}  // namespace gpk
