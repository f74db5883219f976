// stepk_dev.h — device bodies of the step tail (loss, small-parameter Adam, U Adam), shared by
// the standalone kernels (stepk.hip) and the fused tail of the parameter-gradient launch
// (pgrad.hip).  References: code/model_GP_solver_2d.py:145-183, code/model_GP_solver_1d.py:123-158.
#pragma once
#include "gpk_internal.h"
#include "stepk.h"

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

// Single-workgroup tail of the step: scalars, loss, small-parameter gradients + Adam.
__device__ inline void finalize_body(const FinalizeArgs& f) {
  __shared__ double sh[4];
  const int t = threadIdx.x;
  const Layout& L = f.L;
  double quad = 0.0, egap = 0.0, bgap = 0.0;
  for (int i = t; i < f.nquad; i += 256) quad += f.red_quad[i];
  for (int i = t; i < f.negap; i += 256) egap += f.red_egap[i];
  quad = block_sum(quad, sh);
  egap = block_sum(egap, sh);
  bgap = *f.bgap;  // boundary gap of U at the start of the step (assembly launch)
  if (t == 0 && f.viol)
    for (int a = 0; a < L.naxes; ++a)
      if (f.watch[a] && gate_open(f.watch[a])) atomicOr(f.viol, 1u);

  const double tau = f.sc->tau, v = f.sc->v;
  const double log_tau = f.params[L.off_tau], log_v = f.params[L.off_v];
  const double wb = f.llk_weight, c = f.logdet;
  if (t == 0) {
    double ld[2] = {0.0, 0.0};
    for (int a = 0; a < L.naxes; ++a)
      for (int k = 0; k < f.nldet[a]; ++k) ld[a] += f.ldet[a][k];
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
    f.grad[L.off_tau] = wb * (-0.5 * Nb + 0.5 * tau * bgap);
    f.grad[L.off_v] = -0.5 * Nc + 0.5 * v * egap;
    const int slot = *f.loss_slot;
    f.losses[slot] = loss;
    *f.loss_slot = slot + 1;
    double* diag = f.diag;
    diag[0] = loss; diag[1] = ld[0]; diag[2] = ld[1]; diag[3] = quad; diag[4] = egap; diag[5] = bgap;
  }
  // kernel-parameter gradients: fields were contracted without the weight w_q
  for (int a = 0; a < L.naxes; ++a) {
    const double* pg = f.pg + a * 3 * QMAX;
    for (int k = t; k < L.q; k += 256) {
      const double w = f.kc[a].w[k];
      const int off = L.off_kp[a];
      f.grad[off + k] = f.has_cos ? pg[k] * w : 0.0;          // freq
      f.grad[off + L.q + k] = pg[QMAX + k] * w;                // log-ls
      f.grad[off + 2 * L.q + k] = pg[2 * QMAX + k] * w;        // log-w
    }
  }
  __syncthreads();
  if (f.apply) {
    const double bc1 = f.sc->bc1, bc2 = f.sc->bc2;
    for (int k = t; k < L.nsmall; k += 256) {
      const int idx = L.off_small + k;
      double p = f.params[idx], m = f.m[idx], vv = f.v[idx];
      adam1(f.grad[idx], p, m, vv, f.hyper, bc1, bc2);
      f.params[idx] = p; f.m[idx] = m; f.v[idx] = vv;
    }
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
