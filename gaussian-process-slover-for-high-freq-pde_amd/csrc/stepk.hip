// stepk.hip — loss assembly, deterministic reductions and on-device Adam (gfx950).
//
// Replaces the scalar tail of loss() and the optax.adam update of step():
//   code/model_GP_solver_2d.py:145-174 (loss), :176-183 (step: value_and_grad + adam)
//   code/model_GP_solver_1d.py:123-158
// Adam follows optax 0.1.4 scale_by_adam + scale(-lr) + apply_updates (eps_root = 0):
//   mu = (1-b1) g + b1 mu;  nu = (1-b2) g^2 + b2 nu;  t += 1
//   p += -lr * (mu/(1-b1^t)) / (sqrt(nu/(1-b2^t)) + eps)
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

__global__ void prep2_kernel(const double* __restrict__ params, int off0, int off1, int off_tau,
                             int off_v, int naxes, int q, AxisConst* kc, StepScalars* sc,
                             int* count, int apply, double b1, double b2) {
  const int t = threadIdx.x;
  for (int ax = 0; ax < naxes; ++ax) {
    const int off = ax == 0 ? off0 : off1;
    for (int c = t; c < q; c += blockDim.x) {
      kc[ax].om[c] = TWO_PI * params[off + c];      // freq
      kc[ax].a[c] = exp(params[off + q + c]);      // log-ls
      kc[ax].w[c] = exp(params[off + 2 * q + c]);  // log-w
    }
  }
  if (t == 0) {
    sc->tau = exp(params[off_tau]);
    sc->v = exp(params[off_v]);
    int n = *count + 1;
    if (apply) *count = n;
    sc->bc1 = 1.0 - pow(b1, (double)n);
    sc->bc2 = 1.0 - pow(b2, (double)n);
  }
}

hipError_t launch_prep2(const double* params, const Layout& L, AxisConst* kc, StepScalars* sc,
                        int* count, int apply, double b1, double b2, hipStream_t s) {
  hipLaunchKernelGGL(prep2_kernel, dim3(1), dim3(64), 0, s, params, L.off_kp[0], L.off_kp[1],
                     L.off_tau, L.off_v, L.naxes, L.q, kc, sc, count, apply, b1, b2);
  return hipGetLastError();
}

// out[axis][x] = sum_b part[(axis*bpa + b)*3*QMAX + x]   (fixed order: deterministic)
__global__ __launch_bounds__(256) void reduce_parts_kernel(const double* __restrict__ part, int bpa,
                                                           int q, double* out) {
  const int x = blockIdx.x, axis = blockIdx.y;
  const int qi = x % QMAX;
  __shared__ double s[4];
  double acc = 0.0;
  if (qi < q)
    for (int b = threadIdx.x; b < bpa; b += 256)
      acc += part[((size_t)axis * bpa + b) * (3 * QMAX) + x];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[axis * 3 * QMAX + x] = (s[0] + s[1]) + (s[2] + s[3]);
}

hipError_t launch_reduce_parts(const double* part, int bpa, int naxes, int q, double* out,
                               hipStream_t s) {
  hipLaunchKernelGGL(reduce_parts_kernel, dim3(3 * QMAX, naxes), dim3(256), 0, s, part, bpa, q, out);
  return hipGetLastError();
}

__device__ double block_sum(double v, double* sh) {
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
__global__ __launch_bounds__(256) void finalize_kernel(FinalizeArgs f) {
  __shared__ double sh[4];
  const int t = threadIdx.x;
  const Layout& L = f.L;
  double quad = 0.0, egap = 0.0, bgap = 0.0;
  for (int i = t; i < f.nquad; i += 256) quad += f.red_quad[i];
  for (int i = t; i < f.negap; i += 256) egap += f.red_egap[i];
  if (L.dim == 2) {
    // u_b = hstack(U[0,:], U[-1,:], U[:,0], U[:,-1])  (model_GP_solver_2d.py:126)
    const int n1 = L.n1, n2 = L.n2, nb = 2 * n2 + 2 * n1;
    for (int k = t; k < nb; k += 256) {
      int i, j;
      if (k < n2) { i = 0; j = k; }
      else if (k < 2 * n2) { i = n1 - 1; j = k - n2; }
      else if (k < 2 * n2 + n1) { i = k - 2 * n2; j = 0; }
      else { i = k - 2 * n2 - n1; j = n2 - 1; }
      const double r = f.Up[(size_t)i * L.p2 + j] - f.bvals[k];
      bgap += r * r;
    }
  } else {
    for (int k = t; k < f.nb; k += 256) {
      const double r = f.Up[f.bidx[k]] - f.bvals[k];
      bgap += r * r;
    }
  }
  quad = block_sum(quad, sh);
  egap = block_sum(egap, sh);
  bgap = block_sum(bgap, sh);

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

hipError_t launch_finalize(const FinalizeArgs& f, hipStream_t s) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, f);
  return hipGetLastError();
}

// dL/dU and Adam on the solution grid.  2D: gU = S + v(X1 + X2)
//   [+ v(3U^2-1)R for Allen-Cahn] + w*tau*scatter(u_b - b);  1D: gu = alpha + v*beta [+...].
__global__ __launch_bounds__(256) void adam_u_kernel(AdamUArgs A) {
  const Layout& L = A.L;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nu = (L.dim == 2) ? L.n1 * L.n2 : L.n1;
  if (e >= nu) return;
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
    if (A.ac) g += v * (3.0 * u * u - 1.0) * A.R[pi];
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

hipError_t launch_adam_u(const AdamUArgs& a, hipStream_t s) {
  const int nu = (a.L.dim == 2) ? a.L.n1 * a.L.n2 : a.L.n1;
  hipLaunchKernelGGL(adam_u_kernel, dim3((nu + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}

// params -> padded working copy of U (after gpk_set_params)
__global__ void sync_u_kernel(const double* __restrict__ params, Layout L, double* Up) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nu = (L.dim == 2) ? L.n1 * L.n2 : L.n1;
  if (e >= nu) return;
  if (L.dim == 2)
    Up[(size_t)(e / L.n2) * L.p2 + e % L.n2] = params[L.off_u + e];
  else
    Up[e] = params[L.off_u + e];
}

hipError_t launch_sync_u(const double* params, const Layout& L, double* Up, hipStream_t s) {
  const int nu = (L.dim == 2) ? L.n1 * L.n2 : L.n1;
  hipLaunchKernelGGL(sync_u_kernel, dim3((nu + 255) / 256), dim3(256), 0, s, params, L, Up);
  return hipGetLastError();
}

}  // namespace gpk
