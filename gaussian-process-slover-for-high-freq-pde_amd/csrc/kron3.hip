// kron3.hip — elementwise / reduction / tail kernels of the 3-axis Kronecker step (gfx950).
//
// the d > 2 generalisation of GP_solver_2d_single's log joint
// (code/model_GP_solver_2d.py:87-183; the 2-axis special case of the log-det weights :157-162)
// for K = K1 (x) K2 (x) K3 on a tensor grid.  The dense work (assembly, SPD inverses, the
// mode-k products as GEMMs over unfoldings) reuses the 2-axis kernels (gpk_kron3.cpp); this file
// holds what is 3-axis specific:
//   k3_prep      step constants: exp of the three axes' kernel params, tau, v, Adam count and
//                bias corrections, ||u_b - b||^2 over the six faces of U
//   k3_permute   mode-2 unfolding: T[i1][i2][i3] <-> Tp[i2][i1][i3] (padded grids)
//   k3_combine   R = U_xx + U_zz + permute(U_yy) - F [+ U(U^2-1)], S = permute(Sp), the permuted
//                copy Rp of R, and per-block partials of ||R||^2 and <U, S>
//   k3_finalize  loss, small-parameter gradients and Adam (one workgroup)
//   k3_adam_u    dL/dU = S + v (X1 + X2 + X3) [+ v(3U^2-1)R] + w tau scatter(u_b - b), Adam on U
// Grids are padded per axis to P_k (multiple of 32); pads of every tensor are zero.
#include "gpk_internal.h"
#include "gpk_kron3.h"
#include "prep_dev.h"
#include "stepk_dev.h"

namespace gpk {

__device__ __forceinline__ double k3_block_sum(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int t = threadIdx.x;
  __syncthreads();
  if ((t & 63) == 0) sh[t >> 6] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// the six faces' entry index of boundary value k (oracle boundary_3d order)
__device__ __forceinline__ void k3_face(const K3Geom& g, int k, int& i1, int& i2, int& i3) {
  const int n1 = g.n[0], n2 = g.n[1], n3 = g.n[2];
  const int f0 = n2 * n3, f2 = n1 * n3, f4 = n1 * n2;
  if (k < 2 * f0) {
    i1 = k < f0 ? 0 : n1 - 1;
    const int r = k % f0;
    i2 = r / n3; i3 = r % n3;
  } else if (k < 2 * f0 + 2 * f2) {
    const int kk = k - 2 * f0;
    i2 = kk < f2 ? 0 : n2 - 1;
    const int r = kk % f2;
    i1 = r / n3; i3 = r % n3;
  } else {
    const int kk = k - 2 * f0 - 2 * f2;
    i3 = kk < f4 ? 0 : n3 - 1;
    const int r = kk % f4;
    i1 = r / n2; i2 = r % n2;
  }
}

__global__ __launch_bounds__(256) void k3_prep_kernel(K3Prep P) {
  const int t = threadIdx.x;
  for (int ax = 0; ax < 3; ++ax)
    for (int c = t; c < P.q; c += 256) {
      const int off = P.off_kp[ax];
      P.kc[ax].om[c] = TWO_PI * P.params[off + c];
      P.kc[ax].oml[c] = om_low(P.params[off + c], P.kc[ax].om[c]);
      P.kc[ax].a[c] = exp(P.params[off + P.q + c]);
      P.kc[ax].w[c] = exp(P.params[off + 2 * P.q + c]);
    }
  if (t == 0) {
    P.sc->tau = exp(P.params[P.off_tau]);
    P.sc->v = exp(P.params[P.off_v]);
    const int n = *P.count + 1;
    if (P.apply) *P.count = n;
    P.sc->bc1 = 1.0 - pow(P.b1, (double)n);
    P.sc->bc2 = 1.0 - pow(P.b2, (double)n);
  }
  double acc = 0.0;
  for (int k = t; k < P.nb; k += 256) {
    int i1, i2, i3;
    k3_face(P.g, k, i1, i2, i3);
    const double d = P.Up[P.g.at(i1, i2, i3)] - P.bvals[k];
    acc += d * d;
  }
  __shared__ double sh[4];
  acc = k3_block_sum(acc, sh);
  if (t == 0) *P.bgap = acc;
}

// dst[i2][i1][i3] = src[i1][i2][i3] over the padded grid (rows of P3 stay contiguous)
__global__ __launch_bounds__(256) void k3_permute_kernel(const double* __restrict__ src,
                                                         double* __restrict__ dst, K3Geom g) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long tot = (long)g.p[0] * g.p[1] * g.p[2];
  if (e >= tot) return;
  const int i3 = (int)(e % g.p[2]);
  const long r = e / g.p[2];
  const int i2 = (int)(r % g.p[1]), i1 = (int)(r / g.p[1]);
  dst[g.atp(i1, i2, i3)] = src[e];
}

__global__ __launch_bounds__(256) void k3_combine_kernel(K3Combine C) {
  const K3Geom& g = C.g;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long tot = (long)g.p[0] * g.p[1] * g.p[2];
  double r2 = 0.0, us = 0.0;
  if (e < tot) {
    const int i3 = (int)(e % g.p[2]);
    const long rr = e / g.p[2];
    const int i2 = (int)(rr % g.p[1]), i1 = (int)(rr / g.p[1]);
    const size_t ep = g.atp(i1, i2, i3);
    const bool real = i1 < g.n[0] && i2 < g.n[1] && i3 < g.n[2];
    double R = 0.0, S = 0.0;
    if (real) {
      R = C.Rx[e] + C.Rz[e] + C.Ryp[ep] - C.F[e];
      const double u = C.Up[e];
      if (C.ac) R += u * (u * u - 1.0);
      S = C.Sp[ep];
      r2 = R * R;
      us = u * S;
    }
    C.R[e] = R;
    C.Rp[ep] = R;
    C.S[e] = S;
  }
  __shared__ double sh[4];
  r2 = k3_block_sum(r2, sh);
  us = k3_block_sum(us, sh);
  if (threadIdx.x == 0) {
    C.red_egap[blockIdx.x] = r2;
    C.red_quad[blockIdx.x] = us;
  }
}

// one workgroup: loss (model_GP_solver_2d.py:145-174 with three log-det weights), the small
// parameters' gradients and their Adam update (optax.adam, :179-182)
__global__ __launch_bounds__(256) void k3_finalize_kernel(K3Final F) {
  const int t = threadIdx.x;
  __shared__ double sh[4], sg[2];
  double quad = 0.0, egap = 0.0;
  for (int i = t; i < F.nred; i += 256) {
    quad += F.red_quad[i];
    egap += F.red_egap[i];
  }
  quad = k3_block_sum(quad, sh);
  egap = k3_block_sum(egap, sh);
  double ld[3];
  for (int a = 0; a < 3; ++a) {
    double x = 0.0;
    for (int k = t; k < F.nldet[a]; k += 256) x += F.ldet[a][k];
    ld[a] = k3_block_sum(x, sh);
  }
  const double tau = F.sc->tau, v = F.sc->v, bc1 = F.sc->bc1, bc2 = F.sc->bc2;
  const double wb = F.llk_weight, c = F.logdet;
  const double n1 = F.g.n[0], n2 = F.g.n[1], n3 = F.g.n[2];
  const double Nc = n1 * n2 * n3;
  const double Nb = 2.0 * (n2 * n3 + n1 * n3 + n1 * n2);
  const double log_tau = F.params[F.off_tau], log_v = F.params[F.off_v];
  if (t == 0) {
    const double bgap = *F.bgap;
    const double log_prior = -0.5 * c * (n2 * n3 * ld[0] + n1 * n3 * ld[1] + n1 * n2 * ld[2]) - 0.5 * quad;
    const double log_b = 0.5 * Nb * log_tau - 0.5 * tau * bgap;
    const double eq_ll = 0.5 * Nc * log_v - 0.5 * v * egap;
    const double loss = -(log_prior + log_b * wb + eq_ll);
    sg[0] = wb * (-0.5 * Nb + 0.5 * tau * bgap);
    sg[1] = -0.5 * Nc + 0.5 * v * egap;
    const int slot = *F.loss_slot;
    F.losses[slot] = loss;
    *F.loss_slot = slot + 1;
    F.diag[0] = loss; F.diag[1] = ld[0]; F.diag[2] = ld[1]; F.diag[3] = ld[2];
    F.diag[4] = quad; F.diag[5] = egap; F.diag[6] = bgap;
  }
  __syncthreads();
  for (int k = t; k < F.nsmall; k += 256) {
    const int idx = F.off_small + k;
    double g;
    if (idx == F.off_tau) {
      g = sg[0];
    } else if (idx == F.off_v) {
      g = sg[1];
    } else {
      const int a = idx >= F.off_kp[2] ? 2 : idx >= F.off_kp[1] ? 1 : 0;
      const int rr = idx - F.off_kp[a], ty = rr / F.q, cq = rr % F.q;  // freq, log-ls, log-w
      g = (ty == 0 && !F.has_cos) ? 0.0 : F.pg[a * 3 * QMAX + ty * QMAX + cq] * F.kc[a].w[cq];
    }
    F.grad[idx] = g;
    if (F.apply) {
      double p = F.params[idx], m = F.m[idx], vv = F.v[idx];
      adam1(g, p, m, vv, F.hyper, bc1, bc2);
      F.params[idx] = p; F.m[idx] = m; F.v[idx] = vv;
    }
  }
}

__global__ __launch_bounds__(256) void k3_adam_u_kernel(K3AdamU A) {
  const K3Geom& g = A.g;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long nu = (long)g.n[0] * g.n[1] * g.n[2];
  if (e >= nu) return;
  const int i3 = (int)(e % g.n[2]);
  const long rr = e / g.n[2];
  const int i2 = (int)(rr % g.n[1]), i1 = (int)(rr / g.n[1]);
  const size_t pi = g.at(i1, i2, i3), pp = g.atp(i1, i2, i3);
  const double tau = A.sc->tau, v = A.sc->v, wt = A.llk_weight * tau;
  const double u = A.Up[pi];
  double gr = A.S[pi] + v * (A.X1[pi] + A.X2p[pp] + A.X3[pi]);
  if (A.ac) gr += v * (3.0 * u * u - 1.0) * A.R[pi];
  const int n1 = g.n[0], n2 = g.n[1], n3 = g.n[2];
  const int f0 = n2 * n3, f2 = n1 * n3, f4 = n1 * n2;
  const int b2 = 2 * f0, b4 = 2 * f0 + 2 * f2;
  if (i1 == 0) gr += wt * (u - A.bvals[i2 * n3 + i3]);
  if (i1 == n1 - 1) gr += wt * (u - A.bvals[f0 + i2 * n3 + i3]);
  if (i2 == 0) gr += wt * (u - A.bvals[b2 + i1 * n3 + i3]);
  if (i2 == n2 - 1) gr += wt * (u - A.bvals[b2 + f2 + i1 * n3 + i3]);
  if (i3 == 0) gr += wt * (u - A.bvals[b4 + i1 * n2 + i2]);
  if (i3 == n3 - 1) gr += wt * (u - A.bvals[b4 + f4 + i1 * n2 + i2]);
  const long idx = A.off_u + e;
  A.grad[idx] = gr;
  if (A.apply) {
    double p = A.params[idx], m = A.m[idx], vv = A.v[idx];
    adam1(gr, p, m, vv, A.hyper, A.sc->bc1, A.sc->bc2);
    A.params[idx] = p; A.m[idx] = m; A.v[idx] = vv;
    A.Up[pi] = p;
  }
}

// flat params (U unpadded) -> padded working copy
__global__ __launch_bounds__(256) void k3_sync_u_kernel(const double* __restrict__ params, long off_u,
                                                        K3Geom g, double* __restrict__ Up) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long nu = (long)g.n[0] * g.n[1] * g.n[2];
  if (e >= nu) return;
  const int i3 = (int)(e % g.n[2]);
  const long rr = e / g.n[2];
  const int i2 = (int)(rr % g.n[1]), i1 = (int)(rr / g.n[1]);
  Up[g.at(i1, i2, i3)] = params[off_u + e];
}

static unsigned blocks_of(long n) { return (unsigned)((n + 255) / 256); }

hipError_t k3_launch_prep(const K3Prep& P, hipStream_t s) {
  hipLaunchKernelGGL(k3_prep_kernel, dim3(1), dim3(256), 0, s, P);
  return hipGetLastError();
}
hipError_t k3_launch_permute(const double* src, double* dst, const K3Geom& g, hipStream_t s) {
  hipLaunchKernelGGL(k3_permute_kernel, dim3(blocks_of(g.padded())), dim3(256), 0, s, src, dst, g);
  return hipGetLastError();
}
int k3_combine_blocks(const K3Geom& g) { return (int)blocks_of(g.padded()); }
hipError_t k3_launch_combine(const K3Combine& C, hipStream_t s) {
  hipLaunchKernelGGL(k3_combine_kernel, dim3(blocks_of(C.g.padded())), dim3(256), 0, s, C);
  return hipGetLastError();
}
hipError_t k3_launch_finalize(const K3Final& F, hipStream_t s) {
  hipLaunchKernelGGL(k3_finalize_kernel, dim3(1), dim3(256), 0, s, F);
  return hipGetLastError();
}
hipError_t k3_launch_adam_u(const K3AdamU& A, hipStream_t s) {
  hipLaunchKernelGGL(k3_adam_u_kernel, dim3(blocks_of(A.g.real())), dim3(256), 0, s, A);
  return hipGetLastError();
}
hipError_t k3_launch_sync_u(const double* params, long off_u, const K3Geom& g, double* Up, hipStream_t s) {
  hipLaunchKernelGGL(k3_sync_u_kernel, dim3(blocks_of(g.real())), dim3(256), 0, s, params, off_u, g, Up);
  return hipGetLastError();
}

}  // namespace gpk
