// prep_dev.h — the step constants, computed on device at the start of a step by one
// workgroup of the step's first (or, with the chain inverse, second) launch: the exp of the
// kernel parameters per axis, tau, v, the Adam step count and bias corrections, and the
// boundary gap of U before the step's update (code/model_GP_solver_2d.py:123-128, 179-182).
#pragma once
#include "gpk_internal.h"

namespace gpk {

// exp of the params -> axis constants of component c (prep2 semantics, bitwise)
__device__ __forceinline__ void axis_component(const PrepArgs& P, int axis, int q, int c, double& w,
                                               double& a, double& om, double& oml) {
  const int off = P.off_kp[axis];
  const double f = P.params[off + c];       // freq
  om = TWO_PI * f;
  oml = om_low(f, om);
  a = exp(P.params[off + q + c]);           // log-ls
  w = exp(P.params[off + 2 * q + c]);       // log-w
}

// the rollback snapshot of a folded batch begin (PrepArgs.snap), spread over nwg workgroups
__device__ inline void copy_snapshot(const PrepArgs& P, int wg, int nwg) {
  if (!P.snap) return;
  const size_t np = P.snap_np;
  for (size_t i = (size_t)wg * blockDim.x + threadIdx.x; i < np; i += (size_t)nwg * blockDim.x) {
    P.snap[i] = P.params[i];
    P.snap[np + i] = P.snap_m[i];
    P.snap[2 * np + i] = P.snap_v[i];
  }
}

// Part w of the boundary gap ||u_b - b||^2 (u_b = hstack(U[0,:], U[-1,:], U[:,0], U[:,-1]) in
// 2D, u[Xind] in 1D; PrepArgs::bgap): entries w BGAP_CHUNK + [0, BGAP_CHUNK), then every
// bgap_parts chunks; 8 entries per thread per chunk, their loads issued before the sums; fixed
// order (thread sums, wave butterflies, waves in order).  One part: the whole sum.  Every caller
// runs 256-thread workgroups (BGAP_CHUNK = 8 x 256).
__device__ inline void bgap_part(const PrepArgs& P, int w) {
  const int t = threadIdx.x;
  const int parts = P.bgap_parts > 0 ? P.bgap_parts : 1;
  double acc = 0.0;
  if (P.dim == 2) {
    const int n1 = P.n1, n2 = P.n2, nb = 2 * n2 + 2 * n1;
    for (int k0 = w * BGAP_CHUNK + t; k0 < nb; k0 += parts * BGAP_CHUNK) {
      double uu[8], bb[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int k = k0 + r * 256;
        const bool ok = k < nb && k < (k0 - t) + BGAP_CHUNK;
        int i, j;
        if (k < n2) { i = 0; j = k; }
        else if (k < 2 * n2) { i = n1 - 1; j = k - n2; }
        else if (k < 2 * n2 + n1) { i = k - 2 * n2; j = 0; }
        else { i = k - 2 * n2 - n1; j = n2 - 1; }
        uu[r] = ok ? P.Up[(size_t)i * P.p2 + j] : 0.0;
        bb[r] = ok ? P.bvals[k] : 0.0;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const double d = uu[r] - bb[r];
        acc += d * d;
      }
    }
  } else if (w == 0) {
    for (int k = t; k < P.nb; k += blockDim.x) {
      const double r = P.Up[P.bidx[k]] - P.bvals[k];
      acc += r * r;
    }
  }
  __shared__ double sb[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((t & 63) == 0) sb[t >> 6] = acc;
  __syncthreads();
  if (t == 0) P.bgap[w] = (sb[0] + sb[1]) + (sb[2] + sb[3]);
  __syncthreads();  // (sb reused by the next part)
}

// workgroup (0, 0): publish the step constants for the later kernels of the step, and every
// part of the boundary gap unless the caller spreads them over its workgroups (bgap_all false:
// class_eval_kernel)
__device__ inline void publish_prep(const PrepArgs& P, int q, bool bgap_all = true) {
  if (P.skip) return;  // published by another launch of the step
  const int t = threadIdx.x;
  for (int ax = 0; ax < P.naxes; ++ax)
    for (int c = t; c < q; c += blockDim.x) {
      double w, a, om, oml;
      axis_component(P, ax, q, c, w, a, om, oml);
      P.kc[ax].om[c] = om;
      P.kc[ax].oml[c] = oml;
      P.kc[ax].a[c] = a;
      P.kc[ax].w[c] = w;
    }
  if (t == 0) {
    P.sc->tau = exp(P.params[P.off_tau]);
    P.sc->v = exp(P.params[P.off_v]);
    const int c0 = *P.count, n = c0 + 1;
    if (P.snap_count) *P.snap_count = c0;
    if (P.viol0) *P.viol0 = 0u;
    if (P.slot0) *P.slot0 = 0;
    if (P.apply) *P.count = n;
    P.sc->bc1 = 1.0 - pow(P.b1, (double)n);
    P.sc->bc2 = 1.0 - pow(P.b2, (double)n);
  }
  if (P.bgap && bgap_all)
    for (int w = 0; w < (P.bgap_parts > 0 ? P.bgap_parts : 1); ++w) bgap_part(P, w);
}

}  // namespace gpk
