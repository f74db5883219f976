// prep_dev.h — the step constants, computed on device at the start of a step by one
// workgroup of the step's first (or, with the chain inverse, second) launch: the exp of the
// kernel parameters per axis, tau, v, the Adam step count and bias corrections, and the
// boundary gap of U before the step's update (code/model_GP_solver_2d.py:123-128, 179-182).
#pragma once
#include "gpk_internal.h"

namespace gpk {

// exp of the params -> axis constants of component c (prep2 semantics, bitwise)
// (from the values: freq f, log-ls ll, log-w lw)
__device__ __forceinline__ void axis_component_v(double f, double ll, double lw, double& w, double& a,
                                                 double& om, double& oml) {
  om = TWO_PI * f;
  oml = om_low(f, om);
  a = exp(ll);
  w = exp(lw);
}

__device__ __forceinline__ void axis_component(const PrepArgs& P, int axis, int q, int c, double& w,
                                               double& a, double& om, double& oml) {
  const int off = P.off_kp[axis];
  axis_component_v(P.params[off + c], P.params[off + q + c], P.params[off + 2 * q + c], w, a, om, oml);
}

// Partial sums over components c = c0, c0 + cs, ... (cs = stride) of K and D at one pair.
template <bool MATERN, bool COS, int DERIV>
__device__ __forceinline__ void eval_kd_part(double diff, const double* w, const double* a,
                                             const double* om, const double* oml, int c0, int cs,
                                             int q, double& K, double& D) {
  double d = fabs(diff);
  double k = 0.0, dv = 0.0;
  for (int c = c0; c < q; c += cs) {
    double m0, m1, m2;
    radial<MATERN>(d, a[c], m0, m1, m2);
    if (COS) {
      double S, C;
      phase_sincos(om[c], oml[c], d, S, C);
      double o = om[c];
      k += w[c] * (m0 * C);
      if (DERIV == 2) dv += w[c] * (m2 * C - 2.0 * m1 * (o * S) - m0 * (o * o * C));
      if (DERIV == 1) dv += w[c] * (m1 * C - m0 * (o * S));
    } else {
      k += w[c] * m0;
      if (DERIV == 2) dv += w[c] * m2;
      if (DERIV == 1) dv += w[c] * m1;
    }
  }
  K = k;
  D = dv;  // unsigned: the D_x1 sign s_ij is applied by the caller
}

// Class u's values (class_eval_kernel; pgrad.hip next_class_values): K and the derivative field
// at the class distance d, one mixture component per lane of a 32-lane half-wave (component c
// and c + 32, ...), the terms added by a fixed xor butterfly (deterministic); lane 0 stores.
template <bool MATERN, bool COS, int DERIV>
__device__ __forceinline__ void class_value_store(const ClassArgs& C, int u, double d, const double* sw,
                                                  const double* sa, const double* so,
                                                  const double* sol, int q) {
  const int c = threadIdx.x & 31;
  double kv = 0.0, dv = 0.0;
  if (u < C.ncls) eval_kd_part<MATERN, COS, DERIV>(d, sw, sa, so, sol, c, 32, q, kv, dv);
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    kv += __shfl_xor(kv, o, 64);
    dv += __shfl_xor(dv, o, 64);
  }
  if (c == 0 && u < C.ncls) {
    C.kval[u] = kv;
    C.dval[u] = dv;
  }
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
    if (P.nce_flag) *P.nce_flag = 0u;
    if (P.apply) *P.count = n;
    P.sc->bc1 = 1.0 - pow(P.b1, (double)n);
    P.sc->bc2 = 1.0 - pow(P.b2, (double)n);
  }
  if (P.bgap && bgap_all)
    for (int w = 0; w < (P.bgap_parts > 0 ? P.bgap_parts : 1); ++w) bgap_part(P, w);
}

}  // namespace gpk
