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
#include "stepk_dev.h"

namespace gpk {

__global__ void prep2_kernel(const double* __restrict__ params, int off0, int off1, int off_tau,
                             int off_v, int naxes, int q, AxisConst* kc, StepScalars* sc,
                             int* count, int apply, double b1, double b2) {
  const int t = threadIdx.x;
  for (int ax = 0; ax < naxes; ++ax) {
    const int off = ax == 0 ? off0 : off1;
    for (int c = t; c < q; c += blockDim.x) {
      kc[ax].om[c] = TWO_PI * params[off + c];      // freq
      kc[ax].oml[c] = om_low(params[off + c], kc[ax].om[c]);
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

__global__ __launch_bounds__(256) void finalize_kernel(FinalizeArgs f) { finalize_body(f); }

hipError_t launch_finalize(const FinalizeArgs& f, hipStream_t s) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, f);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void adam_u_kernel(AdamUArgs A) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (A.e1 > 0 && (e < A.e0 || e >= A.e1)) return;  // another rank's rows
  if (e < tail_nu(A.L)) adam_u_elem(A, e);
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

namespace gpk {

// padded working copy of U -> flat params (row-sharded handles gather U rows into Up every step;
// the flat params are refreshed from it before they are read back)
__global__ void params_from_up_kernel(const double* __restrict__ Up, Layout L, double* params) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nu = L.n1 * L.n2;
  if (e >= nu) return;
  params[L.off_u + e] = Up[(size_t)(e / L.n2) * L.p2 + e % L.n2];
}

hipError_t launch_params_from_up(const double* Up, const Layout& L, double* params, hipStream_t s) {
  const int nu = L.n1 * L.n2;
  hipLaunchKernelGGL(params_from_up_kernel, dim3((nu + 255) / 256), dim3(256), 0, s, Up, L, params);
  return hipGetLastError();
}

// dst[i] += src[i]  (the in-process all-reduce of a local rank group)
__global__ void add_into_kernel(double* __restrict__ dst, const double* __restrict__ src, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] += src[i];
}

hipError_t launch_add_into(double* dst, const double* src, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(add_into_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

// Status word <-> two doubles (bit 1: non-positive pivot, bit 2: hand-off timeout), so that a
// summing all-reduce makes the status of a split-factor rank group group-wide (gpk_api.cpp
// split_broadcast): mode 0 packs, mode 1 ORs the summed bits back into the word.
__global__ void status_f64_kernel(int* st, double* x, int mode) {
  if (threadIdx.x != 0) return;
  if (mode == 0) {
    const int v = *st;
    x[0] = (v & 1) ? 1.0 : 0.0;
    x[1] = (v & 2) ? 1.0 : 0.0;
  } else {
    *st |= (x[0] > 0.0 ? 1 : 0) | (x[1] > 0.0 ? 2 : 0);
  }
}

hipError_t launch_status_f64(int* st, double* x, int mode, hipStream_t s) {
  hipLaunchKernelGGL(status_f64_kernel, dim3(1), dim3(64), 0, s, st, x, mode);
  return hipGetLastError();
}

// Start of a gpk_step batch, one launch instead of five copies / memsets: the rollback snapshot
// of params, m, v and the Adam count (snap != nullptr), the refinement-violation flag and the
// loss-ring slot zeroed.
__global__ __launch_bounds__(256) void step_begin_kernel(StepBegin b) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (b.snap && i < b.np) {
    b.snap[i] = b.params[i];
    b.snap[b.np + i] = b.m[i];
    b.snap[2 * b.np + i] = b.v[i];
  }
  if (i == 0) {
    if (b.snap) *b.snap_count = *b.count;
    if (b.viol) *b.viol = 0u;
    *b.loss_slot = 0;
  }
}

hipError_t launch_step_begin(const StepBegin& b, hipStream_t s) {
  const size_t n = b.snap ? b.np : 1;
  hipLaunchKernelGGL(step_begin_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b);
  return hipGetLastError();
}

// End of a batch: the status word, the violation flag, the refinement gates of both axes and the
// batch's losses in one record written straight into pinned host memory (no device-to-host copies)
__global__ void step_report_kernel(StepReport r) {
  for (int k = threadIdx.x; k < r.nloss; k += blockDim.x) r.out[8 + k] = r.losses[k];
  if (threadIdx.x == 0) {
    r.out[0] = (double)*r.status;
    r.out[1] = r.viol ? (double)*r.viol : 0.0;
    for (int a = 0; a < 2; ++a) {
      r.out[2 + 2 * a] = r.pst[a] ? r.pst[a][0] : 0.0;
      r.out[3 + 2 * a] = r.pst[a] ? r.pst[a][1] : 0.0;  // (bits of max diag K^{-1})
    }
  }
  __threadfence_system();  // every thread's record stores, then one barrier for the whole block
  __syncthreads();
  if (threadIdx.x == 0) report_ready(r.out);
}

hipError_t launch_step_report(const StepReport& r, hipStream_t s) {
  hipLaunchKernelGGL(step_report_kernel, dim3(1), dim3(256), 0, s, r);
  return hipGetLastError();
}

}  // namespace gpk
