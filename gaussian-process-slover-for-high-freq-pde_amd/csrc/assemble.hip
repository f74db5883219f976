// assemble.hip — fused covariance + derivative-covariance block assembly (gfx950).
//
// Replaces, per axis and per step,
//   K  = vmap(kappa)(X1, X2) + jitter*I         code/kernel_matrix.py:21-30
//   D  = vmap(DD_x1_kappa) or vmap(D_x1_kappa)  code/model_GP_solver_2d.py:107-117,
//                                               code/model_GP_solver_advection.py:107-117
// with closed-form fields instead of nested jax.grad.
//
// Design: d = |x_i - x_j| is exactly symmetric, so K and DD are bitwise symmetric and D_x1
// bitwise antisymmetric.  One workgroup computes a 32x32 tile of the LOWER tile triangle and
// writes it twice (direct + LDS-transposed mirror): half the exp/sincos work of a full
// sweep.  Every thread evaluates 4 elements x Q components; per-axis constants (w, a, 2*pi*f)
// sit in LDS.  Pads (i or j >= n) are written as identity (K) / zero (D) so the padded SPD
// inverse stays block-diagonal.
#include "gpk_internal.h"

namespace gpk {

template <bool MATERN, bool COS, int DERIV>
__device__ __forceinline__ void eval_kd(double diff, const double* w, const double* a,
                                        const double* om, int q, double& K, double& D) {
  double d = fabs(diff);
  double k = 0.0, dv = 0.0;
  for (int c = 0; c < q; ++c) {
    double m0, m1, m2;
    radial<MATERN>(d, a[c], m0, m1, m2);
    if (COS) {
      double S, C;
      sincos(om[c] * d, &S, &C);
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
  // JAX abs JVP: select(x >= 0, g, -g) -> sign(0) = +1
  D = (DERIV == 1) ? (diff >= 0.0 ? dv : -dv) : dv;
}

struct AssembleBatch {
  AssembleArgs ax[2];
  int tiles[2];   // lower-triangle tile count per axis
};

template <bool MATERN, bool COS, int DERIV>
__global__ __launch_bounds__(256) void assemble_kernel(AssembleBatch b, int q) {
  const int axis = blockIdx.y;
  const AssembleArgs& A = b.ax[axis];
  int tile = blockIdx.x;
  if (tile >= b.tiles[axis]) return;
  // lower-triangle tile index -> (I, J), I >= J
  int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= tile) ++I;
  while (I * (I + 1) / 2 > tile) --I;
  int J = tile - I * (I + 1) / 2;

  __shared__ double sw[QMAX], sa[QMAX], so[QMAX];
  __shared__ double tK[32][33], tD[32][33];
  const int t = threadIdx.x;
  if (t < q) {
    sw[t] = A.kc->w[t];
    sa[t] = A.kc->a[t];
    so[t] = A.kc->om[t];
  }
  __syncthreads();
  const int tx = t & 31, ty = t >> 5;
  const int j = J * 32 + tx;
  const double xj = j < A.n ? A.x[j] : 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int li = ty + 8 * r;
    const int i = I * 32 + li;
    double kv, dv;
    if (i < A.n && j < A.n) {
      eval_kd<MATERN, COS, DERIV>(A.x[i] - xj, sw, sa, so, q, kv, dv);
      if (i == j) kv += A.jitter;
    } else {
      kv = (i == j) ? 1.0 : 0.0;
      dv = 0.0;
    }
    A.K[(size_t)i * A.p + j] = kv;
    if (DERIV) A.D[(size_t)i * A.p + j] = dv;
    tK[li][tx] = kv;
    tD[li][tx] = dv;
  }
  if (I == J) return;  // block-uniform
  __syncthreads();
  // mirror tile (J, I): element (J*32+row, I*32+col) = tile(I,J)[col][row]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = ty + 8 * r;
    const size_t o = (size_t)(J * 32 + row) * A.p + I * 32 + tx;
    A.K[o] = tK[tx][row];
    if (DERIV == 2) A.D[o] = tD[tx][row];
    if (DERIV == 1) A.D[o] = -tD[tx][row];  // D_x1 is antisymmetric (pads are 0 either way)
  }
}

// rectangular block (preds' Kmn, gpk_kernel_matrices): no symmetry assumed
template <bool MATERN, bool COS, int DERIV>
__global__ __launch_bounds__(256) void cross_kernel(const double* __restrict__ xr, int nr,
                                                    const double* __restrict__ xc, int nc, int ld,
                                                    const AxisConst* kc, int q, double jitter,
                                                    double* K, double* D) {
  __shared__ double sw[QMAX], sa[QMAX], so[QMAX];
  const int t = threadIdx.x;
  if (t < q) {
    sw[t] = kc->w[t];
    sa[t] = kc->a[t];
    so[t] = kc->om[t];
  }
  __syncthreads();
  const int j = blockIdx.x * 64 + (t & 63);
  const int i = blockIdx.y * 4 + (t >> 6);
  if (i >= nr || j >= nc) return;
  double kv, dv;
  eval_kd<MATERN, COS, DERIV>(xr[i] - xc[j], sw, sa, so, q, kv, dv);
  if (i == j) kv += jitter;
  K[(size_t)i * ld + j] = kv;
  if (DERIV) D[(size_t)i * ld + j] = dv;
}

template <bool MATERN, bool COS>
static void launch_assemble_t(const AssembleBatch& b, int naxes, int maxt, int q, int deriv,
                              hipStream_t s) {
  dim3 grid(maxt, naxes);
  if (deriv == 2)
    hipLaunchKernelGGL((assemble_kernel<MATERN, COS, 2>), grid, dim3(256), 0, s, b, q);
  else if (deriv == 1)
    hipLaunchKernelGGL((assemble_kernel<MATERN, COS, 1>), grid, dim3(256), 0, s, b, q);
  else
    hipLaunchKernelGGL((assemble_kernel<MATERN, COS, 0>), grid, dim3(256), 0, s, b, q);
}

hipError_t launch_assemble(int kind, int q, const AssembleArgs* a, int naxes, hipStream_t s) {
  AssembleBatch b{};
  int maxt = 0;
  for (int k = 0; k < naxes; ++k) {
    b.ax[k] = a[k];
    int T = a[k].p / 32;
    b.tiles[k] = T * (T + 1) / 2;
    if (b.tiles[k] > maxt) maxt = b.tiles[k];
  }
  int deriv = a[0].deriv;
  switch (kind) {
    case SE_COS: launch_assemble_t<false, true>(b, naxes, maxt, q, deriv, s); break;
    case MATERN52_COS: launch_assemble_t<true, true>(b, naxes, maxt, q, deriv, s); break;
    case SE: launch_assemble_t<false, false>(b, naxes, maxt, q, deriv, s); break;
    default: launch_assemble_t<true, false>(b, naxes, maxt, q, deriv, s); break;
  }
  return hipGetLastError();
}

template <bool MATERN, bool COS>
static void launch_cross_t(const double* xr, int nr, const double* xc, int nc, int ld,
                           const AxisConst* kc, int q, double jitter, int deriv, double* K,
                           double* D, hipStream_t s) {
  dim3 grid((nc + 63) / 64, (nr + 3) / 4);
  if (deriv == 2)
    hipLaunchKernelGGL((cross_kernel<MATERN, COS, 2>), grid, dim3(256), 0, s, xr, nr, xc, nc, ld,
                       kc, q, jitter, K, D);
  else if (deriv == 1)
    hipLaunchKernelGGL((cross_kernel<MATERN, COS, 1>), grid, dim3(256), 0, s, xr, nr, xc, nc, ld,
                       kc, q, jitter, K, D);
  else
    hipLaunchKernelGGL((cross_kernel<MATERN, COS, 0>), grid, dim3(256), 0, s, xr, nr, xc, nc, ld,
                       kc, q, jitter, K, D);
}

hipError_t launch_cross(int kind, int q, const double* xr, int nr, const double* xc, int nc,
                        int ld, const AxisConst* kc, double jitter, int deriv, double* K,
                        double* D, hipStream_t s) {
  switch (kind) {
    case SE_COS: launch_cross_t<false, true>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
    case MATERN52_COS: launch_cross_t<true, true>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
    case SE: launch_cross_t<false, false>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
    default: launch_cross_t<true, false>(xr, nr, xc, nc, ld, kc, q, jitter, deriv, K, D, s); break;
  }
  return hipGetLastError();
}

}  // namespace gpk
