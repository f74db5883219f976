// gpk_kron3.h — argument blocks of the 3-axis Kronecker step's own kernels (kron3.hip).
#pragma once
#include "gpk_internal.h"
#include "stepk.h"

namespace gpk {

// Tensor grid: true sizes n[k], padded sizes p[k] (multiples of 32).  A grid tensor is stored
// row-major [p1][p2][p3]; its mode-2 permutation (the mode-2 unfolding, contiguous) [p2][p1][p3].
struct K3Geom {
  int n[3], p[3];
  __host__ __device__ size_t at(int i1, int i2, int i3) const {
    return ((size_t)i1 * p[1] + i2) * p[2] + i3;
  }
  __host__ __device__ size_t atp(int i1, int i2, int i3) const {
    return ((size_t)i2 * p[0] + i1) * p[2] + i3;
  }
  __host__ __device__ long padded() const { return (long)p[0] * p[1] * p[2]; }
  __host__ __device__ long real() const { return (long)n[0] * n[1] * n[2]; }
};

struct K3Prep {
  K3Geom g;
  const double* params;
  int off_kp[3], off_tau, off_v, q;
  AxisConst* kc;        // out [3]
  StepScalars* sc;      // out
  int* count;
  int apply;
  double b1, b2;
  const double* Up; const double* bvals; int nb;
  double* bgap;         // out [1]
};

struct K3Combine {
  K3Geom g;
  const double *Rx, *Rz, *Ryp, *F, *Up, *Sp;  // U_xx, U_zz (natural), U_yy, S (permuted)
  int ac;
  double *R, *Rp, *S;                         // out: R (natural and permuted), S (natural)
  double *red_egap, *red_quad;                // out: per-block partials
};

struct K3Final {
  K3Geom g;
  AdamHyper hyper;
  double llk_weight, logdet;
  int apply, has_cos, q;
  const double* red_quad; const double* red_egap; int nred;
  const double* ldet[3]; int nldet[3];
  const double* pg;          // [3][3*QMAX]
  const AxisConst* kc;
  const StepScalars* sc;
  const double* bgap;
  int off_kp[3], off_tau, off_v, off_small, nsmall;
  double *params, *grad, *m, *v;
  double* losses; int* loss_slot;
  double* diag;              // [8]: loss, logdet1..3, quad, egap, bgap
};

struct K3AdamU {
  K3Geom g;
  AdamHyper hyper;
  double llk_weight;
  int apply, ac;
  const StepScalars* sc;
  const double *S, *X1, *X2p, *X3, *R;  // X2 in the permuted layout
  double* Up;
  const double* bvals;
  long off_u;
  double *params, *grad, *m, *v;
};

hipError_t k3_launch_prep(const K3Prep& P, hipStream_t s);
hipError_t k3_launch_permute(const double* src, double* dst, const K3Geom& g, hipStream_t s);
int k3_combine_blocks(const K3Geom& g);
hipError_t k3_launch_combine(const K3Combine& C, hipStream_t s);
hipError_t k3_launch_finalize(const K3Final& F, hipStream_t s);
hipError_t k3_launch_adam_u(const K3AdamU& A, hipStream_t s);
hipError_t k3_launch_sync_u(const double* params, long off_u, const K3Geom& g, double* Up, hipStream_t s);

}  // namespace gpk
